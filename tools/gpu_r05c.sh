# round 5: in-kernel split-K combine (tickets) — isolated A/B, tests, bench A/B
set -u
export TMPDIR=/tmp
timeout -k 10 120 ./tools/convbench5 20 layer4 > gpurun_out/r05c_convbench5.txt 2>&1 || { echo "convbench5 failed"; tail -20 gpurun_out/r05c_convbench5.txt; exit 1; }
cat gpurun_out/r05c_convbench5.txt
timeout -k 10 600 python -u -m pytest tests/test_abi.py tests/test_gpu_model.py tests/test_gpu_bench_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05c_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05c_tests.txt; exit 1; }
tail -2 gpurun_out/r05c_tests.txt
bash tools/ab_env.sh SFA_SPLITK_TICKETS=0,SFA_SPLITK_TICKETS=1 || exit 1
rm -rf gpurun_out/prof_r05c
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05c -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bp_r05c.json 2> gpurun_out/bp_r05c.err || { echo "rocprof failed"; exit 1; }
python3 tools/rocprof_summary.py "$(ls gpurun_out/prof_r05c/*kernel_trace.csv | head -1)" > gpurun_out/prof_summary_r05c.txt
grep -A9 "^# per-stage" gpurun_out/prof_summary_r05c.txt
echo done
