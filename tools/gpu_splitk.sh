set -u
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bench_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_splitk.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/t_splitk.txt; exit 1; }
tail -1 gpurun_out/t_splitk.txt
bash tools/ab_env.sh SFA_TUNE=1024,SFA_TUNE=0,SFA_TUNE=3072
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_splitk -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bp_splitk.json 2> gpurun_out/bp_splitk.err || { echo "rocprof failed"; exit 1; }
echo done
