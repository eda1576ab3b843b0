set -u
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/t_gpu.txt; exit 1; }
tail -2 gpurun_out/t_gpu.txt
timeout -k 10 300 python bench.py > gpurun_out/b_main.json 2> gpurun_out/b_main.err || { echo "bench failed"; tail gpurun_out/b_main.err; exit 1; }
cat gpurun_out/b_main.json
rm -rf gpurun_out/prof_cur
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cur -o run --output-format csv -- python bench.py --inflight 1 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b_prof.json 2> gpurun_out/b_prof.err || { echo "rocprof failed"; tail gpurun_out/b_prof.err; exit 1; }
f=$(find gpurun_out/prof_cur -name "*kernel_trace.csv" | head -1)
python3 tools/rocprof_summary.py "$f" > gpurun_out/prof_cur_summary.txt
head -70 gpurun_out/prof_cur_summary.txt
