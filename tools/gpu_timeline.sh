# kernel trace of the default bench (2 steps in flight, graphs) -> busy fraction / concurrency
set -u
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl -o run --output-format csv -- python bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/tl_bench.json 2> gpurun_out/tl_bench.err || { echo "rocprof failed"; tail gpurun_out/tl_bench.err; exit 1; }
f=$(find gpurun_out/tl -name "*kernel_trace.csv" | head -1)
python3 tools/timeline_busy.py "$f" 0 > gpurun_out/tl_summary.txt
cat gpurun_out/tl_summary.txt
# side-stream priority A/B (SFA_SIDE_PRIO: 1 = lowest, -1 = highest, 0 = default)
bash tools/ab_env.sh SFA_SIDE_PRIO=0,SFA_SIDE_PRIO=1,SFA_SIDE_PRIO=-1
