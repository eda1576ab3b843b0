set -u
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_h3m -o run --output-format csv -- python bench.py --inflight 1 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b_prof.json 2> gpurun_out/b_prof.err || { echo "rocprof failed"; tail gpurun_out/b_prof.err; exit 1; }
f=$(find gpurun_out/prof_h3m -name "*kernel_trace.csv" | head -1)
python3 tools/rocprof_summary.py "$f" > gpurun_out/prof_h3m_summary.txt
cat gpurun_out/prof_h3m_summary.txt | head -80
