# grouped heads (SFA_HEADS_GROUPED): bit-identity tests, bench A/B interleaved (value, single-flight
# forward, heads roofline), rocprof single-flight kernel summary with grouped heads (GPU box)
set -u
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread -k "grouped or probe or stagger" > gpurun_out/t_grp.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_grp.txt; exit 1; }
tail -1 gpurun_out/t_grp.txt
for rep in 1 2; do
  for g in 0 1; do
    SFA_HEADS_GROUPED=$g timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/grp_${g}_$rep.json 2> gpurun_out/grp_$g.err || { echo "bench failed: $g"; tail -3 gpurun_out/grp_$g.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('grouped', sys.argv[2], d['value'], d['stages_ms']['forward'], r['frac'], r['launch_us'])" gpurun_out/grp_${g}_$rep.json $g
  done
done
SFA_HEADS_GROUPED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_grp -o run --output-format csv -- python bench.py --inflight 1 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bp_grp.json 2> gpurun_out/bp_grp.err || { echo "rocprof failed"; exit 1; }
python3 tools/rocprof_summary.py $(find gpurun_out/prof_grp -name "*kernel_trace.csv" | head -1) > gpurun_out/prof_grp_summary.txt 2>&1 || true
head -30 gpurun_out/prof_grp_summary.txt
echo done
