# FPN skip convs: residual taps before the K loop (tune bit 1048576) vs in the epilogue: test, bench A/B,
# rocprof single flight of both (GPU box)
set -u
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread -k "prefetch or residual" > gpurun_out/t_rup.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_rup.txt; exit 1; }
tail -1 gpurun_out/t_rup.txt
bash tools/ab_env.sh SFA_TUNE=0,SFA_TUNE=1048576
for t in 0 1048576; do
  SFA_TUNE=$t timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rup_$t -o run --output-format csv -- python bench.py --inflight 1 --steps 20 --warmup 3 --no-cpu-baseline --probe-forwards 0 > gpurun_out/bp_rup_$t.json 2> gpurun_out/bp_rup_$t.err || { echo "rocprof failed"; exit 1; }
  f=$(find gpurun_out/prof_rup_$t -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$t" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "35072" in r["Name"] or "4229376" in r["Name"] or "4229440" in r["Name"] or "4194304" in r["Name"]:
        print(sys.argv[2], "%-100s %5s %8.1f us" % (r["Name"][:100], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
echo done
