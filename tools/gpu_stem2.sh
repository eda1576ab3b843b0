# stem v2: bit-identity tests, then the bench A/B (default / old stem / MFMAs-first variant) and a rocprof summary
set -u
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread -k "stem or fpn or round2" > gpurun_out/t_stem2.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_stem2.txt; exit 1; }
tail -1 gpurun_out/t_stem2.txt
bash tools/ab_env.sh SFA_TUNE=0,SFA_TUNE=262144,SFA_TUNE=524288,SFA_TUNE=1048576 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stem2 -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b_stem2.json 2> gpurun_out/b_stem2.err || { echo "rocprof failed"; tail gpurun_out/b_stem2.err; exit 1; }
f=$(find gpurun_out/prof_stem2 -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:24]:
    print("%-110s %6s %10.1f us" % (r["Name"][:110], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
