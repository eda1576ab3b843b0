# one-barrier stem: bit-identity tests, bench A/B, rocprof of the one-barrier variants
set -u
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread -k "stem_one_barrier" > gpurun_out/t_stem3.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_stem3.txt; exit 1; }
tail -1 gpurun_out/t_stem3.txt
bash tools/ab_env.sh SFA_TUNE=0,SFA_TUNE=262144,SFA_TUNE=524288 || exit 1
for T in 262144 524288; do
SFA_TUNE=$T timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stem3_$T -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b_stem3_$T.json 2> gpurun_out/b_stem3_$T.err || { echo "rocprof failed"; tail gpurun_out/b_stem3_$T.err; exit 1; }
f=$(find gpurun_out/prof_stem3_$T -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if "stem" in r["Name"]:
        print("%-80s %6s %10.1f us" % (r["Name"][:80], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
