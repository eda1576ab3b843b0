# quick loop: selected GPU tests, the default bench, a single-flight rocprof kernel summary
# usage: bash tools/gpu_quick.sh TAG "pytest -k expression or test files"
set -u
export TMPDIR=/tmp
TAG="${1:-q}"
TESTS="${2:-tests}"
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tq_$TAG.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/tq_$TAG.txt; exit 1; }
tail -1 gpurun_out/tq_$TAG.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bq_$TAG.json 2> gpurun_out/bq_$TAG.err || { echo "bench failed"; tail gpurun_out/bq_$TAG.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('value', d['value'], 'fwd', d['stages_ms'], 'heads', d['roofline'].get('launch_us'))" gpurun_out/bq_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profq_$TAG -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bpq_$TAG.json 2> gpurun_out/bpq_$TAG.err || { echo "rocprof failed"; tail gpurun_out/bpq_$TAG.err; exit 1; }
f=$(find gpurun_out/profq_$TAG -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:40]:
    print("%-110s %6s %10.1f us" % (r["Name"][:110], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
