# stream workload variants: steps in flight x HIP graph (run on the GPU box)
set -u
export TMPDIR=/tmp
for v in "--inflight 1 --no-graph" "--inflight 1" "--inflight 2 --no-graph" "--inflight 2"; do
  timeout -k 10 300 python bench.py --workload stream --no-cpu-baseline $v > gpurun_out/sv.json 2> gpurun_out/sv.err || { echo "failed: $v"; tail -3 gpurun_out/sv.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/sv.json')); print(sys.argv[1], d['value'], d['ms_per_step'])" "$v"
done
