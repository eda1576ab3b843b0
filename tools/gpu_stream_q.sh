# stream workload: pipelines in flight x side streams x hardware queues, interleaved twice (GPU box)
set -u
export TMPDIR=/tmp
run() {  # label, env..., -- bench args
  local label="$1"; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py --workload stream --no-cpu-baseline "$@" > gpurun_out/sq.json 2> gpurun_out/sq.err || { echo "failed: $label"; tail -3 gpurun_out/sq.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/sq.json')); print(sys.argv[1], d['value'], d['ms_per_step'])" "$label"
}
for rep in 1 2; do
  run "1pipe,side" X=1 --
  run "2pipe,side" X=1 -- --stream-inflight 2
  run "2pipe,noside" SFA_SIDE_STREAMS=0 -- --stream-inflight 2
  run "2pipe,side,hwq8" GPU_MAX_HW_QUEUES=8 -- --stream-inflight 2
  run "1pipe,noside" SFA_SIDE_STREAMS=0 --
done
