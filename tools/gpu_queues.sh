# steps in flight x side streams x hardware queues, interleaved twice (run on the GPU box)
set -u
export TMPDIR=/tmp
run() {  # label, env..., -- bench args
  local label="$1"; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --probe-forwards 0 "$@" > gpurun_out/q.json 2>/dev/null || { echo "failed: $label"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/q.json')); print(sys.argv[1], d['value'], d['stages_ms']['forward'])" "$label"
}
for rep in 1 2; do
  run "default(2inflight,side)" X=1 --
  run "noside,2inflight" SFA_SIDE_STREAMS=0 --
  run "noside,3inflight" SFA_SIDE_STREAMS=0 -- --inflight 3
  run "hwq8,2inflight,side" GPU_MAX_HW_QUEUES=8 --
  run "hwq8,2inflight,side+fpn3" GPU_MAX_HW_QUEUES=8 SFA_FPN3_SIDE=1 --
  run "hwq8,3inflight,side" GPU_MAX_HW_QUEUES=8 -- --inflight 3
done
