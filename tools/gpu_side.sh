# side-stream toggle: its GPU tests, then the stream workload (default now 2 pipelines, no side
# streams) against 1 pipeline with side streams, interleaved (run on the GPU box)
set -u
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_side.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/t_side.txt; exit 1; }
tail -1 gpurun_out/t_side.txt
for rep in 1 2; do
  for v in "--stream-inflight 1" ""; do
    timeout -k 10 200 python bench.py --workload stream --no-cpu-baseline $v > gpurun_out/ss.json 2> gpurun_out/ss.err || { echo "failed: $v"; tail -3 gpurun_out/ss.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ss.json')); print(repr(sys.argv[1]), d['value'], d['ms_per_step'], d['config']['steps_in_flight'])" "$v"
  done
done
cp gpurun_out/ss.json gpurun_out/stream_default.json
