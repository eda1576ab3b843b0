# end-of-round bundle on the final binary: GPU tests, smoke, headline bench (cpu_baseline + parity),
# the other BASELINE workloads, serial-heads rocprof (roofline agreement) (GPU box)
set -u
export TMPDIR=/tmp
TAG="${1:-r04z}"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_gpu_$TAG.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/t_gpu_$TAG.txt; exit 1; }
tail -1 gpurun_out/t_gpu_$TAG.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.txt 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke_$TAG.txt; exit 1; }
tail -1 gpurun_out/smoke_$TAG.txt
timeout -k 10 400 python bench.py > gpurun_out/b_$TAG.json 2> gpurun_out/b_$TAG.err || { echo "bench failed"; tail gpurun_out/b_$TAG.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], d['stages_ms']['forward'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['parity']['ok'], d['parity']['max_rel_logit_err'], d['cpu_baseline']['value'])" gpurun_out/b_$TAG.json
timeout -k 10 400 python bench.py --workload e2e > gpurun_out/e2e_$TAG.json 2> gpurun_out/e2e_$TAG.err || { echo "e2e failed"; tail gpurun_out/e2e_$TAG.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('e2e', d['value'], d['bev_roofline']['us_per_batch'], d['bev_roofline']['frac'], d['parity']['ok'], d['parity']['bev_equal'])" gpurun_out/e2e_$TAG.json
timeout -k 10 300 python bench.py --workload stream --no-cpu-baseline > gpurun_out/stream_$TAG.json 2> gpurun_out/stream_$TAG.err || { echo "stream failed"; tail gpurun_out/stream_$TAG.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('stream', d['value'])" gpurun_out/stream_$TAG.json
timeout -k 10 300 python bench.py --workload fusion --batch 8 --no-cpu-baseline > gpurun_out/fusion_$TAG.json 2> gpurun_out/fusion_$TAG.err || { echo "fusion failed"; tail gpurun_out/fusion_$TAG.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('fusion', d['value'])" gpurun_out/fusion_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bp_$TAG.json 2> gpurun_out/bp_$TAG.err || { echo "rocprof failed"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('probe', d['roofline']['launch_us'], d['roofline']['avg_launch_us'])" gpurun_out/bp_$TAG.json
echo done
