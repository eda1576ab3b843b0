# binned BEV voxeliser: its GPU tests, the e2e bench (bev_roofline) binned vs atomic, rocprof (GPU box)
set -u
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bev.py tests/test_gpu_back.py tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_bev.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/t_bev.txt; exit 1; }
tail -1 gpurun_out/t_bev.txt
for rep in 1 2; do
  for e in 0 1; do
    SFA_BEV_ATOMIC=$e timeout -k 10 200 python bench.py --workload e2e --no-cpu-baseline > gpurun_out/bev_$e.json 2> gpurun_out/bev_$e.err || { echo "bench failed"; tail -3 gpurun_out/bev_$e.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['bev_roofline']; print('SFA_BEV_ATOMIC=' + sys.argv[2], d['value'], r['us_per_batch'], r['achieved'], r['frac'])" gpurun_out/bev_$e.json $e
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bev -o run --output-format csv -- python bench.py --workload e2e --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/bev_p.json 2> gpurun_out/bev_p.err || { echo "rocprof failed"; exit 1; }
echo done
