# round 3 BEV: tests, e2e bench NCHW3 vs NHWC4 (interleaved), PMC traffic of one call (GPU box)
set -u
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bev.py tests/test_gpu_back.py tests/test_gpu_stream.py tests/test_gpu_bench_parity.py tests/test_gpu_fusion_pipeline.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_bev3.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/t_bev3.txt; exit 1; }
tail -1 gpurun_out/t_bev3.txt
for rep in 1 2; do
  for l in nhwc4 nchw3; do
    timeout -k 10 200 python bench.py --workload e2e --bev-layout $l --no-cpu-baseline > gpurun_out/bev3_${l}_${rep}.json 2> gpurun_out/bev3_${l}.err || { echo "bench failed"; tail -3 gpurun_out/bev3_${l}.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['bev_roofline']; print(sys.argv[2], d['value'], d['stages_ms']['forward'], r['us_per_batch'], r['achieved'], r['frac'])" gpurun_out/bev3_${l}_${rep}.json $l
  done
done
bash tools/pmc_bev.sh gpurun_out/pmc_bev3 && python3 tools/pmc_bev_summary.py gpurun_out/pmc_bev3 gpurun_out/pmc_bev3.json > /dev/null && cat gpurun_out/pmc_bev3.json | head -5
echo done
