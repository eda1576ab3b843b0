# round 3c BEV (4-row strips, strip-major table): BEV tests, e2e bench A/B against 8-row strips
# (SFA_BEV_STRIP8=1), interleaved; PMC traffic of one call (GPU box)
set -u
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bev.py tests/test_gpu_back.py tests/test_gpu_stream.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_bev4.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/t_bev4.txt; exit 1; }
tail -1 gpurun_out/t_bev4.txt
for rep in 1 2; do
  for v in 0 1; do
    SFA_BEV_STRIP8=$v timeout -k 10 200 python bench.py --workload e2e --no-cpu-baseline > gpurun_out/bev4_${v}_${rep}.json 2> gpurun_out/bev4.err || { echo "bench failed"; tail -3 gpurun_out/bev4.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['bev_roofline']; print('strip8', sys.argv[2], d['value'], d['stages_ms']['forward'], r['us_per_batch'], r['achieved'], r['frac'],)" gpurun_out/bev4_${v}_${rep}.json $v
  done
done
bash tools/pmc_bev.sh gpurun_out/pmc_bev4 && python3 tools/pmc_bev_summary.py gpurun_out/pmc_bev4 gpurun_out/pmc_bev4.json > /dev/null && head -c 1500 gpurun_out/pmc_bev4.json
echo done
