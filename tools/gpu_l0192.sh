# level-0 heads on 192x320 tiles (tune bit 33554432): bit-identity tests (608 incl.), bench A/B interleaved x3,
# probe launch times (GPU box)
set -u
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread -k "stagger" > gpurun_out/t_l0.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_l0.txt; exit 1; }
tail -1 gpurun_out/t_l0.txt
for rep in 1 2 3; do
  for t in 0 33554432; do
    SFA_TUNE=$t timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/l0_${t}_$rep.json 2> gpurun_out/l0.err || { echo "bench failed"; tail -3 gpurun_out/l0.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('tune', sys.argv[2], d['value'], d['stages_ms']['forward'], r['frac'], r['launch_us'])" gpurun_out/l0_${t}_$rep.json $t
  done
done
echo done
