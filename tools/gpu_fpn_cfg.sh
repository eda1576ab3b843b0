# FPN skip-conv tile variants (SFA_FPN_CFG): parity tests, then per-kernel rocprof averages (GPU box)
set -u
export TMPDIR=/tmp
for c in 0 1 2 3 4; do
  SFA_FPN_CFG=$c timeout -k 10 200 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -k "fpn_commute or small_inputs or round2" > gpurun_out/t_fpn_$c.txt 2>&1 || { echo "pytest failed cfg $c"; tail -20 gpurun_out/t_fpn_$c.txt; exit 1; }
  echo "cfg $c: $(tail -1 gpurun_out/t_fpn_$c.txt)"
  SFA_FPN_CFG=$c timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fpn_$c -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 20 --warmup 3 --no-cpu-baseline --probe-forwards 0 > gpurun_out/fpn_$c.json 2> gpurun_out/fpn_$c.err || { echo "rocprof failed cfg $c"; exit 1; }
done
echo done
