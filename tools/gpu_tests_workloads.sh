# GPU tests + the other BASELINE workloads (run on the GPU box)
set -u
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/t_gpu.txt; exit 1; }
tail -2 gpurun_out/t_gpu.txt
for w in e2e stream; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/w_$w.json 2> gpurun_out/w_$w.err || { echo "bench $w failed"; tail gpurun_out/w_$w.err; exit 1; }
  cut -c1-200 gpurun_out/w_$w.json
done
timeout -k 10 300 python bench.py --workload fusion --batch 8 --no-cpu-baseline > gpurun_out/w_fusion.json 2> gpurun_out/w_fusion.err || { echo "bench fusion failed"; tail gpurun_out/w_fusion.err; exit 1; }
cut -c1-200 gpurun_out/w_fusion.json
