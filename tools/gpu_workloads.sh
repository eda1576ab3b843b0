# PMC traffic of the bench forward + the other BASELINE workloads (run on the GPU box)
set -u
export TMPDIR=/tmp
bash tools/pmc_forward.sh gpurun_out/pmc_cur || { echo "pmc failed"; exit 1; }
for w in e2e stream; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/w_$w.json 2> gpurun_out/w_$w.err || { echo "bench $w failed"; tail gpurun_out/w_$w.err; exit 1; }
  cut -c1-160 gpurun_out/w_$w.json
done
timeout -k 10 300 python bench.py --workload fusion --batch 8 --no-cpu-baseline > gpurun_out/w_fusion.json 2> gpurun_out/w_fusion.err || { echo "bench fusion failed"; tail gpurun_out/w_fusion.err; exit 1; }
cut -c1-160 gpurun_out/w_fusion.json
