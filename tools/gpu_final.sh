# end-of-round evidence: tests, default bench, single-flight rocprof, PMC traffic (run on the GPU box)
set -u
export TMPDIR=/tmp
TAG="${1:-final}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_gpu.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/t_gpu.txt; exit 1; }
tail -1 gpurun_out/t_gpu.txt
timeout -k 10 300 python bench.py > gpurun_out/b_$TAG.json 2> gpurun_out/b_$TAG.err || { echo "bench failed"; tail gpurun_out/b_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/b_$TAG.json
# --serial-heads: every launch on the caller's stream, the configuration the bench's head probe
# times, so rocprof's average head-launch duration is comparable with roofline.avg_launch_us
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bp_$TAG.json 2> gpurun_out/bp_$TAG.err || { echo "rocprof failed"; exit 1; }
bash tools/pmc_forward.sh gpurun_out/pmc_$TAG || { echo "pmc failed"; exit 1; }
for w in e2e stream; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/w_${w}_$TAG.json 2> gpurun_out/w_$w.err || { echo "bench $w failed"; tail gpurun_out/w_$w.err; exit 1; }
done
timeout -k 10 300 python bench.py --workload fusion --batch 8 --no-cpu-baseline > gpurun_out/w_fusion_$TAG.json 2> gpurun_out/w_fusion.err || { echo "bench fusion failed"; tail gpurun_out/w_fusion.err; exit 1; }
echo done
