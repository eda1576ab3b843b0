# round 4: full-row FPN level-2 skip conv (fpn_row_kernel): bits (the FPN kernel-choice test), serial
# rocprof with it on / off, bench A/B
set -u
export TMPDIR=/tmp
TAG="${1:-r04k}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread -k "fpn" > gpurun_out/t_$TAG.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_$TAG.txt; exit 1; }
tail -1 gpurun_out/t_$TAG.txt
for mask in 61 37; do
  SFA_FPN_GEMM=$mask timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_m$mask -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bp_${TAG}_m$mask.json 2> gpurun_out/bp_${TAG}_m$mask.err || { echo "rocprof failed $mask"; tail gpurun_out/bp_${TAG}_m$mask.err; exit 1; }
  KT=$(find gpurun_out/prof_${TAG}_m$mask -name "*kernel_trace.csv" -print -quit); python3 tools/rocprof_summary.py "$KT" > gpurun_out/prof_summary_${TAG}_m$mask.txt 2>&1 || true
  echo "== mask $mask"; grep -A40 "one forward in issue order" gpurun_out/prof_summary_${TAG}_m$mask.txt | grep -E "fpn_row|35072|fpn_gemm|conv_h3_kernel<128, 128, 32, 0, 2, 32, 2, 1"
done
bash tools/ab_env.sh SFA_FPN_GEMM=61,SFA_FPN_GEMM=37,SFA_FPN_GEMM=61,SFA_FPN_GEMM=37 || exit 1
echo done
