# round 4: FPN kernel choice (SFA_FPN_GEMM) and stem form A/B on one box — the option tests, serial
# rocprof per mask, interleaved bench A/B
set -u
export TMPDIR=/tmp
TAG="${1:-r04d}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_abi.py -x -q --timeout 300 --timeout-method thread -k "fpn or stem or option or abi" > gpurun_out/t_$TAG.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_$TAG.txt; exit 1; }
tail -1 gpurun_out/t_$TAG.txt
for mask in 0 63 5; do
  SFA_FPN_GEMM=$mask timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_m$mask -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bp_${TAG}_m$mask.json 2> gpurun_out/bp_${TAG}_m$mask.err || { echo "rocprof failed $mask"; tail gpurun_out/bp_${TAG}_m$mask.err; exit 1; }
  KT=$(find gpurun_out/prof_${TAG}_m$mask -name "*kernel_trace.csv" -print -quit); python3 tools/rocprof_summary.py "$KT" > gpurun_out/prof_summary_${TAG}_m$mask.txt 2>&1 || true
  echo "== mask $mask"; grep -A40 "one forward in issue order" gpurun_out/prof_summary_${TAG}_m$mask.txt | grep -v -E "conv_h3s|rocclr" | tail -16
done
bash tools/ab_env.sh SFA_FPN_GEMM=5,SFA_FPN_GEMM=0,SFA_FPN_GEMM=63,SFA_STEM_PATCH=2 || exit 1
echo done
