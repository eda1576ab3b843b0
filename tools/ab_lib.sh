# Same-box A/B of the in-tree library against a previous build (run on the GPU box), the form of every
# round-5 kernel change (profiles/r05*):
#   cp <pkg>/sfa/sfa_hip/libsfa_hip.so tools/prev_lib/libsfa_hip_prev.so   # before the change, here
#   <edit, build>                                                                  # then
#   gpurun -- 'bash tools/ab_lib.sh TAG "KERNEL_REGEX" [stamps,hstamps,tests,bits,ab,prof]'
# Parts (default all but stamps / hstamps): tests = the model + timed-config parity GPU tests; bits =
# tools/ab_lib_bits.py over the full forward, previous vs new; ab = tools/ab_env.sh bench A/B (2 x 2
# interleaved); prof = rocprofv3 kernel trace of the serial forward for both libraries, the lines of
# KERNEL_REGEX and the per-stage times; stamps / hstamps = the s_memtime diagnostics of the strip /
# heads kernels (tools/stampbench, tools/headstampbench: tools/build_stamps.sh regenerates the stamped copies from
# the product headers and builds them, beforehand).
set -u
export TMPDIR=/tmp
TAG="$1"
RX="${2:-conv_}"
PARTS=",${3:-tests,bits,ab,prof},"
has() { [[ "$PARTS" == *",$1,"* ]]; }
PREV=tools/prev_lib/libsfa_hip_prev.so
NEW=lidar-image_object-detection_-fpn_resnet-yolov8_amd/sfa/sfa_hip/libsfa_hip.so
if has stamps; then
  timeout -k 10 120 ./tools/stampbench > gpurun_out/${TAG}_stampbench.txt 2>&1 || { echo "stampbench failed"; exit 1; }
  python3 tools/stamp_summary.py gpurun_out/stamps_layer1.bin gpurun_out/stamps_layer2.bin > gpurun_out/${TAG}_stamps.txt 2>&1
  rm -f gpurun_out/stamps_*.bin
  grep -h "prologue" gpurun_out/${TAG}_stamps.txt
fi
if has hstamps; then
  timeout -k 10 120 ./tools/headstampbench > gpurun_out/${TAG}_headstampbench.txt 2>&1 || { echo "headstampbench failed"; exit 1; }
  python3 tools/head_stamp_summary.py gpurun_out/hstamps_L0.bin gpurun_out/hstamps_L1.bin gpurun_out/hstamps_L2.bin > gpurun_out/${TAG}_hstamps.txt 2>&1
  rm -f gpurun_out/hstamps_*.bin
  grep -E "bin:|prologue  |epilogue  |shares" gpurun_out/${TAG}_hstamps.txt
fi
if has tests; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bench_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.txt
fi
if has bits; then
  SFA_HIP_LIB=$PREV timeout -k 10 200 python tools/ab_lib_bits.py run gpurun_out/bits_prev_${TAG}.npz > gpurun_out/${TAG}_bits.txt 2>&1 || { echo "bits prev failed"; exit 1; }
  timeout -k 10 200 python tools/ab_lib_bits.py run gpurun_out/bits_new_${TAG}.npz >> gpurun_out/${TAG}_bits.txt 2>&1 || { echo "bits new failed"; exit 1; }
  python tools/ab_lib_bits.py compare gpurun_out/bits_prev_${TAG}.npz gpurun_out/bits_new_${TAG}.npz >> gpurun_out/${TAG}_bits.txt 2>&1
  tail -1 gpurun_out/${TAG}_bits.txt
  rm -f gpurun_out/bits_*_${TAG}.npz
fi
if has ab; then
  bash tools/ab_env.sh SFA_HIP_LIB=$PREV,SFA_HIP_LIB=$NEW || exit 1
fi
if has prof; then
  for m in prev new; do
    rm -rf gpurun_out/prof_$m
    if [ $m = prev ]; then E="SFA_HIP_LIB=$PREV"; else E="SFA_HIP_LIB=$NEW"; fi
    env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$m -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bp_$m.json 2> gpurun_out/bp_$m.err || { echo "rocprof failed"; tail gpurun_out/bp_$m.err; exit 1; }
    python3 tools/rocprof_summary.py "$(ls gpurun_out/prof_$m/*kernel_trace.csv | head -1)" --title "$E rocprofv3 --kernel-trace -- python bench.py --inflight 1 --serial-heads --steps 10 --warmup 3 --no-cpu-baseline" > gpurun_out/${TAG}_prof_summary_$m.txt
    rm -rf gpurun_out/prof_$m
    echo "== $m"
    grep -E "^sfa::.*($RX).*[0-9]$" gpurun_out/${TAG}_prof_summary_$m.txt | head -16
    grep -E "^#   [a-z]" gpurun_out/${TAG}_prof_summary_$m.txt
  done
fi
echo done
