# round 5: conv_r3 prologue: the first W DMA and A loads issued before the frame-scale loads
# between the K loop and the heads epilogue; stamps, tests, bits vs the previous library, bench A/B
set -u
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bench_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05af_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05af_tests.txt; exit 1; }
tail -1 gpurun_out/r05af_tests.txt
SFA_HIP_LIB=tools/experiments/r05/libsfa_hip_prev.so timeout -k 10 200 python tools/ab_lib_bits.py run gpurun_out/bits_prev_r05af.npz > gpurun_out/r05af_bits.txt 2>&1 || { echo "bits prev failed"; tail gpurun_out/r05af_bits.txt; exit 1; }
timeout -k 10 200 python tools/ab_lib_bits.py run gpurun_out/bits_new_r05af.npz >> gpurun_out/r05af_bits.txt 2>&1 || { echo "bits new failed"; tail gpurun_out/r05af_bits.txt; exit 1; }
python tools/ab_lib_bits.py compare gpurun_out/bits_prev_r05af.npz gpurun_out/bits_new_r05af.npz >> gpurun_out/r05af_bits.txt 2>&1; tail -1 gpurun_out/r05af_bits.txt
rm -f gpurun_out/bits_*_r05af.npz
bash tools/ab_env.sh SFA_HIP_LIB=tools/experiments/r05/libsfa_hip_prev.so,SFA_HIP_LIB=lidar-image_object-detection_-fpn_resnet-yolov8_amd/sfa/sfa_hip/libsfa_hip.so || exit 1
for m in prev new; do
  rm -rf gpurun_out/prof_$m
  if [ $m = prev ]; then E="SFA_HIP_LIB=tools/experiments/r05/libsfa_hip_prev.so"; else E="SFA_NOOP=1"; fi
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$m -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bp_$m.json 2> gpurun_out/bp_$m.err || { echo "rocprof failed"; tail gpurun_out/bp_$m.err; exit 1; }
  python3 tools/rocprof_summary.py "$(ls gpurun_out/prof_$m/*kernel_trace.csv | head -1)" --title "$E rocprofv3 --kernel-trace -- python bench.py --inflight 1 --serial-heads --steps 10 --warmup 3 --no-cpu-baseline" > gpurun_out/r05af_prof_summary_$m.txt
  rm -rf gpurun_out/prof_$m
  echo "== $m"; grep -E "^sfa::conv_r3_kernel.*[0-9]$|^#   (layer2|heads)" gpurun_out/r05af_prof_summary_$m.txt | head -16
done
echo done
timeout -k 10 120 ./tools/headstampbench > gpurun_out/r05af_headstampbench.txt 2>&1 || { echo "headstampbench failed"; exit 1; }
python3 tools/head_stamp_summary.py gpurun_out/hstamps_L0.bin gpurun_out/hstamps_L1.bin gpurun_out/hstamps_L2.bin > gpurun_out/r05af_hstamps.txt 2>&1
rm -f gpurun_out/hstamps_*.bin
grep -E "bin:|prologue  |epilogue  |shares" gpurun_out/r05af_hstamps.txt
