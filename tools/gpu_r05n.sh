# round 5: FPN kernels stage their weight slice by LDS-DMA (all pieces in flight) instead of a
# load -> ds_write loop (one latency per iteration); + the flat-step fpn_seg_kernel for the level-0 / 1
# skip convs (SFA_FPN_GEMM 61 vs 37); tests, bits vs the previous library, bench A/B, serial rocprof
set -u
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bench_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05n_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05n_tests.txt; exit 1; }
tail -1 gpurun_out/r05n_tests.txt
SFA_HIP_LIB=tools/experiments/r05/libsfa_hip_prev.so timeout -k 10 200 python tools/ab_lib_bits.py run gpurun_out/bits_prev_r05n.npz > gpurun_out/r05n_bits.txt 2>&1 || { echo "bits prev failed"; tail gpurun_out/r05n_bits.txt; exit 1; }
timeout -k 10 200 python tools/ab_lib_bits.py run gpurun_out/bits_new_r05n.npz >> gpurun_out/r05n_bits.txt 2>&1 || { echo "bits new failed"; tail gpurun_out/r05n_bits.txt; exit 1; }
python tools/ab_lib_bits.py compare gpurun_out/bits_prev_r05n.npz gpurun_out/bits_new_r05n.npz >> gpurun_out/r05n_bits.txt 2>&1; tail -1 gpurun_out/r05n_bits.txt
rm -f gpurun_out/bits_*_r05n.npz
bash tools/ab_env.sh SFA_HIP_LIB=tools/experiments/r05/libsfa_hip_prev.so,SFA_HIP_LIB=lidar-image_object-detection_-fpn_resnet-yolov8_amd/sfa/sfa_hip/libsfa_hip.so || exit 1
bash tools/ab_env.sh SFA_FPN_GEMM=37,SFA_FPN_GEMM=61,SFA_FPN_GEMM=63 || exit 1
for m in prev 37 61 63; do
  rm -rf gpurun_out/prof_fpn$m
  if [ $m = prev ]; then E="SFA_HIP_LIB=tools/experiments/r05/libsfa_hip_prev.so"; else E="SFA_FPN_GEMM=$m"; fi
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fpn$m -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bp_fpn$m.json 2> gpurun_out/bp_fpn$m.err || { echo "rocprof failed"; tail gpurun_out/bp_fpn$m.err; exit 1; }
  python3 tools/rocprof_summary.py "$(ls gpurun_out/prof_fpn$m/*kernel_trace.csv | head -1)" --title "$E rocprofv3 --kernel-trace -- python bench.py --inflight 1 --serial-heads --steps 10 --warmup 3 --no-cpu-baseline" > gpurun_out/r05n_prof_summary_fpn$m.txt
  rm -rf gpurun_out/prof_fpn$m
  echo "== $E"; grep -E "fpn|upsample|conv_r3_kernel<128, 128, 32, 0, 2, 2, 1, 35072>|conv_h3_kernel<128, 128, 32, 0, 2, 32, 2, 1, false, 2, 1, 128, false> |^#   fpn" gpurun_out/r05n_prof_summary_fpn$m.txt | grep -v "^ " | head -12
done
echo done
