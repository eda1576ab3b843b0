# round 5: fp16x3 scales of both frames from one 16-load group (strip, r3, h3 prologues) vs the previous
# library; the level-0 / level-1 FPN skip convs on fpn_seg_kernel (SFA_FPN_GEMM 61 vs 37)
set -u
export TMPDIR=/tmp
timeout -k 10 120 ./tools/stampbench > gpurun_out/r05m_stampbench.txt 2>&1 || { echo "stampbench failed"; tail gpurun_out/r05m_stampbench.txt; exit 1; }
python3 tools/stamp_summary.py gpurun_out/stamps_layer1.bin gpurun_out/stamps_layer2.bin > gpurun_out/r05m_stamps.txt 2>&1
rm -f gpurun_out/stamps_*.bin
grep -h "prologue" gpurun_out/r05m_stamps.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bench_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05m_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05m_tests.txt; exit 1; }
tail -2 gpurun_out/r05m_tests.txt
SFA_HIP_LIB=tools/experiments/r05/libsfa_hip_prev.so timeout -k 10 200 python tools/ab_lib_bits.py run gpurun_out/bits_prev_r05m.npz > gpurun_out/r05m_bits.txt 2>&1 || { echo "bits prev failed"; tail gpurun_out/r05m_bits.txt; exit 1; }
timeout -k 10 200 python tools/ab_lib_bits.py run gpurun_out/bits_new_r05m.npz >> gpurun_out/r05m_bits.txt 2>&1 || { echo "bits new failed"; tail gpurun_out/r05m_bits.txt; exit 1; }
python tools/ab_lib_bits.py compare gpurun_out/bits_prev_r05m.npz gpurun_out/bits_new_r05m.npz >> gpurun_out/r05m_bits.txt 2>&1; tail -1 gpurun_out/r05m_bits.txt
rm -f gpurun_out/bits_*_r05m.npz
bash tools/ab_env.sh SFA_HIP_LIB=tools/experiments/r05/libsfa_hip_prev.so,SFA_HIP_LIB=lidar-image_object-detection_-fpn_resnet-yolov8_amd/sfa/sfa_hip/libsfa_hip.so || exit 1
bash tools/ab_env.sh SFA_FPN_GEMM=37,SFA_FPN_GEMM=61 || exit 1
for m in 37 61; do
  rm -rf gpurun_out/prof_fpn$m
  SFA_FPN_GEMM=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fpn$m -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bp_fpn$m.json 2> gpurun_out/bp_fpn$m.err || { echo "rocprof failed"; tail gpurun_out/bp_fpn$m.err; exit 1; }
  python3 tools/rocprof_summary.py "$(ls gpurun_out/prof_fpn$m/*kernel_trace.csv | head -1)" --title "SFA_FPN_GEMM=$m rocprofv3 --kernel-trace -- python bench.py --inflight 1 --serial-heads --steps 10 --warmup 3 --no-cpu-baseline" > gpurun_out/r05m_prof_summary_fpn$m.txt
  rm -rf gpurun_out/prof_fpn$m
  grep -E "fpn|upsample|conv_r3_kernel<128, 128, 32, 0, 2, 2, 1, 35072>|fpn\+aux" gpurun_out/r05m_prof_summary_fpn$m.txt | head -12
done
echo done
