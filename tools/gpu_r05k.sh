# round 5: strip kernel: PS + RESPF on the 128-wide tiles, epilogue columns staged in LDS
# isolated times (the product kernels), GPU model tests, bench A/B against the previous library
set -u
export TMPDIR=/tmp
timeout -k 10 120 ./tools/stampbench > gpurun_out/r05k_stampbench.txt 2>&1 || { echo "stampbench failed"; tail gpurun_out/r05k_stampbench.txt; exit 1; }
python3 tools/stamp_summary.py gpurun_out/stamps_layer1.bin gpurun_out/stamps_layer2.bin > gpurun_out/r05k_stamps.txt 2>&1
rm -f gpurun_out/stamps_*.bin
cat gpurun_out/r05k_stamps.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bench_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05k_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05k_tests.txt; exit 1; }
tail -2 gpurun_out/r05k_tests.txt
SFA_HIP_LIB=tools/experiments/r05/libsfa_hip_prev.so timeout -k 10 200 python tools/ab_lib_bits.py run gpurun_out/bits_prev_r05k.npz > gpurun_out/r05k_bits.txt 2>&1 || { echo "bits prev failed"; tail gpurun_out/r05k_bits.txt; exit 1; }
timeout -k 10 200 python tools/ab_lib_bits.py run gpurun_out/bits_new_r05k.npz >> gpurun_out/r05k_bits.txt 2>&1 || { echo "bits new failed"; tail gpurun_out/r05k_bits.txt; exit 1; }
python tools/ab_lib_bits.py compare gpurun_out/bits_prev_r05k.npz gpurun_out/bits_new_r05k.npz >> gpurun_out/r05k_bits.txt 2>&1; tail -3 gpurun_out/r05k_bits.txt
rm -f gpurun_out/bits_*_r05k.npz
bash tools/ab_env.sh SFA_HIP_LIB=tools/experiments/r05/libsfa_hip_prev.so,SFA_HIP_LIB=lidar-image_object-detection_-fpn_resnet-yolov8_amd/sfa/sfa_hip/libsfa_hip.so || exit 1
echo done
