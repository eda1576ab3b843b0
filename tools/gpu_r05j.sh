# round 5: (1) PS / RESPF on the 128-wide strip tiles, isolated; (2) conv_r3 / conv_h3 prologue
# diet: bits vs the previous library, GPU model tests, bench A/B
set -u
export TMPDIR=/tmp
timeout -k 10 180 ./tools/convbench5 20 layer2 > gpurun_out/r05j_convbench5.txt 2>&1 || { echo "convbench5 failed"; tail -20 gpurun_out/r05j_convbench5.txt; exit 1; }
timeout -k 10 180 ./tools/convbench5 20 layer3 >> gpurun_out/r05j_convbench5.txt 2>&1 || { echo "convbench5 failed"; tail -20 gpurun_out/r05j_convbench5.txt; exit 1; }
cat gpurun_out/r05j_convbench5.txt
SFA_HIP_LIB=tools/experiments/r05/libsfa_hip_prev.so timeout -k 10 200 python tools/ab_lib_bits.py run gpurun_out/bits_prev_r05j.npz > gpurun_out/r05j_bits.txt 2>&1 || { echo "bits prev failed"; tail gpurun_out/r05j_bits.txt; exit 1; }
timeout -k 10 200 python tools/ab_lib_bits.py run gpurun_out/bits_new_r05j.npz >> gpurun_out/r05j_bits.txt 2>&1 || { echo "bits new failed"; tail gpurun_out/r05j_bits.txt; exit 1; }
python tools/ab_lib_bits.py compare gpurun_out/bits_prev_r05j.npz gpurun_out/bits_new_r05j.npz >> gpurun_out/r05j_bits.txt 2>&1; tail -2 gpurun_out/r05j_bits.txt
rm -f gpurun_out/bits_*_r05j.npz
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bench_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05j_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05j_tests.txt; exit 1; }
tail -2 gpurun_out/r05j_tests.txt
bash tools/ab_env.sh SFA_HIP_LIB=tools/experiments/r05/libsfa_hip_prev.so,SFA_HIP_LIB=lidar-image_object-detection_-fpn_resnet-yolov8_amd/sfa/sfa_hip/libsfa_hip.so || exit 1
echo done
