# round 4: VALU diet of the strip kernel prologue / transposed epilogue — bits vs the previous build,
# isolated timing, instruction census, bench A/B of the two builds
set -u
export TMPDIR=/tmp
TAG="${1:-r04n}"
PRE=tools/experiments/r04/libsfa_hip_prev.so
timeout -k 10 300 python tools/ab_lib_bits.py run gpurun_out/bits_new_$TAG.npz > gpurun_out/bits_$TAG.log 2>&1 || { echo "bits new failed"; tail gpurun_out/bits_$TAG.log; exit 1; }
SFA_HIP_LIB=$PRE timeout -k 10 300 python tools/ab_lib_bits.py run gpurun_out/bits_pre_$TAG.npz >> gpurun_out/bits_$TAG.log 2>&1 || { echo "bits pre failed"; tail gpurun_out/bits_$TAG.log; exit 1; }
python tools/ab_lib_bits.py compare gpurun_out/bits_pre_$TAG.npz gpurun_out/bits_new_$TAG.npz 2>&1 | tail -2
timeout -k 10 200 ./tools/convbench4 20 layer > gpurun_out/cb4_$TAG.txt 2>&1 || { echo "convbench4 failed"; tail -20 gpurun_out/cb4_$TAG.txt; exit 1; }
grep -E "==|us " gpurun_out/cb4_$TAG.txt | grep -v "weight-stationary\|abl266\|abl398\|64x128\|128x64 w32 occ3 abl10"
bash tools/pmc_forward_insts.sh gpurun_out/pmc_insts_$TAG || { echo "insts failed"; exit 1; }
python3 tools/pmc_insts_summary.py gpurun_out/pmc_insts_$TAG > gpurun_out/pmc_insts_$TAG.txt 2>&1 || true
head -24 gpurun_out/pmc_insts_$TAG.txt
bash tools/ab_env.sh SFA_HIP_LIB=$PRE,SFA_HIP_LIB=lidar-image_object-detection_-fpn_resnet-yolov8_amd/sfa/sfa_hip/libsfa_hip.so,SFA_HIP_LIB=$PRE,SFA_HIP_LIB=lidar-image_object-detection_-fpn_resnet-yolov8_amd/sfa/sfa_hip/libsfa_hip.so || exit 1
echo done
