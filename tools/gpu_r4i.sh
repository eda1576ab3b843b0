# round 4: bench A/B of the LDS bank-conflict fixes (previous build vs this one), interleaved
set -u
export TMPDIR=/tmp
bash tools/ab_env.sh SFA_HIP_LIB=tools/experiments/r04/libsfa_hip_pre_swz.so,SFA_HIP_LIB=lidar-image_object-detection_-fpn_resnet-yolov8_amd/sfa/sfa_hip/libsfa_hip.so,SFA_HIP_LIB=tools/experiments/r04/libsfa_hip_pre_swz.so,SFA_HIP_LIB=lidar-image_object-detection_-fpn_resnet-yolov8_amd/sfa/sfa_hip/libsfa_hip.so || exit 1
echo done
