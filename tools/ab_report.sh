# Summary of a tools/ab_lib.sh run (here, after gpurun merged gpurun_out/):
#   bash tools/ab_report.sh TAG "KERNEL_REGEX"
TAG="$1"
RX="${2:-conv_}"
for m in prev new; do
  echo "== $m"
  grep -E "^sfa::($RX).*[0-9]$" gpurun_out/${TAG}_prof_summary_$m.txt | head -8
  grep -E "^#   [a-z]" gpurun_out/${TAG}_prof_summary_$m.txt
done
tail -1 gpurun_out/${TAG}_tests.txt
tail -1 gpurun_out/${TAG}_bits.txt
for f in gpurun_out/ab_SFA_HIP_LIB=tools_experiments_r05_libsfa_hip_prev.so_1.json \
         gpurun_out/ab_SFA_HIP_LIB=lidar-image_object-detection_-fpn_resnet-yolov8_amd_sfa_sfa_hip_libsfa_hip.so_1.json \
         gpurun_out/ab_SFA_HIP_LIB=tools_experiments_r05_libsfa_hip_prev.so_2.json \
         gpurun_out/ab_SFA_HIP_LIB=lidar-image_object-detection_-fpn_resnet-yolov8_amd_sfa_sfa_hip_libsfa_hip.so_2.json; do
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', 'prev' if 'prev' in sys.argv[1] else 'new', sys.argv[1][-6:-5], d['value'])" "$f"
done
