# round 5: heads without s_setprio 1 on the delayed half (ABL 4 off) vs the product (bench A/B, serial rocprof, bits)
set -u
export TMPDIR=/tmp
SFA_HIP_LIB=tools/experiments/r05/libsfa_hip_prev.so timeout -k 10 200 python tools/ab_lib_bits.py run gpurun_out/bits_prev_r05aa.npz > gpurun_out/r05aa_bits.txt 2>&1 || { echo "bits prev failed"; tail gpurun_out/r05aa_bits.txt; exit 1; }
timeout -k 10 200 python tools/ab_lib_bits.py run gpurun_out/bits_new_r05aa.npz >> gpurun_out/r05aa_bits.txt 2>&1 || { echo "bits new failed"; tail gpurun_out/r05aa_bits.txt; exit 1; }
python tools/ab_lib_bits.py compare gpurun_out/bits_prev_r05aa.npz gpurun_out/bits_new_r05aa.npz >> gpurun_out/r05aa_bits.txt 2>&1; tail -1 gpurun_out/r05aa_bits.txt
rm -f gpurun_out/bits_*_r05aa.npz
bash tools/ab_env.sh SFA_HIP_LIB=tools/experiments/r05/libsfa_hip_prev.so,SFA_HIP_LIB=lidar-image_object-detection_-fpn_resnet-yolov8_amd/sfa/sfa_hip/libsfa_hip.so || exit 1
for m in prev new; do
  rm -rf gpurun_out/prof_$m
  if [ $m = prev ]; then E="SFA_HIP_LIB=tools/experiments/r05/libsfa_hip_prev.so"; else E="SFA_NOOP=1"; fi
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$m -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bp_$m.json 2> gpurun_out/bp_$m.err || { echo "rocprof failed"; tail gpurun_out/bp_$m.err; exit 1; }
  python3 tools/rocprof_summary.py "$(ls gpurun_out/prof_$m/*kernel_trace.csv | head -1)" --title "$E" > gpurun_out/r05aa_prof_summary_$m.txt
  rm -rf gpurun_out/prof_$m
  echo "== $m"; grep -E "^sfa::conv_r3_kernel<256.*\('|^#   heads" gpurun_out/r05aa_prof_summary_$m.txt | head -4
done
echo done
