# round 4 (late): layer4 strip convs on 128 x 64 split-K tiles — bits vs the previous build, the
# forward's kernel times (rocprof, serial heads) and an interleaved bench A/B of the two builds
set -u
export TMPDIR=/tmp
TAG="${1:-r04p}"
PRE=tools/experiments/r04/libsfa_hip_prev.so
NEW=lidar-image_object-detection_-fpn_resnet-yolov8_amd/sfa/sfa_hip/libsfa_hip.so
timeout -k 10 300 python tools/ab_lib_bits.py run gpurun_out/bits_new_$TAG.npz > gpurun_out/bits_$TAG.log 2>&1 || { echo "bits new failed"; tail gpurun_out/bits_$TAG.log; exit 1; }
SFA_HIP_LIB=$PRE timeout -k 10 300 python tools/ab_lib_bits.py run gpurun_out/bits_pre_$TAG.npz >> gpurun_out/bits_$TAG.log 2>&1 || { echo "bits pre failed"; tail gpurun_out/bits_$TAG.log; exit 1; }
python tools/ab_lib_bits.py compare gpurun_out/bits_pre_$TAG.npz gpurun_out/bits_new_$TAG.npz 2>&1 | tail -2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bp_$TAG.json 2> gpurun_out/bp_$TAG.err || { echo "rocprof failed"; exit 1; }
bash tools/ab_env.sh SFA_HIP_LIB=$PRE,SFA_HIP_LIB=$NEW,SFA_HIP_LIB=$PRE,SFA_HIP_LIB=$NEW || exit 1
echo done
