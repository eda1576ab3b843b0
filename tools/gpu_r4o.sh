# round 4 (late): layer4 split-K grids (strip convs and the stride-2 conv1) in convbench4
set -u
export TMPDIR=/tmp
TAG="${1:-r04o}"
timeout -k 10 300 ./tools/convbench4 20 "${2:-layer4}" > gpurun_out/cb4_$TAG.txt 2>&1 || { echo "convbench4 failed"; tail -20 gpurun_out/cb4_$TAG.txt; exit 1; }
grep -E "==|us " gpurun_out/cb4_$TAG.txt
echo done
