set -u
export TMPDIR=/tmp
timeout -k 10 120 ./tools/decodebench 200 > gpurun_out/decodebench.txt 2>&1 || { echo "decodebench failed"; cat gpurun_out/decodebench.txt; exit 1; }
cat gpurun_out/decodebench.txt
bash tools/gpu_quick.sh "$1" "tests"
