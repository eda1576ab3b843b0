# convbench: strip-kernel ablations on the body shapes (isolated launches, GPU box)
set -u
export TMPDIR=/tmp
timeout -k 10 300 ./tools/convbench 20 "layer" > gpurun_out/cb_strip.txt 2>&1 || { echo "convbench failed"; tail gpurun_out/cb_strip.txt; exit 1; }
cat gpurun_out/cb_strip.txt
