set -u
export TMPDIR=/tmp
timeout -k 10 300 ./tools/convbench 20 "layer1" > gpurun_out/cb_l1.txt 2>&1 || { echo "convbench failed"; tail gpurun_out/cb_l1.txt; exit 1; }
cat gpurun_out/cb_l1.txt
timeout -k 10 300 ./tools/convbench 20 "head L" > gpurun_out/cb_heads_x.txt 2>&1 || { echo "convbench failed"; tail gpurun_out/cb_heads_x.txt; exit 1; }
cat gpurun_out/cb_heads_x.txt
