# convbench heads candidates (isolated, checked against the first) (GPU box)
set -u
export TMPDIR=/tmp
timeout -k 10 300 ./tools/convbench 20 "head L" > gpurun_out/cb_h.txt 2>&1 || { echo "convbench failed"; tail gpurun_out/cb_h.txt; exit 1; }
cat gpurun_out/cb_h.txt
