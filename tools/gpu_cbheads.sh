# convbench heads only (isolated; each candidate checked against the first)
set -u
export TMPDIR=/tmp
timeout -k 10 300 ./tools/convbench 20 "head L" > gpurun_out/cb_heads_x.txt 2>&1 || { echo "convbench failed"; tail gpurun_out/cb_heads_x.txt; exit 1; }
cat gpurun_out/cb_heads_x.txt
