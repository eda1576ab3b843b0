# round 5: strip tiles of 64 rows at 4 blocks per CU (layer1 / layer2), isolated
set -u
export TMPDIR=/tmp
timeout -k 10 120 ./tools/convbench5 20 layer1 > gpurun_out/r05i_convbench5.txt 2>&1 || { echo "convbench5 failed"; tail -20 gpurun_out/r05i_convbench5.txt; exit 1; }
timeout -k 10 120 ./tools/convbench5 20 layer2 >> gpurun_out/r05i_convbench5.txt 2>&1 || { echo "convbench5 failed"; tail -20 gpurun_out/r05i_convbench5.txt; exit 1; }
cat gpurun_out/r05i_convbench5.txt
echo done
