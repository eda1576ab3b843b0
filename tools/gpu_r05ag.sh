# round 5: layer1 strip convs on 256-row tiles (8 waves, 1 / 2 blocks per CU) vs the product 128 x 64 at 3 (isolated)
set -u
export TMPDIR=/tmp
timeout -k 10 300 ./tools/convbench5 20 "layer1" > gpurun_out/r05ag_convbench5_layer1_256rows.txt 2>&1 || { echo "convbench5 failed"; tail gpurun_out/r05ag_convbench5_layer1_256rows.txt; exit 1; }
cat gpurun_out/r05ag_convbench5_layer1_256rows.txt
