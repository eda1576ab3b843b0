# round 5: conv_h3 (layer3 / 4 stride-2 conv1) with 3- and 4-stage rings at one block per CU vs the product's 2 stages at 2 (isolated)
set -u
export TMPDIR=/tmp
timeout -k 10 300 ./tools/convbench4 20 "s2 layer" > gpurun_out/r05u_convbench4_h3_stages.txt 2>&1 || { echo "convbench4 failed"; tail gpurun_out/r05u_convbench4_h3_stages.txt; exit 1; }
cat gpurun_out/r05u_convbench4_h3_stages.txt
