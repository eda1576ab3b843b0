# round 5: per-k-step s_memtime stamps of the strip kernel (diagnostic build, tools only)
set -u
export TMPDIR=/tmp
timeout -k 10 120 ./tools/stampbench > gpurun_out/r05g_stampbench.txt 2>&1 || { echo "stampbench failed"; tail gpurun_out/r05g_stampbench.txt; exit 1; }
cat gpurun_out/r05g_stampbench.txt
python3 tools/stamp_summary.py gpurun_out/stamps_layer1.bin gpurun_out/stamps_layer2.bin gpurun_out/stamps_layer4.bin
echo done
