# round 5: s_memtime stamps of the fused heads kernel (prologue / K loop / epilogue / block turnover)
set -u
export TMPDIR=/tmp
timeout -k 10 120 ./tools/headstampbench > gpurun_out/r05q_headstampbench.txt 2>&1 || { echo "headstampbench failed"; tail gpurun_out/r05q_headstampbench.txt; exit 1; }
cat gpurun_out/r05q_headstampbench.txt
python3 tools/head_stamp_summary.py gpurun_out/hstamps_L0.bin gpurun_out/hstamps_L1.bin gpurun_out/hstamps_L2.bin > gpurun_out/r05q_hstamps.txt 2>&1
rm -f gpurun_out/hstamps_*.bin
cat gpurun_out/r05q_hstamps.txt
