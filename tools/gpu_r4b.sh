# round 4: stem band vs patch kernel timing + PMC passes on the convbench4 stem shape
set -u
export TMPDIR=/tmp
TAG="${1:-r04b}"
timeout -k 10 120 ./tools/convbench4 20 stem > gpurun_out/cb4stem_$TAG.txt 2>&1 || { echo "convbench4 stem failed"; tail gpurun_out/cb4stem_$TAG.txt; exit 1; }
grep -E "==|us " gpurun_out/cb4stem_$TAG.txt
OUT=gpurun_out/pmcstem_$TAG; mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- ./tools/convbench4 3 stem > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed: $grp"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 tools/pmc_table.py $OUT 2>&1 | head -40 || true
echo done
