# round 4: stall census of one bench forward (SQ wait / LDS bank-conflict counters, one pass each)
set -u
export TMPDIR=/tmp
TAG="${1:-r04g}"
OUT=gpurun_out/pmcwait_$TAG; mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
    python bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --probe-forwards 1 > "$OUT/p$i.log" 2>&1 \
    || { echo "pass $i failed: $grp"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 tools/pmc_table.py $OUT > gpurun_out/pmcwait_$TAG.txt 2>&1 || true
echo done
