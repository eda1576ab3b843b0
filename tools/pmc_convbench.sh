#!/bin/bash
# PMC passes over one convbench shape (run on the GPU box). Usage: tools/pmc_convbench.sh "<shape substring>" outdir
set -u
SHAPE="$1"; OUT="$2"
export TMPDIR=/tmp
mkdir -p "$OUT"
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- ./tools/convbench 3 "$SHAPE" > "$OUT/p$i.log" 2>&1 || echo "pass $i failed: $grp" >> "$OUT/failed.txt"
done
exit 0
