#!/bin/bash
# HBM traffic of one bench forward from PMC counters (run on the GPU box).
# Separate passes per the MI355X guide (FETCH_SIZE and WRITE_SIZE do not fit one pass).
set -u
OUT="${1:-gpurun_out/pmc_fwd}"
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
    python bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --probe-forwards 1 > "$OUT/p$i.log" 2>&1 \
    || { echo "pass $i failed: $grp" >> "$OUT/failed.txt"; exit 1; }
done
