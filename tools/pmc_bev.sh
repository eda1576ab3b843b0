#!/bin/bash
# HBM traffic of one BEV voxelisation (16 sweeps) from PMC counters, bench --workload e2e (GPU box).
# Separate FETCH_SIZE / WRITE_SIZE passes (MI355X guide); summarised by tools/pmc_bev_summary.py.
set -u
OUT="${1:-gpurun_out/pmc_bev}"
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
    python bench.py --workload e2e --steps 2 --warmup 1 --no-graph --no-cpu-baseline --probe-forwards 0 > "$OUT/p$i.log" 2>&1 \
    || { echo "pass $i failed: $grp" >> "$OUT/failed.txt"; exit 1; }
done
