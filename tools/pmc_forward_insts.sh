#!/bin/bash
# Instruction census of one bench forward (run on the GPU box): VALU / MFMA / LDS / VMEM / SALU
# instruction counts per launch, one PMC pass (8 SQ counters), bench.py --no-graph.
set -u
OUT="${1:-gpurun_out/pmc_insts}"
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/p1" -o run -- \
  python bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline > "$OUT/p1.log" 2>&1
