#!/bin/bash
# Regenerates the DIAGNOSTIC stamped copies of the product strip / heads kernels from the current
# product headers (tools/experiments/r05/make_*stamp_variant.py -> conv_h3s_stamp.h, conv_r3_stamp.h;
# generated, never committed: .gitignore) and builds tools/stampbench, tools/headstampbench
# (used by tools/ab_lib.sh parts stamps / hstamps). Run here, before the GPU call.
set -eu
cd "$(dirname "$0")/.."
python3 tools/experiments/r05/make_stamp_variant.py
python3 tools/experiments/r05/make_heads_stamp_variant.py
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -pthread tools/stampbench.hip -o tools/stampbench
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -pthread tools/headstampbench.hip -o tools/headstampbench
