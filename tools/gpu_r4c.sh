# round 4, second GPU pass: stem band vs patch (convbench4 + PMC), PMC forward (HBM, MFMA busy) and the
# instruction census of one bench forward with the round-4 kernels
set -u
export TMPDIR=/tmp
TAG="${1:-r04c}"
bash tools/gpu_r4b.sh "$TAG" || { echo "stem pass failed"; exit 1; }
bash tools/pmc_forward.sh gpurun_out/pmc_fwd_$TAG || { echo "pmc forward failed"; cat gpurun_out/pmc_fwd_$TAG/failed.txt; exit 1; }
python3 tools/pmc_forward_summary.py gpurun_out/pmc_fwd_$TAG gpurun_out/pmc_fwd_$TAG.json > gpurun_out/pmc_fwd_$TAG.txt 2>&1 || true
head -c 1500 gpurun_out/pmc_fwd_$TAG.txt
bash tools/pmc_forward_insts.sh gpurun_out/pmc_insts_$TAG || { echo "insts failed"; exit 1; }
python3 tools/pmc_insts_summary.py gpurun_out/pmc_insts_$TAG > gpurun_out/pmc_insts_$TAG.txt 2>&1 || true
head -50 gpurun_out/pmc_insts_$TAG.txt
echo done
