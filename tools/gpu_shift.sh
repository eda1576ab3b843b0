# heads shifted-A (tune bit 16777216): bit-identity tests, convbench heads (isolated, interleaved),
# bench A/B (GPU box)
set -u
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread -k "stagger" > gpurun_out/t_shift.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_shift.txt; exit 1; }
tail -1 gpurun_out/t_shift.txt
timeout -k 10 300 ./tools/convbench 20 "head L" > gpurun_out/cb_shift.txt 2>&1 || { echo "convbench failed"; tail gpurun_out/cb_shift.txt; exit 1; }
cat gpurun_out/cb_shift.txt
bash tools/ab_env.sh SFA_TUNE=0,SFA_TUNE=16777216
echo done
