# heads stagger A/B: convbench heads (isolated, checked against the first candidate), then the
# bench with SFA_TUNE 0 / 65536 / 131072 interleaved
set -u
export TMPDIR=/tmp
timeout -k 10 300 ./tools/convbench 20 "head L" > gpurun_out/cb_stag.txt 2>&1 || { echo "convbench failed"; tail gpurun_out/cb_stag.txt; exit 1; }
cat gpurun_out/cb_stag.txt
timeout -k 10 200 python -u -m pytest tests/test_gpu_model.py -m gpu -x -q --timeout 120 --timeout-method thread -k "stagger or round2" > gpurun_out/t_stag.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_stag.txt; exit 1; }
tail -1 gpurun_out/t_stag.txt
bash tools/ab_env.sh SFA_TUNE=0,SFA_TUNE=65536,SFA_TUNE=131072
