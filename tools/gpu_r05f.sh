# round 5: the full GPU suite on the current tree, then FPN commute masks re-measured (bench A/B)
set -u
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05f_gpu_tests.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r05f_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r05f_gpu_tests.txt
bash tools/ab_env.sh SFA_FPN_COMMUTE=7,SFA_FPN_COMMUTE=6,SFA_FPN_COMMUTE=4,SFA_FPN_COMMUTE=0 || exit 1
echo done
