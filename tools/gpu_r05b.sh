# round 5: persistent strip kernel — isolated A/B (bit-identity + time), GPU model tests, bench A/B
set -u
export TMPDIR=/tmp
timeout -k 10 120 ./tools/convbench5 20 > gpurun_out/r05b_convbench5.txt 2>&1 || { echo "convbench5 failed"; tail -20 gpurun_out/r05b_convbench5.txt; exit 1; }
cat gpurun_out/r05b_convbench5.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bench_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05b_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05b_tests.txt; exit 1; }
tail -2 gpurun_out/r05b_tests.txt
bash tools/ab_env.sh SFA_BODY_PERSIST=0,SFA_BODY_PERSIST=1 || exit 1
echo done
