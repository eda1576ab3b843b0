# round 5: tickets on the strip convs only; wide register-A tiles on layer3 (isolated)
set -u
export TMPDIR=/tmp
timeout -k 10 120 ./tools/convbench5 20 layer3 > gpurun_out/r05d_convbench5.txt 2>&1 || { echo "convbench5 failed"; tail -20 gpurun_out/r05d_convbench5.txt; exit 1; }
cat gpurun_out/r05d_convbench5.txt
timeout -k 10 600 python -u -m pytest tests/test_abi.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread -k "splitk or batch_invariance or bench" > gpurun_out/r05d_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05d_tests.txt; exit 1; }
tail -2 gpurun_out/r05d_tests.txt
bash tools/ab_env.sh SFA_SPLITK_TICKETS=0,SFA_SPLITK_TICKETS=1 || exit 1
echo done
