# 256x128 strip tiles for the body convs (tune bits 2097152: 256-wide, 8388608: 128-wide):
# bit-identity test + bench A/B interleaved (GPU box)
set -u
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread -k "strip256 or batch_invariance" > gpurun_out/t_s256.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_s256.txt; exit 1; }
tail -1 gpurun_out/t_s256.txt
bash tools/ab_env.sh SFA_TUNE=0,SFA_TUNE=2097152,SFA_TUNE=10485760
echo done
