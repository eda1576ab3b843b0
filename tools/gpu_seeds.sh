# the multi-seed full-size parity test (GPU box)
set -u
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k "weight_seeds" > gpurun_out/t_seeds.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_seeds.txt; exit 1; }
grep -E "max rel err|passed|failed" gpurun_out/t_seeds.txt
