# round 4: band stem with paired block chains — bits (tests) and isolated timing vs the patch stem
set -u
export TMPDIR=/tmp
TAG="${1:-r04f}"
timeout -k 10 120 ./tools/convbench4 20 stem > gpurun_out/cb4_$TAG.txt 2>&1 || { echo "convbench4 failed"; tail -20 gpurun_out/cb4_$TAG.txt; exit 1; }
grep -E "==|us " gpurun_out/cb4_$TAG.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread -k "stem" > gpurun_out/t_$TAG.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_$TAG.txt; exit 1; }
tail -1 gpurun_out/t_$TAG.txt
echo done
