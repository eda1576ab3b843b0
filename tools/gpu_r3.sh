# round 3: GPU tests (new bench-parity tests first) + the default bench line (run on the GPU box)
set -u
export TMPDIR=/tmp
TAG="${1:-r3}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_parity.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_parity_$TAG.txt 2>&1 || { echo "parity tests failed"; tail -40 gpurun_out/t_parity_$TAG.txt; exit 1; }
grep -E "passed|failed|err per" gpurun_out/t_parity_$TAG.txt | tail -4
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_gpu_$TAG.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/t_gpu_$TAG.txt; exit 1; }
tail -1 gpurun_out/t_gpu_$TAG.txt
timeout -k 10 400 python bench.py > gpurun_out/b_$TAG.json 2> gpurun_out/b_$TAG.err || { echo "bench failed"; tail gpurun_out/b_$TAG.err; exit 1; }
cat gpurun_out/b_$TAG.json
