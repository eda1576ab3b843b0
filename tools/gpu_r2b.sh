# tests + bench (with the head probe) + same-box A/B of the chunk-major K order (run on the GPU box)
set -u
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/t_gpu.txt; exit 1; }
tail -2 gpurun_out/t_gpu.txt
timeout -k 10 300 python bench.py > gpurun_out/b_main.json 2> gpurun_out/b_main.err || { echo "bench failed"; tail gpurun_out/b_main.err; exit 1; }
cat gpurun_out/b_main.json
bash tools/ab_env.sh SFA_TUNE=256,SFA_TUNE=0
