set -u
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t_gpu.txt 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/b_main.json 2> gpurun_out/b_main.err || { echo "bench failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_h3 -o run --output-format csv -- python bench.py --inflight 1 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b_prof.json 2> gpurun_out/b_prof.err || { echo "rocprof failed"; exit 1; }
bash tools/pmc_forward.sh gpurun_out/pmc_h3 || { echo "pmc failed"; exit 1; }
