# final-tree check: GPU tests, smoke, default bench (GPU box)
set -u
export TMPDIR=/tmp
TAG="${1:-r03u}"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_gpu_$TAG.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/t_gpu_$TAG.txt; exit 1; }
tail -1 gpurun_out/t_gpu_$TAG.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.txt 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke_$TAG.txt; exit 1; }
tail -1 gpurun_out/smoke_$TAG.txt
timeout -k 10 400 python bench.py > gpurun_out/b_$TAG.json 2> gpurun_out/b_$TAG.err || { echo "bench failed"; tail gpurun_out/b_$TAG.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], d['stages_ms']['forward'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['parity']['ok'], d['cpu_baseline']['value'])" gpurun_out/b_$TAG.json
echo done
