# stem-patch check: model tests (verbose), full GPU suite, bench A/B (run on the GPU box)
set -u
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py -x -v -s --timeout 200 --timeout-method thread -k "stem or 608" > gpurun_out/t_stem.txt 2>&1 || { echo "stem tests failed"; tail -40 gpurun_out/t_stem.txt; exit 1; }
grep "stem patch\|passed\|failed" gpurun_out/t_stem.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_gpu.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/t_gpu.txt; exit 1; }
tail -2 gpurun_out/t_gpu.txt
for v in 1 0 1 0; do
  SFA_STEM_PATCH=$v timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b_sp$v.json 2> gpurun_out/b_sp$v.err || { echo "bench failed"; tail gpurun_out/b_sp$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_sp$v.json'));print('stem_patch=$v', d['value'], d['stages_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sp -o run --output-format csv -- python bench.py --inflight 1 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bp_sp.json 2> gpurun_out/bp_sp.err || { echo "rocprof failed"; exit 1; }
