set -u
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_parity.py tests/test_gpu_model.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r06_t3.txt 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r06_t3.txt | head; tail -30 gpurun_out/r06_t3.txt; exit 1; }
grep -E "PASS|FAIL|passed|failed|timed batch|tie-free|bench N" gpurun_out/r06_t3.txt | tail -60
timeout -k 10 400 python bench.py > gpurun_out/r06_b.json 2> gpurun_out/r06_b.err || { tail gpurun_out/r06_b.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('gpurun_out/r06_b.json')); print('bench', d['value'], d['stages_ms']['forward'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['parity'], d['cpu_baseline']['value'])"
