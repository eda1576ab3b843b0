# round-3 final evidence: GPU tests, default bench (cpu_baseline + parity), e2e bench, BEV PMC,
# PMC of the serial forward (HBM traffic / MFMA busy per launch), single-flight serial-heads rocprof
# (roofline agreement), decodebench (GPU box)
set -u
export TMPDIR=/tmp
TAG="${1:-r03q}"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_gpu_$TAG.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/t_gpu_$TAG.txt; exit 1; }
tail -1 gpurun_out/t_gpu_$TAG.txt
timeout -k 10 400 python bench.py > gpurun_out/b_$TAG.json 2> gpurun_out/b_$TAG.err || { echo "bench failed"; tail gpurun_out/b_$TAG.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], d['stages_ms'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['parity'], d['cpu_baseline']['value'])" gpurun_out/b_$TAG.json
timeout -k 10 400 python bench.py --workload e2e > gpurun_out/e2e_$TAG.json 2> gpurun_out/e2e_$TAG.err || { echo "e2e failed"; tail gpurun_out/e2e_$TAG.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('e2e', d['value'], d['bev_roofline']['us_per_batch'], d['bev_roofline']['frac'], d['parity'])" gpurun_out/e2e_$TAG.json
bash tools/pmc_bev.sh gpurun_out/pmc_bev_$TAG && python3 tools/pmc_bev_summary.py gpurun_out/pmc_bev_$TAG gpurun_out/pmc_bev_$TAG.json > /dev/null || { echo "pmc bev failed"; exit 1; }
bash tools/pmc_forward.sh gpurun_out/pmc_fwd_$TAG && python3 tools/pmc_forward_summary.py gpurun_out/pmc_fwd_$TAG gpurun_out/pmc_fwd_$TAG.json > gpurun_out/pmc_fwd_$TAG.txt 2>&1 || { echo "pmc forward failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bp_$TAG.json 2> gpurun_out/bp_$TAG.err || { echo "rocprof failed"; exit 1; }
timeout -k 10 120 ./tools/decodebench 200 > gpurun_out/decodebench_$TAG.txt 2>&1 || { echo "decodebench failed"; exit 1; }
head -4 gpurun_out/decodebench_$TAG.txt

timeout -k 10 300 ./tools/convbench 20 "layer" > gpurun_out/cb_strip_$TAG.txt 2>&1 || { echo "convbench failed"; exit 1; }
grep -v unsupported gpurun_out/cb_strip_$TAG.txt | head -20
echo done
