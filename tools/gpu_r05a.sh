set -u
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05a_b.json 2> gpurun_out/r05a_b.err || { echo "bench failed"; tail gpurun_out/r05a_b.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], d['stages_ms']['forward'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['parity']['ok'])" gpurun_out/r05a_b.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05a -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r05a_bp.json 2> gpurun_out/r05a_bp.err || { echo "rocprof failed"; exit 1; }
echo done
