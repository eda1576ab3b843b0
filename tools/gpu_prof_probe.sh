# PMC traffic of one forward (refreshes profiles/*_pmc_forward_fp16x3.json) and a rocprofv3
# kernel-trace summary of the head-probe configuration (run on the GPU box)
set -u
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_fwd
bash tools/pmc_forward.sh gpurun_out/pmc_fwd || { echo "pmc failed"; cat gpurun_out/pmc_fwd/failed.txt; exit 1; }
python3 tools/pmc_forward_summary.py gpurun_out/pmc_fwd gpurun_out/pmc_forward_fp16x3.json > /dev/null || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_serial -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_serial.json 2> gpurun_out/b_serial.err || { echo "rocprof failed"; tail gpurun_out/b_serial.err; exit 1; }
cat gpurun_out/b_serial.json
