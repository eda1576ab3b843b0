# remainder of the round-3 evidence: single-flight serial-heads rocprof (roofline agreement),
# decodebench, strip-kernel W ablations (GPU box)
set -u
export TMPDIR=/tmp
TAG="${1:-r03q}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bp_$TAG.json 2> gpurun_out/bp_$TAG.err || { echo "rocprof failed"; exit 1; }
timeout -k 10 120 ./tools/decodebench 200 > gpurun_out/decodebench_$TAG.txt 2>&1 || { echo "decodebench failed"; exit 1; }
head -4 gpurun_out/decodebench_$TAG.txt
timeout -k 10 300 ./tools/convbench 20 "layer" > gpurun_out/cb_strip_$TAG.txt 2>&1 || { echo "convbench failed"; exit 1; }
grep -v unsupported gpurun_out/cb_strip_$TAG.txt | head -24
echo done
