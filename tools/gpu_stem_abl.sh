# stem-patch timing ablations (SFA_STEM_ABL; results wrong by design), rocprof per variant
set -u
export TMPDIR=/tmp
for v in ${ABLS:-0 1 2 4 3}; do
  SFA_STEM_ABL=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_abl$v -o run --output-format csv -- python bench.py --inflight 1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bp_abl$v.json 2> gpurun_out/bp_abl$v.err || { echo "abl $v failed"; tail -5 gpurun_out/bp_abl$v.err; exit 1; }
  echo "abl=$v $(grep stem_patch gpurun_out/prof_abl$v/run_kernel_stats.csv | cut -d, -f2-4)"
done
