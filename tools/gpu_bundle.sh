# Evidence bundle on the GPU box (replaces the per-round gpu_final*.sh / gpu_r*_evidence*.sh /
# gpu_prof*.sh scripts of rounds 1-4):
#   bash tools/gpu_bundle.sh TAG [PARTS]
# PARTS: comma list of tests, smoke, bench, e2e, stream, fusion, prof (serial-heads rocprofv3 kernel
# trace + summary), pmc (HBM traffic + instruction census of one forward); default: all but pmc.
# Outputs under gpurun_out/ (*_TAG.*); every GPU step has its own time limit and the script stops at
# the first failure.
set -u
export TMPDIR=/tmp
TAG="${1:-cur}"
PARTS=",${2:-tests,smoke,bench,e2e,stream,fusion,prof},"
has() { [[ "$PARTS" == *",$1,"* ]]; }
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_gpu_$TAG.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/t_gpu_$TAG.txt; exit 1; }
  tail -1 gpurun_out/t_gpu_$TAG.txt
fi
if has smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.txt 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke_$TAG.txt; exit 1; }
  tail -1 gpurun_out/smoke_$TAG.txt
fi
if has bench; then
  timeout -k 10 400 python bench.py > gpurun_out/b_$TAG.json 2> gpurun_out/b_$TAG.err || { echo "bench failed"; tail gpurun_out/b_$TAG.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], d['stages_ms']['forward'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['parity']['ok'], d['parity']['max_rel_logit_err'], d['cpu_baseline']['value'])" gpurun_out/b_$TAG.json
fi
if has e2e; then
  timeout -k 10 400 python bench.py --workload e2e --no-cpu-baseline > gpurun_out/e2e_$TAG.json 2> gpurun_out/e2e_$TAG.err || { echo "e2e failed"; tail gpurun_out/e2e_$TAG.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('e2e', d['value'], d['bev_roofline']['us_per_batch'], d['bev_roofline']['frac'])" gpurun_out/e2e_$TAG.json
fi
if has stream; then
  timeout -k 10 300 python bench.py --workload stream --no-cpu-baseline > gpurun_out/stream_$TAG.json 2> gpurun_out/stream_$TAG.err || { echo "stream failed"; tail gpurun_out/stream_$TAG.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('stream', d['value'])" gpurun_out/stream_$TAG.json
fi
if has fusion; then
  timeout -k 10 300 python bench.py --workload fusion --batch 8 --no-cpu-baseline > gpurun_out/fusion_$TAG.json 2> gpurun_out/fusion_$TAG.err || { echo "fusion failed"; tail gpurun_out/fusion_$TAG.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('fusion', d['value'])" gpurun_out/fusion_$TAG.json
fi
if has prof; then
  rm -rf gpurun_out/prof_$TAG
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bp_$TAG.json 2> gpurun_out/bp_$TAG.err || { echo "rocprof failed"; tail gpurun_out/bp_$TAG.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('probe', d['roofline']['launch_us'], d['roofline']['avg_launch_us'])" gpurun_out/bp_$TAG.json
  python3 tools/rocprof_summary.py "$(ls gpurun_out/prof_$TAG/*kernel_trace.csv | head -1)" --title "rocprofv3 --kernel-trace --stats -- python bench.py --inflight 1 --serial-heads --steps 20 --warmup 3 --no-cpu-baseline (tools/gpu_bundle.sh $TAG)" > gpurun_out/prof_summary_$TAG.txt
  grep -A9 "^# per-stage" gpurun_out/prof_summary_$TAG.txt
fi
if has pmc; then
  rm -rf gpurun_out/pmc_fwd_$TAG
  bash tools/pmc_forward.sh gpurun_out/pmc_fwd_$TAG || { echo "pmc failed"; cat gpurun_out/pmc_fwd_$TAG/failed.txt; exit 1; }
  python3 tools/pmc_forward_summary.py gpurun_out/pmc_fwd_$TAG gpurun_out/pmc_forward_$TAG.json > /dev/null || exit 1
  bash tools/pmc_forward_insts.sh gpurun_out/pmc_insts_$TAG || { echo "pmc insts failed"; exit 1; }
fi
echo done
