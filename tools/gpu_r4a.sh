# round 4, first GPU pass: GPU tests (incl. the shared-scratch BEV test), headline bench, and the
# N > 1 paths self-launched by bench.py (2 ranks on one GPU over gloo: SFA_BENCH_SHARE_DEVICE)
set -u
export TMPDIR=/tmp
TAG="${1:-r04a}"
# the pruned product library against the round-3 build (tools/experiments/r03/libsfa_hip_r03.so)
timeout -k 10 300 python tools/ab_lib_bits.py run gpurun_out/bits_new_$TAG.npz > gpurun_out/bits_$TAG.log 2>&1 || { echo "bits new failed"; tail gpurun_out/bits_$TAG.log; exit 1; }
SFA_HIP_LIB=tools/experiments/r03/libsfa_hip_r03.so SFA_ABI_EXPECT=1 timeout -k 10 300 python tools/ab_lib_bits.py run gpurun_out/bits_r03_$TAG.npz >> gpurun_out/bits_$TAG.log 2>&1 || { echo "bits r03 failed"; tail gpurun_out/bits_$TAG.log; exit 1; }
python tools/ab_lib_bits.py compare gpurun_out/bits_r03_$TAG.npz gpurun_out/bits_new_$TAG.npz | tail -5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_gpu_$TAG.txt 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/t_gpu_$TAG.txt; exit 1; }
tail -1 gpurun_out/t_gpu_$TAG.txt
timeout -k 10 400 python bench.py > gpurun_out/b_$TAG.json 2> gpurun_out/b_$TAG.err || { echo "bench failed"; tail gpurun_out/b_$TAG.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], d['stages_ms']['forward'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['parity']['ok'], d['parity']['max_rel_logit_err'], d['cpu_baseline']['value'])" gpurun_out/b_$TAG.json
export SFA_BENCH_SHARE_DEVICE=1 SFA_DIST_BACKEND=gloo
for w in "bev_infer" "stream" "fusion --batch 8"; do
  timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --workload $w > gpurun_out/g2_$TAG.json 2> gpurun_out/g2_$TAG.err || { echo "self-launched gloo rehearsal failed: $w"; tail -20 gpurun_out/g2_$TAG.err; exit 1; }
  python3 -c "import json,sys; L=[l for l in open('gpurun_out/g2_$TAG.json') if l.startswith('{')]; assert len(L)==1, L; d=json.loads(L[0]); print(sys.argv[1], d['n_gpus'], d['value'], d['config']['workload'][:120])" "$w"
done

timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bp_$TAG.json 2> gpurun_out/bp_$TAG.err || { echo "rocprof failed"; tail gpurun_out/bp_$TAG.err; exit 1; }
KT=$(find gpurun_out/prof_$TAG -name "*kernel_trace.csv" -print -quit); python3 tools/rocprof_summary.py "$KT" > gpurun_out/prof_summary_$TAG.txt 2>&1 || true
head -30 gpurun_out/prof_summary_$TAG.txt
timeout -k 10 300 ./tools/convbench4 20 > gpurun_out/cb4_$TAG.txt 2>&1 || { echo "convbench4 failed"; tail gpurun_out/cb4_$TAG.txt; exit 1; }
grep -E "==|us " gpurun_out/cb4_$TAG.txt
echo done
