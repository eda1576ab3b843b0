# round 4: weight-stationary layer1 kernel — isolated timing + bits (convbench4), the equivalence
# test, then the bench A/B and a serial rocprof with it on
set -u
export TMPDIR=/tmp
TAG="${1:-r04e}"
timeout -k 10 120 ./tools/convbench4 20 layer1 > gpurun_out/cb4_$TAG.txt 2>&1 || { echo "convbench4 failed"; tail -20 gpurun_out/cb4_$TAG.txt; exit 1; }
grep -E "==|us " gpurun_out/cb4_$TAG.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_abi.py -x -q --timeout 300 --timeout-method thread -k "weight_stationary or abi or option" > gpurun_out/t_$TAG.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_$TAG.txt; exit 1; }
tail -1 gpurun_out/t_$TAG.txt
SFA_CONV_WS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --inflight 1 --serial-heads --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bp_$TAG.json 2> gpurun_out/bp_$TAG.err || { echo "rocprof failed"; tail gpurun_out/bp_$TAG.err; exit 1; }
KT=$(find gpurun_out/prof_$TAG -name "*kernel_trace.csv" -print -quit); python3 tools/rocprof_summary.py "$KT" > gpurun_out/prof_summary_$TAG.txt 2>&1 || true
head -24 gpurun_out/prof_summary_$TAG.txt
bash tools/ab_env.sh SFA_CONV_WS=1,SFA_CONV_WS=0 || exit 1
echo done
