# grouped heads, auto mode (SFA_HEADS_GROUPED=2: grouped when the model has no side stream): stream
# and fusion workloads (no side streams) A/B against per-level launches (0), headline unchanged (GPU box)
set -u
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_stream.py tests/test_gpu_fusion_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread -k "grouped or probe or side_streams or stream or pipeline" > gpurun_out/t_grp2.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_grp2.txt; exit 1; }
tail -1 gpurun_out/t_grp2.txt
for rep in 1 2; do
  for g in 0 2; do
    for w in "--workload stream" "--workload fusion --batch 8" ""; do
      tag=$(echo "$w" | tr -d ' -')
      SFA_HEADS_GROUPED=$g timeout -k 10 200 python bench.py $w --no-cpu-baseline > gpurun_out/grp2_${g}_${tag}_$rep.json 2> gpurun_out/grp2.err || { echo "bench failed: $g $w"; tail -3 gpurun_out/grp2.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('grouped', sys.argv[2], sys.argv[3], d['value'], d.get('stages_ms', {}).get('forward'))" gpurun_out/grp2_${g}_${tag}_$rep.json $g "$tag"
    done
  done
done
echo done
