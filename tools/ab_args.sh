# A/B of bench.py argument sets, interleaved (run on the GPU box):
#   bash tools/ab_args.sh "ARGS1" "ARGS2" ...   (each set benched twice, alternating)
set -u
export TMPDIR=/tmp
for rep in 1 2; do
  i=0
  for args in "$@"; do
    i=$((i + 1))
    timeout -k 10 200 python bench.py --no-cpu-baseline $args > gpurun_out/aba_${i}_$rep.json 2> gpurun_out/aba_${i}_$rep.err || { echo "bench failed: $args"; tail -5 gpurun_out/aba_${i}_$rep.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(repr(sys.argv[2]), sys.argv[3], d['value'], d.get('stages_ms', {}).get('forward'))" gpurun_out/aba_${i}_$rep.json "$args" $rep
  done
done
