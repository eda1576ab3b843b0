# headline bench at longer runs (steady state at the power limit) (GPU box)
set -u
export TMPDIR=/tmp
for s in 20 500 2000; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps $s > gpurun_out/sus_$s.json 2> gpurun_out/sus.err || { echo "bench failed"; tail -3 gpurun_out/sus.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('steps', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/sus_$s.json $s
done
echo done
