set -u
export TMPDIR=/tmp
for n in 2 3 4 2 3; do
  timeout -k 10 200 python bench.py --inflight $n --no-cpu-baseline --steps 40 > gpurun_out/if_$n.json 2> gpurun_out/if_$n.err || { echo "bench $n failed"; tail gpurun_out/if_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/if_$n.json'));print($n, d['value'], d['ms_per_step'])"
done
