# bench.py with dense U[0,1) frames vs the sparse BEV maps of synthetic sweeps: throughput and the
# board's clock / power mid-run (run on the GPU box)
set -u
export TMPDIR=/tmp
for rep in 1 2; do
  for inp in uniform sweeps; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --input $inp > gpurun_out/in.json 2>/dev/null || { echo "failed $inp"; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/in.json')); print(sys.argv[1], d['value'], d['stages_ms']['forward'], d['roofline']['launch_us'])" $inp
  done
done
for inp in uniform sweeps; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --probe-forwards 0 --input $inp --steps 3000 > gpurun_out/in_long_$inp.json 2>/dev/null &
  pid=$!
  sleep 14
  echo "== $inp (3000 steps, mid-run)"; rocm-smi --showpower --showclocks 2>/dev/null | grep -E 'sclk|Power \(W\)' || true
  sleep 3
  rocm-smi --showpower --showclocks 2>/dev/null | grep -E 'sclk|Power \(W\)' || true
  wait $pid || { echo "long run failed"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('value', d['value'])" gpurun_out/in_long_$inp.json
done
