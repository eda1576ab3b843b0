# A/B of bench.py under environment settings, interleaved (run on the GPU box):
#   bash tools/ab_env.sh NAME=V1,NAME=V2,...   (each setting benched twice, alternating)
set -u
export TMPDIR=/tmp
IFS=',' read -ra SETS <<< "$1"
for rep in 1 2; do
  for kv in "${SETS[@]}"; do
    f=gpurun_out/ab_$(echo "$kv" | tr '/' '_')_$rep.json
    env "$kv" timeout -k 10 200 python bench.py --no-cpu-baseline > "$f" 2>/dev/null || { echo "bench failed: $kv"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['stages_ms']['forward'])" "$f" "$kv" $rep
  done
done
