# 2-rank rehearsal of bench.py's N > 1 paths on one GPU (gloo instead of RCCL, both ranks on
# the same device): the headline, the KITTI .bin stream (per-batch gather), the fused path
set -u
export TMPDIR=/tmp
export SFA_BENCH_SHARE_DEVICE=1 SFA_DIST_BACKEND=gloo
port=29541
for w in "bev_infer" "stream" "fusion --batch 8"; do
  port=$((port + 1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --steps 10 --warmup 3 --workload $w > gpurun_out/g2.json 2> gpurun_out/g2.err || { echo "gloo rehearsal failed: $w"; tail -20 gpurun_out/g2.err; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/g2.json') if l.startswith('{')][-1]); print(sys.argv[1], d['n_gpus'], d['value'], d['config']['workload'][:200])" "$w"
done
