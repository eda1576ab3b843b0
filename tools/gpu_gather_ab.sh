# N > 1 stream layout rehearsed on one GPU (--sim-gather: a device copy where the all-gather
# goes), interleaved A/B; then a 2-rank gloo rehearsal of the real N > 1 path (run on the GPU box)
set -u
export TMPDIR=/tmp
bash tools/ab_args.sh "" "--sim-gather --gather-stream comm --side-streams on" "--sim-gather --side-streams on" "--sim-gather --side-streams off" || exit 1
SFA_BENCH_SHARE_DEVICE=1 SFA_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/gloo2.json 2> gpurun_out/gloo2.err || { echo "gloo rehearsal failed"; tail -20 gpurun_out/gloo2.err; exit 1; }
cut -c1-400 gpurun_out/gloo2.json
