set -u
export TMPDIR=/tmp
timeout -k 10 300 ./tools/convbench 20 "head L" > gpurun_out/cb_l0.txt 2>&1 || { echo "convbench failed"; tail gpurun_out/cb_l0.txt; exit 1; }
cat gpurun_out/cb_l0.txt
SFA_BENCH_SHARE_DEVICE=1 SFA_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/b_gloo2.json 2> gpurun_out/b_gloo2.err || { echo "gloo2 failed"; tail -20 gpurun_out/b_gloo2.err; exit 1; }
cut -c1-600 gpurun_out/b_gloo2.json
