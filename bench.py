#!/usr/bin/env python3
"""Benchmark of the MI355X hot path — BEV frames/s at 608x608, bs=16 per GPU.

One step = one batch of 16 synthetic 3x608x608 BEV frames, resident in HBM,
through the KFPN FPN-ResNet-18 forward (23 implicit-GEMM conv launches — split-operand
MFMA, ``--math fp16x3|bf16x6|f32`` (include/sfa_hip.h sfa_math) — + maxpool /
upsample / KFPN kernels) and the fused sigmoid + decode (K=50), each
captured as a HIP graph; with N > 1 the step also all-gathers the (16, 50, 10)
detections over RCCL (frames are sharded: rank r owns its own 16 frames).
``--workload e2e`` starts each step from raw point clouds (BEV voxelisation on
the GPU as well).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       N > 1: either launched per rank by torch.distributed.run (RANK / WORLD_SIZE set), or
       self-launched: with WORLD_SIZE unset the process touches no GPU, starts N rank processes
       of itself (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT) and exits with
       the first failing rank's status (launch_ranks; the reference's own multi-process entry
       spawns its ranks too: train.py:58-67 mp.spawn).
Prints ONE JSON line on rank 0.
"""

from __future__ import annotations

import argparse
import json
import os
import platform
import signal
import socket
import subprocess
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
SFA_ROOT = os.path.join(REPO, "lidar-image_object-detection_-fpn_resnet-yolov8_amd", "sfa")
sys.path.insert(0, SFA_ROOT)

from sfa_hip import _lib, synthetic  # noqa: E402
from sfa_hip.runtime import (DEFAULT_BOUNDARY, DEFAULT_HEADS, DetectorPipeline, KfpnEngine,  # noqa: E402
                             pack_state_dict)

# Algorithmic work per frame at 608x608: 53 convs.
CONV_MACS_PER_FRAME = 31_283_555_328
CONV_FLOP_PER_FRAME = 2 * CONV_MACS_PER_FRAME
PEAK_FP32_MFMA_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32, dense
PEAK_BF16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA
# bf16x6 computes each f32 MAC as 6 bf16 MFMA products: its f32-equivalent ceiling
PEAK_BF16X6_TFLOPS = PEAK_BF16_MFMA_TFLOPS / 6
# fp16x3: 3 fp16 MFMA products per f32 MAC (fp16 MFMA has the bf16 rate)
PEAK_FP16X3_TFLOPS = PEAK_BF16_MFMA_TFLOPS / 3
# measured on MI355X: pure v_mfma_f32_16x16x32_f16 chains over the whole chip settle at the
# board's power / current limit (~1,990 MHz, 1,300 W): tools/micro/mfma_power.hip,
# profiles/r02_power_cap.txt. The practical ceiling the bench (itself at the 1,375 W limit) sees.
MEASURED_FP16_MFMA_CAPPED_TFLOPS = 1883.0
PEAKS_CAPPED = {"fp16x3": MEASURED_FP16_MFMA_CAPPED_TFLOPS / 3, "bf16x6": MEASURED_FP16_MFMA_CAPPED_TFLOPS / 6}
MATHS = {"fp16x3": _lib.MATH_FP16X3, "bf16x6": _lib.MATH_BF16X6, "f32": _lib.MATH_F32}
PEAKS = {"fp16x3": (PEAK_FP16X3_TFLOPS, "dense fp16 MFMA 2500 TF / 3 fp16 products per f32 MAC"),
         "bf16x6": (PEAK_BF16X6_TFLOPS, "dense bf16 MFMA 2500 TF / 6 bf16 products per f32 MAC"),
         "f32": (PEAK_FP32_MFMA_TFLOPS, "dense f32 MFMA (v_mfma_f32_32x32x2_f32)")}
DTYPES = {"fp16x3": "f32 (fp16x3: power-of-two-scaled operands split into 2 fp16 terms, "
                    "3 products, f32 accumulate)",
          "bf16x6": "f32 (bf16x6: operands split into 3 bf16 terms, 6 products, f32 accumulate)",
          "f32": "f32"}
METRIC = "BEV frames/sec (608x608, bs=16)"
# Synthetic weights of every workload (sfa_hip.synthetic.synthetic_state_dict seed).  Seed 2, not 0:
# on the uniform BEV frames seed 0's heatmaps put every top-51 score at the decode's 1 - 1e-4 clamp
# (~5,000 tied peaks per frame), so its detections were a tie order and the timed batch could not be
# compared with the reference's own detections; seed 2's top scores (~0.95) are distinct and
# tests/golden/bench_golden.npz holds the reference's forward + decode of this exact batch.
BENCH_WEIGHT_SEED = 2


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--K", type=int, default=50)
    ap.add_argument("--workload", choices=["bev_infer", "e2e", "stream", "fusion"],
                    default="bev_infer",
                    help="bev_infer: resident BEV frames (the headline); e2e: resident raw sweeps; "
                         "stream: KITTI .bin files read + DMA'd per batch (SURVEY §8(f) #3); "
                         "fusion: BASELINE configs[4] chain up to camera-LiDAR fusion + NMS "
                         "(use --batch 8)")
    env_math = {v: k for k, v in MATHS.items()}[_lib.math_from_env()]
    ap.add_argument("--math", choices=list(MATHS), default=env_math,
                    help="convolution arithmetic (include/sfa_hip.h sfa_math; default: SFA_MATH "
                         "or the library default)")
    ap.add_argument("--input", choices=["uniform", "sweeps"], default="uniform",
                    help="bev_infer frames: U[0,1) in every cell (dense, the default), or the BEV maps "
                         "of synthetic 132,880-point sweeps (sparse like KITTI; made on the GPU before "
                         "the timed region)")
    ap.add_argument("--bev-layout", choices=["nchw3", "nhwc4"], default="nchw3",
                    help="--workload e2e: the voxeliser's output / model input layout (the patch stem reads "
                         "either; NCHW3 moves 3/4 of NHWC4's bytes)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--inflight", type=int, default=None,
                    help="steps in flight on separate streams (each with its own buffers and "
                         "model handle); >1 lets one step's kernel tails overlap the next's. "
                         "Default 2; 3 for --workload fusion (bs=8: profiles/r02c_ab_fusion_inflight3.txt)")
    ap.add_argument("--fusion-nms", choices=["greedy", "gaussian"], default="greedy",
                    help="--workload fusion: test6.py's greedy NMS or the README's Gaussian soft-NMS "
                         "(README.md:250-261)")
    ap.add_argument("--stream-inflight", type=int, default=2,
                    help="--workload stream: pipelines in flight; with 2+ the engines run without "
                         "side streams (profiles/r02b_stream_side_streams.txt)")
    ap.add_argument("--side-streams", choices=["auto", "on", "off"], default="auto",
                    help="the models' level-0-heads side streams (sfa_model_set_side_streams); auto: "
                         "on at N = 1 with at most 2 steps in flight, else off (side_streams_for)")
    ap.add_argument("--gather-stream", choices=["step", "comm"], default="step",
                    help="N > 1: the detections' all-gather on each step's own stream, or on one "
                         "extra stream")
    ap.add_argument("--sim-gather", action="store_true",
                    help="N = 1: rehearse the N > 1 layout on one GPU: the models without side "
                         "streams (side_streams_for) and, where the all-gather goes, a device copy of "
                         "the detections enqueued the way torch's RCCL process group enqueues a "
                         "collective (its own stream, created on first use, joined to the step's stream "
                         "before and after)")
    ap.add_argument("--dump-dets", default=None, metavar="NPZ",
                    help="after the timed region, every pipeline runs one more step and rank 0 writes "
                         "the gathered detections (nf, world*B, K, 10), frame ids (nf, world*B) and each "
                         "rank's input seed to NPZ (tests/test_gpu_bench_multirank.py)")
    ap.add_argument("--share-weights", action="store_true",
                    help="the in-flight pipelines share one device copy of the packed weights "
                         "(KfpnEngine.twin) instead of one copy each")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--serial-heads", action="store_true",
                    help="keep the level-0 heads on the main stream (no side stream) for the whole "
                         "run: with --inflight 1 every head launch then has the chip to itself, "
                         "the configuration the roofline probe measures (for rocprof agreement)")
    ap.add_argument("--probe-forwards", type=int, default=10,
                    help="un-captured forwards timed per head launch for the roofline")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: every rank joins a gloo group and runs --steps all-gathers of "
                         "rank-coded (B, K, 10) detections through sfa_hip.dist (rank wiring, the "
                         "gather and the single JSON line; tests/test_bench_launcher.py)")
    args = ap.parse_args(argv)
    if args.inflight is None:
        args.inflight = 3 if args.workload == "fusion" else 2
    return args


def side_streams_for(args, world, nf):
    """The models' side streams: every stream of the process takes one of HIP's 4 hardware
    queues, so "auto" keeps them only while the pipelines' streams and theirs fit (N = 1, at
    most 2 pipelines); RCCL's own stream at N > 1 and a third pipeline do not
    (profiles/r02b_ab_gather_streams.txt, r02c_ab_fusion_inflight3.txt)."""
    return {"on": True, "off": False,
            "auto": world == 1 and not getattr(args, "sim_gather", False) and nf <= 2}[args.side_streams]


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv, poll_s: float = 0.05) -> int:
    """--gpus N > 1 started without a launcher: start N rank processes of this script (same
    argv) and wait for them.  Called before anything touches a GPU (no torch.cuda call, no HIP
    library load), so every child initialises its own device from a fresh process.  Rank r gets
    RANK = LOCAL_RANK = r, WORLD_SIZE = LOCAL_WORLD_SIZE = N, MASTER_ADDR = 127.0.0.1 and a free
    MASTER_PORT (kept if the caller set one).  Rank 0's stdout is this process's (its JSON line
    goes out unchanged; the other ranks print none).  The first rank to exit non-zero ends the
    others (SIGTERM, then SIGKILL after 10 s) so no survivor waits on a collective forever, and
    its status is returned; 0 when every rank exits 0.  The ranks stay in this process's
    process group (a timeout that kills the group ends them too), a SIGTERM / SIGINT to this
    process is passed on to them, and each rank gets SIGTERM if this process dies
    (PR_SET_PDEATHSIG)."""
    port = os.environ.get("MASTER_PORT") or str(_free_port())

    def _pdeathsig():
        try:
            import ctypes
            ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, int(signal.SIGTERM))  # PR_SET_PDEATHSIG
        except OSError:
            pass

    procs = []

    def _end(live, sig):
        for q in live:
            try:
                q.send_signal(sig)
            except ProcessLookupError:
                pass

    def _forward(signo, _frame):
        _end([p for p in procs if p.poll() is None], signo)
        raise SystemExit(128 + signo)

    old = {s: signal.signal(s, _forward) for s in (signal.SIGTERM, signal.SIGINT)}
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                       LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                          preexec_fn=_pdeathsig))
        status = 0
        live = list(procs)
        while live:
            for p in list(live):
                rc = p.poll()
                if rc is None:
                    continue
                live.remove(p)
                if rc != 0 and status == 0:
                    status = rc if rc > 0 else 128 - rc  # killed by a signal: 128 + signo, as a shell reports
                    _end(live, signal.SIGTERM)
                    deadline = time.time() + 10
                    for q in live:
                        try:
                            q.wait(timeout=max(0.1, deadline - time.time()))
                        except subprocess.TimeoutExpired:
                            q.kill()
                            q.wait()
                    live = []
                    break
            if live:
                time.sleep(poll_s)
        return status
    finally:
        for s, h in old.items():
            signal.signal(s, h)


def run_dry(args):
    """--dry-run: the N > 1 wiring without a GPU.  Each rank joins a gloo group, enqueues
    --warmup + --steps all-gathers of its (B, K, 10) detections whose values encode (rank, step)
    through sfa_hip.dist.gather_detections (the bench's collective, CPU tensors), checks every
    gathered row and id, and the max-over-ranks time gives the JSON line rank 0 prints.
    SFA_BENCH_FAIL_RANK=r makes rank r exit 3 after joining the group (exit-status tests)."""
    import torch.distributed as dist
    from sfa_hip import dist as sdist
    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        dist.init_process_group("gloo")
    if os.environ.get("SFA_BENCH_FAIL_RANK", "") == str(rank):
        sys.stderr.write(f"rank {rank}: SFA_BENCH_FAIL_RANK\n")
        sys.stderr.flush()
        os._exit(3)
    B, K = args.batch, args.K

    def step(k):
        dets = torch.zeros((B, K, 10), dtype=torch.float32)
        dets[:, :, 0] = float(rank)
        dets[:, :, 1] = float(k)
        ids = torch.arange((k * world + rank) * B, (k * world + rank + 1) * B, dtype=torch.int64)
        if world == 1:
            return dets, ids
        d, i = sdist.gather_detections(dets, ids)
        exp = torch.cat([torch.arange((k * world + r) * B, (k * world + r + 1) * B) for r in range(world)])
        if not torch.equal(i, exp) or not torch.equal(d[:, :, 0], torch.arange(world).repeat_interleave(B)
                                                        .float()[:, None].expand(-1, K)) \
                or not bool(torch.all(d[:, :, 1] == float(k))):
            raise SystemExit(f"rank {rank}: gathered detections / ids of step {k} are wrong")
        return d, i

    for k in range(args.warmup):
        step(k)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        frames = world * B * args.steps
        print(json.dumps({
            "metric": METRIC, "value": round(frames / max(elapsed, 1e-9), 2), "unit": "frames/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / max(1, args.steps) * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "dry_run": True,
            "config": {"workload": "dry run: gloo all-gather of rank-coded (B, K, 10) detections only "
                                   "(no GPU, no model)", "global_batch": world * B,
                       "parallelism": f"dp{world}", "launcher": os.environ.get("SFA_BENCH_LAUNCHER", "external")},
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


def init_dist(n):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != n:
        raise SystemExit(f"--gpus {n} but WORLD_SIZE={world}: start the ranks with torch.distributed.run "
                         "--nproc-per-node N, or run without WORLD_SIZE set and bench.py launches them")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # SFA_BENCH_SHARE_DEVICE=1 + SFA_DIST_BACKEND=gloo: rehearse the N>1 path on one GPU
    if os.environ.get("SFA_BENCH_SHARE_DEVICE") == "1":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("SFA_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, torch.device("cuda", local)


def build_pipeline(dev, args, rank, engine=None):
    if engine is None:
        arch = _lib.make_arch(DEFAULT_HEADS)
        spec = _lib.state_layout(arch)
        sd = synthetic.synthetic_state_dict(spec, seed=BENCH_WEIGHT_SEED)
        engine = KfpnEngine(arch, pack_state_dict(sd, arch), dev,
                            math=MATHS[args.math])
    if args.workload == "e2e":
        clouds = [synthetic.synthetic_point_cloud(1000 * rank + i + 1) for i in range(args.batch)]
        pipe = DetectorPipeline(engine, args.batch, K=args.K, with_bev=True,
                                max_points=sum(c.shape[0] for c in clouds), bev_layout=args.bev_layout)
        pipe.set_points(clouds)
    else:
        pipe = DetectorPipeline(engine, args.batch, K=args.K)
        if args.input == "sweeps":
            from sfa_hip.runtime import BevVoxelizer
            clouds = [synthetic.synthetic_point_cloud(1000 * rank + i + 1) for i in range(args.batch)]
            offs = np.cumsum([0] + [c.shape[0] for c in clouds])
            pts = torch.from_numpy(np.concatenate(clouds)).to(dev)
            BevVoxelizer(dev, args.batch)(pts, offs, layout=_lib.BEV_NCHW3_F32, out=pipe.x)
            torch.cuda.synchronize()
        else:
            pipe.x.copy_(torch.from_numpy(synthetic.synthetic_bev(args.batch, seed=1 + rank)))
    return pipe


class StepGraphs:
    """forward and decode captured as two graphs so HIP events can bracket each."""

    def __init__(self, pipe: DetectorPipeline, use_graph: bool):
        self.pipe = pipe
        p = pipe
        o = p.outs
        from sfa_hip.runtime import _decoder

        def fwd():
            st = _lib.stream_ptr(p.dev)
            if p.with_bev:
                p.vox(p.points, p.offsets, layout=p.bev_fmt, flags=_lib.BEV_RAW, out=p.bev, stream=st)
                p.engine.forward_into(p.bev, o, p.in_fmt, p.ws, st)
            else:
                p.engine.forward_into(p.x, o, _lib.IN_NCHW3, p.ws, st)

        def dec():
            _decoder(o["hm_cen"], o["cen_offset"], o["direction"], o["z_coor"], o["dim"], K=p.K,
                     apply_sigmoid=True, out=p.dets, stream=_lib.stream_ptr(p.dev), workspace=p.dec_ws)

        self.fns = [fwd, dec]
        self.graphs = None
        if use_graph:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                fwd()
                dec()
            torch.cuda.current_stream().wait_stream(s)
            self.graphs = []
            for fn in self.fns:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    fn()
                self.graphs.append(g)

    def run(self, i):
        if self.graphs is None:
            self.fns[i]()
        else:
            self.graphs[i].replay()


class BevInferBench:
    """The timed configuration of the bev_infer / e2e workloads: ``--inflight`` pipelines (own
    model handle, buffers and stream each), forward and decode captured as HIP graphs, the
    models' side streams per ``side_streams_for``; at N > 1 each step all-gathers its detections.
    ``one_step(k)`` enqueues step k on stream k % nf.  tests/test_gpu_bench_parity.py builds this
    same object and checks every frame of it against the oracle."""

    def __init__(self, args, rank, world, dev):
        self.args, self.rank, self.world, self.dev = args, rank, world, dev
        nf = self.nf = max(1, args.inflight)
        pipes = self.pipes = [build_pipeline(dev, args, rank)]
        for _ in range(nf - 1):  # own model handle each; weights shared (--share-weights) or a copy each
            pipes.append(build_pipeline(dev, args, rank, pipes[0].engine.twin() if args.share_weights else None))
        # side streams: every stream of the process takes one of HIP's 4 hardware queues; with
        # N > 1 RCCL adds its own stream, so the models run without theirs
        # (profiles/r02b_ab_gather_streams.txt: the N > 1 layout rehearsed with --sim-gather).
        self.side = side_streams_for(args, world, nf)
        for p in pipes:
            p.engine.set_side_streams(self.side)
        if args.serial_heads:
            for p in pipes:
                p.engine.set_probe(_lib.PROBE_SERIAL)
        self.steps = [StepGraphs(p, not args.no_graph) for p in pipes]
        self.streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(nf - 1)]
        # --sim-gather (N = 1): a device copy of the detections in place of the all-gather, on a
        # stream of its own joined to the step's stream as ProcessGroupNCCL joins its RCCL stream
        # (the N > 1 stream layout rehearsed on one GPU)
        self.gather = world > 1 or args.sim_gather
        self.last_gathered = [None] * nf
        if self.gather:
            self.frame_ids = torch.arange(rank * args.batch, (rank + 1) * args.batch, device=dev)
            self.sim_out = torch.empty((world * args.batch,) + tuple(pipes[0].dets.shape[1:]),
                                       dtype=torch.float32, device=dev)
            self.sim_stream = None
        self.comm_mode = self.gather and args.gather_stream == "comm"
        if self.comm_mode:
            # all-gathers on one extra stream in step order (the same collective order on every
            # rank); a pipeline's detections are overwritten only after their gather finished
            self.comm = torch.cuda.Stream()
            self.step_done = [torch.cuda.Event() for _ in range(nf)]
            self.comm_done = [torch.cuda.Event() for _ in range(nf)]
            self.gathered = [0] * nf

    def do_gather(self, dets):
        if self.world > 1:
            from sfa_hip import dist as sdist
            return sdist.gather_detections(dets, self.frame_ids)
        cur = torch.cuda.current_stream()
        if self.sim_stream is None:  # created on first use, after every pipeline's streams
            self.sim_stream = torch.cuda.Stream()
        self.sim_stream.wait_stream(cur)
        with torch.cuda.stream(self.sim_stream):
            self.sim_out.copy_(dets)
        cur.wait_stream(self.sim_stream)
        return self.sim_out, self.frame_ids

    def one_step(self, k, ev=None):
        i = k % self.nf
        with torch.cuda.stream(self.streams[i]):
            if self.comm_mode and self.gathered[i]:
                self.streams[i].wait_event(self.comm_done[i])
            if ev is not None:
                ev[0].record()
            self.steps[i].run(0)
            if ev is not None:
                ev[1].record()
            self.steps[i].run(1)
            if ev is not None:
                ev[2].record()
            if self.comm_mode:
                self.step_done[i].record()
            elif self.gather:
                # on the step's own stream, in step order (the same collective order on every
                # rank); RCCL's stream waits for this step only, the other pipeline runs on
                self.last_gathered[i] = self.do_gather(self.pipes[i].dets)
        if self.comm_mode:
            with torch.cuda.stream(self.comm):
                self.comm.wait_event(self.step_done[i])
                self.last_gathered[i] = self.do_gather(self.pipes[i].dets)
                self.comm_done[i].record()
            self.gathered[i] = 1


def dump_gathered(args, bench, rank, world):
    """--dump-dets: one more step per pipeline after the timed region (every rank, so the
    collectives pair up); rank 0 writes what each step's gather returned."""
    dets, ids, local = [], [], []
    for i in range(bench.nf):
        bench.one_step(i)
        torch.cuda.synchronize()
        d, fid = bench.last_gathered[i] if bench.gather else (bench.pipes[i].dets, None)
        dets.append(d.cpu().numpy())
        ids.append(fid.cpu().numpy() if fid is not None else np.arange(args.batch, dtype=np.int64))
        local.append(bench.pipes[i].dets.cpu().numpy())
    if rank == 0:
        np.savez(args.dump_dets, dets=np.stack(dets), ids=np.stack(ids), local=np.stack(local),
                 input_seed=np.array([1 + r for r in range(world)], np.int64), world=np.int64(world),
                 side_streams=np.int64(bench.side))


def _lib_sha256():
    import hashlib
    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def _pmc_forward_file(args):
    """The newest committed PMC pass (tools/pmc_forward.sh -> tools/pmc_forward_summary.py ->
    profiles/r*_pmc_forward_<math>.json) that ran THIS library build (its lib_sha256 equals the
    loaded libsfa_hip.so's): traffic measured on other kernels is never reported.  rocprofv3 cannot
    run inside this process, so the counters come from that separate pass of the same command."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_pmc_forward_{args.math}.json")))
    if not files and args.math == "f32":
        files = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc_forward.json")))
    sha = _lib_sha256()
    for fn in reversed(files):
        with open(fn) as f:
            d = json.load(f)
        if d.get("lib_sha256") == sha:
            return fn, d
    return None, None


def traffic_per_forward(args):
    """HBM bytes of the conv launches of one forward (PMC pass of this library build), or None."""
    if args.workload != "bev_infer" or args.batch != 16:
        return None
    _, d = _pmc_forward_file(args)
    return int(d["conv_hbm_bytes_per_forward"]) if d else None


def head_traffic_per_launch(args):
    """HBM bytes per head launch (mean over the 3 levels) from the PMC pass of this library build
    (tools/pmc_forward.sh: FETCH_SIZE x2 + WRITE_SIZE per dispatch, the probe's serial forward)."""
    if args.workload != "bev_infer" or args.batch != 16 or args.math != "fp16x3":
        return None
    fn, d = _pmc_forward_file(args)
    if not d:
        return None
    rows = [r for r in d["per_launch"] if r["kernel"].startswith("sfa::conv_r3_kernel<256, 320")]
    return {"bytes": int(sum(r["hbm_MB"] for r in rows) * 1e6 / len(rows)), "file": os.path.relpath(fn, REPO),
            "kernel": rows[0]["kernel"]} if len(rows) == 3 else None


def head_flop_per_launch(args):
    """Algorithmic f32 FLOP of one head-level launch: the 5 heads' 3x3 convs
    (C_l -> 64 each, as one N = 320 GEMM) + their 1x1 convs (64 -> c_h), over B frames."""
    hc = sum(c for c in DEFAULT_HEADS.values())
    n = 64 * len(DEFAULT_HEADS)
    out = []
    for c_in, div in ((256, 8), (128, 4), (64, 4)):
        px = args.batch * (608 // div) ** 2
        out.append(2 * px * (n * 9 * c_in + hc * 64))
    return out


def probe_heads(args, pipe, step):
    """Per-launch durations of the dominant kernel (the fused detection heads, one launch per
    KFPN level, 54.6 % of the FLOPs) from HIP events the library records on the launching
    stream around each launch (sfa_model_set_probe): un-captured forwards, one step in flight,
    all launches on one stream, so each head launch has the chip to itself."""
    if args.workload != "bev_infer":
        return None
    eng = pipe.engine
    eng.set_probe(_lib.PROBE_HEADS | _lib.PROBE_SERIAL)
    try:
        torch.cuda.synchronize()
        per = []
        for _ in range(args.probe_forwards):
            step.fns[0]()
            per.append(eng.probe_times(3))
    finally:
        eng.set_probe(_lib.PROBE_SERIAL if args.serial_heads else 0)
    return np.median(np.array(per), axis=0).tolist()  # ms per level


def probe_bev(args, pipe, reps=20):
    """configs[2]: the BEV voxelisation pass alone (filter fused; sfa_bev_voxelize's blocked
    bin + strip kernels) on the pipeline's resident sweeps, HIP events on the launching stream,
    against the HBM roofline: algorithmic bytes = N * 16 (xyzi read) + 3 * 608^2 * 4 (f32 map
    written) per frame; scratch key / count traffic is not algorithmic."""
    if args.workload != "e2e":
        return None
    st = _lib.stream_ptr(pipe.dev)

    def vox():
        pipe.vox(pipe.points, pipe.offsets, layout=pipe.bev_fmt, flags=_lib.BEV_RAW, out=pipe.bev,
                 stream=st)

    vox()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        vox()
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    npts = int(pipe.offsets[-1])
    algo = npts * 16 + pipe.B * 3 * 608 * 608 * 4
    ach = algo / (ms * 1e-3) / 1e9
    traffic = None  # PMC HBM bytes per call (tools/pmc_bev.sh) of this library build at this batch
    import glob
    sha = _lib_sha256()
    for fn in reversed(sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc_bev.json")))):
        with open(fn) as f:
            d = json.load(f)
        if pipe.B == 16 and d.get("lib_sha256") == sha:
            traffic = int(d["bev_hbm_bytes_per_call"])
            break
    return {"bound": "hbm", "unit": "GB/s", "achieved": round(ach, 1), "peak": 8000.0,
            "frac": round(ach / 8000.0, 4), "traffic": traffic,
            "traffic_basis": "PMC 2 x FETCH_SIZE + WRITE_SIZE of one call (profiles/r*_pmc_bev.json): points read "
                             "once by the bin pass, 8-B records written and read once, the top points' intensities "
                             "gathered, the NCHW3 f32 map written",
            "kernel": "sfa_bev_voxelize (SFA_BEV_RAW: filter fused; bev_blk_bin_kernel: 1024 points per block "
                      "binned by 4-row strip into the block's record region of 8-B records; bev_blk_strip_kernel: "
                      "each strip reduced in LDS)",
            "us_per_batch": round(1e3 * ms, 1), "points_per_batch": npts,
            "algorithmic_bytes_per_batch": algo,
            "measured": "HIP events around %d back-to-back voxelisations of the step's %d sweeps, "
                        "one stream, nothing else running" % (reps, pipe.B)}


def roofline_line(args, heads, forward_roofline, fwd_achieved, peak, peak_basis, capped):
    line = {"bound": "mfma", "unit": "TFLOP/s", "peak": round(peak, 2), "peak_basis": peak_basis,
            "peak_power_capped": round(capped, 2) if capped else None,
            "peak_power_capped_basis": "measured pure-MFMA chip ceiling at the board power limit "
                                       "(1883 TF fp16 / products per MAC; profiles/r02_power_cap.txt)",
            "traffic": None, "forward": forward_roofline}
    fwd_traffic = traffic_per_forward(args)
    forward_roofline["traffic"] = fwd_traffic
    if heads is None:  # no probe: the whole forward is the unit
        line.update({"kernel": "the whole forward (math %s)" % args.math, "achieved": round(fwd_achieved, 3),
                     "frac": round(fwd_achieved / peak, 4), "traffic": fwd_traffic})
        return line
    flops = head_flop_per_launch(args)
    ach = sum(flops) / (sum(heads) * 1e-3) / 1e12
    line.update({
        "kernel": {"fp16x3": "conv_r3_kernel<256, 320, ...> (fused detection heads: 3x3 conv C->5x64 + bias + "
                             "ReLU + the 5 heads' 1x1 convs; one launch per KFPN level)",
                   "bf16x6": "conv_x6g_kernel<256, 320, ...> (fused detection heads)",
                   "f32": "conv_mfma_kernel<128, 64, ...> (detection heads)"}[args.math],
        "achieved": round(ach, 3), "frac": round(ach / peak, 4),
        "frac_of_power_capped": round(ach / capped, 4) if capped else None,
        "frac_of_f32_mfma_peak": round(ach / PEAK_FP32_MFMA_TFLOPS, 4),
        "measured": "HIP events on the launching stream around each head launch, median of %d "
                    "un-captured forwards, one step in flight, no side stream (sfa_model_set_probe); "
                    "achieved = algorithmic FLOP of the 3 launches / their summed durations" % args.probe_forwards,
        "launch_us": [round(1e3 * v, 1) for v in heads],
        "avg_launch_us": round(1e3 * sum(heads) / 3, 1),
        "algorithmic_flop_per_launch": flops,
    })
    ht = head_traffic_per_launch(args)
    line["traffic"] = ht["bytes"] if ht else None
    line["traffic_basis"] = (
        "HBM bytes per launch, mean of the 3 levels: PMC 2 x FETCH_SIZE + WRITE_SIZE of %s (tools/pmc_forward.sh "
        "on this library build, sha256 matched; kernel %s)" % (ht["file"], ht["kernel"]) if ht else
        "null: no committed PMC pass (profiles/r*_pmc_forward_%s.json) ran this library build "
        "(lib_sha256 %s...)" % (args.math, _lib_sha256()[:16]))
    return line


def _cpu_model_name():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def _cpu_threads():
    """Host threads for the CPU baseline: every core this process may run on
    (len(sched_getaffinity)) -- unless OMP_NUM_THREADS caps the process' CPU
    share (the GPU box sets it to that share: its affinity mask lists the whole machine)."""
    ncores = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    threads = min(ncores, int(omp)) if omp.isdigit() and int(omp) > 0 else ncores
    return threads, ncores


def cpu_baseline(args, bench=None):
    """The CPU leg: the oracle -- the torch fp32 CPU restatement of the reference
    forward, verified bit-for-bit against reference-generated fixtures, + the numpy restatement
    of _sigmoid / decode (+ makeBEVMap for e2e) -- on the SAME batch of 16 frames the GPU step
    processes, 2 warm-ups then the median of 5 batches, all allotted host threads.

    Outside the timed region it doubles as the parity check of the timed configuration: the
    GPU's logits for those frames (pipeline 0, one more graph replay) against the oracle's
    (``max_rel_logit_err``, bar 1e-4 * max(1, |ref|)), the GPU's detections against the oracle
    decode of the GPU's own sigmoid maps (bit-exact: same maps in, same top-K / gathers out), for
    e2e the GPU BEV maps against the oracle's makeBEVMap (bit-exact)."""
    sys.path.insert(0, REPO)
    from oracle import bev_oracle, decode_oracle, model_oracle
    threads, ncores = _cpu_threads()
    torch.set_num_threads(threads)
    arch = _lib.make_arch(DEFAULT_HEADS)
    sd = model_oracle.state_dict_torch(synthetic.synthetic_state_dict(_lib.state_layout(arch), BENCH_WEIGHT_SEED))
    B = args.batch
    e2e = args.workload == "e2e"
    clouds = [synthetic.synthetic_point_cloud(i + 1) for i in range(B)] if e2e else None
    x_uniform = None if e2e or args.input != "uniform" else torch.from_numpy(synthetic.synthetic_bev(B, seed=1))

    def one_batch():
        if e2e or x_uniform is None:
            cl = clouds if clouds is not None else [synthetic.synthetic_point_cloud(i + 1) for i in range(B)]
            maps = [bev_oracle.makeBEVMap(bev_oracle.get_filtered_lidar(c, DEFAULT_BOUNDARY), DEFAULT_BOUNDARY)
                    for c in cl]
            x = torch.from_numpy(np.stack(maps).astype(np.float32))
        else:
            maps, x = None, x_uniform
        with torch.no_grad():
            out = model_oracle.forward(sd, x)
        hm = decode_oracle.sigmoid_clamp(out["hm_cen"].numpy())
        off = decode_oracle.sigmoid_clamp(out["cen_offset"].numpy())
        dets = decode_oracle.decode(hm, off, out["direction"].numpy(), out["z_coor"].numpy(),
                                    out["dim"].numpy(), K=args.K)
        return maps, out, dets

    for _ in range(2):
        one_batch()
    times = []
    for _ in range(5):
        t0 = time.perf_counter()
        maps, out, dets = one_batch()
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    cpu = {"value": round(B / med, 3), "unit": "frames/s", "cores": threads, "kind": "port",
           "sample": (f"bs={B} batch of the timed workload ({'16 synthetic 132,880-pt sweeps: makeBEVMap + ' if e2e else ''}"
                      f"3x608x608 forward + sigmoid + decode K={args.K}), 2 warm-ups, median of 5 batches "
                      f"({med:.2f} s/batch); oracle = torch {torch.__version__} fp32 CPU forward + numpy "
                      f"decode; host {_cpu_model_name()}, {threads} threads (affinity {ncores} cores, "
                      f"OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')})")}
    if bench is None:
        return cpu, None
    # parity of the timed configuration (pipeline 0 of the in-flight set, its captured graphs)
    pipe = bench.pipes[0]
    torch.cuda.synchronize()
    bench.one_step(0)
    torch.cuda.synchronize()
    worst = 0.0
    for h, _ in pipe.engine.heads:
        g = pipe.outs[h].cpu().numpy()
        r = out[h].numpy()
        worst = max(worst, float(np.max(np.abs(g - r) / np.maximum(1.0, np.abs(r)))))
    gd = pipe.dets.cpu().numpy()
    o = {h: pipe.outs[h].cpu().numpy() for h, _ in pipe.engine.heads}
    from sfa_hip.runtime import sigmoid_clamp_
    hm = sigmoid_clamp_(pipe.outs["hm_cen"].clone()).cpu().numpy()
    off = sigmoid_clamp_(pipe.outs["cen_offset"].clone()).cpu().numpy()
    ref_dec = decode_oracle.decode(hm, off, o["direction"], o["z_coor"], o["dim"], K=args.K)
    par = {"frames": B, "max_rel_logit_err": float(f"{worst:.3e}"), "logit_tol": 1e-4,
           "dets_equal_oracle_decode_of_gpu_maps": bool(np.array_equal(gd, ref_dec)),
           "max_abs_det_err_vs_oracle_forward": float(f"{float(np.max(np.abs(gd - dets))):.3e}"),
           "scope": "pipeline 0 of the timed set (HIP graphs, %d in flight, side streams %s, math %s) "
                    "after the timed region, against the oracle batch timed above" % (bench.nf, bench.side, args.math)}
    if e2e:
        gb = pipe.bev[:B].cpu().numpy()
        ref = np.stack(maps).astype(np.float32)
        if pipe.bev_layout == "nchw3":
            par["bev_equal"] = bool(np.array_equal(gb, ref))
        else:
            par["bev_equal"] = bool(np.array_equal(gb[..., :3], ref.transpose(0, 2, 3, 1)) and not np.any(gb[..., 3]))
    par["ok"] = bool(worst <= 1e-4 and par["dets_equal_oracle_decode_of_gpu_maps"] and par.get("bev_equal", True))
    return cpu, par


def run_stream(args, rank, world, dev):
    """.bin files (written once to /tmp, then served from the page cache) -> native reader
    pool -> pinned DMA -> BEV -> forward -> decode, reads/H2D of batch k+1 overlapping the
    GPU work of batch k (sfa_hip.stream.StreamingDetector).  Returns (frames, seconds)."""
    import shutil
    import tempfile
    from sfa_hip.stream import StreamingDetector
    arch = _lib.make_arch(DEFAULT_HEADS)
    sd = synthetic.synthetic_state_dict(_lib.state_layout(arch), seed=BENCH_WEIGHT_SEED)
    # several pipelines in flight + the copy stream: no side streams ("auto"), so every stream
    # keeps a hardware queue of its own (profiles/r02b_stream_side_streams.txt)
    side = {"on": True, "off": False, "auto": world == 1 and args.stream_inflight < 2}[args.side_streams]
    engine = KfpnEngine(arch, pack_state_dict(sd, arch), dev, math=MATHS[args.math], side_streams=side)
    tmp = tempfile.mkdtemp(prefix=f"sfa_bins_r{rank}_", dir="/tmp")
    try:
        files = []
        for i in range(4 * args.batch):
            p = os.path.join(tmp, f"{i:06d}.bin")
            synthetic.synthetic_point_cloud(1000 * rank + i + 1).tofile(p)
            files.append(p)
        threads = max(1, min(16, len(os.sched_getaffinity(0)) // max(1, world)))
        warm = StreamingDetector(engine, [files[i % len(files)] for i in range(args.batch * args.warmup)],
                                 args.batch, args.K, threads, inflight=args.stream_inflight, graph=not args.no_graph)
        warm.run()
        torch.cuda.synchronize()
        warm.close()
        det = StreamingDetector(engine, [files[i % len(files)] for i in range(args.batch * args.steps)],
                                args.batch, args.K, threads, inflight=args.stream_inflight, graph=not args.no_graph)
        gather_cb = None
        if world > 1:
            import torch.distributed as dist
            from sfa_hip import dist as sdist
            slot = torch.arange(args.batch, device=dev)

            def gather_cb(dets, n, k):
                # configs[3]: each batch's decoded boxes all-gathered on the batch's own stream
                # (global frame ids; -1 marks the slots of a short last batch)
                ids = torch.where(slot < n, (k * world + rank) * args.batch + slot, torch.full_like(slot, -1))
                sdist.gather_detections(dets, ids)
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        det.run(gather_cb)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        det.close()
        return elapsed, threads
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def build_fusion(args, rank, world, dev):
    """BASELINE configs[4]'s timed configuration: ``--inflight`` FusionPipelines (the first engine
    and its twins: own model handle, buffers, stream and HIP graph each; side streams per
    side_streams_for), the same sweeps and 30 synthetic camera boxes per frame.  Returns the
    pipelines and their streams (tests/test_gpu_bench_parity.py checks them)."""
    import project_cases
    from sfa_hip.runtime import FusionPipeline
    arch = _lib.make_arch(DEFAULT_HEADS)
    sd = synthetic.synthetic_state_dict(_lib.state_layout(arch), seed=BENCH_WEIGHT_SEED)
    engine = KfpnEngine(arch, pack_state_dict(sd, arch), dev,
                        math=MATHS[args.math])
    cal = project_cases.calibs()["avg"]
    calib = runtime_make_calib(cal)
    clouds = [synthetic.synthetic_point_cloud(1000 * rank + i + 1) for i in range(args.batch)]
    cams = []
    for i in range(args.batch):
        u = synthetic.hash_uniform(77, i, 30 * 6).reshape(30, 6)
        boxes = np.stack([u[:, 0] * 1150, u[:, 1] * 320, 10 + u[:, 2] * 120, 10 + u[:, 3] * 90], 1)
        cams.append((boxes.astype(np.int64), u[:, 4].astype(np.float32).astype(np.float64),
                     (u[:, 5] * 80).astype(np.int64)))
    # --inflight pipelines (each with its own model handle and buffers) replayed on their own
    # streams in turn, as in the bev_infer workload: one step's kernel tails and its small
    # latency-bound post-processing / fusion launches overlap the other step's convolutions
    nf = max(1, args.inflight)
    engine.set_side_streams(side_streams_for(args, world, nf))
    fps = []
    for i in range(nf):
        fp = FusionPipeline(engine if i == 0 else engine.twin(), args.batch, [calib], K=args.K,
                            nms=args.fusion_nms, max_points=sum(c.shape[0] for c in clouds),
                            conf_source=_lib.CONF_SCORE)
        fp.set_points(clouds)
        fp.set_camera(cams)
        if not args.no_graph:
            fp.capture()
        fps.append(fp)
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(nf - 1)]
    return fps, streams, (clouds, cams, calib)


def run_fusion(args, rank, world, dev):
    """BASELINE configs[4]: sweeps -> BEV -> forward -> decode -> post_process -> camera boxes
    -> association / Bayesian fusion / NMS against camera boxes, all on the GPU in one HIP
    graph (runtime.FusionPipeline).  The camera detector (YOLOv8n) is not in this framework:
    its boxes are synthetic inputs, 30 per frame."""
    fps, streams, _ = build_fusion(args, rank, world, dev)
    nf = len(fps)

    def step(k):
        with torch.cuda.stream(streams[k % nf]):
            fps[k % nf].replay()

    for k in range(args.warmup):
        step(k)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    return time.perf_counter() - t0


def runtime_make_calib(c):
    from sfa_hip.runtime import make_calib
    return make_calib(c["V2C"], c["R0"], c["P2"], c["img_shape"])


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: this process only starts the ranks (it never touches a GPU)
        os.environ["SFA_BENCH_LAUNCHER"] = "bench.py"
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.dry_run:
        world = int(os.environ.get("WORLD_SIZE", "1"))
        if world != args.gpus:
            raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
        run_dry(args)
        return
    rank, world, dev = init_dist(args.gpus)
    if args.workload in ("stream", "fusion"):
        if args.workload == "fusion":
            sys.path.insert(0, os.path.join(REPO, "tests"))
            elapsed, threads = run_fusion(args, rank, world, dev), None
        else:
            elapsed, threads = run_stream(args, rank, world, dev)
        if world > 1:
            import torch.distributed as dist
            t = torch.tensor([elapsed], dtype=torch.float64,
                             device=dev if dist.get_backend() == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        if rank == 0:
            frames = world * args.batch * args.steps
            if args.workload == "stream":
                data = "synthetic 132,880-pt sweeps written as KITTI .bin files (page cache)"
                cfg = {"workload": "KITTI .bin stream -> pinned DMA -> BEV -> fpn_resnet_18 "
                                   "forward -> decode K=%d, bs=%d per GPU (forward + decode as a "
                                   "HIP graph, BEV eager: per-batch frame offsets)%s"
                                   % (args.K, args.batch, " -> all-gather of each batch's detections"
                                      if world > 1 else ""),
                       "reader_threads": threads, "global_batch": world * args.batch,
                       "steps_in_flight": max(1, args.stream_inflight)}
            else:
                data = ("synthetic 132,880-pt sweeps + 30 synthetic camera boxes per frame "
                        "(YOLOv8n itself not in the framework)")
                cfg = {"workload": "BASELINE configs[4]: sweeps -> BEV -> fpn_resnet_18 forward -> "
                                   "decode K=%d -> post_process -> camera boxes -> Bayesian "
                                   "fusion + %s NMS, bs=%d per GPU, one HIP graph"
                                   % (args.K, args.fusion_nms, args.batch),
                       "global_batch": world * args.batch, "steps_in_flight": max(1, args.inflight)}
            print(json.dumps({
                "metric": METRIC, "value": round(frames / elapsed, 2), "unit": "frames/s",
                "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None,
                "dtype": DTYPES[args.math],
                "data": data, "config": cfg,
            }), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    bench = BevInferBench(args, rank, world, dev)
    nf, pipes, steps, side, one_step = bench.nf, bench.pipes, bench.steps, bench.side, bench.one_step
    if world > 1:
        import torch.distributed as dist
    for k in range(args.warmup):
        one_step(k)
    torch.cuda.synchronize()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        one_step(k, ev[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if args.dump_dets:
        dump_gathered(args, bench, rank, world)
    if nf > 1:
        # per-stage times with one step in flight (the in-flight events overlap): a short
        # untimed-for-value pass on stream 0 only, for the roofline and stages_ms
        torch.cuda.synchronize()
        for k in range(args.steps):
            one_step(k * nf, ev[k])
        torch.cuda.synchronize()
    fwd_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev]))
    dec_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in ev]))
    heads = probe_heads(args, pipes[0], steps[0]) if rank == 0 and args.probe_forwards > 0 else None
    bev_roof = probe_bev(args, pipes[0]) if rank == 0 else None
    if world > 1:
        t = torch.tensor([elapsed, fwd_ms, dec_ms], dtype=torch.float64,
                         device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, fwd_ms, dec_ms = (float(v) for v in t.tolist())
    frames = world * args.batch * args.steps
    value = frames / elapsed
    if rank == 0:
        flop_step = CONV_FLOP_PER_FRAME * args.batch
        # the forward's own event time with one step in flight (the conv launches + aux)
        achieved = flop_step / (fwd_ms * 1e-3) / 1e12
        peak, peak_basis = PEAKS[args.math]
        capped = PEAKS_CAPPED.get(args.math)
        forward_roofline = {
            "scope": "the whole forward (22 implicit-GEMM launches + the stem + aux kernels), "
                     "algorithmic f32 FLOP over its event time with one step in flight",
            "achieved": round(achieved, 3), "frac": round(achieved / peak, 4),
            "frac_of_power_capped": round(achieved / capped, 4) if capped else None,
            "algorithmic_flop_per_step": flop_step}
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": DTYPES[args.math],
            "data": ("synthetic (hash-RNG U[0,1) BEV frames; synthetic He-uniform weights seed %d, BN folded)" % BENCH_WEIGHT_SEED
                     if args.input == "uniform" else
                     "synthetic (BEV maps of synthetic 132,880-pt sweeps, SURVEY §8(d); synthetic weights)")
                    if args.workload == "bev_infer" else
                    "synthetic (132,880-pt LiDAR sweeps per frame, SURVEY §8(d); synthetic weights)",
            "config": {
                "workload": ("fpn_resnet_18 KITTI BEV inference: forward + sigmoid + decode K=%d, "
                             "bs=%d per GPU, 3x608x608 (BASELINE configs[1])" % (args.K, args.batch))
                if args.workload == "bev_infer" else
                ("points -> BEV voxelisation -> fpn_resnet_18 forward -> decode K=%d, bs=%d per GPU "
                 "(BASELINE configs[2])" % (args.K, args.batch)),
                "global_batch": world * args.batch,
                "input": "3x608x608",
                "parallelism": f"dp{world} (frame-sharded replicas; RCCL all_gather of detections)",
                "hip_graph": not args.no_graph,
                "steps_in_flight": nf,
                "side_streams": side,
                "gather": ("RCCL all_gather_into_tensor of the (B, K, 10) detections + frame ids per step"
                           if world > 1 else "simulated: device copy on a lazily created stream joined "
                           "like ProcessGroupNCCL's (--sim-gather)" if args.sim_gather else None),
            },
            "stages_ms": {"forward": round(fwd_ms, 4), "decode": round(dec_ms, 4),
                          "note": "one step in flight; value/ms_per_step use %d in flight" % nf},
            "roofline": roofline_line(args, heads, forward_roofline, achieved, peak, peak_basis, capped),
        }
        if bev_roof is not None:
            line["bev_roofline"] = bev_roof
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"], line["parity"] = cpu_baseline(args, bench)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
