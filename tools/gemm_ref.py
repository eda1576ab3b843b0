"""Library GEMM reference points (hipBLASLt via torch) at the conv implicit-GEMM shapes:
what a vendor-tuned fp16 GEMM sustains on this chip (tools only)."""
import torch, time
shapes = [("head L1", 369664, 320, 1152), ("head L2", 369664, 320, 576), ("head L0", 92416, 320, 2304),
          ("layer1", 369664, 64, 576), ("layer2", 92416, 128, 1152), ("layer3", 23104, 256, 2304),
          ("layer4", 5776, 512, 4608), ("square 8192", 8192, 8192, 8192)]
dev = torch.device("cuda")
for name, M, N, K in shapes:
    a = torch.randn(M, K, device=dev, dtype=torch.float16)
    b = torch.randn(K, N, device=dev, dtype=torch.float16)
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(10):
        e0.record(); c = a @ b; e1.record(); e1.synchronize(); ts.append(e0.elapsed_time(e1))
    t = sorted(ts)[len(ts) // 2] * 1e-3
    fl = 2.0 * M * N * K
    print(f"{name:12s} M={M} N={N} K={K}: {t*1e6:8.1f} us  {fl/t/1e12:7.1f} TF/s fp16 "
          f"(x3 products: {3*t*1e6:8.1f} us = {fl/(3*t)/1e12:6.1f} f32-eq TF/s)", flush=True)
