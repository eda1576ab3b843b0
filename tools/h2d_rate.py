"""Host -> device copy rate of one stream-workload batch (16 frames x 132,880 points x 16 B) from
pinned memory (the BinStream staging slots' path), median of 20 copies timed with HIP events."""
import json

import torch

nbytes = 16 * 132880 * 16
src = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
st = torch.cuda.Stream()
ts = []
with torch.cuda.stream(st):
    for i in range(25):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        dst.copy_(src, non_blocking=True)
        e1.record(st)
        e1.synchronize()
        if i >= 5:
            ts.append(e0.elapsed_time(e1))
ts.sort()
ms = ts[len(ts) // 2]
print(json.dumps({"bytes_per_batch": nbytes, "ms_median": round(ms, 4), "GB_per_s": round(nbytes / ms / 1e6, 2)}))
