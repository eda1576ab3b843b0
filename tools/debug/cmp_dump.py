"""Compare the pipelines of a bench --dump-dets file with each other (rank-0 slice) and with a
reference dump (the first argument)."""
import sys

import numpy as np

ref = np.load(sys.argv[1])["local"][0]
for f in sys.argv[2:]:
    d = np.load(f)
    out = []
    for p in range(d["local"].shape[0]):
        out.append("p%d:%s%s" % (p, "=" if np.array_equal(d["local"][p], ref) else "DIFF(%.2e)" % float(np.abs(d["local"][p] - ref).max()),
                                 "" if np.array_equal(d["dets"][p][:16], d["local"][p]) else "/gather-differs"))
    print(f, " ".join(out))
