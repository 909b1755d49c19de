"""Compare two bwd_pair_probe.py runs (on the GPU box's /tmp): where the pair kernel differs."""
import sys

import numpy as np

out = sys.argv[1]
a, b = np.load("/tmp/%s_pair.npz" % out), np.load("/tmp/%s_single.npz" % out)
n = 207
for k in ("dh", "dfg"):
    d = np.abs(a[k] - b[k])
    print(k, d.max(), (d > 0).sum(), d.size)
    if d.max() > 0:
        r = np.nonzero(d.max(1) > 1e-3)[0]
        print(" bad rows", len(r), "slices", np.unique(r // n)[:60], "nodes", np.unique(r % n)[:60])
t = a["tg4"].astype(np.int32) != b["tg4"].astype(np.int32)
print("tg4 diff", t.sum(), t.size)
if t.any():
    nt = 13
    S = a["dh"].shape[0] // n
    idx = np.nonzero(t)[0]
    blk = idx // 512
    print(" which/slice/tile", np.unique(blk // (S * nt))[:4], np.unique((blk % (S * nt)) // nt)[:60],
          np.unique(blk % nt))
