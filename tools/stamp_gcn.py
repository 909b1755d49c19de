"""Phase timing of the fused GCN forward from in-kernel s_memtime stamps (diagnostic build:
build.sh with EXTRA=-DGWN_EXP=64, loaded through GWN_LIB).  The stamps land over z; this prints
the mean cycles per phase, per wave slot, over all slices.  Usage:
  GWN_LIB=.../libgwn_e64.so python tools/stamp_gcn.py [--ts 1,12]"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-wavenet_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gwn_amd import _lib  # noqa: E402

NAMES = {0: "start", 1: "load xs + barrier", 2: "mlp piece 0"}
for k in range(3):
    b = 3 + 8 * k
    NAMES.update({b: "s%d hop1 diffuse" % k, b + 1: "s%d hop1 mlp (W loads)" % k, b + 2: "s%d barrier A" % k,
                  b + 3: "s%d x1 -> lds + global" % k, b + 4: "s%d barrier B" % k, b + 5: "s%d hop2 diffuse" % k,
                  b + 6: "s%d hop2 mlp (W loads)" % k, b + 7: "s%d x2 -> global" % k})
NAMES.update({27: "final barrier + hacc -> lds", 28: "(stamp)", 29: "barrier"})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ts", default="1,12")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    N, C, K, B = 207, 32, 3, 64
    NP = (N + 31) // 32 * 32
    W = (2 * K + 1) * C
    torch.manual_seed(0)
    sups = []
    for _ in range(K):
        s = torch.zeros(NP, NP, device=dev)
        s[:N, :N] = torch.rand(N, N, device=dev) / N
        sups.append(s)
    arr = (ctypes.c_void_p * K)(*[s.data_ptr() for s in sups])
    wm = torch.randn(C, W, device=dev) * 0.05
    bm = torch.randn(C, device=dev)
    seed = torch.zeros(1, device=dev, dtype=torch.int64)
    st = _lib.stream()
    for T in [int(t) for t in args.ts.split(",")]:
        rows = T * B * N
        h = torch.randn(rows, W, device=dev)
        res = torch.randn(rows, C, device=dev)
        z = torch.zeros(rows, C, device=dev)
        bnp = torch.empty(T * B * 3 * C, device=dev)
        ga = _lib.GcnArgs(rows=rows, n=N, c=C, nsup=K, sup=ctypes.cast(arr, ctypes.POINTER(ctypes.c_void_p)),
                          ld_sup=NP, h=h.data_ptr(), ld_h=W, w_mlp=wm.data_ptr(), b_mlp=bm.data_ptr(),
                          residual=res.data_ptr(), z=z.data_ptr(), seed_ptr=seed.data_ptr(), salt=0, drop_p=0.3,
                          bn_partials=bnp.data_ptr())
        for _ in range(5):
            _lib.call("gwn_gcn_fwd", ctypes.byref(ga), st)
        torch.cuda.synchronize()
        raw = z.cpu().numpy().view(np.uint64).reshape(T * B, N * C // 2)[:, :7 * 32].reshape(T * B, 7, 32)
        st_ = raw[:, :, :30].astype(np.int64)
        d = np.diff(st_, axis=2)  # [slices, waves, 29]
        tot = (st_[:, :, 29] - st_[:, :, 0])
        print("T=%d slices=%d: mean slice-wave lifetime %.0f cycles" % (T, T * B, tot.mean()))
        for i in range(1, 30):
            m = d[:, :, i - 1].mean(axis=0)
            print("  %-30s %8.0f   per wave: %s" % (NAMES.get(i, str(i)), d[:, :, i - 1].mean(),
                                                     " ".join("%6.0f" % v for v in m)))
        # block start skew: spread of start stamps within slices
        print("  start skew within block (max-min) %.0f" % (st_[:, :, 0].max(1) - st_[:, :, 0].min(1)).mean())
        rt = raw[:, 0, 30:32].astype(np.int64)  # s_memrealtime (100 MHz) at block start / end
        dur_us = (rt[:, 1] - rt[:, 0]) / 100.0
        clk = (st_[:, 0, 29] - st_[:, 0, 0]) / (dur_us * 1e3)
        span = (rt[:, 1].max() - rt[:, 0].min()) / 100.0
        print("  shader clock %.2f GHz (median over blocks); block lifetime %.1f us mean; kernel span %.1f us;"
              " sum of block lifetimes / (span * resident slots) = %.2f"
              % (np.median(clk), dur_us.mean(), span, dur_us.sum() / (span * min(T * B, 512))))
        starts = np.sort(rt[:, 0] - rt[:, 0].min()) / 100.0
        print("  block start times (us): first %.1f, 512th %.1f, last %.1f"
              % (starts[0], starts[min(511, len(starts) - 1)], starts[-1]))


if __name__ == "__main__":
    main()
