"""Shader clock during the fused GCN forward (diagnostic build: build.sh with EXTRA=-DGWN_EXP=256,
loaded through GWN_LIB): each workgroup writes its s_memtime and s_memrealtime (100 MHz) deltas
over z; clock = cycles / ticks * 100 MHz.  Usage: GWN_LIB=... python tools/clock_gcn.py [--ts 12,4,1]"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-wavenet_amd"))

import torch  # noqa: E402

from gwn_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ts", default="12,4,1")
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
        z = torch.empty(rows, C, device=dev)
        S = T * B
        diag = torch.zeros(S * 3 * C + 4 * S, device=dev)
        ga = _lib.GcnArgs(rows=rows, n=N, c=C, nsup=K, sup=ctypes.cast(arr, ctypes.POINTER(ctypes.c_void_p)),
                          ld_sup=NP, h=h.data_ptr(), ld_h=W, w_mlp=wm.data_ptr(), b_mlp=bm.data_ptr(),
                          residual=res.data_ptr(), z=z.data_ptr(), seed_ptr=seed.data_ptr(), salt=0, drop_p=0.3,
                          bn_partials=diag.data_ptr())
        for _ in range(30):
            _lib.call("gwn_gcn_fwd", ctypes.byref(ga), st)
        torch.cuda.synchronize()
        v = diag[S * 3 * C:].view(-1, 4).double().cpu()
        cyc, ticks, t0 = v[:, 0], v[:, 1], v[:, 2]
        span = float(((t0 + ticks).max() - t0.min()) / 100.0)
        ghz = (cyc / ticks * 0.1)
        print("T=%2d slices=%4d: workgroup life %.1f us (median; min %.1f max %.1f), launch span %.1f us, clock "
              "%.2f GHz (median; min %.2f max %.2f)"
              % (T, S, float(ticks.median()) / 100.0, float(ticks.min()) / 100.0, float(ticks.max()) / 100.0, span,
                 float(ghz.median()), float(ghz.min()), float(ghz.max())), flush=True)


if __name__ == "__main__":
    main()
