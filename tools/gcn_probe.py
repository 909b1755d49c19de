"""Probe of the fused diffusion-GCN kernels at METR-LA layer shapes (B = 64, N = 207): forward and
backward (data path: gwn_gcn_fwd / gwn_gcn_bwd with skip_weight_grads), power or chained schedule,
timed with HIP events on the launch stream.  GWN_LIB selects an experiment build of libgwn.
    python tools/gcn_probe.py [--ts 12,7,1] [--reps 20] [--chain] [--no-pieces] [--nodes 207]"""
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
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--ts", default="12,7,1")
    ap.add_argument("--nodes", type=int, default=207)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--chain", action="store_true")
    ap.add_argument("--no-pieces", action="store_true")
    ap.add_argument("--tag", default="")
    ap.add_argument("--no-bn", action="store_true", help="no BN partials (forward)")
    ap.add_argument("--drop", type=float, default=0.3)
    ap.add_argument("--stamps", default=None, help="with an experiment build that writes per-wave stamps "
                    "past the BN partials (tools/exp/stamp_pow.py): save them to this .npy (forward, first T)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    N, C, K, B = args.nodes, 32, 3, args.batch
    NP = (N + 31) // 32 * 32
    W = (2 * K + 1) * C
    P = ctypes.POINTER(ctypes.c_void_p)
    torch.manual_seed(0)
    sups = []
    for _ in range(K):
        s = torch.zeros(NP, NP, device=dev)
        s[:N, :N] = torch.rand(N, N, device=dev) / N
        sups.append(s)
    supT = [s.t().contiguous() for s in sups]
    sq, sqt = [], []
    for s in sups:
        a2, a2t = torch.empty_like(s), torch.empty_like(s)
        _lib.call("gwn_support_square", s.data_ptr(), NP, NP, a2.data_ptr(), a2t.data_ptr(), None, _lib.stream())
        sq.append(a2)
        sqt.append(a2t)
    arr = (ctypes.c_void_p * K)(*[s.data_ptr() for s in sups])
    arrT = (ctypes.c_void_p * K)(*[s.data_ptr() for s in supT])
    arr2 = (ctypes.c_void_p * K)(*[s.data_ptr() for s in sq])
    arr2T = (ctypes.c_void_p * K)(*[s.data_ptr() for s in sqt])
    # gwn_support_g4 copies (the 16-node tile kernels): forward [A_k, A_k^2], backward [A_k^T, (A_k^2)^T]
    fl = _lib.load().gwn_support_g4_floats(N)
    g4 = []
    for mats in ([m for a_, b_ in zip(sups, sq) for m in (a_, b_)], [m for a_, b_ in zip(supT, sqt) for m in (a_, b_)]):
        buf = torch.empty(len(mats), fl, device=dev)
        src = (ctypes.c_void_p * len(mats))(*[m.data_ptr() for m in mats])
        _lib.call("gwn_support_g4", ctypes.cast(src, P), len(mats), N, NP, buf.data_ptr(), fl, _lib.stream())
        g4.append((buf, (ctypes.c_void_p * len(mats))(*[buf[i].data_ptr() for i in range(len(mats))])))
    wm = torch.randn(C, W, device=dev) * 0.05
    wmt = wm.t().contiguous()
    bm = torch.randn(C, device=dev)
    seed = torch.zeros(1, device=dev, dtype=torch.int64)
    lib = _lib.load()
    st = _lib.stream()
    for T in [int(t) for t in args.ts.split(",")]:
        rows = T * B * N
        h = torch.randn(rows, W, device=dev)
        res = torch.randn(rows, C, device=dev)
        z = torch.empty(rows, C, device=dev)
        nwaves = T * B * ((N + 31) // 32)
        # BN partial slots (gwn_gcn_bn_partial_count) + room for experiment-build stamps
        bnp = torch.zeros(lib.gwn_gcn_bn_partial_count(rows, N, C, K, NP) * 3 * C + 8 * nwaves, device=dev)
        ga = _lib.GcnArgs(rows=rows, n=N, c=C, nsup=K, sup=ctypes.cast(arr, P), ld_sup=NP, h=h.data_ptr(), ld_h=W,
                          w_mlp=wm.data_ptr(), b_mlp=bm.data_ptr(), residual=res.data_ptr(), z=z.data_ptr(),
                          seed_ptr=seed.data_ptr(), salt=0, drop_p=args.drop,
                          bn_partials=None if args.no_bn else bnp.data_ptr(),
                          no_pieces=1 if args.no_pieces else 0,
                          sup2=None if args.chain else ctypes.cast(arr2, P), w_mlp_t=wmt.data_ptr(), ksplit=1,
                          sup_g4=None if args.chain else ctypes.cast(g4[0][1], P))
        dh = torch.randn(rows, C, device=dev)
        dhc = torch.empty(rows, W, device=dev)
        gb = _lib.GcnBwdArgs(rows=rows, n=N, c=C, nsup=K, sup=ctypes.cast(arr, P), ld_sup=NP, h=h.data_ptr(),
                             ld_h=W, w_mlp=wm.data_ptr(), dh=dh.data_ptr(), dhcat=dhc.data_ptr(), ld_dhcat=W,
                             adp_index=K - 1, accumulate_dadp=0, sup_t=ctypes.cast(arrT, P), skip_weight_grads=1,
                             sup2_t=None if args.chain else ctypes.cast(arr2T, P), ksplit=1,
                             sup_g4_t=None if args.chain else ctypes.cast(g4[1][1], P))
        flop = T * B * (K * 2 * 2.0 * C * N * N + 2.0 * (2 * K + 1) * C * C * N)
        for name, fn, a in (("fwd", "gwn_gcn_fwd", ga), ("bwd", "gwn_gcn_bwd", gb)):
            for _ in range(3):
                _lib.call(fn, ctypes.byref(a), st)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(args.reps):
                _lib.call(fn, ctypes.byref(a), st)
            e1.record()
            torch.cuda.synchronize()
            us = 1000.0 * e0.elapsed_time(e1) / args.reps
            print("%s T=%2d slices=%4d %s %8.1f us  %6.1f TFLOP/s (%.3f of 157.3)"
                  % (args.tag, T, T * B, name, us, flop / us / 1e6, flop / us / 1e6 / 157.3), flush=True)
            if args.stamps and name == "fwd":
                import numpy as np
                st_ = bnp[lib.gwn_gcn_bn_partial_count(rows, N, C, K, NP) * 3 * C:].view(torch.int32).view(nwaves, 8).cpu().numpy()
                np.save(args.stamps.replace(".npy", "_T%d.npy" % T), st_)
    del lib


if __name__ == "__main__":
    main()
