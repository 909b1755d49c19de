"""Micro-benchmark of the diffusion GCN layer (gwn_gcn_fwd / gwn_gcn_bwd through the C-ABI) at
METR-LA layer shapes, timed with HIP events on the launch stream.  The backward includes the
mlp weight gradient and the adaptive-support grams (separate kernels in a kernel trace).
Usage: python tools/bench_gcn.py [--reps R] [--ts 12,7,1]"""
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
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    N, C, K, B = args.nodes, 32, 3, 64
    NP = (N + 31) // 32 * 32
    W = (2 * K + 1) * C
    torch.manual_seed(0)
    sups = []
    for _ in range(K):
        s = torch.zeros(NP, NP, device=dev)
        s[:N, :N] = torch.rand(N, N, device=dev) / N
        sups.append(s)
    supT = [s.t().contiguous() for s in sups]
    arr = (ctypes.c_void_p * K)(*[s.data_ptr() for s in sups])
    arrT = (ctypes.c_void_p * K)(*[s.data_ptr() for s in supT])
    wm = torch.randn(C, W, device=dev) * 0.05
    bm = torch.randn(C, device=dev)
    seed = torch.zeros(1, device=dev, dtype=torch.int64)
    st = _lib.stream()
    lib = _lib.load()
    for T in [int(t) for t in args.ts.split(",")]:
        rows = T * B * N
        h = torch.randn(rows, W, device=dev)
        res = torch.randn(rows, C, device=dev)
        z = torch.empty(rows, C, device=dev)
        bnp = torch.empty(T * B * 3 * C, device=dev)
        ga = _lib.GcnArgs(rows=rows, n=N, c=C, nsup=K, sup=ctypes.cast(arr, ctypes.POINTER(ctypes.c_void_p)),
                          ld_sup=NP, h=h.data_ptr(), ld_h=W, w_mlp=wm.data_ptr(), b_mlp=bm.data_ptr(),
                          residual=res.data_ptr(), z=z.data_ptr(), seed_ptr=seed.data_ptr(), salt=0, drop_p=0.3,
                          bn_partials=bnp.data_ptr())
        dh = torch.randn(rows, C, device=dev)
        dhc = torch.empty(rows, W, device=dev)
        dwm = torch.empty(C, W, device=dev)
        dbm = torch.empty(C, device=dev)
        dadp = torch.zeros(NP, NP, device=dev)
        ws = torch.empty(lib.gwn_gcn_bwd_workspace_floats(rows, N, C, K) + 16, device=dev)
        gb = _lib.GcnBwdArgs(rows=rows, n=N, c=C, nsup=K, sup=ctypes.cast(arr, ctypes.POINTER(ctypes.c_void_p)),
                             ld_sup=NP, h=h.data_ptr(), ld_h=W, w_mlp=wm.data_ptr(), dh=dh.data_ptr(),
                             dhcat=dhc.data_ptr(), ld_dhcat=W, dw_mlp=dwm.data_ptr(), db_mlp=dbm.data_ptr(),
                             adp_index=K - 1, dadp=dadp.data_ptr(), accumulate_dadp=0, workspace=ws.data_ptr(),
                             sup_t=ctypes.cast(arrT, ctypes.POINTER(ctypes.c_void_p)))
        flop = T * B * (K * 2 * 2.0 * C * N * N + 2.0 * (2 * K + 1) * C * C * N)
        # data path only, plain and with the BN-backward prologue + gate-backward epilogue
        gd = _lib.GcnBwdArgs.from_buffer_copy(gb)
        gd.skip_weight_grads = 1
        gf = _lib.GcnBwdArgs.from_buffer_copy(gd)
        zb, dres, dho = torch.randn(rows, C, device=dev), torch.empty(rows, C, device=dev), torch.empty(rows, C, device=dev)
        gam, mu, rs, sums = (torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev), torch.rand(C, device=dev) + 0.5,
                             torch.randn(2 * C, device=dev))
        dgam, dbet = torch.empty(C, device=dev), torch.empty(C, device=dev)
        fgb, dskb, dfgb = torch.rand(rows, 2 * C, device=dev), torch.randn(rows, 8 * C, device=dev), torch.empty(rows, 2 * C, device=dev)
        gf.bn_dy, gf.bn_z, gf.bn_gamma, gf.bn_mean, gf.bn_rstd, gf.bn_sums = (dh.data_ptr(), zb.data_ptr(), gam.data_ptr(),
                                                                              mu.data_ptr(), rs.data_ptr(), sums.data_ptr())
        gf.bn_dgamma, gf.bn_dbeta, gf.dres, gf.dh_out = dgam.data_ptr(), dbet.data_ptr(), dres.data_ptr(), dho.data_ptr()
        gf.seed_ptr, gf.salt, gf.drop_p = seed.data_ptr(), 3, 0.3
        gf.fg, gf.dskip, gf.ld_dskip, gf.skip_row0, gf.dfg = fgb.data_ptr(), dskb.data_ptr(), 8 * C, 0, dfgb.data_ptr()
        variants = []
        for lay in ((0, 1, 3) if NP <= 256 else (0, 1)):
            tag = "" if lay == 0 else " L%d" % lay
            ga_l = _lib.GcnArgs.from_buffer_copy(ga)
            ga_l.layout = lay
            gd_l = _lib.GcnBwdArgs.from_buffer_copy(gd)
            gd_l.layout = lay
            gf_l = _lib.GcnBwdArgs.from_buffer_copy(gf)
            gf_l.layout = lay
            variants += [("fwd" + tag, lambda a=ga_l: _lib.call("gwn_gcn_fwd", ctypes.byref(a), st)),
                         ("bwd-data" + tag, lambda a=gd_l: _lib.call("gwn_gcn_bwd", ctypes.byref(a), st)),
                         ("bwd-data+bn+gate" + tag, lambda a=gf_l: _lib.call("gwn_gcn_bwd", ctypes.byref(a), st))]
        variants.append(("bwd (+wgrad, gram)", lambda: _lib.call("gwn_gcn_bwd", ctypes.byref(gb), st)))
        for lay in ((0, 3) if NP <= 256 else (0,)):
            ga_np = _lib.GcnArgs.from_buffer_copy(ga)
            ga_np.no_pieces = 1
            ga_np.layout = lay
            variants.append(("fwd no pieces" + ("" if lay == 0 else " L%d" % lay),
                             lambda a=ga_np: _lib.call("gwn_gcn_fwd", ctypes.byref(a), st)))
        wws = torch.empty(lib.gwn_wgrad_workspace_floats(rows, C, W) + 16, device=dev)
        variants.append(("wgrad mlp", lambda wws=wws: _lib.call(
            "gwn_wgrad", dh.data_ptr(), C, C, h.data_ptr(), W, rows, W, 1, 0, rows, dwm.data_ptr(), W,
            dbm.data_ptr(), wws.data_ptr(), st)))
        gx = [torch.randn(rows, C, device=dev) for _ in range(4)]
        gws = torch.empty(lib.gwn_gram_workspace_floats(N, T * B) + 16, device=dev)
        variants.append(("gram (2 pairs)", lambda gx=gx, gws=gws: _lib.call(
            "gwn_gram", gx[0].data_ptr(), gx[1].data_ptr(), gx[2].data_ptr(), gx[3].data_ptr(), C, C, N, T * B,
            dadp.data_ptr(), NP, 0, gws.data_ptr(), st)))
        for planes in (3, 2):
            if not lib.gwn_gcn_split_supported(C, N, planes):
                continue
            sup_el = lib.gwn_split_support_elems(N, planes)
            w_el = (lib.gwn_split_mlp_elems(K, planes) + 7) // 8 * 8
            ssup = torch.empty(K * sup_el, device=dev, dtype=torch.int16)
            sw = torch.empty(w_el, device=dev, dtype=torch.int16)
            warr = (ctypes.c_void_p * 1)(wm.data_ptr())
            _lib.call("gwn_split_supports", ctypes.cast(arr, ctypes.c_void_p), K, N, NP, planes, ssup.data_ptr(),
                      sup_el, NP, st)
            _lib.call("gwn_split_mlp_weights", ctypes.cast(warr, ctypes.c_void_p), 1, K, planes, sw.data_ptr(),
                      w_el, st)
            ga_s = _lib.GcnArgs.from_buffer_copy(ga)
            ga_s.split_planes, ga_s.sup_split, ga_s.sup_split_stride = planes, ssup.data_ptr(), sup_el
            ga_s.ld_split, ga_s.w_split = NP, sw.data_ptr()
            variants.append(("fwd split%d" % planes,
                             lambda a=ga_s, keep=(ssup, sw): _lib.call("gwn_gcn_fwd", ctypes.byref(a), st)))
        for name, fn in variants:
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = 1000.0 * e0.elapsed_time(e1) / args.reps
            print("gcn %-20s T=%2d slices=%4d: %8.1f us  %6.1f TFLOP/s (fwd-equivalent flops)"
                  % (name, T, T * B, us, flop / us / 1e6), flush=True)
        del dh, dhc


if __name__ == "__main__":
    main()
