"""Probe: can the backward's side work (mlp weight-gradient partials, adaptive-support gram) run in
the idle capacity of the fused GCN backward's last (lone-workgroup) round?  Times the GCN backward
(BN prologue + gate epilogue), the mlp wgrad and the gram serially on one stream and concurrently on
two streams (one event edge each way per repetition).  Usage: python tools/overlap_probe.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-wavenet_amd"))

import torch  # noqa: E402

from gwn_amd import _lib  # noqa: E402


def main():
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
    supT = [s.t().contiguous() for s in sups]
    arr = (ctypes.c_void_p * K)(*[s.data_ptr() for s in sups])
    arrT = (ctypes.c_void_p * K)(*[s.data_ptr() for s in supT])
    wm = torch.randn(C, W, device=dev) * 0.05
    seed = torch.zeros(1, device=dev, dtype=torch.int64)
    lib = _lib.load()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for T in (12, 10, 7, 4, 3):
        rows = T * B * N
        h = torch.randn(rows, W, device=dev)
        dh = torch.randn(rows, C, device=dev)
        dhc = torch.empty(rows, W, device=dev)
        dwm = torch.empty(C, W, device=dev)
        dbm = torch.empty(C, device=dev)
        dadp = torch.zeros(NP, NP, device=dev)
        ws = torch.empty(lib.gwn_gcn_bwd_workspace_floats(rows, N, C, K) + 16, device=dev)
        gf = _lib.GcnBwdArgs(rows=rows, n=N, c=C, nsup=K, sup=ctypes.cast(arr, ctypes.POINTER(ctypes.c_void_p)),
                             ld_sup=NP, h=h.data_ptr(), ld_h=W, w_mlp=wm.data_ptr(), dh=dh.data_ptr(),
                             dhcat=dhc.data_ptr(), ld_dhcat=W, dw_mlp=dwm.data_ptr(), db_mlp=dbm.data_ptr(),
                             adp_index=K - 1, dadp=dadp.data_ptr(), accumulate_dadp=0, workspace=ws.data_ptr(),
                             sup_t=ctypes.cast(arrT, ctypes.POINTER(ctypes.c_void_p)))
        gf.skip_weight_grads = 1
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
        # side work of the layer above (same shapes: T + d rows; close enough for a probe)
        h2 = torch.randn(rows, W, device=dev)
        dy2 = torch.randn(rows, C, device=dev)
        npart = lib.gwn_wgrad_partial_count(rows, C, W)
        part = torch.empty(max(npart, 1) * (C * W + C) + 16, device=dev)
        gx = [torch.randn(rows, C, device=dev) for _ in range(4)]
        gws = torch.empty(lib.gwn_gram_workspace_floats(N, T * B) + 16, device=dev)

        def gcn(st):
            _lib.call("gwn_gcn_bwd", ctypes.byref(gf), st)

        def side(st):
            _lib.call("gwn_wgrad_partials", dy2.data_ptr(), C, C, h2.data_ptr(), W, rows, W, 1, 0, rows,
                      None, None, None, part.data_ptr(), st)
            _lib.call("gwn_gram", gx[0].data_ptr(), gx[1].data_ptr(), gx[2].data_ptr(), gx[3].data_ptr(), C, C, N,
                      T * B, dadp.data_ptr(), NP, 0, gws.data_ptr(), st)

        def timed(fn, reps=20):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s1)
            for _ in range(reps):
                fn()
            e1.record(s1)
            torch.cuda.synchronize()
            return 1000.0 * e0.elapsed_time(e1) / reps

        def serial():
            gcn(s1.cuda_stream)
            side(s1.cuda_stream)

        def conc():
            ev = torch.cuda.Event()
            ev.record(s1)
            s2.wait_event(ev)
            gcn(s1.cuda_stream)
            side(s2.cuda_stream)
            ev2 = torch.cuda.Event()
            ev2.record(s2)
            s1.wait_event(ev2)

        t_g = timed(lambda: gcn(s1.cuda_stream))
        t_s = timed(lambda: side(s1.cuda_stream))
        t_ser = timed(serial)
        t_con = timed(conc)
        print("T=%2d slices=%4d: gcn bwd %6.1f  side %6.1f  serial %6.1f  concurrent %6.1f us"
              % (T, T * B, t_g, t_s, t_ser, t_con), flush=True)


if __name__ == "__main__":
    main()
