"""Where the 16-node tile forward's time goes, per workgroup (GWN_T16_PROBE build: s_memrealtime
stamps, 100 MHz, into gwn_gcn_args.ksplit_ws).  METR-LA layer shapes (n = 207, 3 supports).

    OUT=$PWD/exp/libgwn_probe.so EXTRA=-DGWN_T16_PROBE bash build.sh
    GWN_LIB=exp/libgwn_probe.so python tools/exp/t16_probe.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "graph-wavenet_amd"), os.path.join(ROOT, "tests")]
from gwn_amd import _lib  # noqa: E402
from test_gpu_kernels import _g4s, _squares  # noqa: E402


def run(S, gpu, n=207, K=3, C=32):
    NP = (n + 31) // 32 * 32
    W = (2 * K + 1) * C
    rows = S * n
    torch.manual_seed(0)
    sups = []
    for _ in range(K):
        s_ = torch.zeros(NP, NP, device=gpu)
        a = torch.rand(n, n, device=gpu)
        s_[:n, :n] = a / a.sum(1, keepdim=True)
        sups.append(s_)
    sq = _squares(gpu, sups)
    g4f, _ = _g4s(gpu, n, sups, sq, [s_.t().contiguous() for s_ in sups])
    P = ctypes.POINTER(ctypes.c_void_p)
    arr = (ctypes.c_void_p * K)(*[s_.data_ptr() for s_ in sups])
    wm = torch.randn(C, W, device=gpu) * 0.1
    wmt = wm.t().contiguous()
    bm = torch.randn(C, device=gpu)
    res = torch.randn(rows, C, device=gpu)
    h = torch.zeros(rows, W, device=gpu)
    h[:, :C] = torch.randn(rows, C, device=gpu)
    z = torch.empty(rows, C, device=gpu)
    seed = torch.zeros(1, device=gpu, dtype=torch.int64)
    bnp = torch.zeros(max(_lib.load().gwn_gcn_bn_partial_count(rows, n, C, K, NP), 256) * 3 * C, device=gpu)
    probe = torch.zeros(256 * 20, device=gpu, dtype=torch.int64)
    ga = _lib.GcnArgs(rows=rows, n=n, c=C, nsup=K, sup=ctypes.cast(arr, P), ld_sup=NP, h=h.data_ptr(), ld_h=W,
                      w_mlp=wm.data_ptr(), b_mlp=bm.data_ptr(), residual=res.data_ptr(), z=z.data_ptr(),
                      seed_ptr=seed.data_ptr(), salt=0, drop_p=0.3, bn_partials=bnp.data_ptr(),
                      w_mlp_t=wmt.data_ptr(), sup_g4=g4f[1], ksplit=1, ksplit_ws=probe.data_ptr())
    grid = min(S * ((n + 15) // 16), 256)
    res_ = []
    for it in range(5):
        probe.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.call("gwn_gcn_fwd", ctypes.byref(ga), _lib.stream())
        e1.record()
        torch.cuda.synchronize()
        t = probe.view(256, 20)[:grid].cpu().numpy().astype(np.float64) * 0.01  # us
        t0 = t[:, 0].min()
        t = t - t0
        waves = t[:, 2:18]
        nw = (waves > 0).sum(1)
        wmax, wmin = waves.max(1), np.where(waves > 0, waves, np.inf).min(1)
        res_.append((e0.elapsed_time(e1) * 1000, t[:, 0].max(), np.median(t[:, 1] - t[:, 0]), np.median(wmax - t[:, 1]),
                     np.median(wmax - wmin), np.median(t[:, 18] - wmax), t[:, 18].max(), np.argmax(t[:, 18]),
                     np.percentile(t[:, 18], 10)))
    r = np.median(np.array(res_), 0)
    print("S=%4d grid %3d: event %.1f us | start skew %.1f, staging %.1f, loop %.1f (wave spread %.1f), flush %.1f,"
          " last WG ends %.1f (10%% of WGs by %.1f)" % (S, grid, r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[8]))


def main():
    gpu = torch.device("cuda:0")
    for S in [int(v) for v in os.environ.get("SLICES", "768,640,448,192,64").split(",")]:
        run(S, gpu)


if __name__ == "__main__":
    main()
