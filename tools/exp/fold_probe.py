"""Timing probe of the gcn forward's in-launch BatchNorm finalize (gwn_gcn_args.bn_fold) at the
METR-LA first-layer shape (768 slices x 207 nodes, 3 supports).  Run with GWN_LIB pointing at a
build made with EXTRA=-DGWN_FOLD_EXP=3: the last workgroup's phase timestamps (s_memrealtime,
100 MHz) are read back from past the grid's partial slots.  Prints per-launch event times too.

    OUT=$PWD/exp/libgwn_f3.so EXTRA=-DGWN_FOLD_EXP=3 bash build.sh
    GWN_LIB=exp/libgwn_f3.so python tools/exp/fold_probe.py
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "graph-wavenet_amd"), os.path.join(ROOT, "tests")]
from gwn_amd import _lib  # noqa: E402
from test_gpu_kernels import _g4s, _squares  # noqa: E402


def main():
    gpu = torch.device("cuda:0")
    n, K, S, C = 207, 3, int(os.environ.get("SLICES", "768")), 32
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
    slots = max(_lib.load().gwn_gcn_bn_partial_count(rows, n, C, K, NP), 512)
    bnp = torch.zeros(slots * 3 * C, device=gpu)
    vec = lambda: torch.randn(C, device=gpu)  # noqa: E731
    gamma, beta, rm, rv = vec(), vec(), vec(), torch.rand(C, device=gpu) + 0.5
    mean, rstd, scale = vec(), vec(), vec()
    wfg, bfg = torch.randn(2 * C, 2 * C, device=gpu), torch.randn(2 * C, device=gpu)
    wfold, bfold = torch.empty_like(wfg), torch.empty_like(bfg)
    nbt = torch.zeros(1, device=gpu, dtype=torch.int64)
    arrive = torch.zeros(1, device=gpu, dtype=torch.int32)
    bf = _lib.BnFold(gamma=gamma.data_ptr(), beta=beta.data_ptr(), running_mean=rm.data_ptr(),
                     running_var=rv.data_ptr(), momentum=0.1, eps=1e-5, save_mean=mean.data_ptr(),
                     save_rstd=rstd.data_ptr(), scale=scale.data_ptr(), w_next=wfg.data_ptr(), b_next=bfg.data_ptr(),
                     w_fold=wfold.data_ptr(), b_fold=bfold.data_ptr(), num_batches_tracked=nbt.data_ptr(),
                     arrive=arrive.data_ptr())
    fold = os.environ.get("FOLD", "1") == "1"
    ga = _lib.GcnArgs(rows=rows, n=n, c=C, nsup=K, sup=ctypes.cast(arr, P), ld_sup=NP, h=h.data_ptr(), ld_h=W,
                      w_mlp=wm.data_ptr(), b_mlp=bm.data_ptr(), residual=res.data_ptr(), z=z.data_ptr(),
                      seed_ptr=seed.data_ptr(), salt=0, drop_p=0.0, bn_partials=bnp.data_ptr(),
                      w_mlp_t=wmt.data_ptr(), sup_g4=g4f[1], bn_fold=ctypes.pointer(bf) if fold else None)
    grid = min(S * ((n + 15) // 16), torch.cuda.get_device_properties(0).multi_processor_count)
    for it in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.call("gwn_gcn_fwd", ctypes.byref(ga), _lib.stream())
        e1.record()
        torch.cuda.synchronize()
        ts = bnp[grid * 3 * C:grid * 3 * C + 8].view(torch.int64).cpu().tolist()
        ph = [(ts[k + 1] - ts[k]) * 10 for k in range(3)]
        print("launch %d: %.1f us (events)  phases ns: loads+merge %d, tree+stats %d, fold+stores %d"
              % (it, e0.elapsed_time(e1) * 1000, ph[0], ph[1], ph[2]))


if __name__ == "__main__":
    main()
