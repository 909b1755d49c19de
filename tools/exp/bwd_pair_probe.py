"""Probe (GWN_LIB selects the library): gwn_gcn_bwd in the bf16-mlp mode at n = 207 on S slices with
the BN-backward prologue and the gate epilogue, inputs seeded on the CPU; saves dfg and tg4 to
gpurun_out/<out>/<tag>.npz for a CPU comparison of two libraries."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, "graph-wavenet_amd")
sys.path.insert(0, "tests")
from gwn_amd import _lib  # noqa: E402
from test_gpu_kernels import _squares  # noqa: E402

out, tag, S = sys.argv[1], sys.argv[2], int(sys.argv[3])
gpu = torch.device("cuda", 0)
n, C, K = 207, 32, 3
NP = (n + 31) // 32 * 32
W = (2 * K + 1) * C
rows = S * n
nt = (n + 15) // 16
g = torch.Generator().manual_seed(5)
cpu = lambda *s_: torch.rand(*s_, generator=g)  # noqa: E731
sups = []
for _ in range(K):
    s_ = torch.zeros(NP, NP)
    a = cpu(n, n)
    s_[:n, :n] = a / a.sum(1, keepdim=True)
    sups.append(s_.to(gpu))
supT = [s_.t().contiguous() for s_ in sups]
sq = _squares(gpu, sups)
P = ctypes.POINTER(ctypes.c_void_p)
el = _lib.load().gwn_support_g4_bf16_elems(n)
mats = [m for t_, q in zip(supT, sq) for m in (t_, q[1])]
g4bt = torch.zeros(len(mats), el // 2, device=gpu)
src = (ctypes.c_void_p * len(mats))(*[m.data_ptr() for m in mats])
_lib.call("gwn_support_g4_bf16", ctypes.cast(src, P), len(mats), n, NP, g4bt.data_ptr(), el, _lib.stream())
arrb = (ctypes.c_void_p * len(mats))(*[g4bt[i].data_ptr() for i in range(len(mats))])
arr = (ctypes.c_void_p * K)(*[s_.data_ptr() for s_ in sups])
arrT = (ctypes.c_void_p * K)(*[s_.data_ptr() for s_ in supT])
wm = ((cpu(C, W) - 0.5) * 0.3).to(gpu)
h = torch.zeros(rows, W, device=gpu)
dhc = torch.zeros(rows, W, device=gpu)
seed = torch.full((1,), 77, device=gpu, dtype=torch.int64)
bn_dy, bn_z = (cpu(rows, C) - 0.5).to(gpu), (cpu(rows, C) * 2).to(gpu)
gamma, bmean, brstd = cpu(C).to(gpu), cpu(C).to(gpu), (cpu(C) + 0.5).to(gpu)
sums = ((cpu(2 * C) - 0.5) * 50).to(gpu)
fg = cpu(rows, 2 * C).to(gpu)
dskip = (cpu(rows, C) - 0.5).to(gpu)
skip_row0 = (S - 3) * n
dres, dh_out = torch.zeros(rows, C, device=gpu), torch.zeros(rows, C, device=gpu)
dfg = torch.zeros(rows, 2 * C, device=gpu)
dg, db = torch.zeros(C, device=gpu), torch.zeros(C, device=gpu)
tg4 = torch.full((2 * S * nt * 512,), -1, device=gpu, dtype=torch.int16)
gb = _lib.GcnBwdArgs(rows=rows, n=n, c=C, nsup=K, sup=ctypes.cast(arr, P), ld_sup=NP, h=h.data_ptr(), ld_h=W,
                     w_mlp=wm.data_ptr(), dhcat=dhc.data_ptr(), ld_dhcat=W, adp_index=K - 1, accumulate_dadp=0,
                     sup_t=ctypes.cast(arrT, P), skip_weight_grads=1, split_planes=2, sup_g4b_t=ctypes.cast(arrb, P),
                     dh=None, bn_dy=bn_dy.data_ptr(), bn_z=bn_z.data_ptr(), bn_gamma=gamma.data_ptr(),
                     bn_mean=bmean.data_ptr(), bn_rstd=brstd.data_ptr(), bn_sums=sums.data_ptr(),
                     bn_dgamma=dg.data_ptr(), bn_dbeta=db.data_ptr(), dres=dres.data_ptr(), dh_out=dh_out.data_ptr(),
                     seed_ptr=seed.data_ptr(), salt=4, drop_p=0.3, fg=fg.data_ptr(), dskip=dskip.data_ptr(),
                     ld_dskip=C, skip_row0=skip_row0, dfg=dfg.data_ptr(), tg4=tg4.data_ptr())
_lib.call("gwn_gcn_bwd", ctypes.byref(gb), _lib.stream())
torch.cuda.synchronize()
first = dfg.clone()
for rep in range(3):  # determinism: the same launch again
    dfg.zero_()
    _lib.call("gwn_gcn_bwd", ctypes.byref(gb), _lib.stream())
    torch.cuda.synchronize()
    d = (dfg - first).abs()
    print("rerun %d: %d elements differ (max %.3g)" % (rep, int((d > 0).sum()), float(d.max())))
    bad = torch.nonzero(d.max(1).values > 0).flatten().cpu().tolist()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    nt_ = 13
    units = ((S + 1) // 2) * nt_
    grid = min(units, cus)
    seen = set()
    for r in bad:
        sl, node = r // n, r % n
        u = (sl // 2) * nt_ + node // 16
        wg = next(w for w in range(grid) if units * w // grid <= u < units * (w + 1) // grid)
        tb = units * wg // grid
        key = (sl, node // 16)
        if key in seen:
            continue
        seen.add(key)
        cols = torch.nonzero((dfg[r] - first[r]).abs() > 0).flatten().cpu().tolist()
        print("  slice %d (%s) tile %d unit %d wg %d pos %d of %d, cols %s" % (
            sl, "A" if sl % 2 == 0 else "B", node // 16, u, wg, u - tb, units * (wg + 1) // grid - tb, cols[:8]))
dfg.copy_(first)
os.makedirs("gpurun_out/" + out, exist_ok=True)
np.savez("/tmp/%s_%s.npz" % (out, tag), dfg=dfg.cpu().numpy(), tg4=tg4.cpu().numpy(), dh=dh_out.cpu().numpy())
print("saved", tag, S)
