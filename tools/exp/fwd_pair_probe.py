"""Probe: determinism of the bf16-mlp forward (gwn_gcn_fwd, split_planes 2, n = 207) on S slices:
the same launch four times, h / z / BN partials compared bitwise."""
import ctypes
import sys

import torch

sys.path.insert(0, "graph-wavenet_amd")
sys.path.insert(0, "tests")
from gwn_amd import _lib  # noqa: E402
from test_gpu_kernels import _squares  # noqa: E402

S = int(sys.argv[1])
gpu = torch.device("cuda", 0)
n, C, K = 207, 32, 3
NP = (n + 31) // 32 * 32
W = (2 * K + 1) * C
rows = S * n
torch.manual_seed(3)
sups = []
for _ in range(K):
    s_ = torch.zeros(NP, NP, device=gpu)
    a = torch.rand(n, n, device=gpu)
    s_[:n, :n] = a / a.sum(1, keepdim=True)
    sups.append(s_)
sq = _squares(gpu, sups)
P = ctypes.POINTER(ctypes.c_void_p)
el = _lib.load().gwn_support_g4_bf16_elems(n)
mats = [m for s_, q in zip(sups, sq) for m in (s_, q[0])]
g4b = torch.zeros(len(mats), el // 2, device=gpu)
src = (ctypes.c_void_p * len(mats))(*[m.data_ptr() for m in mats])
_lib.call("gwn_support_g4_bf16", ctypes.cast(src, P), len(mats), n, NP, g4b.data_ptr(), el, _lib.stream())
arrb = (ctypes.c_void_p * len(mats))(*[g4b[i].data_ptr() for i in range(len(mats))])
arr = (ctypes.c_void_p * K)(*[s_.data_ptr() for s_ in sups])
wm = torch.randn(C, W, device=gpu) * 0.1
wmt = wm.t().contiguous()
bm = torch.randn(C, device=gpu)
res = torch.randn(rows, C, device=gpu)
xg = torch.randn(rows, C, device=gpu)
seed = torch.zeros(1, device=gpu, dtype=torch.int64)
outs = []
for rep in range(4):
    h = torch.zeros(rows, W, device=gpu)
    h[:, :C] = xg
    z = torch.empty(rows, C, device=gpu)
    bnp = torch.zeros(_lib.load().gwn_gcn_bn_partial_count(rows, n, C, K, NP) * 3 * C, device=gpu)
    ga = _lib.GcnArgs(rows=rows, n=n, c=C, nsup=K, sup=ctypes.cast(arr, P), ld_sup=NP, h=h.data_ptr(), ld_h=W,
                      w_mlp=wm.data_ptr(), b_mlp=bm.data_ptr(), residual=res.data_ptr(), z=z.data_ptr(),
                      seed_ptr=seed.data_ptr(), salt=0, drop_p=0.0, bn_partials=bnp.data_ptr(), w_mlp_t=wmt.data_ptr(),
                      split_planes=2, sup_g4b=ctypes.cast(arrb, P))
    _lib.call("gwn_gcn_fwd", ctypes.byref(ga), _lib.stream())
    torch.cuda.synchronize()
    outs.append((h, z, bnp))
for rep in range(1, 4):
    print("fwd S=%d rerun %d: h %d z %d bnp %d elements differ" % (
        S, rep, int((outs[rep][0] != outs[0][0]).sum()), int((outs[rep][1] != outs[0][1]).sum()),
        int((outs[rep][2] != outs[0][2]).sum())))
