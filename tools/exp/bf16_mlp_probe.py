"""Which bf16 emulation does the HIP bf16 train step follow?  One train step on the PEMS-BAY
fixture (tests/golden/g13_train_n325.npz) in bf16 mode, its gradients against the oracle's
bf16 emulation with the per-piece mlp rounding switched on in the forward and / or backward
(4 variants); prints norm-rel per parameter for each.

    python tools/exp/bf16_mlp_probe.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "graph-wavenet_amd"), os.path.join(ROOT, "tests"), ROOT]
from conftest import load_golden, norm_rel, state_dict_of  # noqa: E402
from oracle import gwnet_oracle as orc  # noqa: E402
from test_gpu_bf16 import _trainer  # noqa: E402


class _Split(torch.autograd.Function):
    """_GcnBf16 with separate mlp roundings for the forward (mf) and backward (mb)."""

    @staticmethod
    def forward(ctx, g, w, rnd, mpair, *sups):  # same input positions as _GcnBf16
        y = orc._GcnBf16.forward(ctx, g, w, rnd, mpair[0], *sups)
        ctx.mrnd = mpair[1]
        return y

    @staticmethod
    def backward(ctx, dy):
        return orc._GcnBf16.backward(ctx, dy)


def main():
    gpu = torch.device("cuda:0")
    g = load_golden("g13_train_n325.npz")
    eng = _trainer(gpu, g, 325)
    eng.train(torch.tensor(g["x"], device=gpu), torch.tensor(g["y"], device=gpu))
    got = {k: p.grad.detach().cpu().numpy() for k, p in eng.model.named_parameters() if p.grad is not None}
    sd = state_dict_of(g)
    keys = [k for k in got if not k.endswith("mlp.bias") and np.linalg.norm(got[k]) > 0]
    rows = {}
    for mf in (False, True):
        for mb in (False, True):
            def fn(gg, w, sups, rnd=orc.bf16_round, mrnd=None, _mf=mf, _mb=mb):
                return _Split.apply(gg, w, rnd, (orc.bf16_round if _mf else None, orc.bf16_round if _mb else None), *sups)
            old = orc.gcn_bf16
            orc.gcn_bf16 = fn
            try:
                _, met, gr, _ = orc.grads(sd, [g["sup0"], g["sup1"]], g["x"], g["y"], orc.Cfg(325, gcn_bf16=True), 54.4, 19.5)
            finally:
                orc.gcn_bf16 = old
            rows[(mf, mb)] = {k: norm_rel(got[k], gr[k].numpy()) for k in keys}
            e = rows[(mf, mb)]
            print("fwd-mlp %d bwd-mlp %d: median %.2e worst %.2e (%s)" % (mf, mb, np.median(list(e.values())),
                                                                         max(e.values()), max(e, key=e.get)), flush=True)
    for k in keys:
        print("%-34s" % k, " ".join("%.2e" % rows[v][k] for v in sorted(rows)))


if __name__ == "__main__":
    main()
