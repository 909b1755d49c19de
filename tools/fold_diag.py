"""Layer-by-layer forward (and gradient) comparison of BatchNorm applied on load (GWN_BN_FOLD=1)
against the materialised bn(z) path (=0), same weights and input: locates the first buffer whose
values differ beyond fp32 rounding.  Usage: python tools/fold_diag.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "graph-wavenet_amd"), os.path.join(ROOT, "tests"), ROOT]

from conftest import load_golden, state_dict_of  # noqa: E402
from test_gpu_headline import _loader_views, _trainer  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def main():
    from gwn_amd import synthetic
    gpu = torch.device("cuda:0")
    n, B = 207, 64
    g = load_golden("g12_metr_n207.npz")
    sd = state_dict_of(g)
    x, y = synthetic.synthetic_batch(B, n, 12, seed=64)
    eng = _trainer(gpu, n, [g["sup0"], g["sup1"]], sd)
    tx, _ = _loader_views(x, y, gpu)
    model = eng.model
    ex = model.executor()
    res = {}
    for fold in ("0", "1"):
        os.environ["GWN_BN_FOLD"] = fold
        out, acts = ex.forward(model._flat, model._fixed_supports(), tx, True, model._bn_bufs(), acts=None, lead_pad=1)
        torch.cuda.synchronize()
        gout = torch.sin(torch.arange(out.numel(), device=out.device, dtype=out.dtype).view_as(out)) * 1e-3
        ex.backward(acts, gout)
        torch.cuda.synchronize()
        res[fold] = (out.clone(), acts, ex.gpacked.clone())
    o0, a0, g0 = res["0"]
    o1, a1, g1 = res["1"]
    print("out", rel(o1, o0))
    for i in range(ex.cfg.L):
        line = "layer %d: FG %.2e H %.2e Z %.2e mean %.2e rstd %.2e" % (
            i, rel(a1.FG[i], a0.FG[i]), rel(a1.H[i], a0.H[i]), rel(a1.Z[i], a0.Z[i]),
            rel(a1.mean[i], a0.mean[i]), rel(a1.rstd[i], a0.rstd[i]))
        if i + 1 < ex.cfg.L:
            xn = (a1.Z[i] - a1.mean[i]) * a1.bn_scale[i] + model._executor.pk("bn_b%d" % i)
            line += " bn(z) %.2e" % rel(xn, a0.X[i + 1])
        print(line)
    for nm in ("skipcat", "skr", "e1", "y"):
        b0, b1 = getattr(a0, nm), getattr(a1, nm)
        flips = int(((b0 > 0) != (b1 > 0)).sum()) if nm in ("skr", "e1") else -1
        print("%-8s %.2e  relu-mask flips %d of %d" % (nm, rel(b1, b0), flips, b0.numel()))
    print("grads (packed)", rel(g1, g0))
    lay = ex.layout
    for name in sorted(lay.segs):
        try:
            print("  %-8s %.2e" % (name, rel(lay.view(g1, name), lay.view(g0, name))))
        except Exception as e:  # noqa: BLE001
            print("  %-8s ?" % name, e)


if __name__ == "__main__":
    main()
