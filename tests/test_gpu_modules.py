"""The reference's building-block modules used standalone (``from model import *``, engine.py:2):
``linear`` (model.py:24-30) and ``gcn`` (model.py:32-55) on libgwn, NCHW in and out, forward and
backward against the fp64 oracle / the reference's own nconv golden (g6).  Tolerances: forward
max-rel <= 1e-4, gradients norm-rel <= 1e-4."""
import numpy as np
import pytest
import torch

from conftest import load_golden, norm_rel, rel_err

pytestmark = pytest.mark.gpu
F64 = torch.float64


@pytest.mark.parametrize("shape", [(2, 224, 207, 12), (3, 7, 5, 1), (1, 32, 33, 13)])
def test_linear_forward_backward(gpu, shape):
    from gwn_amd.model import linear
    from oracle import gwnet_oracle as orc
    B, ci, H, W = shape
    torch.manual_seed(5)
    m = linear(ci, 32).to(gpu)
    x = torch.randn(*shape, device=gpu, requires_grad=True)
    y = m(x)
    gy = torch.randn_like(y)
    y.backward(gy)
    torch.cuda.synchronize()
    wd = m.mlp.weight.detach().cpu().double().requires_grad_(True)
    bd = m.mlp.bias.detach().cpu().double().requires_grad_(True)
    xd = x.detach().cpu().double().requires_grad_(True)
    yr = orc.pointwise(xd, wd, bd)
    assert rel_err(y.detach().cpu().numpy(), yr.detach().numpy()) <= 1e-4
    yr.backward(gy.cpu().double())
    assert norm_rel(x.grad.cpu().numpy(), xd.grad.numpy()) <= 1e-4
    assert norm_rel(m.mlp.weight.grad.cpu().numpy(), wd.grad.numpy()) <= 1e-4
    assert norm_rel(m.mlp.bias.grad.cpu().numpy(), bd.grad.numpy()) <= 1e-4


def test_linear_rejects_channel_mismatch(gpu):
    from gwn_amd.model import linear
    m = linear(8, 4).to(gpu)
    with pytest.raises(RuntimeError):
        m(torch.randn(1, 7, 3, 3, device=gpu))


def test_gcn_module_forward_backward_vs_oracle(gpu):
    """gcn(x, [A1, A2, adp]) in eval mode: the reference's nconv golden pins hop 1 of A1; the whole
    block (3 supports x 2 hops, concat, 1x1) and its gradients w.r.t. x, every support and the mlp
    against fp64 autograd of the oracle."""
    from gwn_amd.model import gcn
    from oracle import gwnet_oracle as orc
    g = load_golden("g6_ops_n207.npz")
    torch.manual_seed(6)
    m = gcn(32, 32, 0.3, support_len=3).to(gpu)
    m.eval()
    x = torch.tensor(g["x"], device=gpu, requires_grad=True)
    adp = torch.tensor(g["adp"], device=gpu)
    sups = [torch.tensor(g["A"], device=gpu), torch.tensor(g["A"].T.copy(), device=gpu), adp.clone()]
    for s in sups:
        s.requires_grad_(True)
    h1 = m.nconv(x, sups[0])
    assert rel_err(h1.detach().cpu().numpy(), g["nconv"]) <= 1e-4
    y = m(x, sups)
    gy = torch.randn_like(y)
    y.backward(gy)
    torch.cuda.synchronize()
    xd = torch.tensor(g["x"], dtype=F64, requires_grad=True)
    sd = [s.detach().cpu().double().requires_grad_(True) for s in sups]
    wd = m.mlp.mlp.weight.detach().cpu().double().requires_grad_(True)
    bd = m.mlp.mlp.bias.detach().cpu().double().requires_grad_(True)
    pieces = [xd]
    for a in sd:
        y1 = orc.diffuse(xd, a)
        pieces += [y1, orc.diffuse(y1, a)]
    yr = orc.pointwise(torch.cat(pieces, dim=1), wd, bd)
    assert rel_err(y.detach().cpu().numpy(), yr.detach().numpy()) <= 1e-4
    yr.backward(gy.cpu().double())
    assert norm_rel(x.grad.cpu().numpy(), xd.grad.numpy()) <= 1e-4
    for s, r in zip(sups, sd):
        assert norm_rel(s.grad.cpu().numpy(), r.grad.numpy()) <= 1e-4
    assert norm_rel(m.mlp.mlp.weight.grad.cpu().numpy(), wd.grad.numpy()) <= 1e-4
    assert norm_rel(m.mlp.mlp.bias.grad.cpu().numpy(), bd.grad.numpy()) <= 1e-4


def test_gcn_module_train_mode_dropout(gpu):
    from gwn_amd.model import gcn
    torch.manual_seed(7)
    m = gcn(16, 16, 0.3, support_len=1, order=3).to(gpu)   # any diffusion order standalone
    m.train()
    x = torch.randn(4, 16, 40, 6, device=gpu)
    a = torch.softmax(torch.randn(40, 40, device=gpu), dim=1)
    y = m(x, [a])
    m.eval()
    ye = m(x, [a])
    zero = (y == 0).float().mean().item()
    assert 0.25 < zero < 0.35
    kept = y != 0
    np.testing.assert_allclose(y[kept].detach().cpu().numpy(), (ye[kept] / 0.7).detach().cpu().numpy(),
                               rtol=1e-5, atol=1e-6)


def test_gcn2_module_vs_reference(gpu):
    """gcn2 (model.py:57-80, per-sample supports) standalone on libgwn against the reference's own
    outputs and f64 gradients (g9: B=3, C=4, N=37, T=5, two supports, order 2, eval mode)."""
    from gwn_amd.model import gcn2
    g = load_golden("g9_nconv2_n37.npz")
    m = gcn2(4, g["gcn2/w"].shape[0], 0.0, support_len=2).to(gpu)
    with torch.no_grad():
        m.mlp.mlp.weight.copy_(torch.tensor(g["gcn2/w"]).reshape(m.mlp.mlp.weight.shape))
        m.mlp.mlp.bias.copy_(torch.tensor(g["gcn2/b"]))
    m.eval()
    x = torch.tensor(g["x"], device=gpu, dtype=torch.float32, requires_grad=True)
    sups = [torch.tensor(g["gcn2/s0"], device=gpu, dtype=torch.float32),
            torch.tensor(g["gcn2/s1"], device=gpu, dtype=torch.float32)]
    h = m(x, sups)
    assert rel_err(h.detach().cpu().numpy(), g["gcn2/h"]) <= 1e-4
    h.backward(torch.tensor(g["gcn2/gh"], device=gpu, dtype=torch.float32))
    assert norm_rel(x.grad.cpu().numpy(), g["gcn2/dx"]) <= 1e-4
    assert norm_rel(m.mlp.mlp.weight.grad.cpu().numpy().reshape(g["gcn2/dw"].shape), g["gcn2/dw"]) <= 1e-4
    assert norm_rel(m.mlp.mlp.bias.grad.cpu().numpy(), g["gcn2/db"]) <= 1e-4
