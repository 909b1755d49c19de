"""Constructor generality on libgwn (reference model.py:83-171, 244-407) against the reference's own
f64 runs (tests/golden/g17_generality.npz, made by tests/golden/make_golden_r3.py):

* kernel_size 3 with residual_channels 32 != dilation_channels 48 (generic MFMA GEMM path: k-tap
  gated TCN, gcn pieces on the dilation channels, mlp back to the residual channels);
* nhid 64 (train.py:28 --nhid) through trainer.train's captured step;
* gcn_bool False with kernel_size 3 and residual 16 != dilation 32 (residual_convs path);
* gwnet_diff_G called with supports=None (model.py:391-398: residual_convs in every layer).

Same tolerances as tests/test_gpu_model.py: output max-rel <= 1e-4, per-tensor gradient norm-rel
<= 1e-4, BN-cancelled biases within 1e-5 of the gradient scale, BN running stats rel <= 1e-5."""
import numpy as np
import pytest
import torch

from conftest import load_golden, norm_rel, rel_err, state_dict_of
from test_gpu_model import _check_grads

pytestmark = pytest.mark.gpu

KW = {  # tests/golden/make_golden_r3.py CASES
    "k3": dict(n=16, kw=dict(gcn_bool=True, addaptadj=True, kernel_size=3, residual_channels=32,
                             dilation_channels=48, skip_channels=64, end_channels=128, blocks=2, layers=2)),
    "h64": dict(n=37, kw=dict(gcn_bool=True, addaptadj=True, residual_channels=64, dilation_channels=64,
                              skip_channels=512, end_channels=1024)),
    "k3ng": dict(n=16, kw=dict(gcn_bool=False, addaptadj=False, kernel_size=3, residual_channels=16,
                               dilation_channels=32, skip_channels=64, end_channels=128)),
}


def _case(tag):
    g = load_golden("g17_generality.npz")
    p = tag + "/"
    return {k[len(p):]: v for k, v in g.items() if k.startswith(p)}


def _loss(out, y, gpu):
    from gwn_amd import util
    pred = out.transpose(1, 3) * 19.5 + 54.4
    return util.masked_mae(pred, torch.tensor(y, device=gpu).unsqueeze(1), 0.0)


def _check_bn(model, sub):
    sd = model.state_dict()
    for k, v in sub.items():
        if k.startswith("bnpost_f64/"):
            name = k[len("bnpost_f64/"):]
            assert rel_err(sd[name].cpu().numpy(), v) <= 1e-5, name


@pytest.mark.parametrize("tag", sorted(KW))
def test_g17_autograd_step(gpu, tag):
    from gwn_amd.model import gwnet
    sub = _case(tag)
    c = KW[tag]
    sups = [torch.tensor(sub["sup0"], device=gpu), torch.tensor(sub["sup1"], device=gpu)]
    m = gwnet(gpu, c["n"], 0.0, supports=sups, **c["kw"])
    assert m.receptive_field == int(sub["receptive_field"])
    m.load_state_dict({k: torch.tensor(v) for k, v in state_dict_of(sub).items()})
    m.train()
    out = m(torch.nn.functional.pad(torch.tensor(sub["x"], device=gpu), (1, 0, 0, 0)))
    loss = _loss(out, sub["y"], gpu)
    loss.backward()
    torch.cuda.synchronize()
    assert rel_err(out.detach().cpu().numpy(), sub["out_f64"]) <= 1e-4, tag
    assert abs(loss.item() / sub["metrics_f64"][0] - 1) <= 1e-4
    _check_grads(m, {k[len("grad_f64/"):]: v for k, v in sub.items() if k.startswith("grad_f64/")}, tag)
    _check_bn(m, sub)
    ex = m.executor()
    assert ex.cfg.square == (tag == "h64")


def test_g17_nhid64_trainer_step(gpu):
    """trainer(nhid=64): the captured train step (HIP loss, hand-written backward, fused clip+Adam
    with lr 0 and no clip, so the flat gradient buffer holds the raw gradients)."""
    from gwn_amd import util
    from gwn_amd.engine import trainer
    sub = _case("h64")
    sups = [torch.tensor(sub["sup0"], device=gpu), torch.tensor(sub["sup1"], device=gpu)]
    eng = trainer(util.StandardScaler(54.4, 19.5), 2, 12, 37, 64, 0.0, 0.0, 0.0, gpu, sups, True, True, None, 4, 2)
    eng.model.load_state_dict({k: torch.tensor(v) for k, v in state_dict_of(sub).items()})
    eng.clip = None
    met = eng.train(torch.tensor(sub["x"], device=gpu), torch.tensor(sub["y"], device=gpu))
    np.testing.assert_allclose(met, sub["metrics_f64"], rtol=1e-4)
    _check_grads(eng.model, {k[len("grad_f64/"):]: v for k, v in sub.items() if k.startswith("grad_f64/")}, "h64")


def test_g17_diff_g_without_supports(gpu):
    from gwn_amd.model import gwnet_diff_G
    sub = _case("dgres")
    m = gwnet_diff_G(gpu, 16, 0.0, supports_len=2, gcn_bool=True, addaptadj=False, residual_channels=16,
                     dilation_channels=16, skip_channels=64, end_channels=128, blocks=2, layers=2)
    m.load_state_dict({k: torch.tensor(v) for k, v in state_dict_of(sub).items()})
    m.train()
    out = m(torch.nn.functional.pad(torch.tensor(sub["x"], device=gpu), (1, 0, 0, 0)), None, None)
    loss = _loss(out, sub["y"], gpu)
    loss.backward()
    torch.cuda.synchronize()
    assert tuple(out.shape) == (2, 12, 16, 7)
    assert rel_err(out.detach().cpu().numpy(), sub["out_f64"]) <= 1e-4
    assert abs(loss.item() / sub["metrics_f64"][0] - 1) <= 1e-4
    _check_grads(m, {k[len("grad_f64/"):]: v for k, v in sub.items() if k.startswith("grad_f64/")}, "dgres")
    # the gcn mlps exist (gcn_bool) but never run: no gradient, as under reference autograd
    assert all(p.grad is None for n, p in m.named_parameters() if n.startswith("gconv."))


@pytest.mark.parametrize("path", ["autograd", "trainer"])
def test_deep_stack_gram_chunks(gpu, path):
    """blocks=4, layers=3 at C=32: 11 adaptive-support gram layers, more than one
    grouped gram launch takes (8), run as two launches, the second accumulating -- gradients against
    the fp64 oracle like every other C=32 model test."""
    from gwn_amd import synthetic, util
    from gwn_amd.engine import trainer
    from gwn_amd.model import gwnet
    from oracle import gwnet_oracle as orc
    n, B = 40, 2
    adj = synthetic.random_sensor_graph(n, density=0.2, seed=11)
    sups = synthetic.double_transition(adj)
    x, y = synthetic.synthetic_batch(B, n, 12, seed=12)
    torch.manual_seed(7)
    dsups = [torch.tensor(a, device=gpu) for a in sups]
    if path == "autograd":
        m = gwnet(gpu, n, 0.0, supports=dsups, blocks=4, layers=3)
        sd0 = {k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()}
        m.train()
        out = m(torch.nn.functional.pad(torch.tensor(x, device=gpu), (1, 0, 0, 0)))
        loss = _loss(out, y, gpu)
        loss.backward()
    else:
        eng = trainer(util.StandardScaler(54.4, 19.5), 2, 12, n, 32, 0.0, 0.0, 0.0, gpu, dsups, True, True, None,
                      4, 3)
        m = eng.model
        sd0 = {k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()}
        eng.clip = None
        # the trainer's own x layout (train.py:244-247): [B, Cin, N, T] transposed views
        met = eng.train(torch.tensor(x, device=gpu), torch.tensor(y, device=gpu))
    torch.cuda.synchronize()
    cfg = orc.Cfg(n, blocks=4, layers=3)
    ref_out, ref_met, ref_g, _ = orc.grads(sd0, sups, x, y, cfg, 54.4, 19.5)
    if path == "autograd":
        assert rel_err(out.detach().cpu().numpy(), ref_out.numpy()) <= 1e-4
        assert abs(loss.item() - ref_met[0]) <= 1e-4 * abs(ref_met[0])
    else:
        assert abs(met[0] - ref_met[0]) <= 1e-4 * abs(ref_met[0])
    _check_grads(m, {k: v.numpy() for k, v in ref_g.items()}, "deep_" + path)
