"""Parity at the configurations the benchmark runs, through the drop-in trainer.

* METR-LA headline shape (B=64, N=207, T=12): one ``trainer.train`` step (dropout 0, lr 0, no
  clip) -> every parameter gradient against the fp64 oracle (norm-rel <= 1e-4; the BN-cancelled
  gconv biases, analytically 0, absolutely), loss / MAPE / RMSE (rel <= 1e-4) and the BN running
  statistics after the step (rel <= 1e-5).  The step's kinks are pinned: labels within 1e-3 of the
  fp64 prediction are moved off the tie first (``_untie``: the MAE gradient is a sign), and the
  oracle differentiates the head ReLUs on the branch the fp32 step took (``_gpu_branch``; one
  element at a ReLU kink out of 10^7 otherwise moves gradients by ~1e-3).  The adopted branches
  are checked, not trusted: every element where the GPU's ReLU mask differs from the oracle's own
  fp64 ``pre-activation > 0`` must have |pre-activation| <= 1e-5 max|pre-activation| (a tie
  within fp32 rounding), and the B=64 output tensor itself is compared (max-rel <= 1e-4).
* PEMS-BAY shape (N=325): the same against the reference's own f64 run (g13, B=2).
Inputs are passed as the transpose views train.py:244-247 builds (``torch.Tensor(x).transpose(1, 3)``
of the [B, T, N, 2] loader batch; labels ``y.transpose(1, 3)[:, 0]``).
Also: the dropout counter advances per autograd forward (F.dropout draws a fresh mask per call),
eval-mode backward (running-stat BN) against the oracle, nodevec grads stay None when the adaptive
support cannot reach the output, and a real_val shape the fused step cannot index raises."""
import numpy as np
import pytest
import torch

from conftest import load_golden, norm_rel, rel_err, state_dict_of

pytestmark = pytest.mark.gpu


def _loader_views(x, y, device):
    """[B, 2, N, T] / [B, N, T] arrays -> the transpose views train.py:244-247 hands to train()."""
    xl = torch.tensor(np.ascontiguousarray(x.transpose(0, 3, 2, 1)), device=device)          # [B, T, N, 2]
    yl = torch.tensor(np.ascontiguousarray(np.stack([y, y], axis=1).transpose(0, 3, 2, 1)), device=device)
    tx = xl.transpose(1, 3)                 # [B, 2, N, T], non-contiguous
    ty = yl.transpose(1, 3)[:, 0, :, :]     # [B, N, T], non-contiguous
    assert not tx.is_contiguous() and not ty.is_contiguous()
    return tx, ty


def _check(got, ref, tag, dropout=False):
    """Every gradient norm-rel <= 1e-4; the gconv biases (BatchNorm cancels a per-channel constant:
    analytically 0) absolutely -- unless dropout scales them per element (then they are live)."""
    assert set(got) == set(ref), (tag, sorted(set(got) ^ set(ref)))
    scale = max(float(np.max(np.abs(v))) for v in ref.values())
    for k, v in ref.items():
        g = got[k]
        if k.startswith("gconv.") and k.endswith("mlp.bias") and not dropout:
            assert np.max(np.abs(g)) <= 1e-5 * scale, (tag, k)
        elif np.linalg.norm(v) > 0:
            assert norm_rel(g, v) <= 1e-4, (tag, k, norm_rel(g, v))


def _trainer(device, n, sups, sd, dropout=0.0):
    from gwn_amd import util
    from gwn_amd.engine import trainer
    eng = trainer(util.StandardScaler(54.4, 19.5), 2, 12, n, 32, dropout, 0.0, 0.0, device,
                  [torch.tensor(s, device=device) for s in sups], True, True, None, 4, 2)
    eng.model.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
    eng.clip = None
    return eng


def _untie(sd, sups, x, y, n, margin=1e-3, cfg=None, dropout_masks=None):
    """Labels moved away from near-ties with the fp64 prediction.  The masked-MAE gradient is
    sign(pred - real) (util.py:524): a label within fp32 rounding of its prediction takes either
    sign in two equally valid fp32 evaluations, and one flipped element out of B*N*12 moves every
    parameter gradient by ~1e-3 relative at B=64.  Labels with |pred - real| < margin (1e-3 in
    label units, ~20x the fp32-vs-fp64 output difference) move to 2*margin on the side they were
    on; zero (masked) labels stay.  Returns (labels, count moved)."""
    from oracle import gwnet_oracle as orc
    f64 = torch.float64
    p = {k: torch.tensor(np.asarray(v), dtype=f64) for k, v in sd.items() if not orc._is_buffer(k)}
    bn = {k: torch.tensor(np.asarray(v), dtype=f64) for k, v in sd.items() if "running" in k}
    with torch.no_grad():
        out = orc.engine_loss(p, [torch.tensor(np.asarray(a), dtype=f64) for a in sups], torch.tensor(x, dtype=f64),
                              torch.tensor(y, dtype=f64), cfg if cfg is not None else orc.Cfg(n), 54.4, 19.5, bn,
                              dropout_masks=dropout_masks)[0]
    pred = (out.transpose(1, 3) * 19.5 + 54.4)[:, 0].numpy()
    d = pred - y
    tie = (np.abs(d) < margin) & (y != 0)
    y = y.copy()
    y[tie] = np.where(d[tie] >= 0, pred[tie] - 2 * margin, pred[tie] + 2 * margin)
    return y, int(tie.sum())


def _gpu_branch(eng, B, n):
    """The head ReLU branches the fp32 step took (oracle module docstring: branch pinning), in the
    oracle's NCHW layout: masks of relu(skip) and relu(end_conv_1) from the trainer's saved
    activations (rows (t, b, n), channels last)."""
    (acts,) = list(eng._acts.values())

    def nchw(buf):
        tf = buf.shape[0] // (B * n)
        return (buf > 0).double().cpu().view(tf, B, n, buf.shape[1]).permute(1, 3, 2, 0)

    return {"skip": nchw(acts.skr), "e1": nchw(acts.e1)}


def test_headline_b64_train_step_grads_vs_oracle(gpu):
    from gwn_amd import synthetic
    from oracle import gwnet_oracle as orc
    n, B = 207, 64
    g = load_golden("g12_metr_n207.npz")
    sd = state_dict_of(g)
    x, y = synthetic.synthetic_batch(B, n, 12, seed=64)
    y, _ = _untie(sd, [g["sup0"], g["sup1"]], x, y, n)
    eng = _trainer(gpu, n, [g["sup0"], g["sup1"]], sd)
    tx, ty = _loader_views(x, y, gpu)
    met = eng.train(tx, ty)
    masks = _gpu_branch(eng, B, n)
    (acts,) = list(eng._acts.values())
    out_gpu = acts.y.detach().cpu().double().view(1, B, n, 12).permute(1, 3, 2, 0).numpy()
    torch.set_num_threads(max(1, torch.get_num_threads()))
    rec = {}
    rout, rmet, rg, rbn = orc.grads(sd, [g["sup0"], g["sup1"]], x, y, orc.Cfg(n), 54.4, 19.5, masks=masks,
                                    record=rec)
    # the adopted branches differ from the oracle's own only at fp32 ties
    for key in ("skip", "e1"):
        pre = rec[key].numpy()
        flip = masks[key].numpy().astype(bool) != (pre > 0)
        tol = 1e-5 * float(np.max(np.abs(pre)))
        print("%s: %d of %d ReLU branches differ from the fp64 sign (max |pre| there %.3g, tol %.3g)"
              % (key, int(flip.sum()), flip.size, float(np.max(np.abs(pre[flip]), initial=0.0)), tol))
        assert np.all(np.abs(pre[flip]) <= tol), (key, int(flip.sum()))
    assert rel_err(out_gpu, rout.numpy()) <= 1e-4, rel_err(out_gpu, rout.numpy())
    np.testing.assert_allclose(met, rmet, rtol=1e-4)
    got = {k: p.grad.detach().cpu().numpy() for k, p in eng.model.named_parameters() if p.grad is not None}
    _check(got, {k: v.numpy() for k, v in rg.items()}, "b64")
    sdn = eng.model.state_dict()
    for k, v in rbn.items():
        assert rel_err(sdn[k].cpu().numpy(), v.numpy()) <= 1e-5, k
    # the captured-graph replay (second step on the same key) gives the same gradients
    eng.train(tx, ty)
    got2 = {k: p.grad.detach().cpu().numpy() for k, p in eng.model.named_parameters() if p.grad is not None}
    for k in got:
        np.testing.assert_array_equal(got[k], got2[k], err_msg=k)


def host_dropout_masks(seed, cfg, B, n, C, T0):
    """libgwn's dropout keep masks of every layer, rebuilt on the host (gwn_uniform of the device
    counter ``seed``, salt = layer, element index ((t*B + b)*N + node)*C + c of the layer's
    [T][B][N][C] output rows), in the oracle's [B, C, N, T] layout."""
    from test_gpu_model import _np_uniform
    masks, T = [], T0
    for i, d in enumerate(cfg.dilations):
        T -= d
        idx = np.arange(T * B * n * C, dtype=np.int64)
        keep = (_np_uniform(seed, i, idx) >= np.float32(cfg.dropout)).reshape(T, B, n, C)
        masks.append(torch.tensor(keep.transpose(1, 3, 2, 0).astype(np.float64)))
    return masks


def test_headline_b64_dropout_train_step_vs_oracle(gpu):
    """The bench's own step: trainer.train at B=64, N=207, C=32 with dropout 0.3 -- the 16-node tile
    forward (its fused gated TCN on the layers with a slice per CU or more) and backward apply the
    counter masks.  The masks are rebuilt on the host from the step's seed and fed to the fp64
    oracle (forward(dropout_masks=...)); output max-rel <= 1e-4, every gradient norm-rel <= 1e-4,
    metrics and BN running stats as in the dropout-0 headline test, same branch pinning.  The
    dropped fraction is ~0.3 per layer and the step advances the counter by one."""
    from gwn_amd import synthetic
    from oracle import gwnet_oracle as orc
    n, B, drop = 207, 64, 0.3
    g = load_golden("g12_metr_n207.npz")
    sd = state_dict_of(g)
    sups = [g["sup0"], g["sup1"]]
    x, y = synthetic.synthetic_batch(B, n, 12, seed=66)
    eng = _trainer(gpu, n, sups, sd, dropout=drop)
    ex = eng.model.executor()
    seed = int(ex.seed.item())
    cfg = orc.Cfg(n, dropout=drop)
    dmasks = host_dropout_masks(seed, cfg, B, n, 32, 13)
    for mk in dmasks:
        assert 0.29 < 1.0 - float(mk.mean()) < 0.31
    y, _ = _untie(sd, sups, x, y, n, cfg=cfg, dropout_masks=dmasks)
    tx, ty = _loader_views(x, y, gpu)
    met = eng.train(tx, ty)
    assert int(ex.seed.item()) == seed + 1
    masks = _gpu_branch(eng, B, n)
    (acts,) = list(eng._acts.values())
    out_gpu = acts.y.detach().cpu().double().view(1, B, n, 12).permute(1, 3, 2, 0).numpy()
    rec = {}
    rout, rmet, rg, rbn = orc.grads(sd, sups, x, y, cfg, 54.4, 19.5, masks=masks, record=rec, dropout_masks=dmasks)
    for key in ("skip", "e1"):
        pre = rec[key].numpy()
        flip = masks[key].numpy().astype(bool) != (pre > 0)
        assert np.all(np.abs(pre[flip]) <= 1e-5 * float(np.max(np.abs(pre)))), (key, int(flip.sum()))
    assert rel_err(out_gpu, rout.numpy()) <= 1e-4, rel_err(out_gpu, rout.numpy())
    np.testing.assert_allclose(met, rmet, rtol=1e-4)
    got = {k: p.grad.detach().cpu().numpy() for k, p in eng.model.named_parameters() if p.grad is not None}
    _check(got, {k: v.numpy() for k, v in rg.items()}, "b64 dropout", dropout=True)
    sdn = eng.model.state_dict()
    for k, v in rbn.items():
        assert rel_err(sdn[k].cpu().numpy(), v.numpy()) <= 1e-5, k
    # a second (graph-captured) step draws the next masks: the output moves
    eng.train(tx, ty)
    assert int(ex.seed.item()) == seed + 2
    (acts2,) = list(eng._acts.values())
    out2 = acts2.y.detach().cpu().double().view(1, B, n, 12).permute(1, 3, 2, 0).numpy()
    assert rel_err(out2, out_gpu) > 1e-3


def test_pems_n325_train_step_grads_vs_reference(gpu):
    g = load_golden("g13_train_n325.npz")
    eng = _trainer(gpu, 325, [g["sup0"], g["sup1"]], state_dict_of(g))
    tx, ty = _loader_views(g["x"], g["y"], gpu)
    met = eng.train(tx, ty)
    np.testing.assert_allclose(met, g["metrics_f64"], rtol=1e-4)
    ref = {k[len("grad_f64/"):]: v for k, v in g.items() if k.startswith("grad_f64/")}
    got = {k: p.grad.detach().cpu().numpy() for k, p in eng.model.named_parameters() if p.grad is not None}
    _check(got, ref, "n325")
    sdn = eng.model.state_dict()
    for k, v in g.items():
        if k.startswith("bnpost_f64/"):
            name = k[len("bnpost_f64/"):]
            if "num_batches" in name:
                assert int(sdn[name]) == int(v)
            else:
                assert rel_err(sdn[name].cpu().numpy(), v) <= 1e-5, name


def _model(device, n=16, dropout=0.0, **kw):
    from gwn_amd import synthetic
    from gwn_amd.model import gwnet
    adj = synthetic.random_sensor_graph(n, density=0.3, seed=3)
    sups = synthetic.double_transition(adj)
    torch.manual_seed(999)
    m = gwnet(device, n, dropout, supports=[torch.tensor(a, device=device) for a in sups], residual_channels=16,
              dilation_channels=16, skip_channels=128, end_channels=256, **kw)
    return m, sups


def test_autograd_forward_draws_fresh_dropout_masks(gpu):
    from gwn_amd import synthetic
    m, _ = _model(gpu, dropout=0.3)
    m.train()
    x, _ = synthetic.synthetic_batch(2, 16, 13, seed=1)
    xd = torch.tensor(x, device=gpu)
    o1 = m(xd).detach().clone()
    o2 = m(xd).detach().clone()
    assert not torch.equal(o1, o2)
    # and forward / backward of one call share their mask: gradients of a call made between
    # another call's forward and backward are unaffected (covered by the mask snapshot)
    m.eval()
    with torch.no_grad():
        e1, e2 = m(xd), m(xd)
    assert torch.equal(e1, e2)


def test_eval_mode_backward_vs_oracle(gpu):
    """model.eval(); loss.backward(): BatchNorm with running statistics is affine, its backward
    is gamma * rstd_running * dy (no batch-mean terms); compared with fp64 autograd."""
    from gwn_amd import synthetic, util
    from oracle import gwnet_oracle as orc
    m, sups = _model(gpu)
    sd0 = {k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()}
    # non-trivial running statistics
    for k in sd0:
        if "running_mean" in k:
            sd0[k] = np.linspace(-0.2, 0.3, sd0[k].size).astype(np.float32)
        elif "running_var" in k:
            sd0[k] = np.linspace(0.5, 2.0, sd0[k].size).astype(np.float32)
    m.load_state_dict({k: torch.tensor(v) for k, v in sd0.items()})
    m.eval()
    x, y = synthetic.synthetic_batch(2, 16, 12, seed=21)
    out = m(torch.nn.functional.pad(torch.tensor(x, device=gpu), (1, 0, 0, 0)))
    loss = util.masked_mae(out.transpose(1, 3) * 19.5 + 54.4, torch.tensor(y, device=gpu).unsqueeze(1), 0.0)
    loss.backward()
    torch.cuda.synchronize()
    cfg = orc.Cfg(16, nhid=16, skip=128, end=256)
    p = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in sd0.items()
         if "running" not in k and "num_batches" not in k}
    bn = {k: torch.tensor(v, dtype=torch.float64) for k, v in sd0.items() if "running" in k}
    ref_out, mae, _, _ = orc.engine_loss(p, [torch.tensor(a, dtype=torch.float64) for a in sups],
                                         torch.tensor(x, dtype=torch.float64), torch.tensor(y, dtype=torch.float64),
                                         cfg, 54.4, 19.5, bn, training=False)
    assert rel_err(out.detach().cpu().numpy(), ref_out.detach().numpy()) <= 1e-4
    names = list(p)
    gs = torch.autograd.grad(mae, [p[k] for k in names], allow_unused=True)
    ref = {k: gi.numpy() for k, gi in zip(names, gs) if gi is not None}
    got = {k: q.grad.detach().cpu().numpy() for k, q in m.named_parameters() if q.grad is not None}
    assert set(got) == set(ref), sorted(set(got) ^ set(ref))
    for k, v in ref.items():
        if np.linalg.norm(v) > 0:
            assert norm_rel(got[k], v) <= 1e-4, (k, norm_rel(got[k], v))
    # running statistics untouched by an eval forward
    for k, v in sd0.items():
        if "running" in k:
            np.testing.assert_array_equal(m.state_dict()[k].cpu().numpy(), v)


def test_single_layer_nodevecs_get_no_grad(gpu):
    """blocks*layers == 1: the only gcn output is dead, so the adaptive support never reaches the
    loss and nodevec1/2 keep grad None (the reference's Adam then skips them)."""
    from gwn_amd import synthetic, util
    m, _ = _model(gpu, blocks=1, layers=1)
    m.train()
    x, y = synthetic.synthetic_batch(2, 16, 12, seed=2)
    out = m(torch.nn.functional.pad(torch.tensor(x, device=gpu), (1, 0, 0, 0)))
    util.masked_mae(out.transpose(1, 3) * 19.5 + 54.4, torch.tensor(y, device=gpu).unsqueeze(1), 0.0).backward()
    assert m.nodevec1.grad is None and m.nodevec2.grad is None
    assert m.start_conv.weight.grad is not None


def test_trainer_rejects_label_shape_it_cannot_index(gpu):
    from gwn_amd import synthetic, util
    from gwn_amd.engine import trainer
    _, sups = _model(gpu)
    eng = trainer(util.StandardScaler(54.4, 19.5), 2, 12, 16, 16, 0.0, 1e-3, 1e-4, gpu,
                  [torch.tensor(a, device=gpu) for a in sups], True, True, None, 4, 2)
    x, y = synthetic.synthetic_batch(2, 16, 12, seed=2)
    with pytest.raises(RuntimeError):
        eng.train(torch.tensor(x, device=gpu), torch.tensor(y[:, :, :11].copy(), device=gpu))
    with pytest.raises(RuntimeError):   # batch mismatch between input and labels
        eng.train(torch.tensor(x, device=gpu), torch.tensor(np.concatenate([y, y]), device=gpu))
