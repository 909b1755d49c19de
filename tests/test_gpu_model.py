"""gwnet / trainer on libgwn vs the reference's golden vectors and the CPU oracle.

Tolerances (north_star): forward max-rel <= 1e-4 against the fp64 reference;
per-tensor gradient norm-rel <= 1e-4 against fp64 truth; gconv.*.mlp.bias gradients (analytically
0, the following BN cancels them) compared with an absolute bound; masked metrics rel <= 1e-4."""
import numpy as np
import pytest
import torch

from conftest import load_golden, norm_rel, rel_err, state_dict_of

pytestmark = pytest.mark.gpu


def _model(g, device, n, dropout=0.0, sups=2, **kw):
    from gwn_amd.model import gwnet
    supports = [torch.tensor(g["sup0"], device=device), torch.tensor(g["sup1"], device=device)][:sups]
    if sups == 0 and kw.get("addaptadj", True):
        supports = None
    m = gwnet(device, n, dropout, supports=supports, **kw)
    sd = {k: torch.tensor(v) for k, v in state_dict_of(g).items()}
    m.load_state_dict(sd)
    return m


def _bn_cancelled(name):
    """Biases added right before a BatchNorm (no dropout in between) have an analytically zero
    gradient: the batch mean removes any per-channel shift."""
    return (name.startswith("gconv.") and name.endswith("mlp.bias")) or \
        (name.startswith("residual_convs.") and name.endswith(".bias"))


def _check_grads(model, ref, tag, dropout=False):
    got = {n: p.grad for n, p in model.named_parameters() if p.grad is not None}
    assert set(got) == set(ref), (tag, sorted(set(got) ^ set(ref)))
    scale = max(np.max(np.abs(v)) for v in ref.values())
    for k, v in ref.items():
        g = got[k].detach().cpu().numpy()
        if _bn_cancelled(k) and not dropout:
            assert np.max(np.abs(g)) <= 1e-5 * scale, (tag, k)
        elif np.linalg.norm(v) > 0:
            assert norm_rel(g, v) <= 1e-4, (tag, k, norm_rel(g, v))


def test_g1_eval_forward(gpu):
    g = load_golden("g12_metr_n207.npz")
    m = _model(g, gpu, 207, dropout=0.3)
    m.eval()
    with torch.no_grad():
        out = m(torch.tensor(g["g1_x"], device=gpu))
    torch.cuda.synchronize()
    assert tuple(out.shape) == (4, 12, 207, 1)
    assert rel_err(out.cpu().numpy(), g["g1_out_f64"]) <= 1e-4
    np.testing.assert_allclose(out.cpu().numpy(), g["g1_out_f64"], rtol=1e-4, atol=1e-4 * np.abs(g["g1_out_f64"]).max())


def test_g2_autograd_grads_and_bn_stats(gpu):
    from gwn_amd import util
    g = load_golden("g12_metr_n207.npz")
    m = _model(g, gpu, 207, dropout=0.0)
    m.train()
    x = torch.nn.functional.pad(torch.tensor(g["g2_x"], device=gpu), (1, 0, 0, 0))
    out = m(x)
    pred = out.transpose(1, 3) * 19.5 + 54.4
    real = torch.tensor(g["g2_y"], device=gpu).unsqueeze(1)
    loss = util.masked_mae(pred, real, 0.0)
    loss.backward()
    torch.cuda.synchronize()
    assert rel_err(out.detach().cpu().numpy(), g["g2_out_f64"]) <= 1e-4
    assert abs(loss.item() - g["g2_metrics_f64"][0]) <= 1e-4 * g["g2_metrics_f64"][0]
    ref = {k[len("g2_grad_f64/"):]: v for k, v in g.items() if k.startswith("g2_grad_f64/")}
    _check_grads(m, ref, "g2")
    sd = m.state_dict()
    for k, v in g.items():
        if k.startswith("g2_bnpost_f64/"):
            name = k[len("g2_bnpost_f64/"):]
            got = sd[name].cpu().numpy()
            if "num_batches" in name:
                assert int(got) == int(v)
            else:
                assert rel_err(got, v) <= 1e-5, name


def test_g2_fused_trainer_grads(gpu):
    """trainer.train's fused path (HIP loss + hand-written backward) with lr=0 and no clip, so the
    flat gradient buffer holds the raw gradients."""
    from gwn_amd import util
    from gwn_amd.engine import trainer
    g = load_golden("g12_metr_n207.npz")
    sups = [torch.tensor(g["sup0"], device=gpu), torch.tensor(g["sup1"], device=gpu)]
    eng = trainer(util.StandardScaler(54.4, 19.5), 2, 12, 207, 32, 0.0, 0.0, 0.0, gpu, sups, True, True, None, 4, 2)
    eng.model.load_state_dict({k: torch.tensor(v) for k, v in state_dict_of(g).items()})
    eng.clip = None
    x = torch.tensor(g["g2_x"], device=gpu)
    y = torch.tensor(g["g2_y"], device=gpu)
    met = eng.train(x, y)
    np.testing.assert_allclose(met, g["g2_metrics_f64"], rtol=1e-4)
    ref = {k[len("g2_grad_f64/"):]: v for k, v in g.items() if k.startswith("g2_grad_f64/")}
    _check_grads(eng.model, ref, "fused")
    # lr = 0 -> Adam leaves the weights unchanged
    for k, v in state_dict_of(g).items():
        if "running" not in k and "num_batches" not in k:
            np.testing.assert_array_equal(eng.model.state_dict()[k].cpu().numpy(), v, err_msg=k)


def test_g3_trainer_three_steps(gpu):
    from gwn_amd import util
    from gwn_amd.engine import trainer
    g = load_golden("g3_trainer_steps_n16.npz")
    sups = [torch.tensor(g["sup0"], device=gpu), torch.tensor(g["sup1"], device=gpu)]
    torch.manual_seed(999)
    eng = trainer(util.StandardScaler(54.4, 19.5), 2, 12, 16, 16, 0.0, 1e-3, 1e-4, gpu, sups, True, True, None, 4, 2)
    for k, v in state_dict_of(g).items():
        np.testing.assert_array_equal(eng.model.state_dict()[k].cpu().numpy(), v, err_msg=k)
    for s in range(3):
        met = eng.train(torch.tensor(g["x%d" % s], device=gpu), torch.tensor(g["y%d" % s], device=gpu))
        np.testing.assert_allclose(met, g["metrics%d_f64" % s], rtol=1e-4)
    sd = eng.model.state_dict()
    for k, v in g.items():
        if k.startswith("post_f64/"):
            name = k[len("post_f64/"):]
            got = sd[name].cpu().numpy()
            if "num_batches" in name:
                assert int(got) == int(v), name
            elif name.startswith("gconv.") and name.endswith("mlp.bias"):
                # true gradient is 0 (BN cancels it): Adam turns fp noise into +-lr steps
                assert np.max(np.abs(got - v)) <= 2 * 3 * 1e-3 + 1e-6, name
            else:
                assert norm_rel(got, v) <= 1e-4, (name, norm_rel(got, v))


VARIANTS = {
    "nogcn": dict(sups=2, gcn_bool=False),
    "noadp": dict(sups=2, addaptadj=False),
    "aptonly": dict(sups=0),
    "blocks3": dict(sups=2, blocks=3, layers=3),
    "seq24": dict(sups=2, out_dim=24),
}


@pytest.mark.parametrize("name", sorted(VARIANTS))
def test_g5_variants(gpu, name):
    from gwn_amd import util
    g = load_golden("g5_variant_%s_n16.npz" % name)
    kw = dict(VARIANTS[name])
    kw.update(residual_channels=16, dilation_channels=16, skip_channels=128, end_channels=256)
    m = _model(g, gpu, 16, **kw)
    m.eval()
    with torch.no_grad():
        out = m(torch.tensor(g["x"], device=gpu))
    torch.cuda.synchronize()
    assert rel_err(out.cpu().numpy(), g["out_f32"]) <= 1e-4, name
    m2 = _model(g, gpu, 16, **kw)
    m2.train()
    x = torch.nn.functional.pad(torch.tensor(g["x"], device=gpu), (1, 0, 0, 0))
    o2 = m2(x)
    loss = util.masked_mae(o2.transpose(1, 3) * 19.5 + 54.4, torch.tensor(g["y"], device=gpu).unsqueeze(1), 0.0)
    loss.backward()
    torch.cuda.synchronize()
    assert rel_err(o2.detach().cpu().numpy(), g["trainout_f64"]) <= 1e-4
    ref = {k[len("grad_f64/"):]: v for k, v in g.items() if k.startswith("grad_f64/")}
    _check_grads(m2, ref, name)


def test_g5b_pems_forward(gpu):
    g = load_golden("g5b_fwd_eval_n325.npz")
    m = _model(g, gpu, 325, dropout=0.3)
    m.eval()
    with torch.no_grad():
        out = m(torch.tensor(g["x"], device=gpu))
    torch.cuda.synchronize()
    assert rel_err(out.cpu().numpy(), g["out_f64"]) <= 1e-4


def test_g4_aptinit(gpu):
    from gwn_amd.model import gwnet
    g = load_golden("g4_aptinit_n16.npz")
    sups = [torch.tensor(g["sup0"], device=gpu), torch.tensor(g["sup1"], device=gpu)]
    m = gwnet(gpu, 16, 0.3, supports=sups, aptinit=sups[0], residual_channels=16, dilation_channels=16,
              skip_channels=128, end_channels=256)
    e = (m.nodevec1 @ m.nodevec2).detach().cpu().numpy()
    assert rel_err(e, g["e1e2"]) <= 1e-5
    m.load_state_dict({k: torch.tensor(v) for k, v in state_dict_of(g).items()})
    m.eval()
    with torch.no_grad():
        out = m(torch.tensor(g["x"], device=gpu))
    assert rel_err(out.cpu().numpy(), g["out_f32"]) <= 1e-4


def test_g7_data_parallel_shards(gpu):
    """Per-replica BN: the DDP gradient = mean over shards of each shard's gradient."""
    from gwn_amd import util
    g = load_golden("g7_ddp_n16.npz")
    kw = dict(residual_channels=16, dilation_channels=16, skip_channels=128, end_channels=256)
    acc = {}
    for r in range(2):
        m = _model(g, gpu, 16, **kw)
        m.train()
        x = torch.nn.functional.pad(torch.tensor(g["x"][2 * r:2 * r + 2], device=gpu), (1, 0, 0, 0))
        out = m(x)
        real = torch.tensor(g["y"][2 * r:2 * r + 2], device=gpu).unsqueeze(1)
        util.masked_mae(out.transpose(1, 3) * 19.5 + 54.4, real, 0.0).backward()
        for n, p in m.named_parameters():
            if p.grad is not None:
                acc[n] = acc.get(n, 0) + 0.5 * p.grad.double().cpu().numpy()
    for k, v in g.items():
        if k.startswith("gradmean_f64/"):
            name = k[len("gradmean_f64/"):]
            if not name.endswith("mlp.bias") and np.linalg.norm(v) > 0:
                assert norm_rel(acc[name], v) <= 1e-4, name


# ------------------------------------------------------------------------------------------------
def _mix32(h):
    M = np.uint32
    h = h ^ (h >> M(16))
    h = h * M(0x7FEB352D)
    h = h ^ (h >> M(15))
    h = h * M(0x846CA68B)
    return h ^ (h >> M(16))


def _np_uniform(seed, salt, idx):
    """numpy restatement of gwn_uniform (csrc/gwn_internal.h) to rebuild libgwn's dropout masks."""
    with np.errstate(over="ignore"):
        M = np.uint32
        seed = int(seed) & ((1 << 64) - 1)
        key = _mix32(np.array(seed & 0xFFFFFFFF, dtype=M)
                     ^ _mix32(np.array(seed >> 32, dtype=M) + M(0x9E3779B9) * M((int(salt) + 1) & 0xFFFFFFFF)))
        h = _mix32(idx.astype(np.uint64).astype(M) * M(0x9E3779B1) + key)
    return (h >> M(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def test_dropout_forward_backward_exact_masks(gpu):
    """Train mode with dropout 0.3: libgwn's counter-based masks, rebuilt on the host, fed to the
    fp64 oracle -> same output and gradients."""
    from gwn_amd import util
    from oracle import gwnet_oracle as orc
    g = load_golden("g7_ddp_n16.npz")
    kw = dict(residual_channels=16, dilation_channels=16, skip_channels=128, end_channels=256)
    m = _model(g, gpu, 16, dropout=0.3, **kw)
    m.train()
    xin = torch.tensor(g["x"], device=gpu)
    x = torch.nn.functional.pad(xin, (1, 0, 0, 0))
    out = m(x)
    real = torch.tensor(g["y"], device=gpu).unsqueeze(1)
    loss = util.masked_mae(out.transpose(1, 3) * 19.5 + 54.4, real, 0.0)
    loss.backward()
    seed = int(m._executor.seed.item()) - 1  # the forward drew from the counter, then advanced it
    cfg = orc.Cfg(16, nhid=16, skip=128, end=256, dropout=0.3)
    B, N, C = 4, 16, 16
    ts = [13]
    for d in cfg.dilations:
        ts.append(ts[-1] - d)
    masks = []
    for i in range(cfg.L):
        T = ts[i + 1]
        t, b, nn_, c = np.meshgrid(np.arange(T), np.arange(B), np.arange(N), np.arange(C), indexing="ij")
        idx = (((t * B + b) * N + nn_) * C + c).astype(np.uint64)
        keep = (_np_uniform(seed, i, idx) >= np.float32(0.3)).astype(np.float64)  # [T][B][N][C]
        masks.append(torch.tensor(keep.transpose(1, 3, 2, 0)))  # -> [B][C][N][T]
    sd = state_dict_of(g)
    p = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in sd.items()
         if "running" not in k and "num_batches" not in k}
    bn = {k: torch.tensor(v, dtype=torch.float64) for k, v in sd.items() if "running" in k}
    sups = [torch.tensor(g["sup0"], dtype=torch.float64), torch.tensor(g["sup1"], dtype=torch.float64)]
    xpad = torch.nn.functional.pad(torch.tensor(g["x"], dtype=torch.float64), (1, 0, 0, 0))
    ref = orc.forward(p, sups, xpad, cfg, True, bn, dropout_masks=masks)
    kept = sum(float(mk.mean()) for mk in masks) / len(masks)
    assert 0.65 < kept < 0.75
    torch.cuda.synchronize()
    assert rel_err(out.detach().cpu().numpy(), ref.detach().numpy()) <= 1e-4
    rl = orc.masked_metrics(ref.transpose(1, 3) * 19.5 + 54.4, torch.tensor(g["y"], dtype=torch.float64).unsqueeze(1))[0]
    names = list(p)
    gs = torch.autograd.grad(rl, [p[n] for n in names], allow_unused=True)
    refg = {n: gi.numpy() for n, gi in zip(names, gs) if gi is not None}
    _check_grads(m, refg, "dropout", dropout=True)


def test_full_size_forward_and_batch_independence(gpu):
    """METR-LA bench shape B=64: eval forward vs the fp64 oracle, and rows of a B=64 batch equal
    the same samples run at B=4 (eval mode is per-sample)."""
    from gwn_amd import synthetic
    from oracle import gwnet_oracle as orc
    g = load_golden("g12_metr_n207.npz")
    m = _model(g, gpu, 207, dropout=0.3)
    m.eval()
    x, _ = synthetic.synthetic_batch(64, 207, 12, seed=11)
    with torch.no_grad():
        out = m(torch.tensor(x, device=gpu)).cpu().numpy()
        out4 = m(torch.tensor(x[8:12], device=gpu)).cpu().numpy()
    sd = state_dict_of(g)
    p = {k: torch.tensor(v, dtype=torch.float64) for k, v in sd.items()}
    ref = orc.forward(p, [torch.tensor(g["sup0"], dtype=torch.float64), torch.tensor(g["sup1"], dtype=torch.float64)],
                      torch.tensor(x, dtype=torch.float64), orc.Cfg(207), False, p).numpy()
    assert rel_err(out, ref) <= 1e-4
    assert rel_err(out4, out[8:12]) <= 1e-5


def test_trainer_step_is_deterministic(gpu):
    from gwn_amd import synthetic, util
    from gwn_amd.engine import trainer
    adj = synthetic.random_sensor_graph(207, seed=0)
    sups = [torch.tensor(a, device=gpu) for a in synthetic.double_transition(adj)]
    x, y = synthetic.synthetic_batch(16, 207, 12, seed=3)
    res = []
    for _ in range(2):
        torch.manual_seed(999)
        eng = trainer(util.StandardScaler(54.4, 19.5), 2, 12, 207, 32, 0.3, 1e-3, 1e-4, gpu, sups, True, True,
                      None, 4, 2)
        eng.model._executor = None
        ex = eng.model.executor()
        ex.seed.fill_(1234)
        mets = [eng.train(torch.tensor(x, device=gpu), torch.tensor(y, device=gpu)) for _ in range(2)]
        res.append((mets, eng.model._flat.clone()))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1])


@pytest.mark.parametrize("dropout", [0.0, 0.3])
def test_fused_layer_backward_matches_unfused(gpu, monkeypatch, dropout):
    """The fused layer backward (BN backward in the gcn_bwd prologue, gate backward in its
    epilogue, BN statistics in the TCN input-gradient epilogue) against the separate-kernel
    schedule (GWN_FUSE_BWD=0) on the same inputs and dropout masks: only the summation order of
    the BN statistics differs (norm-rel <= 2e-5: the order difference of 7 layers' statistics
    reaches start_conv at ~1.0e-5)."""
    from gwn_amd import synthetic, util
    from gwn_amd.engine import trainer
    adj = synthetic.random_sensor_graph(207, seed=0)
    sups = [torch.tensor(a, device=gpu) for a in synthetic.double_transition(adj)]
    x, y = synthetic.synthetic_batch(8, 207, 12, seed=4)
    grads = []
    for fuse in ("1", "0"):
        monkeypatch.setenv("GWN_FUSE_BWD", fuse)
        monkeypatch.setenv("GWN_GRAPHS", "0")
        torch.manual_seed(999)
        eng = trainer(util.StandardScaler(54.4, 19.5), 2, 12, 207, 32, dropout, 0.0, 0.0, gpu, sups, True, True,
                      None, 4, 2)
        eng.clip = None
        eng.model.executor().seed.fill_(77)
        eng.train(torch.tensor(x, device=gpu), torch.tensor(y, device=gpu))
        torch.cuda.synchronize()
        grads.append({n: p.grad.detach().clone() for n, p in eng.model.named_parameters() if p.grad is not None})
    assert set(grads[0]) == set(grads[1])
    scale = max(float(v.abs().max()) for v in grads[1].values())
    for k in grads[0]:
        a, b = grads[0][k].double(), grads[1][k].double()
        if _bn_cancelled(k) and dropout == 0.0:
            assert float((a - b).abs().max()) <= 1e-5 * scale, k
        elif b.norm() > 0:
            assert float((a - b).norm() / b.norm()) <= 2e-5, k
        else:
            assert float(a.abs().max()) <= 1e-6, k


def test_power_schedule_matches_chained_hops(gpu, monkeypatch):
    """A training step on the power schedule of the fused gcn kernels (GWN_GCN_POW=1, the default:
    x2 = (A^2)^T x, backward W^T after the diffusions) against the chained hops (GWN_GCN_POW=0:
    x2 = A^T (A^T x), the reference's order) on the same inputs and dropout masks: loss and every
    gradient agree to fp32 rounding (the two differ only by reassociation)."""
    from gwn_amd import synthetic, util
    from gwn_amd.engine import trainer
    adj = synthetic.random_sensor_graph(207, seed=0)
    sups = [torch.tensor(a, device=gpu) for a in synthetic.double_transition(adj)]
    x, y = synthetic.synthetic_batch(8, 207, 12, seed=5)
    grads, losses = [], []
    for pw in ("1", "0"):
        monkeypatch.setenv("GWN_GCN_POW", pw)
        monkeypatch.setenv("GWN_GRAPHS", "0")
        torch.manual_seed(999)
        eng = trainer(util.StandardScaler(54.4, 19.5), 2, 12, 207, 32, 0.3, 0.0, 0.0, gpu, sups, True, True,
                      None, 4, 2)
        eng.clip = None
        eng.model.executor().seed.fill_(78)
        losses.append(eng.train(torch.tensor(x, device=gpu), torch.tensor(y, device=gpu))[0])
        torch.cuda.synchronize()
        grads.append({n: p.grad.detach().clone() for n, p in eng.model.named_parameters() if p.grad is not None})
    assert abs(losses[0] - losses[1]) <= 1e-5 * abs(losses[1])
    assert set(grads[0]) == set(grads[1])
    scale = max(float(v.abs().max()) for v in grads[1].values())
    for k in grads[0]:
        a, b = grads[0][k].double(), grads[1][k].double()
        if b.norm() > 1e-3 * scale:
            assert float((a - b).norm() / b.norm()) <= 2e-5, k
        else:
            assert float((a - b).abs().max()) <= 1e-5 * scale, k


def test_num_batches_tracked_counts_train_forwards(gpu):
    """BatchNorm2d.num_batches_tracked is advanced on the device by the BatchNorm finalise
    (gwn_batchnorm_fwd_fold / _partials / the eval-free paths), once per train-mode
    forward as torch does: three trainer.train steps (the first eager, then HIP-graph replays), one
    autograd train-mode forward, eval forwards (no change), and gwnet_diff_G called without
    supports (the residual-only schedule, model.py:391-398)."""
    from gwn_amd import synthetic, util
    from gwn_amd.engine import trainer
    from gwn_amd.model import gwnet_diff_G
    n = 37
    adj = synthetic.random_sensor_graph(n, density=0.2, seed=5)
    sups = [torch.tensor(a, device=gpu) for a in synthetic.double_transition(adj)]
    x, y = synthetic.synthetic_batch(4, n, 12, seed=9)
    torch.manual_seed(3)
    eng = trainer(util.StandardScaler(54.4, 19.5), 2, 12, n, 32, 0.3, 1e-3, 1e-4, gpu, sups, True, True, None, 4, 2)
    bns = [eng.model.bn[i] for i in range(len(eng.model.bn))]
    assert all(int(b.num_batches_tracked) == 0 for b in bns)
    for step in range(3):
        eng.train(torch.tensor(x, device=gpu), torch.tensor(y, device=gpu))
        torch.cuda.synchronize()
        assert [int(b.num_batches_tracked) for b in bns] == [step + 1] * len(bns), step
    m = eng.model
    m.train()
    out = m(torch.nn.functional.pad(torch.tensor(x, device=gpu), (1, 0, 0, 0)))
    out.sum().backward()
    torch.cuda.synchronize()
    assert [int(b.num_batches_tracked) for b in bns] == [4] * len(bns)
    m.eval()
    with torch.no_grad():
        m(torch.tensor(x, device=gpu))
        eng.eval(torch.tensor(x, device=gpu), torch.tensor(y, device=gpu))
    torch.cuda.synchronize()
    assert [int(b.num_batches_tracked) for b in bns] == [4] * len(bns)
    dg = gwnet_diff_G(gpu, 16, 0.0, supports_len=2, gcn_bool=True, addaptadj=False, residual_channels=16,
                      dilation_channels=16, skip_channels=64, end_channels=128, blocks=2, layers=2)
    dg.train()
    xd = torch.randn(2, 2, 16, 31, device=gpu)  # (dilations 4, 8 per block: T >= 25)
    for k in range(2):
        dg(xd, None, None).sum().backward()
    torch.cuda.synchronize()
    assert [int(b.num_batches_tracked) for b in dg.bn] == [2] * len(dg.bn)


def test_sync_check_debug_mode(gpu):
    """GWN_SYNC_CHECK (the debugging aid, gwn_set_sync_check): every launch synchronised and every
    operand / workspace range checked against its device allocation.  A train-mode forward +
    backward runs clean under it and gives the same bits as without it."""
    from gwn_amd import _lib, synthetic, util
    from gwn_amd.model import gwnet
    n = 40
    sups = synthetic.double_transition(synthetic.random_sensor_graph(n, density=0.2, seed=3))
    x, y = synthetic.synthetic_batch(2, n, 12, seed=5)

    def run():
        torch.manual_seed(999)
        m = gwnet(gpu, n, 0.0, supports=[torch.tensor(a, device=gpu) for a in sups])
        m.train()
        out = m(torch.nn.functional.pad(torch.tensor(x, device=gpu), (1, 0, 0, 0)))
        loss = util.masked_mae(out.transpose(1, 3) * 19.5 + 54.4, torch.tensor(y, device=gpu).unsqueeze(1), 0.0)
        loss.backward()
        torch.cuda.synchronize()
        return out.detach().cpu(), {k: p.grad.detach().cpu() for k, p in m.named_parameters() if p.grad is not None}

    ref_out, ref_g = run()
    lib = _lib.load()
    lib.gwn_set_sync_check(1)
    try:
        out, g = run()
    finally:
        lib.gwn_set_sync_check(0)
    assert torch.equal(out, ref_out)
    assert set(g) == set(ref_g)
    for k in g:
        assert torch.equal(g[k], ref_g[k]), k
