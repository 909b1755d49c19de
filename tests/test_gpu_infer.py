"""Inference path and HBM-resident data ingestion on the GPU:
lean eval forward vs the full eval forward and the fp64 reference, per-horizon metrics vs the
reference's util.metric, device loaders vs the reference's loader order."""
import numpy as np
import pandas as pd
import pytest
import torch

from conftest import load_golden, rel_err, state_dict_of

pytestmark = pytest.mark.gpu


def _model(g, gpu, n=207, dropout=0.3):
    from gwn_amd.model import gwnet
    sups = [torch.tensor(g["sup0"], device=gpu), torch.tensor(g["sup1"], device=gpu)]
    m = gwnet(gpu, n, dropout, supports=sups)
    m.load_state_dict({k: torch.tensor(v) for k, v in state_dict_of(g).items()})
    return m


def test_lean_eval_forward_matches_reference_and_full_path(gpu, monkeypatch):
    g = load_golden("g12_metr_n207.npz")
    m = _model(g, gpu)
    m.eval()
    x = torch.tensor(g["g1_x"], device=gpu)
    with torch.no_grad():
        lean = m(x)
    assert m.executor().infer_ok()
    monkeypatch.setenv("GWN_LEAN_EVAL", "0")
    with torch.no_grad():
        full = m(x)
    torch.cuda.synchronize()
    assert rel_err(lean.cpu().numpy(), g["g1_out_f64"]) <= 1e-4
    assert rel_err(lean.cpu().numpy(), full.cpu().numpy()) <= 1e-6


def test_trainer_eval_lean_matches_full(gpu, monkeypatch):
    from gwn_amd import synthetic, util
    from gwn_amd.engine import trainer
    adj = synthetic.random_sensor_graph(207, seed=0)
    sups = [torch.tensor(a, device=gpu) for a in synthetic.double_transition(adj)]
    x, y = synthetic.synthetic_batch(16, 207, 12, seed=9)
    xd, yd = torch.tensor(x, device=gpu), torch.tensor(y, device=gpu)
    torch.manual_seed(999)
    eng = trainer(util.StandardScaler(54.4, 19.5), 2, 12, 207, 32, 0.3, 1e-3, 1e-4, gpu, sups, True, True, None, 4, 2)
    eng.train(xd, yd)  # running statistics move away from (0, 1)
    lean = eng.eval(xd, yd)
    monkeypatch.setenv("GWN_LEAN_EVAL", "0")
    full = eng.eval(xd, yd)
    np.testing.assert_allclose(lean, full, rtol=1e-5)


def test_horizon_metrics_match_reference(gpu):
    from gwn_amd import infer, util
    g = load_golden("g8_data.npz")
    yhat = torch.tensor(g["hm_yhat"], device=gpu)
    real = torch.tensor(g["hm_real"], device=gpu)
    m = infer.horizon_metrics(yhat, real, util.StandardScaler(54.4, 19.5))
    ref = g["hm_metrics"]
    assert np.all(m[5] == 0.0) and np.all(ref[5] == 0.0)  # a horizon without labels
    np.testing.assert_allclose(m, ref, rtol=2e-5, atol=1e-6)
    # strided views (the transposes train.py builds) give the same numbers
    yt = yhat.transpose(1, 2).contiguous().transpose(1, 2)
    np.testing.assert_allclose(infer.horizon_metrics(yt, real, util.StandardScaler(54.4, 19.5)), m, rtol=1e-6)


def test_device_loader_matches_host_loader(gpu):
    from gwn_amd import data, util
    g = load_golden("g8_data.npz")
    xs, ys = g["seq_x"][:203], g["seq_y"][:203]
    np.random.seed(21)
    host = util.DataLoader(xs, ys, 16)
    host.shuffle()
    np.random.seed(21)
    dev = data.DeviceDataLoader(xs, ys, 16, gpu)
    dev.shuffle()
    nb = 0
    for (hx, hy), (dx, dy) in zip(host.get_iterator(), dev.get_iterator()):
        assert torch.equal(dx.cpu(), torch.Tensor(hx)) and torch.equal(dy.cpu(), torch.Tensor(hy))
        nb += 1
    assert nb == host.num_batch == dev.num_batch


def test_series_loader_matches_materialised_pipeline(gpu, tmp_path):
    """load_dataset_series (raw readings in HBM, windows cut per batch) == generate_train_val_test
    + load_dataset_device (windowed arrays) batch for batch, including the scaler."""
    from gwn_amd import data
    g = load_golden("g8_data.npz")
    df = pd.DataFrame(g["df_values"], index=pd.to_datetime(g["df_index_ns"]))
    data.generate_train_val_test(df, str(tmp_path))
    arrays = data.load_dataset_device(str(tmp_path), 8, 8, 8, gpu)
    series = data.load_dataset_series(df, 8, 8, 8, gpu)
    assert arrays["scaler"].mean == series["scaler"].mean and arrays["scaler"].std == series["scaler"].std
    for cat in ("train", "val", "test"):
        np.random.seed(4)
        arrays[cat + "_loader"].shuffle()
        np.random.seed(4)
        series[cat + "_loader"].shuffle()
        for (ax, ay), (sx, sy) in zip(arrays[cat + "_loader"].get_iterator(), series[cat + "_loader"].get_iterator()):
            assert torch.equal(ax, sx), cat
            assert torch.equal(ay, sy), cat


def test_evaluate_test_split_matches_reference_loop(gpu):
    """infer.evaluate (lean forward, device loader, on-device horizon metrics) against the
    reference's own loop of train.py:378-400 run on the same model (host loader, torch.Tensor
    copies, util.metric per horizon)."""
    from gwn_amd import data, infer, synthetic, util
    from gwn_amd.model import gwnet
    N, S = 207, 150
    adj = synthetic.random_sensor_graph(N, seed=1)
    sups = [torch.tensor(a, device=gpu) for a in synthetic.double_transition(adj)]
    torch.manual_seed(0)
    m = gwnet(gpu, N, 0.3, supports=sups)
    rng = np.random.default_rng(0)
    xs = np.zeros((S, 12, N, 2))
    xs[..., 0] = rng.standard_normal((S, 12, N))
    xs[..., 1] = (np.arange(12)[None, :, None] % 288) / 288.0
    ys = np.clip(54.4 + 19.5 * rng.standard_normal((S, 12, N, 2)), 0, 80)
    ys[rng.random(ys.shape) < 0.05] = 0.0
    scaler = util.StandardScaler(54.4, 19.5)
    realy = torch.Tensor(ys).to(gpu).transpose(1, 3)[:, 0, :, :]
    # reference loop
    m.eval()
    outs = []
    with torch.no_grad():
        for x, _ in util.DataLoader(xs, ys, 64).get_iterator():
            outs.append(m(torch.Tensor(x).to(gpu).transpose(1, 3)).transpose(1, 3).squeeze())
    yhat = torch.cat(outs, dim=0)[:S]
    ref = np.array([util.metric(scaler.inverse_transform(yhat[:, :, i]), realy[:, :, i]) for i in range(12)])
    amae, amape, armse = infer.evaluate(m, data.DeviceDataLoader(xs, ys, 64, gpu), realy, scaler, log=None)
    np.testing.assert_allclose(np.stack([amae, amape, armse], 1), ref, rtol=2e-5)
