"""Evaluation / test path on libgwn (reference train.py:377-404, test.py:58-87).

* ``predict(model, loader, n_real)`` -- the eval forward over every batch of a loader under
  ``torch.no_grad()``, outputs transposed / squeezed / concatenated exactly as train.py:382-390
  and trimmed to the real sample count.  A gwn_amd model runs its lean inference schedule there
  (``Executor.infer``: nothing kept for a backward, eval BatchNorm folded into the fused GCN).
  Works with the host ``util.DataLoader`` (numpy batches, copied like train.py:383-384) and with
  ``data.DeviceDataLoader`` / ``data.SeriesDataLoader`` (batches already in HBM).
* ``horizon_metrics(yhat, realy, scaler)`` -- ``util.metric(scaler.inverse_transform(yhat[:, :, i]),
  realy[:, :, i])`` for every horizon i (train.py:392-400) in two libgwn launches and ONE
  device->host copy, where the reference issues 12 x 3 masked-metric reductions and 36 ``.item()``
  syncs; returns an [H, 3] array (mae, mape, rmse).
* ``evaluate(model, loader, realy, scaler)`` -- both, printing the reference's log lines.
"""
import numpy as np
import torch

from . import _lib
from ._lib import ptr


def _device_of(model):
    return next(model.parameters()).device


def _as_device(x, device):
    if isinstance(x, torch.Tensor) and x.is_cuda:
        return x
    return torch.Tensor(x).to(device)  # train.py:383 (float64 numpy -> fp32)


def predict(model, loader, n_real=None):
    """train.py:378-390: yhat [S, N, H] on the device."""
    device = _device_of(model)
    outputs = []
    model.eval()
    with torch.no_grad():
        for x, _ in loader.get_iterator():
            testx = _as_device(x, device).transpose(1, 3)
            preds = model(testx).transpose(1, 3)
            outputs.append(preds.squeeze())
    yhat = torch.cat(outputs, dim=0)
    if n_real is not None:
        yhat = yhat[:n_real, ...]
    return yhat


def horizon_metrics(yhat, realy, scaler):
    """Masked (mae, mape, rmse) per horizon of yhat, realy [S, N, H] (any strides, fp32, on the
    GPU); pred = scaler.inverse_transform(yhat)."""
    if yhat.dim() != 3 or tuple(yhat.shape) != tuple(realy.shape):
        raise RuntimeError("horizon_metrics: yhat and realy must both be [S, N, H], got %s and %s"
                           % (tuple(yhat.shape), tuple(realy.shape)))
    if not (yhat.is_cuda and realy.is_cuda and yhat.dtype == torch.float32 and realy.dtype == torch.float32):
        raise RuntimeError("horizon_metrics: float32 GPU tensors required (there is no CPU fallback)")
    S, N, H = yhat.shape
    lib = _lib.load()
    ws = torch.empty(lib.gwn_horizon_metrics_workspace_floats(H), device=yhat.device, dtype=torch.float32)
    out = torch.empty(3 * H, device=yhat.device, dtype=torch.float32)
    ps, rs = yhat.stride(), realy.stride()
    _lib.call("gwn_horizon_metrics", ptr(yhat), ps[0], ps[2], ps[1], ptr(realy), rs[0], rs[2], rs[1], S, H, N,
              float(scaler.mean), float(scaler.std), ptr(out), ptr(ws), _lib.stream())
    return out.view(H, 3).cpu().numpy().astype(np.float64)


def evaluate(model, loader, realy, scaler, log=print, horizons=None):
    """train.py:377-404: per-horizon and average test metrics; returns (amae, amape, armse)."""
    yhat = predict(model, loader, n_real=realy.size(0))
    m = horizon_metrics(yhat, realy, scaler)
    H = m.shape[0] if horizons is None else horizons
    amae, amape, armse = [], [], []
    for i in range(H):
        if log is not None:
            log('Evaluate best model on test data for horizon {:d}, Test MAE: {:.4f}, Test MAPE: {:.4f}, '
                'Test RMSE: {:.4f}'.format(i + 1, m[i, 0], m[i, 1], m[i, 2]))
        amae.append(float(m[i, 0]))
        amape.append(float(m[i, 1]))
        armse.append(float(m[i, 2]))
    if log is not None:
        log('On average over seq_length horizons, Test MAE: {:.4f}, Test MAPE: {:.4f}, Test RMSE: {:.4f}'.format(
            np.mean(amae), np.mean(amape), np.mean(armse)))
    return amae, amape, armse


__all__ = ["predict", "horizon_metrics", "evaluate"]
