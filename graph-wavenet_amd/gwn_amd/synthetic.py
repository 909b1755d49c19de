"""Seeded synthetic inputs in the METR-LA tensor format.

The real METR-LA / PEMS-BAY files are not available offline, so every test, fixture and
benchmark uses tensors of the exact shapes the reference's loaders produce:

* ``x``        [B, 2, N, T]  (after ``transpose(1, 3)`` in ``train.py:244-245``): channel 0 is the
  standardised speed (``util.py:208-211``), channel 1 the time of day in [0, 1)
  (``generate_training_data.py:36-39``).
* ``real_val`` [B, N, T]  speed labels (``train.py:246-251``), with ~5 % exact zeros that the
  masked metrics treat as missing (``util.py:527-538``).
* ``supports`` ``[D^-1 A, D^-1 A^T]`` of a sparse random sensor graph (``util.py:130-136``,
  ``util.py:187-188``).

Only numpy is used so that the generator is deterministic across machines (PCG64).
"""
import numpy as np

SCALER_MEAN = 54.4
SCALER_STD = 19.5


def random_sensor_graph(num_nodes, density=0.04, seed=0, dense=False):
    """A METR-LA-like weighted adjacency: ~4 % off-diagonal U(0,1) weights plus self loops
    (METR-LA's ``adj_mx`` has a unit diagonal).  ``dense=True`` gives the dense U(0,1)
    graph of the N=2048 stress config."""
    rng = np.random.default_rng(seed)
    if dense:
        adj = rng.random((num_nodes, num_nodes), dtype=np.float64)
    else:
        adj = rng.random((num_nodes, num_nodes)) * (rng.random((num_nodes, num_nodes)) < density)
    np.fill_diagonal(adj, 1.0)
    return adj.astype(np.float32)


def asym_adj(adj):
    """Row-normalised transition matrix D^-1 A (``util.py:130-136``): rows with zero degree stay 0."""
    adj = np.asarray(adj, dtype=np.float64)
    rowsum = adj.sum(1)
    with np.errstate(divide="ignore"):
        d_inv = np.power(rowsum, -1.0)
    d_inv[np.isinf(d_inv)] = 0.0
    return (d_inv[:, None] * adj).astype(np.float32)


def double_transition(adj):
    """``mod_adj(adj, 'doubletransition')`` (``util.py:187-188``)."""
    return [asym_adj(adj), asym_adj(np.transpose(adj))]


def synthetic_batch(batch, num_nodes, seq_len=12, seed=0, zero_frac=0.05):
    """One mini-batch ``(x [B,2,N,T], real_val [B,N,T])`` as float32 numpy arrays."""
    rng = np.random.default_rng(seed)
    x = np.empty((batch, 2, num_nodes, seq_len), dtype=np.float32)
    x[:, 0] = rng.standard_normal((batch, num_nodes, seq_len))
    t0 = rng.integers(0, 288, size=batch)
    tod = ((t0[:, None] + np.arange(seq_len)[None, :]) % 288) / 288.0
    x[:, 1] = tod[:, None, :]
    y = np.clip(SCALER_MEAN + SCALER_STD * rng.standard_normal((batch, num_nodes, seq_len)), 0.0, 80.0)
    y[rng.random(y.shape) < zero_frac] = 0.0
    return x, y.astype(np.float32)
