"""Golden vectors for the data-ingestion and evaluation rows, produced
by the REFERENCE's own functions, imported from /root/reference in the build container only
(same harness-side shims as make_golden.py).  Only numeric outputs are written (g8_data.npz):

* generate_training_data.generate_graph_seq2seq_io_data on a small timestamped DataFrame, with
  and without day-of-week, and generate_train_val_test's split (its ``pd.read_hdf`` is pointed at
  the in-memory frame; the npz files go to a temporary directory);
* Utils.util.DataLoader: the batches after ``np.random.seed(11); shuffle()`` with padding;
* Utils.util.metric per horizon on predictions with exact-zero labels (train.py:392-400).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_data.py
"""
import argparse
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import REF, _install_shims  # noqa: E402


def frame(T=400, N=5, seed=7):
    import pandas as pd
    rng = np.random.default_rng(seed)
    idx = pd.date_range("2012-03-01 00:00:00", periods=T, freq="5min")
    vals = np.clip(55.0 + 12.0 * rng.standard_normal((T, N)), 0.0, 80.0)
    vals[rng.random((T, N)) < 0.05] = 0.0
    return pd.DataFrame(vals, index=idx, columns=["s%d" % i for i in range(N)])


def main():
    _install_shims()
    import pandas as pd
    import torch
    import generate_training_data as gtd  # noqa: E402  (the reference module)
    from Utils import util  # noqa: E402
    for mod in (gtd, util):
        assert os.path.abspath(mod.__file__).startswith(REF + "/"), mod.__file__

    g = {}
    df = frame()
    g["df_values"] = df.values
    g["df_index_ns"] = df.index.values.astype("datetime64[ns]").astype(np.int64)
    xo = np.sort(np.concatenate((np.arange(-11, 1, 1),)))
    yo = np.sort(np.arange(1, 13, 1))
    x, y = gtd.generate_graph_seq2seq_io_data(df, x_offsets=xo, y_offsets=yo, add_time_in_day=True,
                                              add_day_in_week=False)
    g["seq_x"], g["seq_y"] = x, y
    xd, yd = gtd.generate_graph_seq2seq_io_data(df, x_offsets=xo, y_offsets=yo, add_time_in_day=True,
                                                add_day_in_week=True)
    g["seq_x_dow"], g["seq_y_dow"] = xd, yd

    # generate_train_val_test through the reference's own function
    with tempfile.TemporaryDirectory() as tmp:
        orig = pd.read_hdf
        pd.read_hdf = lambda *a, **k: df
        try:
            args = argparse.Namespace(output_dir=tmp, traffic_df_filename="in-memory", seq_length_x=12,
                                      seq_length_y=12, y_start=1, dow=False)
            gtd.generate_train_val_test(args)
        finally:
            pd.read_hdf = orig
        for cat in ("train", "val", "test"):
            d = np.load(os.path.join(tmp, cat + ".npz"))
            g["split_%s_x" % cat] = d["x"]
            g["split_%s_y" % cat] = d["y"]
            g["split_%s_x_offsets" % cat] = d["x_offsets"]

    # DataLoader: padding + shuffle order
    xs, ys = x[:23], y[:23]
    np.random.seed(11)
    dl = util.DataLoader(xs, ys, 5)
    dl.shuffle()
    bx, by = [], []
    for bxi, byi in dl.get_iterator():
        bx.append(bxi)
        by.append(byi)
    g["dl_x"], g["dl_y"] = np.stack(bx), np.stack(by)

    # per-horizon masked metrics (train.py:392-400)
    rng = np.random.default_rng(3)
    S, N, H = 37, 11, 12
    yhat = rng.standard_normal((S, N, H)).astype(np.float32)
    real = np.clip(54.4 + 19.5 * rng.standard_normal((S, N, H)), 0.0, 80.0).astype(np.float32)
    real[rng.random(real.shape) < 0.07] = 0.0
    real[:, :, 5] = 0.0  # a horizon without labels
    scaler = util.StandardScaler(54.4, 19.5)
    mets = []
    for i in range(H):
        pred = scaler.inverse_transform(torch.tensor(yhat)[:, :, i])
        mets.append(util.metric(pred, torch.tensor(real)[:, :, i]))
    g["hm_yhat"], g["hm_real"], g["hm_metrics"] = yhat, real, np.asarray(mets, dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "g8_data.npz"), **g)
    print("wrote g8_data.npz", {k: v.shape for k, v in g.items()})


if __name__ == "__main__":
    main()
