"""Data ingestion on the host: the npz generation and the loader order
against the reference's own outputs (tests/golden/g8_data.npz, made by make_golden_data.py)."""
import numpy as np
import pandas as pd

from conftest import load_golden


def _frame(g):
    idx = pd.to_datetime(g["df_index_ns"])
    return pd.DataFrame(g["df_values"], index=idx)


def test_seq2seq_windows_match_reference():
    from gwn_amd import data
    g = load_golden("g8_data.npz")
    df = _frame(g)
    xo, yo = data.offsets(12, 12, 1)
    x, y = data.generate_graph_seq2seq_io_data(df, xo, yo, add_time_in_day=True, add_day_in_week=False)
    assert x.dtype == g["seq_x"].dtype and x.shape == g["seq_x"].shape
    np.testing.assert_array_equal(x, g["seq_x"])
    np.testing.assert_array_equal(y, g["seq_y"])
    x, y = data.generate_graph_seq2seq_io_data(df, xo, yo, add_time_in_day=True, add_day_in_week=True)
    np.testing.assert_array_equal(x, g["seq_x_dow"])
    np.testing.assert_array_equal(y, g["seq_y_dow"])


def test_train_val_test_npz_match_reference(tmp_path):
    from gwn_amd import data
    g = load_golden("g8_data.npz")
    data.generate_train_val_test(_frame(g), str(tmp_path))
    for cat in ("train", "val", "test"):
        d = np.load(tmp_path / (cat + ".npz"))
        np.testing.assert_array_equal(d["x"], g["split_%s_x" % cat])
        np.testing.assert_array_equal(d["y"], g["split_%s_y" % cat])
        np.testing.assert_array_equal(d["x_offsets"], g["split_%s_x_offsets" % cat])


def test_split_sizes_and_window_edges():
    from gwn_amd import data
    assert data.split_sizes(377) == (264, 38, 75)
    assert data.split_sizes(34249) == (23974, 3425, 6850)  # METR-LA's published split
    xo, yo = data.offsets()
    assert data.window_range(400, xo, yo) == (11, 388)


def test_host_dataloader_shuffle_matches_reference():
    from gwn_amd import util
    g = load_golden("g8_data.npz")
    np.random.seed(11)
    dl = util.DataLoader(g["seq_x"][:23], g["seq_y"][:23], 5)
    dl.shuffle()
    bx = np.stack([b[0] for b in dl.get_iterator()])
    np.testing.assert_array_equal(bx, g["dl_x"])


def test_series_loader_order_matches_array_loader_on_host():
    """The index bookkeeping shared by the device loaders: padding + cumulative permutations
    select the same samples as util.DataLoader's array shuffles (no GPU needed)."""
    from gwn_amd import data, util
    g = load_golden("g8_data.npz")
    xs = g["seq_x"][:23]
    np.random.seed(5)
    ref = util.DataLoader(xs, g["seq_y"][:23], 4)
    ref.shuffle()
    ref.shuffle()
    np.random.seed(5)
    o = data._Order.__new__(data._Order)
    data._Order.__init__(o, 23, 4, "cpu")
    o._upload = lambda: None
    o.shuffle()
    o.shuffle()
    np.testing.assert_array_equal(np.concatenate([xs, xs[-1:]])[o._order], ref.xs)
