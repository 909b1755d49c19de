"""Data ingestion for the METR-LA / PEMS-BAY path, HBM-resident.

Reference: ``generate_training_data.py:12-91`` (sliding windows + 70/10/20 split into npz),
``Utils/util.py:14-54`` (``DataLoader``: pad with the last sample, ``np.random.permutation``
shuffle, contiguous mini-batches) and ``util.py:202-217`` (``load_dataset_metr``: StandardScaler
on channel 0 of x).  The reference keeps the windowed arrays on the host and copies every batch
with ``torch.Tensor(x).to(device)`` plus a transpose (``train.py:244-247``).

Here:
* ``generate_graph_seq2seq_io_data`` / ``generate_train_val_test`` restate the npz generation
  (vectorised; the same arrays bit for bit, pinned by tests/test_data.py against the
  reference's own output);
* ``DeviceDataLoader`` uploads a split once (fp32: exactly ``torch.Tensor(x)``'s rounding) and
  assembles every batch on the GPU with ``gwn_gather_rows`` from a permutation vector drawn by the
  reference's own ``np.random.permutation`` call, so the batch order is the reference's for the
  same numpy seed;
* ``SeriesDataLoader`` keeps only the raw [T, N] readings in HBM (fp64; 12x less memory than the
  windowed arrays) and cuts the windows of each batch with ``gwn_window_batch``; its batches equal
  the ``DeviceDataLoader`` batches of the generated arrays bit for bit.
Batches are device tensors x [B, LX, N, C], y [B, LY, N, C] (the numpy layout of the reference's
loader); ``model_inputs`` turns them into the trainer's (x [B, C, N, LX], real_val [B, N, LY]).
"""
import os

import numpy as np
import torch

from . import _lib
from ._lib import ptr
from .util import StandardScaler


# ---------------------------------------------------------------------------------------------
# generate_training_data.py

def _time_in_day(index):
    idx = np.asarray(index.values if hasattr(index, "values") else index)
    return (idx - idx.astype("datetime64[D]")) / np.timedelta64(1, "D")


def _day_of_week(index):
    if hasattr(index, "dayofweek"):
        return np.asarray(index.dayofweek)
    idx = np.asarray(index).astype("datetime64[D]").astype(np.int64)
    return (idx + 3) % 7  # 1970-01-01 was a Thursday (Monday = 0)


def _features(values, index, add_time_in_day, add_day_in_week):
    values = np.asarray(values)
    num_samples, num_nodes = values.shape
    feats = [values[..., None]]
    if add_time_in_day:
        tod = _time_in_day(index)
        feats.append(np.broadcast_to(tod[:, None, None], (num_samples, num_nodes, 1)))
    if add_day_in_week:
        dow = _day_of_week(index)
        feats.append(np.broadcast_to(dow[:, None, None], (num_samples, num_nodes, 1)))
    return np.concatenate(feats, axis=-1)


def window_range(num_samples, x_offsets, y_offsets):
    """[min_t, max_t): the window end indices t of generate_training_data.py:42-44."""
    min_t = abs(min(x_offsets))
    max_t = abs(num_samples - abs(max(y_offsets)))
    return int(min_t), int(max_t)


def generate_graph_seq2seq_io_data(df, x_offsets, y_offsets, add_time_in_day=True, add_day_in_week=False,
                                   scaler=None):
    """generate_training_data.py:12-49.  ``df``: a pandas DataFrame indexed by timestamps (rows =
    time, columns = sensors).  Returns x (S, len(x_offsets), N, C), y (S, len(y_offsets), N, C)."""
    data = _features(df.values, df.index, add_time_in_day, add_day_in_week)
    x_offsets = np.asarray(x_offsets).reshape(-1)
    y_offsets = np.asarray(y_offsets).reshape(-1)
    min_t, max_t = window_range(data.shape[0], x_offsets, y_offsets)
    t = np.arange(min_t, max_t)
    x = data[t[:, None] + x_offsets[None, :], ...]
    y = data[t[:, None] + y_offsets[None, :], ...]
    return x, y


def offsets(seq_length_x=12, seq_length_y=12, y_start=1):
    """generate_training_data.py:55-58."""
    x_offsets = np.sort(np.concatenate((np.arange(-(seq_length_x - 1), 1, 1),)))
    y_offsets = np.sort(np.arange(y_start, (seq_length_y + 1), 1))
    return x_offsets, y_offsets


def split_sizes(num_samples):
    """generate_training_data.py:71-74: 70 / 10 / 20 % with Python's round()."""
    num_test = round(num_samples * 0.2)
    num_train = round(num_samples * 0.7)
    return num_train, num_samples - num_test - num_train, num_test


def generate_train_val_test(df, output_dir, seq_length_x=12, seq_length_y=12, y_start=1, dow=False):
    """generate_training_data.py:52-91 for an in-memory DataFrame (the reference reads it with
    ``pd.read_hdf``; PyTables is not part of this image): writes {train,val,test}.npz."""
    x_offsets, y_offsets = offsets(seq_length_x, seq_length_y, y_start)
    x, y = generate_graph_seq2seq_io_data(df, x_offsets, y_offsets, add_time_in_day=True, add_day_in_week=dow)
    num_train, num_val, num_test = split_sizes(x.shape[0])
    parts = {"train": (x[:num_train], y[:num_train]),
             "val": (x[num_train:num_train + num_val], y[num_train:num_train + num_val]),
             "test": (x[-num_test:], y[-num_test:])}
    os.makedirs(output_dir, exist_ok=True)
    for cat, (_x, _y) in parts.items():
        np.savez_compressed(os.path.join(output_dir, "%s.npz" % cat), x=_x, y=_y,
                            x_offsets=x_offsets.reshape(list(x_offsets.shape) + [1]),
                            y_offsets=y_offsets.reshape(list(y_offsets.shape) + [1]))
    return parts


# ---------------------------------------------------------------------------------------------
# HBM-resident loaders

class _Order(object):
    """util.DataLoader's sample order (util.py:23-40): padding with the last sample, then
    cumulative ``np.random.permutation`` shuffles, kept as an index vector (host + device)."""

    def __init__(self, count, batch_size, device, pad_with_last_sample=True):
        if count < 1:
            raise ValueError("DataLoader: empty split")
        self.batch_size = batch_size
        self.current_ind = 0
        num_padding = (batch_size - (count % batch_size)) % batch_size if pad_with_last_sample else 0
        self._order = np.concatenate([np.arange(count, dtype=np.int64),
                                      np.full(num_padding, count - 1, dtype=np.int64)])
        self.size = len(self._order)
        self.num_batch = int(self.size // self.batch_size)
        self.device = torch.device(device)

    def _upload(self):
        self._order_dev = torch.tensor(self._order, dtype=torch.int64, device=self.device)

    def shuffle(self):
        permutation = np.random.permutation(self.size)  # the reference's draw (util.py:37)
        self._order = self._order[permutation]
        self._upload()

    def _batches(self, make):
        self.current_ind = 0

        def _wrapper():
            while self.current_ind < self.num_batch:
                lo = self.batch_size * self.current_ind
                hi = min(self.size, self.batch_size * (self.current_ind + 1))
                yield make(lo, hi)
                self.current_ind += 1

        return _wrapper()


class DeviceDataLoader(_Order):
    """util.DataLoader (util.py:14-54) over arrays uploaded to HBM once; batches are gathered on
    the device (gwn_gather_rows)."""

    def __init__(self, xs, ys, batch_size, device="cuda", pad_with_last_sample=True):
        xs, ys = np.asarray(xs), np.asarray(ys)
        if len(xs) != len(ys):
            raise ValueError("DataLoader: xs and ys differ in length")
        super().__init__(len(xs), batch_size, device, pad_with_last_sample)
        self.xs = torch.tensor(xs, dtype=torch.float32).to(self.device)
        self.ys = torch.tensor(ys, dtype=torch.float32).to(self.device)
        self._row_x = int(np.prod(xs.shape[1:]))
        self._row_y = int(np.prod(ys.shape[1:]))
        self._upload()

    def get_iterator(self):
        st = _lib.stream()

        def make(lo, hi):
            idx = self._order_dev[lo:hi]
            x = torch.empty((hi - lo,) + tuple(self.xs.shape[1:]), device=self.device, dtype=torch.float32)
            y = torch.empty((hi - lo,) + tuple(self.ys.shape[1:]), device=self.device, dtype=torch.float32)
            _lib.call("gwn_gather_rows", ptr(self.xs), self._row_x, ptr(idx), hi - lo, ptr(x), st)
            _lib.call("gwn_gather_rows", ptr(self.ys), self._row_y, ptr(idx), hi - lo, ptr(y), st)
            return x, y

        return self._batches(make)


class SeriesDataLoader(_Order):
    """Sliding-window batches cut on the device from the raw readings [T, N] (gwn_window_batch):
    sample s of the split is the window ending at t_last[s]; x channel 0 is standardised with
    ``scaler`` (fp64, as load_dataset_metr does on the float64 arrays), y is raw."""

    def __init__(self, values, index, t_last, batch_size, device="cuda", x_offsets=None, y_offsets=None,
                 scaler=None, add_time_in_day=True, add_day_in_week=False, pad_with_last_sample=True):
        t_last = np.asarray(t_last, dtype=np.int64)
        super().__init__(len(t_last), batch_size, device, pad_with_last_sample)
        if x_offsets is None or y_offsets is None:
            x_offsets, y_offsets = offsets()
        self.x_offsets = np.asarray(x_offsets, dtype=np.int64).reshape(-1)
        self.y_offsets = np.asarray(y_offsets, dtype=np.int64).reshape(-1)
        values = np.asarray(values, dtype=np.float64)
        T, self.N = values.shape
        if t_last.min() + self.x_offsets.min() < 0 or t_last.max() + self.y_offsets.max() >= T:
            raise ValueError("SeriesDataLoader: a window leaves the series")
        dev = self.device
        self.series = torch.tensor(values, dtype=torch.float64, device=dev)
        self.tod = (torch.tensor(_time_in_day(index), dtype=torch.float64, device=dev)
                    if add_time_in_day else None)
        self.dow = (torch.tensor(_day_of_week(index).astype(np.float64), dtype=torch.float64, device=dev)
                    if add_day_in_week else None)
        self.cin = 1 + int(add_time_in_day) + int(add_day_in_week)
        self._t_last = t_last
        self._xoff = torch.tensor(self.x_offsets, dtype=torch.int32, device=dev)
        self._yoff = torch.tensor(self.y_offsets, dtype=torch.int32, device=dev)
        self.scaler = scaler
        self._upload()

    def _upload(self):
        # the window ends in (shuffled) sample order: one index vector per epoch, no per-batch host work
        self._t_dev = torch.tensor(self._t_last[self._order], dtype=torch.int64, device=self.device)

    def get_iterator(self):
        st = _lib.stream()
        LX, LY = len(self.x_offsets), len(self.y_offsets)
        mean = float(self.scaler.mean) if self.scaler is not None else 0.0
        std = float(self.scaler.std) if self.scaler is not None else 1.0

        def make(lo, hi):
            B = hi - lo
            x = torch.empty((B, LX, self.N, self.cin), device=self.device, dtype=torch.float32)
            y = torch.empty((B, LY, self.N, self.cin), device=self.device, dtype=torch.float32)
            _lib.call("gwn_window_batch", ptr(self.series), ptr(self.tod), ptr(self.dow), self.N,
                      ptr(self._t_dev[lo:hi]), B, ptr(self._xoff), LX, ptr(self._yoff), LY, mean, std,
                      1 if self.scaler is not None else 0, ptr(x), ptr(y), st)
            return x, y

        return self._batches(make)


def model_inputs(x, y):
    """train.py:244-251: (x.transpose(1, 3), y.transpose(1, 3)[:, 0, :, :]) as views."""
    return x.transpose(1, 3), y.transpose(1, 3)[:, 0, :, :]


def load_dataset_device(dataset_dir, batch_size, valid_batch_size=None, test_batch_size=None, device="cuda"):
    """util.load_dataset_metr (util.py:202-217) with HBM-resident loaders."""
    data = {}
    for category in ["train", "val", "test"]:
        cat = np.load(os.path.join(dataset_dir, category + ".npz"))
        data["x_" + category] = cat["x"]
        data["y_" + category] = cat["y"]
    scaler = StandardScaler(mean=data["x_train"][..., 0].mean(), std=data["x_train"][..., 0].std())
    for category in ["train", "val", "test"]:
        data["x_" + category][..., 0] = scaler.transform(data["x_" + category][..., 0])
    bs = {"train": batch_size, "val": valid_batch_size, "test": test_batch_size}
    for category in ["train", "val", "test"]:
        data[category + "_loader"] = DeviceDataLoader(data["x_" + category], data["y_" + category], bs[category],
                                                      device)
    data["scaler"] = scaler
    return data


def load_dataset_series(df, batch_size, valid_batch_size=None, test_batch_size=None, device="cuda",
                        seq_length_x=12, seq_length_y=12, y_start=1, dow=False):
    """The generate_training_data.py + load_dataset_metr pipeline without materialising the
    windows in HBM: one device copy of the readings, three SeriesDataLoaders over the 70/10/20
    split of the window ends.  The scaler is computed from the train windows exactly as the
    reference does (same float64 array, same reduction), so batches match bit for bit."""
    x_offsets, y_offsets = offsets(seq_length_x, seq_length_y, y_start)
    values = np.asarray(df.values, dtype=np.float64)
    min_t, max_t = window_range(values.shape[0], x_offsets, y_offsets)
    t_all = np.arange(min_t, max_t, dtype=np.int64)
    num_train, num_val, num_test = split_sizes(len(t_all))
    t_split = {"train": t_all[:num_train], "val": t_all[num_train:num_train + num_val], "test": t_all[-num_test:]}
    data = _features(values, df.index, True, dow)
    x_train = data[t_split["train"][:, None] + x_offsets[None, :], ...]
    scaler = StandardScaler(mean=x_train[..., 0].mean(), std=x_train[..., 0].std())
    del x_train
    out = {"scaler": scaler}
    bs = {"train": batch_size, "val": valid_batch_size, "test": test_batch_size}
    for category in ["train", "val", "test"]:
        out[category + "_loader"] = SeriesDataLoader(values, df.index, t_split[category], bs[category], device,
                                                     x_offsets, y_offsets, scaler, True, dow)
        out["t_" + category] = t_split[category]
    return out


__all__ = ["generate_graph_seq2seq_io_data", "generate_train_val_test", "offsets", "split_sizes", "window_range",
           "DeviceDataLoader", "SeriesDataLoader", "model_inputs", "load_dataset_device", "load_dataset_series"]
