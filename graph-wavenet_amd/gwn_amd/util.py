"""The parts of the reference's ``Utils/util.py`` that the METR-LA training path uses.

* ``StandardScaler``                      util.py:104-117
* ``asym_adj`` / ``sym_adj`` / ``mod_adj`` / ``load_adj``   util.py:121-199 (host, once)
* ``DataLoader`` / ``load_dataset_metr``   util.py:14-54, 202-217 (host-side batching)
* ``masked_mse/rmse/mae/mape``, ``metric`` util.py:510-559

The masked metrics keep the reference's torch formulation so that user code calling them on
arbitrary tensors behaves identically; the trainer's hot path does NOT call them — it uses the
fused ``gwn_masked_loss`` kernel (engine.py).
"""
import os
import pickle

import numpy as np
import torch

from .synthetic import asym_adj as _asym_adj_dense


class DataLoader(object):
    """Mini-batch iterator; pads with the last sample to a multiple of batch_size (util.py:14-54)."""

    def __init__(self, xs, ys, batch_size, pad_with_last_sample=True):
        self.batch_size = batch_size
        self.current_ind = 0
        if pad_with_last_sample:
            num_padding = (batch_size - (len(xs) % batch_size)) % batch_size
            xs = np.concatenate([xs, np.repeat(xs[-1:], num_padding, axis=0)], axis=0)
            ys = np.concatenate([ys, np.repeat(ys[-1:], num_padding, axis=0)], axis=0)
        self.size = len(xs)
        self.num_batch = int(self.size // self.batch_size)
        self.xs = xs
        self.ys = ys

    def shuffle(self):
        permutation = np.random.permutation(self.size)
        self.xs, self.ys = self.xs[permutation], self.ys[permutation]

    def get_iterator(self):
        self.current_ind = 0

        def _wrapper():
            while self.current_ind < self.num_batch:
                lo = self.batch_size * self.current_ind
                hi = min(self.size, self.batch_size * (self.current_ind + 1))
                yield self.xs[lo:hi, ...], self.ys[lo:hi, ...]
                self.current_ind += 1

        return _wrapper()


class StandardScaler:
    def __init__(self, mean, std):
        self.mean = mean
        self.std = std

    def transform(self, data):
        return (data - self.mean) / self.std

    def inverse_transform(self, data):
        return (data * self.std) + self.mean


def asym_adj(adj):
    """D^-1 A (row-normalised), util.py:130-136."""
    return np.asarray(_asym_adj_dense(np.asarray(adj)), dtype=np.float32)


def sym_adj(adj):
    """D^-1/2 A D^-1/2 in the reference's transposed form (util.py:121-128)."""
    adj = np.asarray(adj, dtype=np.float64)
    d = adj.sum(1)
    with np.errstate(divide="ignore"):
        d_inv_sqrt = np.power(d, -0.5)
    d_inv_sqrt[np.isinf(d_inv_sqrt)] = 0.0
    return ((adj * d_inv_sqrt[None, :]).T * d_inv_sqrt[None, :]).astype(np.float32)


def calculate_normalized_laplacian(adj):
    return np.eye(adj.shape[0], dtype=np.float32) - sym_adj(adj)


def calculate_scaled_laplacian(adj_mx, lambda_max=2, undirected=True):
    if undirected:
        adj_mx = np.maximum.reduce([adj_mx, adj_mx.T])
    lap = calculate_normalized_laplacian(adj_mx).astype(np.float64)
    if lambda_max is None:
        lambda_max = float(np.max(np.linalg.eigvalsh(lap)))
    return ((2.0 / lambda_max) * lap - np.eye(lap.shape[0])).astype(np.float32)


def mod_adj(adj_mx, adjtype):
    """Support list for --adjtype (util.py:178-194)."""
    if adjtype == "scalap":
        return [calculate_scaled_laplacian(adj_mx)]
    if adjtype == "normlap":
        return [calculate_normalized_laplacian(adj_mx)]
    if adjtype == "symnadj":
        return [sym_adj(adj_mx)]
    if adjtype == "transition":
        return [asym_adj(adj_mx)]
    if adjtype == "doubletransition":
        return [asym_adj(adj_mx), asym_adj(np.transpose(adj_mx))]
    if adjtype == "identity":
        return [np.diag(np.ones(adj_mx.shape[0])).astype(np.float32)]
    raise AssertionError("adj type not defined")


def load_pickle(pickle_file):
    """The METR-LA ``adj_mx.pkl`` is a pickle (util.py:166-176); load only files you trust."""
    try:
        with open(pickle_file, "rb") as f:
            return pickle.load(f)
    except UnicodeDecodeError:
        with open(pickle_file, "rb") as f:
            return pickle.load(f, encoding="latin1")


def load_adj(pkl_filename, adjtype):
    sensor_ids, sensor_id_to_ind, adj_mx = load_pickle(pkl_filename)
    return sensor_ids, sensor_id_to_ind, mod_adj(adj_mx, adjtype)


def load_dataset_metr(dataset_dir, batch_size, valid_batch_size=None, test_batch_size=None):
    """``{train,val,test}.npz`` with x, y: (S, 12, N, 2) (generate_training_data.py:85-91)."""
    data = {}
    for category in ["train", "val", "test"]:
        cat = np.load(os.path.join(dataset_dir, category + ".npz"))
        data["x_" + category] = cat["x"]
        data["y_" + category] = cat["y"]
    scaler = StandardScaler(mean=data["x_train"][..., 0].mean(), std=data["x_train"][..., 0].std())
    for category in ["train", "val", "test"]:
        data["x_" + category][..., 0] = scaler.transform(data["x_" + category][..., 0])
    data["train_loader"] = DataLoader(data["x_train"], data["y_train"], batch_size)
    data["val_loader"] = DataLoader(data["x_val"], data["y_val"], valid_batch_size)
    data["test_loader"] = DataLoader(data["x_test"], data["y_test"], test_batch_size)
    data["scaler"] = scaler
    return data


# test.py:56 calls ``util.load_dataset``; the reference's util only defines the METR-LA loader
load_dataset = load_dataset_metr


def _mask(labels, null_val):
    if np.isnan(null_val):
        mask = ~torch.isnan(labels)
    else:
        mask = labels != null_val
    mask = mask.float()
    mask /= torch.mean(mask)
    return torch.where(torch.isnan(mask), torch.zeros_like(mask), mask)


def masked_mse(preds, labels, null_val=np.nan):
    loss = (preds - labels) ** 2 * _mask(labels, null_val)
    return torch.mean(torch.where(torch.isnan(loss), torch.zeros_like(loss), loss))


def masked_rmse(preds, labels, null_val=np.nan):
    return torch.sqrt(masked_mse(preds=preds, labels=labels, null_val=null_val))


def masked_mae(preds, labels, null_val=np.nan):
    loss = torch.abs(preds - labels) * _mask(labels, null_val)
    return torch.mean(torch.where(torch.isnan(loss), torch.zeros_like(loss), loss))


def masked_mape(preds, labels, null_val=np.nan):
    loss = torch.abs(preds - labels) / labels * _mask(labels, null_val)
    return torch.mean(torch.where(torch.isnan(loss), torch.zeros_like(loss), loss))


def metric(pred, real):
    mae = masked_mae(pred, real, 0.0).item()
    mape = masked_mape(pred, real, 0.0).item()
    rmse = masked_rmse(pred, real, 0.0).item()
    return mae, mape, rmse
