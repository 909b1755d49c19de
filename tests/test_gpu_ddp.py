"""The data-parallel trainer on the GPU (bench.py --gpus N): two ranks, each a process
with its own HIP trainer on cuda:0, joined by a gloo process group (RCCL refuses two ranks on one
device; the product launches one rank per GPU with the "nccl" backend = RCCL over xGMI, and the
trainer code path is the same).

Step 1 runs eagerly; steps 2 and 3 take the captured path of engine.trainer._capture: graph g0
(forward + loss) -> graph g1 (backward) -> eager all-reduce of the flat gradient -> graph g2 (clip +
Adam; g2 exists only when distributed).

* G7 (B=2 per rank, N=16, C=16): step-1 gradients = the mean of the per-shard f64 reference
  gradients (g7, norm-rel <= 1e-4), step-1 parameters = clip + Adam on those mean gradients
  (norm-rel <= 1e-4; BN-cancelled biases, analytically 0, within 2 lr), and the parameters of both
  ranks bitwise equal after the captured steps.
* Headline shape (B=64 per rank, N=207, C=32: the fused GCN kernels of the bench): the data-parallel
  step-1 gradients equal the mean of two single-process HIP trainer runs on the same shards (each
  of which tests/test_gpu_headline.py pins to the fp64 oracle), and both ranks' parameters are
  bitwise equal after the captured steps.
* ``bench.py --gpus 2`` (self-launched ranks; gloo, both on cuda:0) prints one line with n_gpus 2."""
import math
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG, ROOT, load_golden, norm_rel, state_dict_of

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_q):
    for p in (PKG, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gwn_amd import util
        from gwn_amd.engine import trainer
        dev = torch.device("cuda:0")
        g = load_golden("g7_ddp_n16.npz")
        sups = [torch.tensor(g["sup0"], device=dev), torch.tensor(g["sup1"], device=dev)]
        eng = trainer(util.StandardScaler(54.4, 19.5), 2, 12, 16, 16, 0.0, 1e-3, 1e-4, dev, sups, True, True,
                      None, 4, 2)
        eng.model.load_state_dict({k: torch.tensor(v) for k, v in state_dict_of(g).items()})
        eng.broadcast_parameters(0)
        x = torch.tensor(g["x"][2 * rank:2 * rank + 2], device=dev)
        y = torch.tensor(g["y"][2 * rank:2 * rank + 2], device=dev)
        eng.train(x, y)
        torch.cuda.synchronize()
        grads = {n: p.grad.detach().cpu().numpy().copy() for n, p in eng.model.named_parameters() if p.grad is not None}
        p1 = {n: p.detach().cpu().numpy().copy() for n, p in eng.model.named_parameters()}
        for _ in range(2):
            eng.train(x, y)
        torch.cuda.synchronize()
        captured = _captured_dp(eng)
        p3 = eng.model._flat.detach().cpu().numpy().copy()
        out_q.put((rank, grads, p1, p3, captured))
    finally:
        torch.distributed.destroy_process_group()


def _captured_dp(eng):
    """Steps 2.. replayed the data-parallel graphs: one entry (g0, (g1, g1b), g2, ...) with g2
    present; returns "split" when the backward is two graphs (the early range's all-reduce beside
    the second, engine.trainer._overlap_hook), "whole" for one, False otherwise."""
    if len(eng._graphs) != 1:
        return False
    g0, (g1, g1b), g2 = list(eng._graphs.values())[0][:3]
    if g0 is None or g1 is None or g2 is None:
        return False
    return "split" if g1b is not None else "whole"


def _expected_step1(sd, gmean, lr=1e-3, wd=1e-4, clip=5.0, b1=0.9, b2=0.999, eps=1e-8):
    """clip_grad_norm_(5) + torch.optim.Adam (step 1) on the mean gradient (engine.py:52-55)."""
    total = math.sqrt(sum(float((v.astype(np.float64) ** 2).sum()) for v in gmean.values()))
    coef = min(clip / (total + 1e-6), 1.0)
    out = {}
    for k, g in gmean.items():
        p = sd[k].astype(np.float64)
        gg = g * coef + wd * p
        m = (1 - b1) * gg
        v = (1 - b2) * gg * gg
        out[k] = p - (lr / (1 - b1)) * m / (np.sqrt(v) / math.sqrt(1 - b2) + eps)
    return out


def test_gpu_ddp_two_ranks_captured_step(gpu):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, grads, p1, p3, captured = q.get(timeout=240)
            res[r] = (grads, p1, p3, captured)
    finally:
        for p in procs:
            p.join(timeout=60)
    for p in procs:
        assert p.exitcode == 0
    g = load_golden("g7_ddp_n16.npz")
    ref = {k[len("gradmean_f64/"):]: v for k, v in g.items() if k.startswith("gradmean_f64/")}
    sd = state_dict_of(g)
    exp = _expected_step1(sd, ref)
    for r in range(world):
        grads, p1, p3, captured = res[r]
        assert captured == "split", "steps 2-3 did not take the split data-parallel path (%s)" % captured
        assert set(grads) == set(ref), sorted(set(grads) ^ set(ref))
        for k, v in ref.items():
            if k.endswith("mlp.bias"):
                assert np.max(np.abs(grads[k])) <= 1e-5 * max(np.max(np.abs(x)) for x in ref.values()), k
                assert np.max(np.abs(p1[k] - exp[k])) <= 2e-3 + 1e-6, k
            elif np.linalg.norm(v) > 0:
                assert norm_rel(grads[k], v) <= 1e-4, (r, k, norm_rel(grads[k], v))
                assert norm_rel(p1[k], exp[k]) <= 1e-4, (r, k)
        for k, v in sd.items():  # parameters without a gradient stay where they were
            if k in p1 and k not in ref:
                np.testing.assert_array_equal(p1[k], v, err_msg=k)
    np.testing.assert_array_equal(res[0][1]["start_conv.weight"], res[1][1]["start_conv.weight"])
    np.testing.assert_array_equal(res[0][2], res[1][2])
    assert np.all(np.isfinite(res[0][2]))


HB, HN = 64, 207  # headline shape per rank


def _headline_setup(dev, seed_x):
    from gwn_amd import synthetic, util
    from gwn_amd.engine import trainer
    adj = synthetic.random_sensor_graph(HN, seed=0)
    sups = [torch.tensor(a, device=dev) for a in synthetic.double_transition(adj)]
    torch.manual_seed(999)
    eng = trainer(util.StandardScaler(synthetic.SCALER_MEAN, synthetic.SCALER_STD), 2, 12, HN, 32, 0.0, 1e-3, 1e-4,
                  dev, sups, True, True, None, 4, 2)
    eng.clip = None  # compare raw gradients (clip_grad_norm_ scales grad_flat in place by a norm
    #                  that differs between a shard and the mean)
    x, y = synthetic.synthetic_batch(HB, HN, 12, seed=seed_x)
    return eng, torch.tensor(x, device=dev), torch.tensor(y, device=dev)


def _headline_worker(rank, world, port, out_q, overlap="1"):
    for p in (PKG, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["GWN_DP_OVERLAP"] = overlap
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng, x, y = _headline_setup(torch.device("cuda:0"), 700 + rank)
        eng.broadcast_parameters(0)
        eng.train(x, y)
        torch.cuda.synchronize()
        g1 = eng.optimizer.grad_flat.detach().cpu().numpy().copy()
        for _ in range(2):
            eng.train(x, y)
        torch.cuda.synchronize()
        out_q.put((rank, g1, eng.model._flat.detach().cpu().numpy().copy(), _captured_dp(eng)))
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.parametrize("overlap", ["1", "0"])
def test_gpu_ddp_headline_shape_equals_mean_of_single_runs(gpu, overlap):
    """overlap 1 (default): end_conv_1's gradient all-reduced on a side stream while the layers'
    backward runs (the step split into g1 / g1b around it); 0: one all-reduce after the backward."""
    # the two shards trained by single-process HIP trainers (no process group in this process)
    singles = []
    for r in range(2):
        eng, x, y = _headline_setup(gpu, 700 + r)
        eng.train(x, y)
        torch.cuda.synchronize()
        singles.append(eng.optimizer.grad_flat.detach().cpu().numpy().copy())
        del eng
    mean = (singles[0] + singles[1]) / np.float32(2.0)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_headline_worker, args=(r, world, port, q, overlap)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, g1, p3, captured = q.get(timeout=240)
            res[r] = (g1, p3, captured)
    finally:
        for p in procs:
            p.join(timeout=60)
    for p in procs:
        assert p.exitcode == 0
    scale = float(np.max(np.abs(mean)))
    for r in range(world):
        g1, p3, captured = res[r]
        assert captured == ("split" if overlap == "1" else "whole"), (captured, overlap)
        diff = float(np.max(np.abs(g1.astype(np.float64) - mean)))
        assert diff <= 1e-6 * scale, (r, diff, scale)
        assert np.all(np.isfinite(p3))
    print("DP grads vs mean of single runs: max |diff| %.3g (bitwise %s)"
          % (float(np.max(np.abs(res[0][0] - mean))), bool(np.array_equal(res[0][0], mean))))
    np.testing.assert_array_equal(res[0][1], res[1][1])


def test_bench_gpus_2_self_launch(gpu):
    """bench.py --gpus 2 with no launcher: two ranks (gloo, both on cuda:0 -- RCCL refuses two ranks
    on one device) and one JSON line with n_gpus 2 and global_batch 128."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(GWN_DIST_BACKEND="gloo", GWN_SHARE_DEVICE="1", OMP_NUM_THREADS="8")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
                          "--warmup", "2", "--no-cpu-baseline"], env=env, capture_output=True, text=True,
                         timeout=110)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = lines[0]
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 128 and rec["config"]["parallelism"] == "dp2"
    assert rec["value"] > 0 and rec["mae12_delta"] <= 1e-4
    dist = rec["distributed"]  # what torch.distributed saw (SCALE lines carry the same record)
    assert dist["backend"] == "gloo" and dist["world_seen"] == 2
    assert 0 < dist["rank_seconds_min"] <= dist["rank_seconds_max"]
    assert abs(rec["ms_per_step"] - 1000.0 * dist["rank_seconds_max"] / 3) < 0.01
    # the collectives' device time and the overlapped share of the early all-reduce (outside the
    # timed region): the early range on the side stream, the rest on the main stream
    ar = dist["allreduce"]
    assert ar["overlap"] is True and ar["steps"] == 5 and ar["grad_floats"] > 0
    assert ar["early_allreduce_ms"] > 0 and ar["rest_allreduce_ms"] > 0 and ar["layers_backward_ms"] > 0
    assert 0 <= ar["early_overlapped_ms"] <= ar["early_allreduce_ms"] + 1e-3
