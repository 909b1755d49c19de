"""Inference benchmark (train.py:377-404 / test.py:58-87 workload).

1. eval forward samples/s at METR-LA shape (B=64, N=207, T=12, doubletransition + adaptive):
   the lean inference schedule (Executor.infer) vs the training-shaped eval forward
   (GWN_LEAN_EVAL=0), HIP-event timed, input resident in HBM;
2. a whole test split (6,850 samples, METR-LA's test size; synthetic values in the npz format):
   the reference's loop (host DataLoader, torch.Tensor(x).to(device) per batch, 12 x 3
   util.metric calls) vs infer.evaluate on a DeviceDataLoader (split uploaded once, batches
   gathered on the GPU, per-horizon metrics in two launches + one copy), wall-clock.
Prints one JSON line.  Usage: python tools/bench_infer.py [--reps R]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-wavenet_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--test-samples", type=int, default=6850)
    args = ap.parse_args()
    from gwn_amd import data, infer, synthetic, util
    from gwn_amd.model import gwnet
    dev = torch.device("cuda:0")
    N, B, T = 207, 64, 12
    adj = synthetic.random_sensor_graph(N, seed=0)
    sups = [torch.tensor(a, device=dev) for a in synthetic.double_transition(adj)]
    torch.manual_seed(999)
    m = gwnet(dev, N, 0.3, supports=sups)
    m.eval()
    x, _ = synthetic.synthetic_batch(B, N, T, seed=1)
    xd = torch.nn.functional.pad(torch.tensor(x, device=dev), (1, 0, 0, 0))
    res = {"workload": "eval forward B=64 N=207 T=12 (+1 pad) fp32; test split %d samples" % args.test_samples}

    def time_fwd(lean):
        os.environ["GWN_LEAN_EVAL"] = "1" if lean else "0"
        with torch.no_grad():
            for _ in range(5):
                m(xd)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                m(xd)
            e1.record()
            torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.reps

    ms_lean, ms_full = time_fwd(True), time_fwd(False)
    os.environ["GWN_LEAN_EVAL"] = "1"
    res["eval_forward"] = {"lean_ms": round(ms_lean, 4), "lean_samples_per_s": round(B / ms_lean * 1e3, 1),
                           "full_ms": round(ms_full, 4), "full_samples_per_s": round(B / ms_full * 1e3, 1),
                           "cpu_reference_samples_per_s": 132.5,
                           "cpu_reference_note": "reference eval forward, 8 vCPU Xeon, BASELINE.md §2"}

    # whole test split
    S = args.test_samples
    rng = np.random.default_rng(0)
    xs = np.zeros((S, T, N, 2))
    xs[..., 0] = rng.standard_normal((S, T, N))
    xs[..., 1] = ((rng.integers(0, 288, size=S)[:, None] + np.arange(T)[None, :]) % 288 / 288.0)[:, :, None]
    ys = np.clip(54.4 + 19.5 * rng.standard_normal((S, T, N, 2)), 0, 80)
    ys[rng.random(ys.shape) < 0.05] = 0.0
    scaler = util.StandardScaler(54.4, 19.5)
    realy = torch.Tensor(ys).to(dev).transpose(1, 3)[:, 0, :, :]

    def reference_loop():
        outs = []
        with torch.no_grad():
            for xb, _ in util.DataLoader(xs, ys, B).get_iterator():
                outs.append(m(torch.Tensor(xb).to(dev).transpose(1, 3)).transpose(1, 3).squeeze())
        yhat = torch.cat(outs, dim=0)[:S]
        return [util.metric(scaler.inverse_transform(yhat[:, :, i]), realy[:, :, i]) for i in range(T)]

    dl = data.DeviceDataLoader(xs, ys, B, dev)

    def device_loop():
        return infer.evaluate(m, dl, realy, scaler, log=None)

    for fn in (reference_loop, device_loop):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ref = reference_loop()
    t1 = time.perf_counter()
    got = device_loop()
    t2 = time.perf_counter()
    diff = float(np.max(np.abs(np.stack(got, 1) - np.asarray(ref)) / np.maximum(np.abs(np.asarray(ref)), 1e-12)))
    res["test_split"] = {"reference_loop_s": round(t1 - t0, 4), "device_loop_s": round(t2 - t1, 4),
                         "speedup": round((t1 - t0) / (t2 - t1), 2),
                         "device_samples_per_s": round(S / (t2 - t1), 1),
                         "max_rel_diff_of_metrics": diff,
                         "upload_once_mb": round((xs.nbytes + ys.nbytes) / 2 / 1e6, 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
