"""Probe: host time per trainer.train() call at the headline config, split into the part before the
graph replay is issued (exposed: the GPU idles while the host prepares the next step) and the part
after it.  Usage: python tools/host_probe.py [--steps 200]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-wavenet_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    from gwn_amd import synthetic, util
    from gwn_amd.engine import trainer
    dev = torch.device("cuda:0")
    B, N, T = 64, 207, 12
    torch.manual_seed(999)
    adj = synthetic.random_sensor_graph(N, seed=1, dense=False)
    sups = [torch.tensor(a, device=dev) for a in synthetic.double_transition(adj)]
    scaler = util.StandardScaler(synthetic.SCALER_MEAN, synthetic.SCALER_STD)
    eng = trainer(scaler, 2, T, N, 32, 0.3, 1e-3, 1e-4, dev, sups, True, True, None, 4, 2)
    x, y = synthetic.synthetic_batch(B, N, T, seed=0)
    xl = torch.tensor(np.ascontiguousarray(x.transpose(0, 3, 2, 1)), device=dev)
    yl = torch.tensor(np.ascontiguousarray(np.stack([y, y], 1).transpose(0, 3, 2, 1)), device=dev)
    xs, ys = xl.transpose(1, 3), yl.transpose(1, 3)[:, 0, :, :]
    marks = []
    orig = torch.cuda.CUDAGraph.replay

    def replay(self):
        marks.append(time.perf_counter())
        return orig(self)
    torch.cuda.CUDAGraph.replay = replay
    for _ in range(5):
        eng.train(xs, ys)
    torch.cuda.synchronize()
    marks.clear()
    starts, ends = [], []
    for _ in range(args.steps):
        starts.append(time.perf_counter())
        eng.train(xs, ys)
        ends.append(time.perf_counter())
    marks = marks[::len(marks) // len(starts)]  # the first replay of each step
    pre = np.array(marks) - np.array(starts)
    post = np.array(ends) - np.array(marks)
    gap = np.array(starts[1:]) - np.array(ends[:-1])
    print("per train(): before replay %.1f us (median), replay -> return %.1f us, between calls %.1f us, "
          "wall %.1f us" % (1e6 * np.median(pre), 1e6 * np.median(post), 1e6 * np.median(gap),
                            1e6 * (ends[-1] - starts[0]) / args.steps))
    import cProfile
    import pstats
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(50):
        eng.train(xs, ys)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
