"""Probe: where the time of the f32 16-node tile forward goes, per layer of a METR-LA training step
(B=64, N=207, T=12), from five per-workgroup stamps (GWN_LIB = an exp build made with
tools/exp/t16_phase_stamps.py): start -> staging issued (1) -> first phase staged (2) -> last tile
of wave 0 (3) -> BN flush done (4).  Eager steps (GWN_GRAPHS=0)."""
import os
import sys

os.environ["GWN_GRAPHS"] = "0"
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, "graph-wavenet_amd")
from gwn_amd import _lib, synthetic, util  # noqa: E402
from gwn_amd.engine import trainer  # noqa: E402

print("torch imported", flush=True)
dev = torch.device("cuda", 0)
N, B, T = 207, 64, 12
torch.manual_seed(999)
adj = synthetic.random_sensor_graph(N, seed=3, dense=False)
sups = [torch.tensor(a, device=dev) for a in synthetic.double_transition(adj)]
eng = trainer(util.StandardScaler(synthetic.SCALER_MEAN, synthetic.SCALER_STD), 2, T, N, 32, 0.3, 1e-3, 1e-4,
              dev, sups, True, True, None, 4, 2)
ex = eng.model.executor()
ex.launch_clock = True
ex.launch_clock_slots = 8  # the exp build stamps clk[8 * wg + k], k < 5: sized before the first launch
x, y = synthetic.synthetic_batch(B, N, T, seed=1)
xl = torch.tensor(np.ascontiguousarray(x.transpose(0, 3, 2, 1)), device=dev).transpose(1, 3)
yl = torch.tensor(np.ascontiguousarray(np.stack([y, y], 1).transpose(0, 3, 2, 1)), device=dev).transpose(1, 3)[:, 0]
for k in range(3):
    eng.train(xl, yl)
    torch.cuda.synchronize()
    print("warm-up step", k, flush=True)
acts = [a for k, a in eng._acts.items() if k[2]][0]
cus = torch.cuda.get_device_properties(0).multi_processor_count
assert all(v.numel() == 8 * cus for v in acts.CLK.values())
for rep in range(3):
    for i in acts.CLK:
        acts.CLK[i].zero_()
    eng.train(xl, yl)
    torch.cuda.synchronize()
    khz = _lib.load().gwn_wall_clock_khz()
    print("step %d (us): layer slices | issue stage first-phase tiles flush | span | tiles min..max end" % rep)
    for i in sorted(acts.CLK):
        c = acts.CLK[i].cpu().numpy().reshape(-1, 8).astype(np.float64)
        g = int((c[:, 4] > 0).sum())
        c = c[:g] * 1000.0 / khz
        d = np.diff(c[:, :5], axis=1).mean(0)
        span = c[:, 4].max() - c[:, 0].min()
        print("  %d %4d | %6.1f %6.1f %6.1f %6.1f | %6.1f | %6.1f .. %6.1f  (start spread %.1f)" % (
            i, acts.gcn_args[i].rows // N, d[0], d[1], d[2], d[3], span, c[:, 3].min() - c[:, 0].min(),
            c[:, 3].max() - c[:, 0].min(), c[:, 0].max() - c[:, 0].min()), flush=True)
        if rep == 2:  # per-workgroup: duration and first-staging quantiles, and the slowest ten
            dur = c[:, 4] - c[:, 0]
            stg = c[:, 2] - c[:, 0]
            q = lambda v: " ".join("%.1f" % x for x in np.percentile(v, [0, 10, 50, 90, 100]))  # noqa: E731
            slow = np.argsort(-dur)[:10]
            print("      wg dur q0/10/50/90/100: %s | staged at: %s | slowest wgs %s (dur %s, staged %s)" % (
                q(dur), q(stg), slow.tolist(), " ".join("%.0f" % dur[k] for k in slow),
                " ".join("%.0f" % stg[k] for k in slow)), flush=True)
