"""Measure the bf16-operand path's error against the fp64 references (forward, train grads) at the
fixture shapes; prints one line per check.  GPU box: python tools/bf16_error.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "graph-wavenet_amd"), ROOT, os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from conftest import load_golden, norm_rel, rel_err, state_dict_of  # noqa: E402


def main():
    from gwn_amd import util
    from gwn_amd.engine import trainer
    dev = torch.device("cuda:0")
    for name, n, xkey, okey in (("g5b_fwd_eval_n325.npz", 325, "x", "out_f64"), ("g12_metr_n207.npz", 207, "g1_x", "g1_out_f64")):
        g = load_golden(name)
        for dt in ("fp32", "bf16"):
            eng = trainer(util.StandardScaler(54.4, 19.5), 2, 12, n, 32, 0.3, 0.0, 0.0, dev,
                          [torch.tensor(g["sup0"], device=dev), torch.tensor(g["sup1"], device=dev)], True, True,
                          None, 4, 2)
            eng.model.load_state_dict({k: torch.tensor(v) for k, v in state_dict_of(g).items()})
            eng.model.set_compute_dtype(dt)
            eng.model.eval()
            with torch.no_grad():
                out = eng.model(torch.tensor(g[xkey], device=dev))
            print("fwd", name, dt, "max-rel %.3e" % rel_err(out.cpu().numpy(), g[okey]), flush=True)
    for name, n, pre in (("g13_train_n325.npz", 325, ""), ("g12_metr_n207.npz", 207, "g2_")):
        g = load_golden(name)
        for dt in ("fp32", "bf16"):
            eng = trainer(util.StandardScaler(54.4, 19.5), 2, 12, n, 32, 0.0, 0.0, 0.0, dev,
                          [torch.tensor(g["sup0"], device=dev), torch.tensor(g["sup1"], device=dev)], True, True,
                          None, 4, 2)
            eng.model.load_state_dict({k: torch.tensor(v) for k, v in state_dict_of(g).items()})
            eng.model.set_compute_dtype(dt)
            eng.clip = None
            met = eng.train(torch.tensor(g[pre + "x"], device=dev), torch.tensor(g[pre + "y"], device=dev))
            mkey = "metrics_f64" if pre == "" else "g2_metrics_f64"
            gkey = "grad_f64/" if pre == "" else "g2_grad_f64/"
            ref = {k[len(gkey):]: v for k, v in g.items() if k.startswith(gkey)}
            errs = []
            for k, p in eng.model.named_parameters():
                if p.grad is None or k not in ref or k.endswith("mlp.bias") or np.linalg.norm(ref[k]) == 0:
                    continue
                errs.append((norm_rel(p.grad.cpu().numpy(), ref[k]), k))
            errs.sort(reverse=True)
            print("train", name, dt, "loss rel %.3e" % abs(met[0] / g[mkey][0] - 1),
                  "worst grads", ["%s %.2e" % (k, e) for e, k in errs[:4]], "median %.2e" % np.median([e for e, _ in errs]),
                  flush=True)


if __name__ == "__main__":
    main()
