"""Benchmark: Graph WaveNet training step (fwd+bwd+clip+Adam) on libgwn.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config metr|pems|n2048]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...   (N > 1)

``--gpus N`` with N > 1 and no launcher around it starts the N ranks itself (a child
torch.distributed.run, before anything touches the GPU) and exits with their status; under a
launcher WORLD_SIZE must equal N.

A step is ``trainer.train(x, y)`` (reference engine.py:41-58) on one synthetic batch per GPU, the
batches already resident in HBM and handed over as the transpose views train.py:244-247 builds.
The default config is the headline (BASELINE.json configs[1]): METR-LA shape, B=64 per GPU, N=207
sensors, T=12, doubletransition supports + adaptive adjacency, dropout 0.3, Adam lr 1e-3 wd 1e-4.
``--config pems`` is configs[2]'s graph (N=325), ``--config n2048`` configs[4] (N=2048, T=24,
dense random adjacency, B=32 per GPU).  With N>1 GPUs each rank trains its own shard and the
gradients are averaged by one RCCL all-reduce per step (weak scaling).  Rank 0 prints one JSON line;
see DESIGN.md §5 for the roofline / baseline fields.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "graph-wavenet_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "samples/sec (fwd+bwd) METR-LA B=64 N=207 T=12 at 1/2/4/8 GPUs; 12-step MAE"
FP32_PEAK_TFLOPS = 157.3   # MI355X dense fp32 (vector = MFMA), MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0
BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (MI355X_MICROARCH.md; no sparsity)

CONFIGS = {
    # batch per GPU, nodes, steps, graph, workload label, oracle / CPU sample batch
    "metr": dict(B=64, N=207, T=12, dense=False, graph_seed=0, sample_b=64,
                 workload="METR-LA train step B=64/GPU N=207 T=12 {dtype} (configs[1])"),
    "pems": dict(B=64, N=325, T=12, dense=False, graph_seed=6, sample_b=16, dtype="bf16",
                 workload="PEMS-BAY-shape train step B=64/GPU N=325 T=12 {dtype} (configs[2])"),
    "n2048": dict(B=32, N=2048, T=24, dense=True, graph_seed=15, sample_b=1,
                  workload="synthetic dense-graph train step B=32/GPU N=2048 T=24 {dtype} (configs[4])"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="metr", choices=sorted(CONFIGS))
    ap.add_argument("--dtype", choices=("f32", "bf16"), default=None,
                    help="override the config's arithmetic precision (pems: bf16, others f32)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--plan-only", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


def step_flops(n, t):
    """Algorithmic fwd+bwd FLOP of one sample: the reference's
    full work as torch.utils.flop_counter counts it (incl. full-T skip convs, gconv.7 backward),
    so executed-work savings show up as a higher effective fraction."""
    return {(207, 12): 3.3962e9, (325, 12): 7.0994e9, (2048, 24): 585.82e9}[(n, t)]


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """``--gpus N`` (N > 1) without a launcher around us: start N ranks, one per GPU, as a CHILD
    ``torch.distributed.run`` (never an exec; nothing here has touched the GPU yet), wait for
    them and return their exit status.  Rank 0 prints the one JSON line."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    cfg = CONFIGS[args.config]
    B, N, T = cfg["B"], cfg["N"], cfg["T"]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d (launch one rank per GPU)" % (args.gpus, world))
    if args.plan_only:
        # launcher check without a GPU (tests/test_host.py): every rank reports its place
        print(json.dumps({"plan": True, "rank": rank, "world": world, "local_rank": local,
                          "master": "%s:%s" % (os.environ.get("MASTER_ADDR"), os.environ.get("MASTER_PORT"))}),
              flush=True)
        return
    # rehearsal on a one-GPU box (never the driver's run): GWN_DIST_BACKEND=gloo GWN_SHARE_DEVICE=1
    # puts every rank on cuda:0 over gloo (RCCL refuses two ranks on one device)
    if os.environ.get("GWN_SHARE_DEVICE", "0") != "0":
        local = 0
    backend = None
    if world > 1:
        backend = os.environ.get("GWN_DIST_BACKEND", "nccl")
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.distributed.init_process_group(backend)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from gwn_amd import synthetic, util
    from gwn_amd.engine import trainer

    torch.manual_seed(999)
    np.random.seed(0)
    adj = synthetic.random_sensor_graph(N, seed=cfg["graph_seed"], dense=cfg["dense"])
    sups_np = synthetic.double_transition(adj)
    sups = [torch.tensor(a, device=dev) for a in sups_np]
    scaler = util.StandardScaler(synthetic.SCALER_MEAN, synthetic.SCALER_STD)
    eng = trainer(scaler, 2, T, N, 32, 0.3, 1e-3, 1e-4, dev, sups, True, True, None, 4, 2)
    bf16 = (args.dtype or cfg.get("dtype", "f32")) == "bf16"
    eng.model.set_compute_dtype("bf16" if bf16 else "fp32")
    eng.broadcast_parameters(0)
    ex = eng.model.executor()
    # the operand format the fused GCN kernels actually run (0: fp32, also when bf16 was requested
    # for a shape without a bf16 tile kernel; 1: bf16 diffusion; 2: bf16 diffusion and mlp)
    planes = ex.split_planes()
    bf16 = planes > 0
    ex.seed.fill_(12345 + 7919 * rank)
    # the dominant kernel's own clock stamps (measure_dominant), captured into the step's graphs
    # with the rest of the step: two stores per workgroup and launch
    ex.launch_clock = True

    nb = 8 if N <= 512 else 2  # distinct resident batches, cycled
    xs, ys = [], []
    for i in range(nb):
        x, y = synthetic.synthetic_batch(B, N, T, seed=1000 * rank + i)
        # the reference feeds transpose views of the loader's [B, T, N, 2] batch (train.py:244-247):
        # trainx = x.transpose(1, 3), real_val = y.transpose(1, 3)[:, 0]; same strides here
        xl = torch.tensor(np.ascontiguousarray(x.transpose(0, 3, 2, 1)), device=dev)
        yl = torch.tensor(np.ascontiguousarray(np.stack([y, y], 1).transpose(0, 3, 2, 1)), device=dev)
        xs.append(xl.transpose(1, 3))
        ys.append(yl.transpose(1, 3)[:, 0, :, :])

    def barrier():
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    for i in range(args.warmup):
        eng.train(xs[i % nb], ys[i % nb])
    clocks = [a for k, a in eng._acts.items() if k[2]]
    for ck in (getattr(clocks[0], "CLK", {}) if clocks else {}).values():
        ck.zero_()  # (a kernel path that stamps nothing leaves zeros)
    barrier()
    t0 = time.perf_counter()
    last = None
    for i in range(args.steps):
        last = eng.train(xs[i % nb], ys[i % nb])
    barrier()
    elapsed = time.perf_counter() - t0
    dist_info = None
    if world > 1:
        elapsed, dist_info = rank_timing(elapsed, world, rank, dev)
        dist_info["device_per_rank"] = ("cuda:%d" % local if os.environ.get("GWN_SHARE_DEVICE", "0") == "0"
                                        else "cuda:0 (shared: rehearsal)")
    samples = world * B * args.steps
    value = samples / elapsed
    ms = 1000.0 * elapsed / args.steps

    # 12-step MAE (train.py:392-403 protocol) of the trained weights on a held-out synthetic batch,
    # and the same number from the fp64 CPU oracle on the same weights and batch (north_star: MAE
    # within 1e-4 of the reference)
    sb = cfg["sample_b"]
    xt, yt = synthetic.synthetic_batch(sb, N, T, seed=99999)
    with torch.no_grad():
        eng.model.eval()
        pred = eng.model(torch.tensor(xt, device=dev)).transpose(1, 3)[:, 0]  # [B, N, T]
        real = torch.tensor(yt, device=dev)
        maes = [util.masked_mae(scaler.inverse_transform(pred[:, :, h]), real[:, :, h], 0.0).item() for h in range(T)]
    mae12 = float(np.mean(maes))
    mae12_ref = oracle_mae12(eng, sups_np, xt, yt, N, T) if rank == 0 else None

    # the dominant kernel's timing: the last timed step's stamps, then 9 more steps of the same
    # captured graphs, each read after it (outside the timed region: the reads synchronize)
    roof = measure_dominant(eng, dev, bf16=bf16, steps=args.steps,
                            extra=lambda k: eng.train(xs[k % nb], ys[k % nb]), extra_n=9)
    if dist_info is not None:
        # the collectives' device time and how much of the early all-reduce the layers' backward
        # hid (engine.trainer.dp_probe_summary), over 5 more steps outside the timed region
        eng.dp_probe = []
        for k in range(5):
            eng.dp_probe.append({})
            eng.train(xs[k % nb], ys[k % nb])
        dist_info["allreduce"] = dict(eng.dp_probe_summary(), steps=5,
                                      overlap=os.environ.get("GWN_DP_OVERLAP", "1") != "0",
                                      grad_floats=int(eng.optimizer.grad_flat.numel()))
        eng.dp_probe = None
    result = None
    if rank == 0:
        result = {
            "metric": METRIC, "value": round(value, 2), "unit": "samples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16" if bf16 else "f32",
            "data": "synthetic (%s, seeded; random-init weights)"
                    % ("METR-LA tensor format" if not cfg["dense"] else "METR-LA tensor format, dense random graph"),
            "config": {"workload": cfg["workload"].format(
                           dtype=("bf16 MFMA operands with fp32 accumulation in the diffusion GCN (%s)"
                                  % ("diffusion and per-piece mlp" if planes == 2 else "diffusion; mlp in fp32"))
                           if bf16 else "fp32"),
                       "global_batch": B * world, "nodes": N, "seq_len": T,
                       "parallelism": "dp%d" % world if world > 1 else "single"},
            "mae12": round(mae12, 6), "mae12_oracle_f64": round(mae12_ref, 6),
            "mae12_delta": float("%.3g" % abs(mae12 - mae12_ref)), "mae12_sample_batch": sb,
            "last_train_metrics": [round(v, 5) for v in last],
            "step_effective_tflops": round(step_flops(N, T) * B * world / (elapsed / args.steps) / 1e12 / world, 3),
            "roofline": roof,
        }
        if dist_info is not None:
            result["distributed"] = dist_info
        if world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(args.cpu_seconds, cfg)
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


def rank_timing(elapsed, world, rank, dev):
    """MAX over ranks of the timed region (the contract's whole-job time) and a record of what
    torch.distributed saw: backend, world size, min / max of the per-rank timed regions.  Without
    GWN_DIST_BACKEND (the driver's runs) the backend must be nccl (= RCCL)."""
    t = torch.zeros(world, device=dev, dtype=torch.float64)
    t[rank] = elapsed
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.SUM)
    per_rank = [float(v) for v in t.cpu()]
    seen_backend = str(torch.distributed.get_backend())
    seen_world = torch.distributed.get_world_size()
    if "GWN_DIST_BACKEND" not in os.environ and seen_backend != "nccl":
        raise SystemExit("bench.py: expected the nccl (RCCL) backend, torch.distributed reports %s" % seen_backend)
    if seen_world != world:
        raise SystemExit("bench.py: WORLD_SIZE %d but torch.distributed sees %d ranks" % (world, seen_world))
    return max(per_rank), {"backend": seen_backend, "world_seen": seen_world,
                           "rank_seconds_min": round(min(per_rank), 6), "rank_seconds_max": round(max(per_rank), 6)}


def replay_ms(launches, rounds):
    """The launches captured in one HIP graph (no host launch overhead between kernels) and
    replayed `rounds` times between one HIP event pair on the launch stream (ms)."""
    import ctypes
    from gwn_amd import _lib
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for ga in launches:
            _lib.call("gwn_gcn_fwd", ctypes.byref(ga), _lib.stream())
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for ga in launches:
            _lib.call("gwn_gcn_fwd", ctypes.byref(ga), _lib.stream())
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(rounds):
        graph.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def clock_spans(acts):
    """Durations (us) of the last timed step's gcn forward launches from the kernels' own device
    clock stamps (gwn_gcn_args.clock: every workgroup's start and end on the device wall clock;
    each launch overwrites the previous step's): launch i lasts max(end) - min(start) over its
    workgroups.  None where a layer's kernel path stamps nothing (only the 16-node tile forward
    kernels do)."""
    from gwn_amd import _lib
    khz = _lib.load().gwn_wall_clock_khz()
    ck = getattr(acts, "CLK", {})
    if khz <= 0 or not ck or sorted(ck) != sorted(acts.gcn_args):
        return None
    spans = []
    for i in sorted(ck):
        c = ck[i].cpu().numpy().reshape(-1, 2)
        g = int((c[:, 1] > 0).sum())  # the launch's workgroups, slots [0, g)
        if g == 0 or (c[:g] <= 0).any() or (c[g:] != 0).any():
            return None
        spans.append(float(c[:g, 1].max() - c[:g, 0].min()) * 1000.0 / khz)
    return spans if min(spans) > 0 else None


def measure_dominant(eng, dev, rounds=5, bf16=False, steps=None, extra=None, extra_n=0):
    """The dominant kernel is the diffusion graph convolution forward (gwn_gcn_fwd: 3 supports x 2
    hops of 'ncvl,vw->ncwl' + the 224->32 mlp + residual + dropout + BN partials, one call per
    layer, 8 per step; for N <= 512 ONE fused launch, gcn_fwd_t16_kernel).  Timing: the kernel's
    own device clock stamps in the last timed step's launches and in extra_n more steps run by
    extra(k) and read after each (clock_spans: the training step's own graphs, no replay); where the
    kernel records none, exactly the last training step's 8 calls
    (same arguments and buffers; idempotent) replayed as one captured HIP graph between HIP events
    on the launch stream.  Either way only the gcn kernel: the BN finalize + fold its bn_fold
    argument issues after it, and the TCN it issues before it where it does not fuse it, are left
    out.  achieved = algorithmic FLOP / time, where the algorithmic FLOP of a call = slices *
    (K*order*2*C*N^2 + 2*(2K+1)*C*C*N), plus slices * N * 2*(2C)^2 when the
    kernel runs the layer's gated TCN itself (gwn_gcn_tcn_fused; where it does not -- bf16, or
    fewer slices than CUs -- the TCN is its own rowgemm launch)."""
    import ctypes
    from gwn_amd import _lib
    ex = eng.model._executor
    acts = [a for k, a in eng._acts.items() if k[2]][0]
    cfg = ex.cfg
    C, N, K = cfg.C, cfg.N, cfg.nsup
    # the gcn launches alone (copies: the step's own args stay intact)
    launches = []
    for i in sorted(acts.gcn_args):
        ga = type(acts.gcn_args[i]).from_buffer_copy(acts.gcn_args[i])
        ga.bn_fold = None
        ga.clock = None
        if ga.tcn and not _lib.load().gwn_gcn_tcn_fused(ctypes.byref(ga)):
            ga.tcn = None  # its TCN (and BN finalize) run as launches of their own: not this kernel's work
        if ga.tcn and ga.tcn.contents.bn:
            # the fused TCN's BatchNorm finalize stays in (it is this launch's work) but without
            # the running statistics / num_batches_tracked updates: the replay leaves the model as is
            ta = type(ga.tcn.contents).from_buffer_copy(ga.tcn.contents)
            bfp = _lib.BnFold.from_buffer_copy(_lib.BnFold.from_address(ta.bn))
            bfp.running_mean = bfp.running_var = bfp.num_batches_tracked = None
            ta.bn = ctypes.addressof(bfp)
            ta._bn_keep = bfp
            ga.tcn = ctypes.pointer(ta)
        launches.append(ga)
    spans = clock_spans(acts) if steps else None
    if spans is not None:
        samples = [spans]
        for k in range(extra_n if extra is not None else 0):
            extra(k)
            torch.cuda.synchronize()
            sp = clock_spans(acts)
            if sp is not None:
                samples.append(sp)
        timing = ("device wall-clock stamps of every workgroup (start, end) of the %d launches of the last "
                  "timed step and of %d more steps of the same captured graphs (read after each), inside "
                  "the steps' graphs" % (len(launches), len(samples) - 1))
        total_ms = sum(sum(sp) for sp in samples) / 1000.0
        rounds = len(samples)
        timing = {"method": timing, "steps_sampled": rounds,
                  "launch_us": [round(float(np.mean([sp[i] for sp in samples])), 2) for i in range(len(spans))],
                  "last_timed_step_launch_us": [round(x, 2) for x in spans]}
    else:
        timing = "captured-graph replay of the last step's %d launches x %d, HIP events" % (len(launches), rounds)
        total_ms = replay_ms(launches, rounds)
        timing = {"method": timing}
    total_flop, total_bytes, count = 0.0, 0.0, 0
    for _ in range(rounds):
        for ga in launches:
            slices = ga.rows // N
            total_flop += slices * (K * 2 * 2.0 * C * N * N + 2.0 * (2 * K + 1) * C * C * N)
            # compulsory bytes: xg + residual in, 2K hop outputs + z out (the
            # hop pieces as bf16 where the bf16 mode stores them so, and its bf16 gram operand
            # copies xg4: X and one hop piece); the last layer (output dead but for BN running
            # stats) stores no hop pieces
            piece_b = 0 if ga.no_pieces else 2 * K * (2.0 if ga.pieces_bf16 else 4.0)
            total_bytes += slices * N * C * (4.0 * 3 + piece_b + (4.0 if ga.xg4 else 0.0))
            if ga.tcn:
                # the layer's gated TCN inside the launch (gwn_gcn_args.tcn): 2C x 2C per row, and
                # its tap-0 input in and (tanh, sigmoid) pairs out (the xg it writes replaces the
                # xg read; tap 1 is the residual row)
                total_flop += slices * N * 2.0 * (2 * C) * (2 * C)
                total_bytes += slices * N * C * (4.0 + 8.0)
            count += 1
    avg_us = 1000.0 * total_ms / count
    achieved = total_flop / (total_ms / 1000.0) / 1e12
    fused = N <= 512
    def pmc(name, key):
        # HBM bytes per launch and MFMA busy fraction from the committed PMC passes of this kernel
        # over this bench (tools/gpu.sh pmc:<cfg> + tools/pmc_summary.py: separate --pmc runs for
        # FETCH_SIZE, WRITE_SIZE and the SQ counters; FETCH x2 per the gfx950 correction)
        # (the newest round's committed passes)
        for rnd in ("r06/final", "r05/final", "r04", "r03"):
            path = os.path.join(ROOT, "profiles", rnd, name)
            if os.path.exists(path):
                with open(path) as f:
                    rec = json.load(f).get(key, {})
                if rec:
                    return rec.get("hbm_bytes_per_dispatch"), rec.get("mfma_busy_frac"), "profiles/%s/%s" % (rnd, name)
        return None, None, None

    def rocprof_avg(name, key):
        # the same kernel's average dispatch duration in the committed rocprofv3 --kernel-trace --stats
        # run of this bench (tools/gpu.sh stats:<cfg>): its packet timestamps also hold the dispatch
        # before the first workgroup and the end-of-kernel release after the last
        import csv
        for rnd in ("r06/final", "r05/final", "r04", "r03"):
            path = os.path.join(ROOT, "profiles", rnd, name)
            if os.path.exists(path):
                with open(path) as f:
                    for r in csv.DictReader(f):
                        if key + "<" in r["Name"]:
                            return round(float(r["AverageNs"]) / 1000.0, 3), "profiles/%s/%s" % (rnd, name)
        return None, None

    def step_mix(name, keys):
        # launches per step of each kernel in the committed one-step trace of this bench
        # (tools/step_trace.py: "<name>  <count>  <us>" summary lines); None unless every key is there
        for rnd in ("r06/final", "r05/final"):
            path = os.path.join(ROOT, "profiles", rnd, name)
            if os.path.exists(path):
                mix = {}
                with open(path) as f:
                    for line in f:
                        parts = line.split()
                        for k in keys:
                            if line.startswith(k + "<") and len(parts) >= 3 and k not in mix:
                                mix[k] = int(parts[-2])
                return mix if len(mix) == len(keys) else None
        return None

    if bf16:
        # bf16 operands: arithmetic intensity (~80 FLOP/B algorithmic) sits far below the bf16
        # ridge (2.5 PF / 8 TB/s = 312 FLOP/B): the kernel is bounded by HBM, priced in bytes
        gbs = total_bytes / (total_ms / 1000.0) / 1e9
        t16b = getattr(acts, "g4bf_arr", None) is not None
        mlpb = getattr(acts, "planes", 1) == 2
        kname = ("gcn_fwd_t16b2_kernel<768> (fused diffusion GCN forward, persistent 16-node tile waves, two "
                 "slices per wave, diffusion and per-piece mlp on bf16 MFMA operands, fp32 accumulation, "
                 "8 launches/step)" if mlpb else
                 "gcn_fwd_t16b_kernel<1024> (fused diffusion GCN forward, persistent 16-node tile waves, diffusion "
                 "on bf16 MFMA operands (mlp in fp32), fp32 accumulation, 8 launches/step)") if t16b else \
            ("gcn_fwd_split_kernel<%d, 1, %d> (fused diffusion GCN forward, bf16 operands, 8 launches/step)"
             % ((N + 31) // 32, (N + 31) // 32))
        pkey = ("gcn_fwd_t16b2_kernel" if mlpb else "gcn_fwd_t16b_kernel") if t16b else "gcn_fwd_split_kernel"
        traffic, mfma_busy, src = pmc("pmc_bench_pems.json", pkey) if N == 325 else (None,) * 3
        timing["rocprof_avg_us"], timing["rocprof_source"] = (rocprof_avg("pems_kernel_stats.csv", pkey)
                                                              if N == 325 else (None, None))
        mix = step_mix("step_pems.txt", ("gcn_fwd_t16b2_kernel", "gcn_fwd_t16b_kernel")) \
            if N == 325 and mlpb and t16b else None
        if mix:
            # the step's 8 launches are a mix: two slices per wave where a layer has >= 10 pairs
            # per CU, one slice per wave below (round 6); traffic, MFMA busy and the rocprof
            # average are the launch-weighted means over the committed one-step trace's counts
            recs = [pmc("pmc_bench_pems.json", k) for k in mix]
            avgs = [rocprof_avg("pems_kernel_stats.csv", k) for k in mix]
            if all(r[0] is not None for r in recs) and all(a[0] is not None for a in avgs):
                tot = float(sum(mix.values()))
                traffic = round(sum(mix[k] * r[0] for k, r in zip(mix, recs)) / tot)
                mfma_busy = round(sum(mix[k] * r[1] for k, r in zip(mix, recs)) / tot, 4)
                timing["rocprof_avg_us"] = round(sum(mix[k] * a[0] for k, a in zip(mix, avgs)) / tot, 3)
                timing["launch_mix"] = dict(mix)
                kname = ("gcn_fwd_t16b2_kernel<768> x %d + gcn_fwd_t16b_kernel<1024, true> x %d (fused "
                         "diffusion GCN forward, persistent 16-node tile waves, two slices per wave on "
                         "the layers with >= 10 pairs per CU, one below; diffusion and per-piece mlp on "
                         "bf16 MFMA operands, fp32 accumulation, 8 launches/step)" % tuple(mix.values()))
        return {"kernel": kname,
                "bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": src,
                "pmc_mfma_busy_frac": mfma_busy,
                "mfma_tflops": round(achieved, 3), "mfma_peak_bf16": BF16_PEAK_TFLOPS,
                "avg_launch_us": round(avg_us, 3), "flop_per_launch_avg": round(total_flop / count, 1),
                "algorithmic_bytes_per_launch": round(total_bytes / count), "launches_timed": count,
                "timing": timing}
    t16 = fused and ex._pow_ok(1) and os.environ.get("GWN_GCN_T16", "1") != "0"
    traffic, mfma_busy, src = pmc("pmc_bench_metr.json", "gcn_fwd_t16_kernel") if t16 and N == 207 else (None,) * 3
    # (the committed rocprof pass of the driver's exact command, `python bench.py`, when present:
    # the stats:metr pass also holds the post-timing legs' slower launches)
    if t16 and N == 207:
        timing["rocprof_avg_us"], timing["rocprof_source"] = rocprof_avg("default_cmd_kernel_stats.csv",
                                                                         "gcn_fwd_t16_kernel")
        if timing["rocprof_avg_us"] is None:
            timing["rocprof_avg_us"], timing["rocprof_source"] = rocprof_avg("metr_kernel_stats.csv",
                                                                             "gcn_fwd_t16_kernel")
    else:
        timing["rocprof_avg_us"], timing["rocprof_source"] = None, None
    if fused:
        kname = (("gcn_fwd_t16_kernel<1024> (fused diffusion GCN forward, power schedule, persistent 16-node "
                  "tile waves: one workgroup per CU over an equal tile range; the layer's gated TCN and the "
                  "layer below's BatchNorm finalize in its staging where >= a slice per CU" if t16 else
                  "gcn_fwd_pow_kernel<512> (fused diffusion GCN forward, power schedule")
                 + ", 8 launches/step)" if ex._pow_ok(1) else "gcn_fwd_fused_kernel<512, true> (fused diffusion GCN forward, chained hops, "
                                       "8 launches/step)")
    else:
        kname = "gwn_gcn_fwd large-graph schedule (batched diffusion GEMMs + mlp, 8 calls/step)"
    return {"kernel": kname,
            "bound": "mfma", "achieved": round(achieved, 3), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / FP32_PEAK_TFLOPS, 4), "traffic": traffic,
            "traffic_source": src,
            "pmc_mfma_busy_frac": mfma_busy,
            "avg_launch_us": round(avg_us, 3), "flop_per_launch_avg": round(total_flop / count, 1),
            "algorithmic_bytes_per_launch": round(total_bytes / count),
            "launches_timed": count, "timing": timing}


def oracle_mae12(eng, sups_np, xt, yt, N, T):
    """12-step masked MAE of the fp64 CPU oracle (checker only) on the trained weights."""
    from oracle import gwnet_oracle as orc
    sd = {k: v.detach().cpu().numpy() for k, v in eng.model.state_dict().items()}
    p = {k: torch.tensor(v, dtype=torch.float64) for k, v in sd.items()}
    out = orc.forward(p, [torch.tensor(s, dtype=torch.float64) for s in sups_np],
                      torch.tensor(xt, dtype=torch.float64), orc.Cfg(N, out_dim=T), False, p)
    pred = out.transpose(1, 3)[:, 0] * eng.scaler.std + eng.scaler.mean
    real = torch.tensor(yt, dtype=torch.float64)
    return float(np.mean([orc.masked_metrics(pred[:, :, h], real[:, :, h])[0].item() for h in range(T)]))


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(seconds, cfg):
    """The CPU restatement (oracle/, kind "port") timing the same training step on the host
    cores: fp32, autograd backward, clip + Adam; 3 warm-up steps (1 at N=2048), then the median of
    >= 5 timed steps (>= 3 at N=2048, where a sample step is B=1) -- the BASELINE.md §3 / SURVEY
    §8d protocol.  Threads: os.cpu_count(), capped by the job's CPU share where the launcher states
    one (OMP_NUM_THREADS; the GPU box gives each 1-GPU job 16 of the machine's cores and
    os.cpu_count() reports the whole machine)."""
    from gwn_amd import synthetic
    from gwn_amd.model import gwnet
    from oracle import gwnet_oracle as orc
    N, T = cfg["N"], cfg["T"]
    nproc = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(nproc, share) if share > 0 else nproc
    torch.set_num_threads(threads)
    ocfg = orc.Cfg(N, out_dim=T, dropout=0.3)
    torch.manual_seed(999)
    m = gwnet("cpu", N, 0.3, supports=[torch.zeros(N, N), torch.zeros(N, N)], out_dim=T)
    sd = {k: v.numpy() for k, v in m.state_dict().items()}
    adj = synthetic.random_sensor_graph(N, seed=cfg["graph_seed"], dense=cfg["dense"])
    tr = orc.Trainer(sd, synthetic.double_transition(adj), ocfg, dtype=torch.float32)
    bsz = cfg["sample_b"]
    x, y = synthetic.synthetic_batch(bsz, N, T, seed=5)
    big = N > 512
    for _ in range(1 if big else 3):
        tr.train(x, y)  # warm-up
    times = []
    t0 = time.perf_counter()
    while True:
        t1 = time.perf_counter()
        tr.train(x, y)
        times.append(time.perf_counter() - t1)
        if len(times) >= (3 if big else 5) and (time.perf_counter() - t0 >= seconds or len(times) >= 30):
            break
    med = float(np.median(times))
    return {"value": round(bsz / med, 3), "unit": "samples/s", "cores": threads, "kind": "port",
            "nproc": nproc, "cpu_model": _cpu_model(), "statistic": "median",
            "sample": "median of %d timed train steps of B=%d (N=%d, T=%d, fp32, dropout 0.3, clip + Adam), "
                      "%.2f s/step, %d threads; the oracle was calibrated in the build container at 38.4 vs "
                      "34.9 samples/s for the reference itself (METR-LA B=64, 8 threads)"
                      % (len(times), bsz, N, T, med, threads)}


if __name__ == "__main__":
    main()
