"""Drop-in ``trainer`` (reference engine.py:9-58, 119-130) on the libgwn hot path.

``trainer.train`` is one fused step: pad (engine.py:44) -> gwnet forward -> masked MAE + its
gradient (engine.py:46-51, util.py:527-538) -> hand-written backward -> clip_grad_norm_(5) ->
Adam (engine.py:52-55), all as libgwn launches on the current stream, followed by ONE device->host
copy of (loss, mape, rmse) -- the reference does three ``.item()`` syncs (engine.py:56-58).
"""
import os

import torch

from . import _lib, util
from ._lib import ptr
from .model import gwnet, gwnet_diff_G

F32 = torch.float32
_NO_CLIP = 3.0e38


class FlatAdam(torch.optim.Optimizer):
    """``torch.optim.Adam`` semantics (L2 weight decay, bias correction, amsgrad=False) over the
    model's flat parameter buffer, executed by ``gwn_adam_clipped`` in one launch."""

    def __init__(self, model, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(model.parameters(), dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.model = model
        flat = model._flat
        self.exp_avg = torch.zeros_like(flat)
        self.exp_avg_sq = torch.zeros_like(flat)
        self.grad_flat = torch.zeros_like(flat)
        self.step_t = torch.zeros(1, device=flat.device, dtype=torch.long)
        self.total_norm = torch.zeros(1, device=flat.device, dtype=F32)
        self._ranges_key = None
        self._ws = torch.zeros(_lib.load().gwn_clip_adam_workspace_floats(flat.numel()) + 16,
                               device=flat.device, dtype=F32)

    def _ranges(self, names):
        key = tuple(names)
        if key != self._ranges_key:
            lay = self.model._executor.layout
            rs = []
            for n in names:
                off, shape = lay.flat_off[n]
                numel = 1
                for s in shape:
                    numel *= s
                if rs and rs[-1][1] == off:
                    rs[-1][1] = off + numel
                else:
                    rs.append([off, off + numel])
            dev = self.model._flat.device
            self._lo = torch.tensor([r[0] for r in rs], dtype=torch.long, device=dev)
            self._hi = torch.tensor([r[1] for r in rs], dtype=torch.long, device=dev)
            self._nr = len(rs)
            self._active = sum(r[1] - r[0] for r in rs)
            self._ranges_key = key
        return self._lo, self._hi, self._nr, self._active

    def apply(self, names, max_norm, norm_ready=False, seed=None):
        """clip (max_norm; huge = off) + Adam over the flat ranges of ``names``; grads in grad_flat.
        norm_ready: the clip-norm partials are already in the workspace (gwn_gather_sqnorm wrote them
        while unpacking the gradient): one launch.  seed: a device counter advanced by 1 by the same
        launch (the dropout counter of the step)."""
        g = self.param_groups[0]
        lo, hi, nr, active = self._ranges(names)
        args = (ptr(self.model._flat), ptr(self.grad_flat), ptr(self.exp_avg), ptr(self.exp_avg_sq), ptr(lo), ptr(hi),
                nr, active, float(max_norm), float(g["lr"]), float(g["betas"][0]), float(g["betas"][1]),
                float(g["eps"]), float(g["weight_decay"]), ptr(self.step_t), ptr(self._ws), ptr(self.total_norm))
        if not norm_ready:
            _lib.call("gwn_sqnorm_partials", ptr(self.grad_flat), ptr(lo), ptr(hi), nr, active, ptr(self._ws),
                      _lib.stream())
        _lib.call("gwn_adam_clipped", *args, ptr(seed), 1 if seed is not None else 0, _lib.stream())

    @torch.no_grad()
    def step(self, closure=None):
        """Generic path (grads left in ``p.grad`` by autograd): gather them and run Adam."""
        loss = closure() if closure is not None else None
        model = self.model
        model._ensure_flat()
        lay = model.executor().layout
        names = []
        for name, p in model.named_parameters():
            if p.grad is None:
                continue
            off, shape = lay.flat_off[name]
            self.grad_flat[off:off + p.numel()].copy_(p.grad.reshape(-1))
            names.append(name)
        if names:
            self.apply(names, _NO_CLIP)
        return loss


class trainer():
    def __init__(self, scaler, in_dim, seq_length, num_nodes, nhid, dropout, lrate, wdecay, device, supports,
                 gcn_bool, addaptadj, aptinit, blocks, layers):
        if isinstance(supports, dict):
            # a different graph per sample (engine.py:14-25): supports = {state: [support stacks]}
            supports_len = len(next(iter(supports.values())))
            if gcn_bool and addaptadj:
                supports_len += 1
            self.model = gwnet_diff_G(device, num_nodes, dropout, supports_len, gcn_bool=gcn_bool,
                                      addaptadj=addaptadj, in_dim=in_dim, out_dim=seq_length,
                                      residual_channels=nhid, dilation_channels=nhid, skip_channels=nhid * 8,
                                      end_channels=nhid * 16, blocks=blocks, layers=layers)
        else:
            self.model = gwnet(device, num_nodes, dropout, supports=supports, gcn_bool=gcn_bool,
                               addaptadj=addaptadj, aptinit=aptinit, in_dim=in_dim, out_dim=seq_length,
                               residual_channels=nhid, dilation_channels=nhid, skip_channels=nhid * 8,
                               end_channels=nhid * 16, blocks=blocks, layers=layers)
        self.model.to(device)
        self.optimizer = FlatAdam(self.model, lr=lrate, weight_decay=wdecay)
        self.loss = util.masked_mae
        self.scaler = scaler
        self.clip = 5
        self.supports = supports
        self.aptinit = aptinit
        self.state = None
        self._acts = {}
        self._host_metrics = torch.zeros(4, dtype=F32).pin_memory() if torch.cuda.is_available() else None
        self._metrics_ready = torch.cuda.Event() if torch.cuda.is_available() else None
        self._metrics_early = False
        # HIP-graph replay of the fused training step (GWN_GRAPHS=0 disables): the ~240 launches
        # of a step are captured once per (shape, hyper-parameter) key and replayed
        self.use_graphs = os.environ.get("GWN_GRAPHS", "1") != "0"
        self.dp_probe = None  # data-parallel collective timing (bench.py; _probe_event)
        self._graphs = {}
        self._eager_runs = {}

    # ------------------------------------------------------------------------------------------
    def _phase_grads(self, input, real_val, training):
        """pad -> forward -> masked loss (+ its gradient) -> backward -> flat gradient buffer."""
        m, acts, dout = self._phase_loss(input, real_val, training)
        if training:
            self._phase_backward(acts, dout)
        return m

    def _phase_backward(self, acts, dout):
        ex = self.model._executor
        ex.backward(acts, dout)
        # single process: the unpack also leaves the clip-norm partials for the update; data
        # parallel: the norm is taken after the all-reduce
        self._norm_ready = not self._distributed()
        ex.unpack_grads(self.optimizer.grad_flat, self.optimizer._ws if self._norm_ready else None)

    def _early_range(self, acts):
        """Data parallel: the flat gradient range final after the backward's head stage
        (Executor.early_grad_range), whose all-reduce overlaps the layers' backward; None in a
        single process or without one.
        GWN_DP_OVERLAP=0: one all-reduce of the whole gradient after the backward."""
        ex = self.model._executor
        if not self._distributed() or os.environ.get("GWN_DP_OVERLAP", "1") == "0":
            return None
        return ex.early_grad_range()

    def _backward_split(self, acts, dout, between):
        """The backward in two parts around between(): the head stage plus the gather of the early
        gradient range, then the layers and the gather of the rest (data parallel only)."""
        ex = self.model._executor
        a, b = self._early_range(acts)
        gf = self.optimizer.grad_flat
        stages = ex.backward_stages(acts, dout)
        next(stages)
        ex.unpack_grads_range(gf, a, b)
        between(1)
        for _ in stages:
            pass
        ex.unpack_grads_range(gf, 0, a)
        ex.unpack_grads_range(gf, b, ex.layout.flat_total)
        self._norm_ready = False
        between(2)

    def _phase_loss(self, input, real_val, training):
        """pad -> forward -> masked loss (+ its gradient); returns (metrics, saved state, dout)."""
        model = self.model
        ex = model._executor
        B, _, _, T = input.shape
        ts = ex.cfg.times(T + 1)  # engine.py:44 pads one step on the left before the forward
        key = (B, tuple(ts), training)
        acts = self._acts.get(key)
        out, acts = ex.forward(model._flat, model._fixed_supports(), input, training, model._bn_bufs(),
                               fixed_t=model._fixed_supports_t(),
                               acts=acts, lead_pad=1, want_out=False)
        self._acts[key] = acts
        sc = ex.scratch(B, ts)
        rs = real_val.stride()
        # the loss reads the head's rows and writes the output gradient in the backward's row layout
        # (no NCHW round trip; the gradient stays in scratch "dy")
        cfg = ex.cfg
        _lib.call("gwn_masked_loss_rows", ptr(acts.y), cfg.O, ptr(real_val), rs[0], rs[1], rs[2], B, cfg.O, cfg.N,
                  ts[-1], float(self.scaler.mean), float(self.scaler.std), ptr(sc["metrics"]),
                  ptr(sc["dy"]) if training else None, cfg.OP, ptr(sc["ws"]), _lib.stream())
        return sc["metrics"], acts, None

    def _eval_lean(self, input, real_val):
        """engine.py:119-130 on the lean inference schedule: pad 1, eval forward (no saved state),
        the three masked metrics from one HIP reduction (no gradient)."""
        model = self.model
        ex = model._executor
        out, bf = ex.infer(model._flat, model._fixed_supports(), input, model._bn_bufs(), lead_pad=1)
        B = input.shape[0]
        rs = real_val.stride()
        _lib.call("gwn_masked_loss", ptr(out), ptr(real_val), rs[0], rs[1], rs[2], B, ex.cfg.O, ex.cfg.N,
                  out.shape[3], float(self.scaler.mean), float(self.scaler.std), ptr(bf["metrics"]), None,
                  ptr(bf["ws"]), _lib.stream())
        return bf["metrics"]

    def _phase_update(self):
        """clip_grad_norm_(clip) + Adam on the flat buffers; advance the dropout counter."""
        model = self.model
        ex = model._executor
        clip = self.clip if self.clip is not None else _NO_CLIP
        # one launch: clip + Adam, the step counter and the dropout counter
        self.optimizer.apply(ex.layout.active, clip, norm_ready=getattr(self, "_norm_ready", False),
                             seed=ex.seed if model.dropout > 0 else None)
        self._norm_ready = False

    def _distributed(self):
        dist = torch.distributed
        return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1

    def _step(self, input, real_val, training):
        """Fused step; returns the device metrics tensor [mae, mape, rmse]."""
        model = self.model
        if model.training != training:
            model.train(training)
        ex = model.executor()
        if not training:
            if ex.infer_ok():
                return self._eval_lean(input, real_val)
            return self._phase_grads(input, real_val, False)
        g = self.optimizer.param_groups[0]
        # everything the captured graph bakes in: shapes, hyper-parameters (kernel arguments), the
        # flat parameter buffer and the padded supports (device pointers), scaler and BN constants.
        # The padded supports are rebuilt (new buffers, a new generation) whenever the supports
        # change: every graph and saved activation set that points at the old ones is dropped
        model._fixed_supports()
        sup_key = getattr(model, "_sup_gen", 0)
        if sup_key != getattr(self, "_sup_gen_seen", sup_key):
            self._graphs.clear()
            self._acts.clear()
            self._eager_runs.clear()
        self._sup_gen_seen = sup_key
        bn_key = tuple((m.momentum, m.eps) for m in model.bn)
        key = (tuple(input.shape), tuple(real_val.shape), float(g["lr"]), tuple(g["betas"]), float(g["eps"]),
               float(g["weight_decay"]), self.clip, float(model.dropout), model._flat.data_ptr(), sup_key, bn_key,
               float(self.scaler.mean), float(self.scaler.std), model.compute_dtype)
        if self.use_graphs and key in self._graphs:
            return self._replay(key, input, real_val)
        if self.use_graphs and self._eager_runs.get(key, 0) >= 1:
            self._capture(key, input, real_val)
            return self._replay(key, input, real_val)
        self._eager_runs[key] = self._eager_runs.get(key, 0) + 1
        m, acts, dout = self._phase_loss(input, real_val, True)
        if self._early_range(acts) is not None:
            self._backward_split(acts, dout, self._overlap_hook())
        else:
            self._phase_backward(acts, dout)
            self._allreduce_grads()
        self._phase_update()
        return m

    def _capture(self, key, input, real_val):
        """Capture the step as graphs: g0 = forward + loss, g1 = backward (+ clip + Adam in a single
        process; data parallel: the all-reduce stays eager between g1 and g2 = clip + Adam).  The
        metrics are read back between g0 and g1 (_replay), so train() returns while the GPU still
        runs the backward and the host prepares the next step meanwhile: no idle GPU between steps."""
        sx = torch.empty_like(input).copy_(input)
        sy = torch.empty_like(real_val).copy_(real_val)
        torch.cuda.synchronize()
        g0 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g0):
            m, acts, dout = self._phase_loss(sx, sy, True)
        g1 = torch.cuda.CUDAGraph()
        g1b = None
        if self._early_range(acts) is not None:
            # data parallel: the backward in two graphs; between them the early range's all-reduce
            # is issued on a side stream, beside the second graph (_replay)
            g1b = torch.cuda.CUDAGraph()
            ctx = [torch.cuda.graph(g1, pool=g0.pool())]
            ctx[0].__enter__()

            def between(part):
                if part == 1:
                    ctx[0].__exit__(None, None, None)
                    ctx[0] = torch.cuda.graph(g1b, pool=g0.pool())
                    ctx[0].__enter__()
                else:
                    ctx[0].__exit__(None, None, None)

            self._backward_split(acts, dout, between)
        else:
            with torch.cuda.graph(g1, pool=g0.pool()):
                self._phase_backward(acts, dout)
                if not self._distributed():
                    self._phase_update()
        g2 = None
        if self._distributed():
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2, pool=g0.pool()):
                self._phase_update()
        # acts (and the scratch dy the loss wrote) live on; the entry keeps them referenced
        self._graphs[key] = (g0, (g1, g1b), g2, sx, sy, m, (acts, dout))

    def _replay(self, key, input, real_val):
        g0, g1, g2, sx, sy, m, _ = self._graphs[key]
        if sx.data_ptr() != input.data_ptr():
            sx.copy_(input)
        if sy.data_ptr() != real_val.data_ptr():
            sy.copy_(real_val)
        g0.replay()
        if self._host_metrics is not None:
            # the three metrics leave as soon as the loss is known; _read waits for this event only
            self._host_metrics[:3].copy_(m[:3], non_blocking=True)
            self._metrics_ready.record()
            self._metrics_early = True
        g1, g1b = g1
        g1.replay()
        if g1b is not None:
            hook = self._overlap_hook()
            hook(1)
            self._probe_event("layers_0")
            g1b.replay()
            self._probe_event("layers_1")
            hook(2)
            g2.replay()
        elif g2 is not None:
            self._probe_event("rest_0")
            self._allreduce_grads()
            self._probe_event("rest_1")
            g2.replay()
        return m

    def _probe_event(self, name, stream=None):
        """Data-parallel probe (bench.py, outside the timed region): with ``dp_probe`` a list, a
        timing event per collective boundary into its last dict (dp_probe_summary)."""
        if self.dp_probe is None or not self.dp_probe:
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(stream if stream is not None else torch.cuda.current_stream())
        self.dp_probe[-1][name] = ev

    def dp_probe_summary(self):
        """Mean device times (ms) over the probed steps: the early range's all-reduce on the side
        stream (early_allreduce), the layers' backward it overlaps (layers_backward), the part of the
        early all-reduce that ran inside that backward (early_overlapped), and the all-reduce of the
        rest on the main stream plus the join (rest_allreduce)."""
        torch.cuda.synchronize()
        acc = {}
        for evs in self.dp_probe or []:
            def el(a, b):
                return evs[a].elapsed_time(evs[b]) if a in evs and b in evs else None
            vals = {"early_allreduce": el("early_0", "early_1"), "layers_backward": el("layers_0", "layers_1"),
                    "rest_allreduce": el("rest_0", "rest_1")}
            if vals["early_allreduce"] is not None and vals["layers_backward"] is not None:
                # overlap of [early_0, early_1] with [layers_0, layers_1] on the device clock
                s0, s1 = el("layers_0", "early_0"), el("layers_0", "early_1")
                vals["early_overlapped"] = max(0.0, min(s1, vals["layers_backward"]) - max(s0, 0.0))
            for k, v in vals.items():
                if v is not None:
                    acc.setdefault(k, []).append(v)
        return {k + "_ms": round(sum(v) / len(v), 4) for k, v in acc.items()}

    def _overlap_hook(self):
        """between(part) for _backward_split in a data-parallel step: part 1 (after the head stage
        and the early range's gather) starts that range's all-reduce on a side stream; part 2 (after
        the rest of the backward) all-reduces the rest on the current stream and joins the side
        stream, so clip + Adam see every averaged gradient."""
        ex = self.model._executor
        a, b = ex.early_grad_range()
        gf = self.optimizer.grad_flat
        if getattr(self, "_dp_side", None) is None:
            self._dp_side = torch.cuda.Stream(device=gf.device)
        side = self._dp_side
        main = torch.cuda.current_stream()

        def between(part):
            if part == 1:
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    self._probe_event("early_0", side)
                    self._allreduce(gf[a:b])
                    self._probe_event("early_1", side)
            else:
                self._probe_event("rest_0")
                if a > 0:
                    self._allreduce(gf[:a])
                if b < gf.numel():
                    self._allreduce(gf[b:])
                main.wait_stream(side)
                self._probe_event("rest_1")

        return between

    @staticmethod
    def _allreduce(g):
        dist = torch.distributed
        if dist.get_backend() == "nccl":
            dist.all_reduce(g, op=dist.ReduceOp.AVG)
        else:
            dist.all_reduce(g, op=dist.ReduceOp.SUM)
            g.div_(dist.get_world_size())

    def _allreduce_grads(self):
        """Data parallel (one process per GPU): average the flat gradient over ranks with ONE
        collective (RCCL all-reduce over xGMI for the "nccl" backend), before clip + Adam, i.e.
        DistributedDataParallel semantics with per-replica BatchNorm (the reference has no
        SyncBN).  A no-op without an initialised process group."""
        dist = torch.distributed
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
            return
        g = self.optimizer.grad_flat
        if dist.get_backend() == "nccl":
            dist.all_reduce(g, op=dist.ReduceOp.AVG)
        else:
            dist.all_reduce(g, op=dist.ReduceOp.SUM)
            g.div_(dist.get_world_size())

    def broadcast_parameters(self, src=0):
        """Make every rank start from rank ``src``'s weights (DDP's construction-time broadcast)."""
        dist = torch.distributed
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            dist.broadcast(self.model._flat, src)
            for m in self.model.bn:
                dist.broadcast(m.running_mean, src)
                dist.broadcast(m.running_var, src)

    def _fused_ok(self, input, real_val):
        """The fused step indexes real_val as [B, N, out_dim] (engine.py:47-51 broadcasts the
        prediction [B, T_f, N, out_dim] against real_val[:, None]); any other shape takes the
        autograd path, where torch's broadcasting rules (and errors) apply as in the reference."""
        if isinstance(self.model, gwnet_diff_G):
            return False  # its forward needs per-sample supports: the reference's train() cannot call it
        cfg = self.model.executor().cfg
        return (self.loss is util.masked_mae and input.is_cuda and input.dtype == F32 and input.dim() == 4
                and real_val.dtype == F32 and real_val.is_cuda
                and tuple(real_val.shape) == (input.shape[0], cfg.N, cfg.O))

    def train(self, input, real_val):
        if not self._fused_ok(input, real_val):
            return self._train_autograd(input, real_val)
        m = self._step(input, real_val, True)
        self._expose_grads()
        return self._read(m)

    def eval(self, input, real_val):
        if not self._fused_ok(input, real_val):
            return self._eval_autograd(input, real_val)
        with torch.no_grad():
            m = self._step(input, real_val, False)
        return self._read(m)

    def _read(self, m):
        if self._metrics_early:
            # replayed step: the metrics were copied right after the loss; the backward and the
            # update stay queued behind them (stream order keeps every later use of the parameters
            # and gradients correct, as for any asynchronous torch work)
            self._metrics_early = False
            self._metrics_ready.synchronize()
            v = self._host_metrics.tolist()
        elif self._host_metrics is not None:
            self._host_metrics[:3].copy_(m[:3], non_blocking=True)
            torch.cuda.current_stream().synchronize()
            v = self._host_metrics.tolist()
        else:
            v = m.tolist()
        return v[0], v[1], v[2]

    def _expose_grads(self):
        """Make ``p.grad`` views of the flat gradient buffer (as after the reference's step).
        The (param, view) pairs are built once per (layout, gradient buffer)."""
        lay = self.model._executor.layout
        gf = self.optimizer.grad_flat
        key = (id(lay), gf.data_ptr())
        if getattr(self, "_grad_views_key", None) != key:
            active = set(lay.active)
            views = []
            for name, p in self.model.named_parameters():
                if name in active:
                    off, shape = lay.flat_off[name]
                    views.append((p, gf[off:off + p.numel()].view(shape)))
            self._grad_views, self._grad_views_key = views, key
        for p, g in self._grad_views:
            if p.grad is not g:
                p.grad = g

    # ------------------------------------------------------------------------------------------
    # the synthetic F/E task with per-sample graphs (engine.py:60-117, 132-178)
    def set_state(self, state):
        assert state == 'train' or state == 'val' or state == 'test'
        self.state = state

    def _syn_forward(self, input, adj_idx):
        input = torch.nn.functional.pad(input, (1, 0, 0, 0))
        if adj_idx is None:
            return self.model(input)
        assert self.state is not None, 'set train/val/test state first'
        supports = self.supports[self.state]
        supports = [supports[i][adj_idx] for i in range(len(supports))]
        aptinit = self.aptinit[self.state]
        if aptinit is not None:
            aptinit = aptinit[adj_idx]
        return self.model(input, supports, aptinit)

    @staticmethod
    def _syn_pool(predict, F_t, G, adj_idx, pooltype):
        """F: the prediction averaged over consecutive groups of F_t output steps and expanded back;
        E: every cluster of G.assign_dict replaced by its node mean (engine.py:86-105).  The E pooling
        writes into ``predict`` in place, as the reference does."""
        F = None
        if pooltype == 'avg':
            F = predict.reshape(*predict.shape[:-1], -1, F_t).mean(-1)
            F = F.unsqueeze(-1).repeat(*[1] * len(F.shape), F_t)
            F = F.view(*F.shape[:-2], -1)
            if not isinstance(G, list):
                assign_dict = G.assign_dict
                for k in range(len(assign_dict)):
                    predict[:, :, assign_dict[k], :] = predict[:, :, assign_dict[k], :].mean(
                        2, keepdim=True).repeat(1, 1, len(assign_dict[k]), 1)
            else:
                for sample in range(len(predict)):
                    assign_dict = G[adj_idx[sample]].assign_dict
                    for k in range(len(assign_dict)):
                        predict[sample:sample + 1, :, assign_dict[k], :] = predict[sample:sample + 1, :, assign_dict[k], :].mean(
                            2, keepdim=True).repeat(1, 1, len(assign_dict[k]), 1)
        return F, predict

    def train_syn(self, input, real, F_t, G, adj_idx=None, pooltype='avg'):
        """engine.py:60-117: output p = 1 sequence, pooled to F (time) and E (graph clusters)."""
        self.model.train()
        self.optimizer.zero_grad()
        output = self._syn_forward(input, adj_idx).transpose(1, 3)
        predict = self.scaler.inverse_transform(output)
        F, predict = self._syn_pool(predict, F_t, G, adj_idx, pooltype)
        loss = self.loss(torch.cat((F, predict), 1), real, 0.0)
        loss.backward()
        if self.clip is not None:
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.clip)
        self.optimizer.step()
        mape = util.masked_mape(predict, real, 0.0).item()
        rmse = util.masked_rmse(predict, real, 0.0).item()
        return loss.item(), mape, rmse

    def eval_syn(self, input, real, F_t, G, adj_idx=None, pooltype='avg'):
        """engine.py:132-178: the same pooling in eval mode; also returns (F, predict)."""
        same_G = not isinstance(G, list)
        self.model.eval()
        if not same_G:
            assert adj_idx is not None, 'adj index needed.'
        with torch.no_grad():
            output = self._syn_forward(input, None if same_G else adj_idx)
        output = output.transpose(1, 3)
        predict = self.scaler.inverse_transform(output)
        F, predict = self._syn_pool(predict, F_t, G, adj_idx, pooltype)
        loss = self.loss(torch.cat((F, predict), 1), real, 0.0)
        mape = util.masked_mape(predict, real, 0.0).item()
        rmse = util.masked_rmse(predict, real, 0.0).item()
        return loss.item(), mape, rmse, F, predict

    # ------------------------------------------------------------------------------------------
    # generic path for a user-supplied loss: the model is still one libgwn autograd node
    def _train_autograd(self, input, real_val):
        self.model.train()
        self.optimizer.zero_grad()
        input = torch.nn.functional.pad(input, (1, 0, 0, 0))
        output = self.model(input).transpose(1, 3)
        real = torch.unsqueeze(real_val, dim=1)
        predict = self.scaler.inverse_transform(output)
        loss = self.loss(predict, real, 0.0)
        loss.backward()
        if self.clip is not None:
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.clip)
        self.optimizer.step()
        mape = util.masked_mape(predict, real, 0.0).item()
        rmse = util.masked_rmse(predict, real, 0.0).item()
        return loss.item(), mape, rmse

    def _eval_autograd(self, input, real_val):
        self.model.eval()
        input = torch.nn.functional.pad(input, (1, 0, 0, 0))
        output = self.model(input).transpose(1, 3)
        real = torch.unsqueeze(real_val, dim=1)
        predict = self.scaler.inverse_transform(output)
        loss = self.loss(predict, real, 0.0)
        mape = util.masked_mape(predict, real, 0.0).item()
        rmse = util.masked_rmse(predict, real, 0.0).item()
        return loss.item(), mape, rmse


__all__ = ["trainer", "FlatAdam"]
