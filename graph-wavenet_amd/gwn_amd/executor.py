"""Step executor: runs gwnet's forward / backward as a fixed schedule of libgwn launches.

Reference semantics (model.py:175-241 forward, engine.py:41-58 train step) restated on the
internal "slab-major, channels-last" layout of include/gwn.h: a reference NCHW tensor
[B, C, N, T] lives here as rows (t, b, n) x C channels.  One time step = a slab of P = B*N rows.

Per layer i (input X_i with T_i steps, dilation d_i, output T_{i+1} = T_i - d_i):
  gated TCN   -> xg (piece 0 of the gcn concat H_i), (tanh, sigmoid) saved in FG_i,
                 last T_f slabs copied into SKIPCAT[:, i*C:(i+1)*C]       (model.py:206-222)
  gcn         -> H_i pieces 1..2K by diffusion, Z_i = dropout(mlp(H_i)) + X_i[last T_{i+1}]
                                                                        (model.py:41-55, 234)
  batchnorm   -> X_{i+1}                                                   (model.py:236)
After the layers: SKR = relu(SKIPCAT Wskip^T + sum_i b_i) (only the last T_f steps of every
skip term reach the output, model.py:216-222, 238), E1 = relu(end_conv_1), Y = end_conv_2.
"""
import ctypes
import os
import warnings
from collections import OrderedDict

import torch

from . import _lib
from ._lib import ptr

F32 = torch.float32


class PackedLayout:
    """Kernel-friendly packing of the parameters (and, with the same offsets, of their grads).

    ``pidx``: packed[i] = flat[pidx[i]];  ``uidx``: grad_flat[j] = grad_packed[uidx[j]] (inactive
    parameters point at a trailing zero slot).  ``flat`` is the model's parameter buffer in
    registration (== state_dict) order.
    """

    def __init__(self, model, cfg=None):
        cfg = cfg if cfg is not None else Config(model)
        C, D, K, Cin, S, E, O, L = cfg.C, cfg.D, cfg.K, cfg.Cin, cfg.S, cfg.E, cfg.O, cfg.L
        names = [n for n, _ in model.named_parameters()]
        flat_off = {}
        o = 0
        for n, p in model.named_parameters():
            flat_off[n] = (o, p.shape)
            o += p.numel()
        self.flat_total = o
        segs = OrderedDict()
        pidx = []
        grad_src = {}  # flat param name -> packed index tensor (same shape as the param)

        def add(name, numel):
            segs[name] = (len(pidx), numel)

        def gather_seg(name, src_index):
            # src_index: LongTensor of flat indices, in packed order.  Segments start 16-B aligned
            # (the row-tile GEMMs load weights as float4).
            while len(pidx) % 4:
                pidx.append(0)
            segs[name] = (len(pidx), src_index.numel())
            pidx.extend(src_index.tolist())

        def flat_range(pname):
            off, shape = flat_off[pname]
            n = 1
            for s in shape:
                n *= s
            return torch.arange(off, off + n, dtype=torch.long).view(shape)

        def map_grad(pname, packed_index):
            grad_src[pname] = packed_index

        def seg_index(name, shape):
            start, numel = segs[name]
            return torch.arange(start, start + numel, dtype=torch.long).view(shape)

        # start conv
        gather_seg("start_w", flat_range("start_conv.weight").reshape(C, Cin).reshape(-1))
        map_grad("start_conv.weight", seg_index("start_w", (C, Cin, 1, 1)))
        gather_seg("start_b", flat_range("start_conv.bias"))
        map_grad("start_conv.bias", seg_index("start_b", (C,)))
        if cfg.adp_params:
            gather_seg("nv1", flat_range("nodevec1").reshape(-1))
            gather_seg("nv2", flat_range("nodevec2").reshape(-1))
            if cfg.adp_live:
                map_grad("nodevec1", seg_index("nv1", tuple(flat_off["nodevec1"][1])))
                map_grad("nodevec2", seg_index("nv2", tuple(flat_off["nodevec2"][1])))
        for i in range(L):
            fw = flat_range("filter_convs.%d.weight" % i).reshape(D, C, K)   # [co][ci][tap]
            gw = flat_range("gate_convs.%d.weight" % i).reshape(D, C, K)
            # packed [2D rows j=2co+g][K*C cols k=tap*C+ci]
            both = torch.stack([fw, gw], dim=1)  # [co][g][ci][tap]
            packed = both.permute(0, 1, 3, 2).reshape(2 * D, K * C)
            gather_seg("fg_w%d" % i, packed.reshape(-1))
            idx = seg_index("fg_w%d" % i, (D, 2, K, C))  # [co][g][tap][ci]
            map_grad("filter_convs.%d.weight" % i, idx[:, 0].permute(0, 2, 1).reshape(D, C, 1, K))
            map_grad("gate_convs.%d.weight" % i, idx[:, 1].permute(0, 2, 1).reshape(D, C, 1, K))
            fb = flat_range("filter_convs.%d.bias" % i)
            gb = flat_range("gate_convs.%d.bias" % i)
            gather_seg("fg_b%d" % i, torch.stack([fb, gb], dim=1).reshape(-1))
            bidx = seg_index("fg_b%d" % i, (D, 2))
            map_grad("filter_convs.%d.bias" % i, bidx[:, 0].clone())
            map_grad("gate_convs.%d.bias" % i, bidx[:, 1].clone())
            if cfg.use_gcn:
                wname, bname = "gconv.%d.mlp.mlp.weight" % i, "gconv.%d.mlp.mlp.bias" % i
            else:
                wname, bname = "residual_convs.%d.weight" % i, "residual_convs.%d.bias" % i
            W = cfg.W
            gather_seg("mlp_w%d" % i, flat_range(wname).reshape(-1))
            # transposed copy [W][C] for the power-schedule gcn forward (coalesced fragment rows)
            gather_seg("mlp_wT%d" % i, flat_range(wname).reshape(C, W).t().contiguous().reshape(-1))
            gather_seg("mlp_b%d" % i, flat_range(bname))
            gather_seg("bn_g%d" % i, flat_range("bn.%d.weight" % i))
            gather_seg("bn_b%d" % i, flat_range("bn.%d.bias" % i))
            if i < L - 1:  # the last layer's gcn / bn never reach the output (no grad)
                map_grad(wname, seg_index("mlp_w%d" % i, tuple(flat_off[wname][1])))
                map_grad(bname, seg_index("mlp_b%d" % i, (C,)))
                map_grad("bn.%d.weight" % i, seg_index("bn_g%d" % i, (C,)))
                map_grad("bn.%d.bias" % i, seg_index("bn_b%d" % i, (C,)))
            assert flat_off[wname][1][1] == W
        # skip convs concatenated along K: [S][L*D]
        sk = torch.stack([flat_range("skip_convs.%d.weight" % i).reshape(S, D) for i in range(L)], dim=1)
        gather_seg("skip_w", sk.reshape(-1))
        skidx = seg_index("skip_w", (S, L, D))
        for i in range(L):
            map_grad("skip_convs.%d.weight" % i, skidx[:, i].reshape(S, D, 1, 1).clone())
        gather_seg("skip_b", torch.cat([flat_range("skip_convs.%d.bias" % i) for i in range(L)]))
        # computed slot: sum_i skip bias (and, for grads, the shared bias gradient)
        segs["skip_bsum"] = (len(pidx), S)
        pidx.extend([0] * S)
        for i in range(L):
            map_grad("skip_convs.%d.bias" % i, seg_index("skip_bsum", (S,)))
        gather_seg("e1_w", flat_range("end_conv_1.weight").reshape(-1))
        map_grad("end_conv_1.weight", seg_index("e1_w", (E, S, 1, 1)))
        gather_seg("e1_b", flat_range("end_conv_1.bias"))
        map_grad("end_conv_1.bias", seg_index("e1_b", (E,)))
        gather_seg("e2_w", flat_range("end_conv_2.weight").reshape(-1))
        map_grad("end_conv_2.weight", seg_index("e2_w", (O, E, 1, 1)))
        gather_seg("e2_b", flat_range("end_conv_2.bias"))
        map_grad("end_conv_2.bias", seg_index("e2_b", (O,)))
        # transposed copies of the head weights for the input gradients (NT GEMMs, no grads)
        gather_seg("skip_wT", sk.reshape(S, L * D).t().contiguous().reshape(-1))
        gather_seg("e1_wT", flat_range("end_conv_1.weight").reshape(E, S).t().contiguous().reshape(-1))
        gather_seg("e2_wT", flat_range("end_conv_2.weight").reshape(O, E).t().contiguous().reshape(-1))
        self.zero_slot = len(pidx)
        pidx.append(0)
        self.total = len(pidx)
        self.segs = segs
        uidx = torch.full((self.flat_total,), self.zero_slot, dtype=torch.long)
        self.active = []  # names of parameters that receive gradients
        for n in names:
            if n in grad_src:
                off, shape = flat_off[n]
                src = grad_src[n].reshape(-1)
                uidx[off:off + src.numel()] = src
                self.active.append(n)
        self.flat_off = flat_off
        self.pidx_cpu = torch.tensor(pidx, dtype=torch.int32)
        self.uidx_cpu = uidx.to(torch.int32)
        # contiguous [lo, hi) flat ranges of the active parameters (clip + Adam)
        ranges = []
        for n in names:
            if n not in grad_src:
                continue
            off, shape = flat_off[n]
            numel = 1
            for s in shape:
                numel *= s
            if ranges and ranges[-1][1] == off:
                ranges[-1][1] = off + numel
            else:
                ranges.append([off, off + numel])
        self.ranges = ranges

    def view(self, buf, name, shape=None):
        start, numel = self.segs[name]
        v = buf[start:start + numel]
        return v.view(shape) if shape is not None else v


class Config:
    """Static model configuration (mirrors the gwnet ctor, model.py:83-171)."""

    def __init__(self, model, residual_only=False):
        self.N = model.num_nodes
        self.C = model.residual_channels   # residual / BatchNorm / gcn-output channels
        self.D = model.dilation_channels   # gated-TCN output, gcn input and skip-conv input channels
        self.K = model.kernel_size         # taps of the dilated convs (model.py:135-141)
        self.Cin = model.in_dim
        self.S = model.skip_channels
        self.E = model.end_channels
        self.O = model.out_dim
        self.OP = (self.O + 31) // 32 * 32  # output gradient rows padded to whole 32-column tiles
        self.L = model.blocks * model.layers
        # gwnet: dilations 1, 2, 4, ... per block; gwnet_diff_G starts every block at 4 (model.py:291)
        first = getattr(model, "first_dilation", 1)
        self.dilations = []
        for _ in range(model.blocks):
            d = first
            for _ in range(model.layers):
                self.dilations.append(d)
                d *= 2
        self.R = model.receptive_field
        self.adaptive = bool(model.gcn_bool and model.addaptadj)
        # per-sample graphs (gwnet_diff_G): every support, the adaptive one included, is a
        # [B][N][N] input of the call; the adaptive embeddings are not parameters
        self.per_sample = bool(getattr(model, "per_sample_graphs", False))
        if self.per_sample:
            # residual_only: gwnet_diff_G called without supports (model.py:391-398 takes the
            # residual_convs branch whenever the gcn does not run)
            self.use_gcn = bool(model.gcn_bool) and not residual_only
            self.nsup = model.supports_len if self.use_gcn else 0
            self.nfixed = self.nsup
            self.adp_params = False
        else:
            self.use_gcn = bool(model.gcn_bool and model.supports is not None)
            self.nfixed = len(model.supports) if (self.use_gcn and model.supports is not None) else 0
            self.nsup = self.nfixed + (1 if (self.use_gcn and self.adaptive) else 0)
            self.adp_params = bool(self.use_gcn and self.adaptive)  # trained nodevec1 / nodevec2
        self.W = (2 * self.nsup + 1) * self.D if self.use_gcn else self.D
        # the adaptive support reaches the output only through a gcn of a non-final layer (the
        # last layer's gcn output is dead, model.py:225-236): otherwise nodevec1/2 keep grad None
        self.adp_live = bool(self.adp_params and self.L > 1)
        self.NP = (self.N + 31) // 32 * 32  # padded support side (zero outside N x N)
        if self.C % 16 != 0 or 256 % self.C != 0:
            raise ValueError("gwn_amd: residual channels must be 16, 32, 64, 128 or 256")
        if self.D % 16 != 0 or self.D > 1024:
            raise ValueError("gwn_amd: dilation channels must be a multiple of 16 (<= 1024)")
        if self.K < 1:
            raise ValueError("gwn_amd: kernel_size must be >= 1")
        # the shape of the fused kernels (fused gcn, row-GEMM TCN, BatchNorm fold): the reference
        # default's square layers; any other (residual != dilation channels, kernel_size != 2)
        # runs the generic MFMA GEMM path
        self.square = self.C == self.D and self.K == 2

    def shift(self, i):
        """Steps layer i's dilated conv consumes: T_out = T_in - (kernel_size - 1) * dilation."""
        return (self.K - 1) * self.dilations[i]

    def times(self, t_in):
        t0 = max(t_in, self.R)
        ts = [t0]
        for i in range(len(self.dilations)):
            ts.append(ts[-1] - self.shift(i))
        return ts


class Acts:
    """Activations of one forward (kept for its backward)."""

    def __init__(self, cfg, B, ts, device, training):
        C, D, N, L = cfg.C, cfg.D, cfg.N, cfg.L
        P = B * N
        self.B, self.ts, self.P = B, ts, P
        tf = ts[-1]
        e = lambda *s: torch.empty(*s, device=device, dtype=F32)  # noqa: E731
        self.xin = e(ts[0] * P, cfg.Cin)
        self.X = [e(ts[0] * P, C)]
        self.FG, self.H, self.Z, self.mean, self.rstd = [], [], [], [], []
        for i in range(L):
            rows = ts[i + 1] * P
            self.FG.append(e(rows, 2 * D))
            self.H.append(e(rows, cfg.W))
            self.Z.append(e(rows, C))
            self.X.append(e(rows, C))
            self.mean.append(e(C))
            self.rstd.append(e(C))
        self.skipcat = e(tf * P, L * D)
        self.skr = e(tf * P, cfg.S)
        self.e1 = e(tf * P, cfg.E)
        self.y = e(tf * P, cfg.O)
        self.adp = torch.zeros(cfg.NP, cfg.NP, device=device, dtype=F32) if cfg.adp_params else None
        self.training = training
        # BatchNorm on load (gwn_batchnorm_fwd_fold): per layer the scale of its normalisation
        # (bn(z) = (z - mean) * scale + beta) and the next layer's TCN weights / bias with it folded in
        self.bn_scale = e(L, C)
        self.w_fold = e(L, 4 * C * C)
        self.b_fold = e(L, 2 * C)
        self.bn_fold = False


class _G4Holder:
    """What Executor._g4_bf16 reads and caches for a forward that has no Acts (the lean eval)."""
    adp = supT = None
    training = False


class _HeadBufs:
    def __init__(self, skipcat, skr, e1, y):
        self.skipcat, self.skr, self.e1, self.y = skipcat, skr, e1, y


class Executor:
    def __init__(self, model, residual_only=False):
        self.cfg = Config(model, residual_only)
        self.layout = PackedLayout(model, self.cfg)
        self.dropout = model.dropout
        self.compute_dtype = getattr(model, "compute_dtype", "fp32")
        self.device = None
        self._scratch = {}
        # instrumentation (bench.py): the training gcn forward launches store their workgroups' device
        # clock stamps (gwn_gcn_args.clock, per layer in acts.CLK)
        self.launch_clock = False
        self.launch_clock_slots = 2  # u64 stamps per workgroup (gwn_gcn_args.clock: start, end)

    # ---------------------------------------------------------------------------------------
    def bind(self, device):
        if self.device == device:
            return
        self.device = device
        lay = self.layout
        self.pidx = lay.pidx_cpu.to(device)
        self.uidx = lay.uidx_cpu.to(device)
        self.packed = torch.zeros(lay.total, device=device, dtype=F32)
        self.gpacked = torch.zeros(lay.total, device=device, dtype=F32)
        # the dropout counter's start value comes from the DEVICE generator (seeded by
        # torch.manual_seed like the CPU one): the CPU stream stays exactly the reference's, whose
        # only CPU draws are the model init and gwnet_diff_G's per-call embeddings (model.py:324-329)
        self.seed = torch.randint(0, 2 ** 62, (1,), device=device, dtype=torch.int64)
        self._scratch = {}

    # ---------------------------------------------------------------------------------------
    def split_planes(self):
        """MFMA operand format of the fused gcn kernels (include/gwn.h gwn_dtype):
        * compute dtype bf16 (gwnet.set_compute_dtype): 2 = bf16 operands, fp32 accumulation,
          forward AND backward, on the 16-node tile kernels, the per-hop 1x1 mlp on bf16 MFMA too
          (the mixed-precision path of configs[2]); GWN_BF16_MLP=0 keeps that mlp in f32 (1);
        * else 0: the f32-MFMA kernels (the default: the reference's fp32 arithmetic).
        0 when the shape has no bf16 tile kernel (c != 32, n > 512, no supports, GWN_GCN_T16=0)."""
        cfg = self.cfg
        if self.compute_dtype != "bf16":
            return 0
        planes = 0
        if (cfg.use_gcn and cfg.nsup >= 1 and cfg.square and self._t16_ok() and self._fused_gcn()
                and _lib.load().gwn_gcn_t16b_supported(cfg.N, cfg.nsup)):
            planes = 2 if os.environ.get("GWN_BF16_MLP", "1") != "0" else 1
        if planes == 0 and not getattr(self, "_warned_bf16", False):
            self._warned_bf16 = True
            warnings.warn("gwn_amd: compute dtype bf16 requested, but this shape (C=%d, N=%d, %d supports) has no "
                          "bf16 tile kernel: the diffusion GCN runs in fp32" % (cfg.C, cfg.N, cfg.nsup))
        return planes

    def pk(self, name, buf=None):
        return self.layout.view(self.packed if buf is None else buf, name)

    def gk(self, name):
        return self.layout.view(self.gpacked, name)

    def scratch(self, B, ts):
        key = (B, tuple(ts))
        s = self._scratch.get(key)
        if s is not None:
            return s
        cfg = self.cfg
        C, D, N, L = cfg.C, cfg.D, cfg.N, cfg.L
        P = B * N
        tf = ts[-1]
        e = lambda *s_: torch.empty(*s_, device=self.device, dtype=F32)  # noqa: E731
        maxrows = max(ts[i + 1] for i in range(L)) * P
        s = {
            "dy": e(tf * P, cfg.OP),  # the output gradient, rows padded to 32 columns (zeros)
            "de1": e(tf * P, cfg.E),
            "dsk": e(tf * P, cfg.S),
            "dskipcat": e(tf * P, L * D),
            "dxa": e(ts[0] * P, C),
            "dxb": e(ts[0] * P, C),
            # bf16 mode: t1 / t2 of the adaptive support in the tiled activation layout (gwn_gram_g4_bf16)
            "tg4": e(2 * (maxrows // N) * ((N + 15) // 16) * 256),
            "dfg": e(maxrows, 2 * D),
            "dh": e(maxrows, C),
            "dhc": e(maxrows, cfg.W),
            "dadp": torch.zeros(cfg.NP, cfg.NP, device=self.device, dtype=F32),
            "metrics": e(4),
            "bnsums": e(2 * C),  # BN-backward statistics handed from a layer's TCN backward to the next
            # BN partials of one layer: gwn_gcn_bn_partial_count slots (>= one per slice)
            "bnpart": e(self._bn_parts(ts[0] * B * N) * 3 * C),
            # layer i's partials are finalized by layer i+1's TCN (gwn_tcn_args.bn) while layer i+1's
            # gcn writes its own: alternate buffers
            "bnpart2": e(self._bn_parts(ts[0] * B * N) * 3 * C),
        }
        lib = _lib.load()
        need = [
            lib.gwn_gcn_bwd_workspace_floats_ex(maxrows, N, D, max(cfg.nsup, 0), C),
            lib.gwn_batchnorm_workspace_floats(maxrows, C),
            lib.gwn_colsum_workspace_floats(maxrows, max(cfg.E, cfg.S, cfg.L * D)),
            lib.gwn_masked_loss_workspace_floats(B, cfg.O, N, tf),
            lib.gwn_clip_adam_workspace_floats(self.layout.flat_total),
            cfg.NP * cfg.NP,
            lib.gwn_gram_g4_workspace_floats(N, maxrows // N),
        ]
        # every layer's TCN backward (the largest workspace need may sit at any dilation)
        need += [lib.gwn_gated_tcn_bwd_workspace_floats_ex(ts[i], P, C, cfg.dilations[i], cfg.K, D) for i in range(L)]
        # split-K partials of the head / start weight grads
        for (M_, N_, K_) in ((cfg.O, cfg.E, tf * P), (cfg.E, cfg.S, tf * P), (cfg.S, L * D, tf * P),
                             (C, cfg.Cin, ts[0] * P)):
            need.append(lib.gwn_gemm_workspace_floats(M_, N_, _ksplit(M_, N_, K_)))
        need.append(lib.gwn_gemm_workspace_floats(tf * P, cfg.O, _ksplit_thin(tf * P, cfg.O, cfg.E)))
        s["ws"] = e(int(max(need)) + 16)
        # deferred weight gradients (_defer_ok): per-layer wgrad partials, reduced by one launch at
        # the end of the backward
        if cfg.C == 32 and cfg.square and cfg.W % 32 == 0:
            pm, pt = [], []
            for i in range(L):
                rows = ts[i + 1] * P
                pm.append(e(max(1, lib.gwn_wgrad_partial_count(rows, C, cfg.W)) * (C * cfg.W + C)))
                pt.append(e(max(1, lib.gwn_wgrad_partial_count(rows, 2 * C, 2 * C)) * (4 * C * C + 2 * C)))
            s["part_mlp"], s["part_tcn"] = pm, pt
            # grouped weight gradients (gwn_wgrad_group): every layer's mlp / TCN dW in one launch
            # each at the end of the backward, so each layer keeps its own dh / dfg
            rows_l = [ts[i + 1] * P for i in range(L)]
            gm = self._group_plan(rows_l[:L - 1], C, cfg.W, 1)
            gt = self._group_plan(rows_l, 2 * C, C, 2)
            if gm is not None and gt is not None and L >= 2:
                s["group_mlp"] = [e(n * (C * cfg.W + C)) for n in gm]
                s["group_tcn"] = [e(n * (4 * C * C + 2 * C)) for n in gt]
                s["group_np"] = (gm, gt)
                s["dh_l"] = [e(r, C) for r in rows_l]
                s["dfg_l"] = [e(r, 2 * D) for r in rows_l]
                s["aff_id"] = torch.cat([torch.zeros(C, device=self.device), torch.ones(C, device=self.device),
                                         torch.zeros(C, device=self.device)])
            # grouped adaptive-support gradient (gwn_gram_group, fp32 mode): each layer keeps its
            # t1 / t2 ([rows][96]: the gcn backward's dhcat with only columns 32..96 written)
            if cfg.adp_live and cfg.use_gcn:
                # a launch takes at most GRAM_GL layers: deeper stacks run several launches, the
                # later ones accumulating (the workspace: the largest chunk's need)
                need = [int(lib.gwn_gram_group_workspace_floats(
                    N, (ctypes.c_int * len(ch))(*[rows_l[i] // N for i in ch]), len(ch)))
                    for ch in _layer_chunks(L - 1)]
                if min(need) > 0:
                    s["tt_l"] = [e(rows_l[i], 3 * C) for i in range(L - 1)]
                    s["ws_gram_group"] = e(max(need) + 16)
            if cfg.Cin <= 4 and 256 % C == 0:  # the start conv's weight gradient (narrow form)
                s["part_start"] = e(max(1, lib.gwn_wgrad_partial_count(ts[0] * P, C, cfg.Cin)) * (C * cfg.Cin + C))
            if cfg.E % 32 == 0 and (cfg.OP // 32) * (cfg.E // 32) <= 16:  # end_conv_2's weight gradient
                s["part_e2"] = e(max(1, lib.gwn_wgrad_partial_count(tf * P, cfg.OP, cfg.E)) * (cfg.OP * cfg.E + cfg.OP))
            ge = self._group_plan([tf * P], cfg.OP, cfg.E, 1)
            if ge is not None:
                s["part_e2g"] = (e(ge[0] * (cfg.OP * cfg.E + cfg.OP)), ge[0])

        # support split of the fused gcn kernels (gwn_gcn_args.ksplit): partial sums + per-slice
        # counters (zero, and left zero by every launch)
        if self._fused_gcn() and cfg.use_gcn and cfg.nsup >= 2:
            s["kws"] = e(int(lib.gwn_gcn_ksplit_ws_floats(maxrows, N, cfg.nsup)))
            s["kcnt"] = torch.zeros(maxrows // N, device=self.device, dtype=torch.int32)
        self._scratch[key] = s
        return s

    # ---------------------------------------------------------------------------------------
    def pack_params(self, flat):
        st = _lib.stream()
        lay = self.layout
        cfg = self.cfg
        # one launch: the packing and the summed skip bias (slot skip_bsum)
        _lib.call("gwn_gather_sum", ptr(flat), ptr(self.pidx), ptr(self.packed), lay.total, lay.segs["skip_b"][0],
                  cfg.L, cfg.S, lay.segs["skip_bsum"][0], st)

    def supports(self, fixed, acts):
        sups = list(fixed) if self.cfg.use_gcn else []
        if self.cfg.adp_params:
            sups.append(acts.adp)
        arr = (ctypes.c_void_p * max(len(sups), 1))(*[s.data_ptr() for s in sups])
        return sups, arr

    def forward(self, flat, fixed_sups, x, training, bn_bufs, acts=None, lead_pad=0, seed=None, sup_batch=1,
                fixed_t=None, want_out=True):
        """x: reference NCHW input [B, Cin, N, T] (any strides).  ``lead_pad`` extra zero steps
        are prepended (engine.py:44) before the receptive-field pad (model.py:176-178).
        ``seed``: the dropout counter this forward (and its backward) draws its masks from
        (default: the executor's own, which the trainer advances after each step).
        ``sup_batch`` > 1: per-sample supports (gwnet_diff_G): each of ``fixed_sups`` is a padded
        [B][NP][NP] buffer, sample b of slice (t, b) diffusing with matrix b.
        ``fixed_t``: padded transposes of ``fixed_sups`` kept by the caller (they change only with the
        supports); the backward's transposes of the others are built here.
        ``want_out`` False: the NCHW copy of the output is not made (the fused training step reads
        the head's rows, acts.y, through gwn_masked_loss_rows); out is then None.
        Returns (out [B, O, N, T_f], acts)."""
        cfg = self.cfg
        C, N, L = cfg.C, cfg.N, cfg.L
        if x.dim() != 4:
            raise RuntimeError("gwnet: expected a 4-D input [B, C, N, T], got %d-D" % x.dim())
        B, cin, n, t_in = x.shape
        if n != N or cin != cfg.Cin:
            raise RuntimeError("gwnet: expected input [B, %d, %d, T], got %s" % (cfg.Cin, N, tuple(x.shape)))
        if x.dtype != F32 or not x.is_cuda:
            raise RuntimeError("gwnet (gwn_amd): input must be a float32 CUDA/HIP tensor")
        ts = cfg.times(t_in + lead_pad)
        if acts is not None and (acts.B != B or list(acts.ts) != list(ts)):
            acts = None
        if ts[-1] < 1:
            raise RuntimeError("gwnet: input too short for the receptive field")
        if sup_batch > 1 and sup_batch != B:
            raise RuntimeError("gwnet: per-sample supports for %d samples, input batch %d" % (sup_batch, B))
        st = _lib.stream()
        self.pack_params(flat)
        if acts is None:
            acts = Acts(cfg, B, ts, self.device, training)
        acts.training = training
        acts.seed = self.seed if seed is None else seed
        acts.gcn_args = {}
        P = B * N
        tf = ts[-1]
        lib = _lib
        if cfg.adp_params:
            lib.call("gwn_adaptive_adj_fwd", ptr(self.pk("nv1")), ptr(self.pk("nv2")), N, 10,
                     ptr(acts.adp), cfg.NP, st)
        sups, sup_arr = self.supports(fixed_sups, acts)
        acts.sups, acts.sup_arr = sups, sup_arr
        acts.supT_arr = None
        acts.sup_batch = sup_batch
        sq = cfg.NP * cfg.NP
        # power schedule of the fused gcn kernels: squared supports (and their transposes); the
        # adaptive one's square launch also writes its transpose for the backward
        pw = self._pow_ok(sup_batch)
        acts.sup2_arr = acts.sup2t_arr = acts.g4f_arr = acts.g4b_arr = None
        adp_t_done = False
        if pw:
            sq2, sq2t, g4f, g4b = self._fixed_squares(fixed_sups)
            g4f_p = [t_.data_ptr() for t_ in g4f] if g4f is not None else []
            g4b_p = [t_.data_ptr() for t_ in g4b] if g4b is not None else []
            if cfg.adp_params:
                if getattr(acts, "adp2", None) is None:
                    acts.adp2 = torch.empty(cfg.NP, cfg.NP, device=self.device, dtype=F32)
                    acts.adp2_t = torch.empty(cfg.NP, cfg.NP, device=self.device, dtype=F32)
                adp_t = None
                if training:
                    if getattr(acts, "supT", None) is None or len(acts.supT) != len(sups) or acts.supT[0].numel() != sq:
                        acts.supT = [torch.empty(sq, device=self.device, dtype=F32) for _ in sups]
                    adp_t, adp_t_done = acts.supT[-1], True
                sq2, sq2t = sq2 + [acts.adp2], sq2t + [acts.adp2_t]
                if self._t16_ok():
                    # the square, the transposes and the adaptive support's 16-node tile copies
                    # (A, A^2 and, training, A^T, (A^2)^T), rewritten every step by one launch
                    fl = int(_lib.load().gwn_support_g4_floats(N))
                    if getattr(acts, "g4_adp", None) is None:
                        acts.g4_adp = torch.empty(4, fl, device=self.device, dtype=F32)
                    lib.call("gwn_support_square_g4", ptr(acts.adp), cfg.NP, cfg.NP, ptr(acts.adp2), ptr(acts.adp2_t),
                             ptr(adp_t), N, ptr(acts.g4_adp), fl, 4 if training else 2, st)
                    g4f_p += [acts.g4_adp[0].data_ptr(), acts.g4_adp[1].data_ptr()]
                    g4b_p += [acts.g4_adp[2].data_ptr(), acts.g4_adp[3].data_ptr()]
                else:
                    lib.call("gwn_support_square", ptr(acts.adp), cfg.NP, cfg.NP, ptr(acts.adp2), ptr(acts.adp2_t),
                             ptr(adp_t), st)
            acts.sup2_arr = (ctypes.c_void_p * len(sq2))(*[t_.data_ptr() for t_ in sq2])
            acts.sup2t_arr = (ctypes.c_void_p * len(sq2t))(*[t_.data_ptr() for t_ in sq2t])
            if self._t16_ok() and len(g4f_p) == 2 * len(sups):
                acts.g4f_arr = (ctypes.c_void_p * len(g4f_p))(*g4f_p)
                acts.g4b_arr = (ctypes.c_void_p * len(g4b_p))(*g4b_p)
        if training and sups:
            # transposed supports: the fused backward computes A·x as (A^T)^T·x on the forward kernel path
            if getattr(acts, "supT", None) is None or len(acts.supT) != len(sups) or acts.supT[0].numel() != sq * sup_batch:
                acts.supT = [torch.empty(sup_batch * sq, device=self.device, dtype=F32) for _ in sups]
            nfix = len(fixed_t) if (fixed_t is not None and sup_batch <= 1 and cfg.use_gcn) else 0
            for k, (s_, t_) in enumerate(zip(sups, acts.supT)):
                if k < nfix or (adp_t_done and k == len(sups) - 1):
                    continue  # the caller's cached transpose (below) / written by gwn_support_square
                if sup_batch > 1:
                    lib.call("gwn_pad_square_batched", ptr(s_), sup_batch, sq, N, cfg.NP, ptr(t_), cfg.NP, cfg.NP, sq,
                             1, st)
                else:
                    lib.call("gwn_pad_square", ptr(s_), N, cfg.NP, ptr(t_), cfg.NP, cfg.NP, 1, st)
            acts.supT_arr = (ctypes.c_void_p * len(sups))(*[(fixed_t[k] if k < nfix else acts.supT[k]).data_ptr()
                                                             for k in range(len(sups))])
            acts.supT_keep = fixed_t  # alive as long as the activations reference them
        sx = x.stride()
        lib.call("gwn_start_conv_fwd", ptr(x), sx[0], sx[1], sx[2], sx[3], B, cin, N, t_in, ts[0],
                 ptr(self.pk("start_w")), ptr(self.pk("start_b")), C, ptr(acts.X[0]), ptr(acts.xin), st)
        scr = self.scratch(B, ts)
        ws, bnparts = scr["ws"], (scr["bnpart"], scr["bnpart2"])
        planes = self.split_planes() if sup_batch <= 1 else 0
        acts.g4bt_arr = None
        # (shared supports only: planes is 0 for per-sample graphs, whose padded stacks are fresh per call)
        acts.g4bf_arr = self._g4_bf16(fixed_sups, acts, st) if planes >= 1 and sups and sup_batch <= 1 else None
        planes = planes if acts.g4bf_arr is not None else 0
        acts.planes = planes
        if not training:
            acts.g4bt_arr = None
        # train mode: BatchNorm i is applied on load by its consumers (TCN weights of layer i+1
        # folded, residual affine in gcn epilogue i+1, affine in the TCN weight gradient) instead
        # of materialising bn(z) (one HBM pass and one launch fewer per layer)
        fold = training and self._bn_fold_ok(sup_batch)
        acts.bn_fold = fold
        # bf16 mode: the adaptive-support gram on tiled operands -- the bf16 16-node tile kernels
        # write X and its hop 1 (forward) and t1 / t2 (backward) in gwn_gram_g4_bf16's layout
        gram_g4 = (training and cfg.adp_params and cfg.use_gcn and sup_batch <= 1 and self._fused_gcn()
                   and acts.g4bf_arr is not None and acts.g4bt_arr is not None
                   and _lib.load().gwn_gcn_t16b_supported(N, cfg.nsup) == 1)
        acts.gram_g4 = gram_g4
        if getattr(acts, "XG4", None) is None:
            acts.XG4, acts.TG4, acts.CLK = {}, {}, {}
        # bf16 mode: every layer's adaptive-support gram in one gwn_gram_g4_group launch at the end
        # of the backward
        if gram_g4 and L >= 2 and getattr(acts, "ws_g4g", None) is None:
            need = [int(_lib.load().gwn_gram_g4_group_workspace_floats(
                N, (ctypes.c_int * len(ch))(*[ts[i + 1] * P // N for i in ch]), len(ch)))
                for ch in _layer_chunks(L - 1)]
            acts.ws_g4g = (torch.empty(max(need) + 16, device=self.device, dtype=F32) if min(need) > 0
                           else False)
        # bf16 mode: the hop pieces' only reader is then the grouped mlp weight gradient -- stored
        # as bf16 (half the bytes written here and read there)
        pieces_b = gram_g4 and "group_mlp" in scr and self._defer_ok(scr) and self._fuse_ok(acts)
        acts.pieces_b = pieces_b
        if pieces_b and (getattr(acts, "HB", None) is None or len(acts.HB) != L - 1):
            acts.HB = [torch.empty(ts[i + 1] * P, 2 * cfg.nsup * cfg.D, device=self.device, dtype=torch.int16)
                       for i in range(L - 1)]
        used_prev = 0  # the BN partial slots the previous gcn launch reported (gwn_gcn_args.bn_slots_used)
        for i in range(L):
            d, sh = cfg.dilations[i], cfg.shift(i)
            rows = ts[i + 1] * P
            xin, wfg, bfg, raff = self.layer_input(acts, i)
            ta = _lib.TcnArgs(x=xin, x_mean=raff[0], t_in=ts[i], P=P, c=C, dilation=d, w_fg=wfg, b_fg=bfg,
                              xg=ptr(acts.H[i]), ld_xg=cfg.W, fg=ptr(acts.FG[i]),
                              skipcat=acts.skipcat.data_ptr() + 4 * i * cfg.D, ld_skip=L * cfg.D,
                              skip_row0=(ts[i + 1] - tf) * P, ntaps=cfg.K, c_out=cfg.D)
            if fold and i > 0:
                # BatchNorm i-1 (train mode) finalized by this TCN from layer i-1's partials: inside
                # the fused gcn launch every workgroup merges them (no finalize launch), else
                # gwn_gated_tcn_fwd issues gwn_batchnorm_fwd_fold first (gwn_tcn_args.bn)
                rm_, rv_, mom_, eps_, nbt_ = bn_bufs[i - 1]
                bfp = _lib.BnFold(gamma=ptr(self.pk("bn_g%d" % (i - 1))), beta=ptr(self.pk("bn_b%d" % (i - 1))),
                                  running_mean=ptr(rm_), running_var=ptr(rv_), momentum=mom_, eps=eps_,
                                  save_mean=ptr(acts.mean[i - 1]), save_rstd=ptr(acts.rstd[i - 1]),
                                  scale=acts.bn_scale[i - 1].data_ptr(),
                                  w_next=ptr(self.pk("fg_w%d" % i)), b_next=ptr(self.pk("fg_b%d" % i)),
                                  w_fold=acts.w_fold[i].data_ptr(), b_fold=acts.b_fold[i].data_ptr(),
                                  num_batches_tracked=ptr(nbt_))
                ta.bn, ta.bn_partials = ctypes.addressof(bfp), ptr(bnparts[(i - 1) % 2])
                ta.bn_nparts = used_prev or self._bn_parts(ts[i] * P)  # (the slots layer i-1's gcn filled)
                ta._bn_keep = bfp  # (ctypes keeps no reference through the c_void_p field)
            if i == L - 1 and not training:
                lib.call("gwn_gated_tcn_fwd", ctypes.byref(ta), st)
                continue  # the last gcn / bn output is dead in eval (only skip reaches the output)
            drop = float(self.dropout) if (training and cfg.use_gcn) else 0.0
            xg4 = None
            if gram_g4 and i < L - 1:
                need_x = 2 * (rows // N) * ((N + 15) // 16) * 256  # two bf16 operands, a KiB per tile
                if acts.XG4.get(i) is None or acts.XG4[i].numel() != need_x:
                    acts.XG4[i] = torch.empty(need_x, device=self.device, dtype=F32)
                    # the backward's t1 / t2 of this layer, kept for the grouped gram at its end
                    acts.TG4[i] = torch.empty(need_x, device=self.device, dtype=F32)
                xg4 = acts.XG4[i]
            ga = _lib.GcnArgs(rows=rows, n=N, c=cfg.D, c_out=C, nsup=cfg.nsup if cfg.use_gcn else 0,
                              sup=ctypes.cast(sup_arr, ctypes.POINTER(ctypes.c_void_p)), ld_sup=cfg.NP,
                              h=ptr(acts.H[i]), ld_h=cfg.W,
                              w_mlp=ptr(self.pk("mlp_w%d" % i)), b_mlp=ptr(self.pk("mlp_b%d" % i)),
                              residual=xin + 4 * sh * P * C, z=ptr(acts.Z[i]),
                              seed_ptr=ptr(acts.seed), salt=i, drop_p=drop,
                              bn_partials=ptr(bnparts[i % 2]) if training else None,
                              # the last layer's gcn output only feeds bn[L-1]'s running statistics:
                              # no backward reads its hop pieces
                              no_pieces=1 if i == L - 1 and self._fused_gcn() else 0,
                              sup_bstride=sq if sup_batch > 1 else 0, sup_batch=sup_batch,
                              residual_mean=raff[0], residual_scale=raff[1], residual_shift=raff[2],
                              sup2=self._arr_field(acts.sup2_arr), w_mlp_t=ptr(self.pk("mlp_wT%d" % i)),
                              sup_g4=self._arr_field(acts.g4f_arr),
                              sup_g4b=self._arr_field(acts.g4bf_arr),
                              xg4=ptr(xg4) if xg4 is not None else None, xg4_support=cfg.nsup - 1,
                              split_planes=planes, **self.ksplit_fields(scr))
            if pieces_b and i < L - 1:
                ga.pieces_bf16, ga.ld_pb = acts.HB[i].data_ptr(), 2 * cfg.nsup * cfg.D
            # the gated TCN rides on the gcn call (gwn_gcn_args.tcn: inside the f32 tile kernel's
            # staging where it runs, else its own launch issued by gwn_gcn_fwd)
            ga.tcn = ctypes.pointer(ta)
            if training and self.launch_clock:
                if acts.CLK.get(i) is None:
                    cus = torch.cuda.get_device_properties(self.device).multi_processor_count
                    acts.CLK[i] = torch.zeros(self.launch_clock_slots * cus, device=self.device, dtype=torch.int64)
                ga.clock = ptr(acts.CLK[i])
            rm, rv, mom, eps, nbt = bn_bufs[i]
            if fold and i == L - 1:
                # the last BatchNorm (its output dead but for the running statistics): finalized by
                # the gcn call (gwn_gcn_args.bn_fold, a second launch); the others by the next TCN
                bf = _lib.BnFold(gamma=ptr(self.pk("bn_g%d" % i)), beta=ptr(self.pk("bn_b%d" % i)),
                                 running_mean=ptr(rm), running_var=ptr(rv), momentum=mom, eps=eps,
                                 save_mean=ptr(acts.mean[i]), save_rstd=ptr(acts.rstd[i]),
                                 scale=acts.bn_scale[i].data_ptr(), num_batches_tracked=ptr(nbt))
                ga.bn_fold = ctypes.pointer(bf)
            used = ctypes.c_int(0)
            ga.bn_slots_used, ga._used = ctypes.pointer(used), used
            lib.call("gwn_gcn_fwd", ctypes.byref(ga), st)
            used_prev = used.value  # the BN partial slots this launch can fill (the consumer's nparts)
            acts.gcn_args[i] = ga  # kept for bench.py's per-kernel timing
            if fold:
                pass  # the BatchNorm finalize rides on the next TCN / this gcn call
            elif training:
                lib.call("gwn_batchnorm_fwd_partials", ptr(acts.Z[i]), rows, C, ptr(bnparts[i % 2]), used_prev or self._bn_parts(rows),
                         ptr(self.pk("bn_g%d" % i)), ptr(self.pk("bn_b%d" % i)), ptr(rm), ptr(rv), mom, eps,
                         ptr(acts.X[i + 1]), ptr(acts.mean[i]), ptr(acts.rstd[i]), ptr(nbt), st)
            else:
                lib.call("gwn_batchnorm_fwd", ptr(acts.Z[i]), rows, C, ptr(self.pk("bn_g%d" % i)),
                         ptr(self.pk("bn_b%d" % i)), ptr(rm), ptr(rv), mom, eps, 0,
                         ptr(acts.X[i + 1]), ptr(acts.mean[i]), ptr(acts.rstd[i]), ptr(ws), st)
        rows_f = tf * P
        self._head_fwd(acts.skipcat, acts.skr, acts.e1, acts.y, rows_f, ws)
        out = None
        if want_out:
            out = torch.empty(B, cfg.O, N, tf, device=self.device, dtype=F32)
            lib.call("gwn_to_nchw", ptr(acts.y), B, cfg.O, N, tf, ptr(out), st)
        return out, acts

    def _bn_parts(self, rows):
        cfg = self.cfg
        return int(_lib.load().gwn_gcn_bn_partial_count(rows, cfg.N, cfg.C, cfg.nsup if cfg.use_gcn else 0, cfg.NP))

    @staticmethod
    def _arr_field(arr):
        return ctypes.cast(arr, ctypes.POINTER(ctypes.c_void_p)) if arr is not None else None

    def _pow_ok(self, sup_batch):
        """Power schedule of the fused gcn kernels (both hops of a support against A and A^2 in one
        pass; include/gwn.h sup2 / sup2_t): shared supports, f32 operands.  GWN_GCN_POW=0 selects
        the chained hops (A/B measurements)."""
        cfg = self.cfg
        return (os.environ.get("GWN_GCN_POW", "1") != "0" and self._fused_gcn() and cfg.use_gcn and cfg.nsup >= 1
                and sup_batch <= 1 and self.split_planes() == 0)

    def _t16_ok(self):
        """The persistent 16-node tile gcn kernels (include/gwn.h sup_g4 / sup_g4_t) with the power
        schedule; GWN_GCN_T16=0 selects the 32-node tile power kernels."""
        return os.environ.get("GWN_GCN_T16", "1") != "0"

    def _g4(self, mats):
        """gwn_support_g4 copies of padded supports (one launch): a [len(mats)][floats] tensor."""
        cfg = self.cfg
        fl = int(_lib.load().gwn_support_g4_floats(cfg.N))
        out = torch.empty(len(mats), fl, device=self.device, dtype=F32)
        self._g4_into(mats, out)
        return out

    def _g4_into(self, mats, out):
        cfg = self.cfg
        arr = (ctypes.c_void_p * len(mats))(*[ptr(m_) for m_ in mats])
        _lib.call("gwn_support_g4", ctypes.cast(arr, ctypes.POINTER(ctypes.c_void_p)), len(mats), cfg.N, cfg.NP,
                  ptr(out), out.shape[1], _lib.stream())

    def _g4_bf16(self, fixed_sups, acts, st):
        """bf16 mode: gwn_support_g4_bf16 copies of (A_k, A_k^2) for the bf16 16-node tile forward
        (include/gwn.h sup_g4b) -- the fixed supports' cached, the adaptive one's (square and copy)
        rebuilt every step; None where the t16 kernels are off."""
        cfg = self.cfg
        if not self._t16_ok() or not cfg.use_gcn:
            return None
        lib = _lib.load()
        el = int(lib.gwn_support_g4_bf16_elems(cfg.N))
        sq, sqt, _, _ = self._fixed_squares(fixed_sups)
        at = self._sq_cache[6]
        fixed = list(fixed_sups)
        key = tuple(s_.data_ptr() for s_ in fixed)
        c = getattr(self, "_g4b_cache", None)
        if c is None or c[0] != key:
            # rows: [A_k, A_k^2] (forward), then [A_k^T, (A_k^2)^T] (backward)
            mats = [m for s_, q in zip(fixed, sq) for m in (s_, q)] + [m for t_, q in zip(at, sqt) for m in (t_, q)]
            buf = torch.empty(max(len(mats), 1), el // 2, device=self.device, dtype=F32)  # bf16 pairs
            if mats:
                arr = (ctypes.c_void_p * len(mats))(*[ptr(m) for m in mats])
                _lib.call("gwn_support_g4_bf16", ctypes.cast(arr, ctypes.POINTER(ctypes.c_void_p)), len(mats), cfg.N,
                          cfg.NP, ptr(buf), el, st)
            c = (key, fixed, buf, len(fixed))
            self._g4b_cache = c
        nf = c[3]
        fw = [c[2][i].data_ptr() for i in range(2 * nf)]
        bw = [c[2][2 * nf + i].data_ptr() for i in range(2 * nf)]
        acts.g4bt_arr = None
        if cfg.adp_params:
            if getattr(acts, "adp2b", None) is None:
                acts.adp2b = torch.empty(cfg.NP, cfg.NP, device=self.device, dtype=F32)
                acts.adp2b_t = torch.empty(cfg.NP, cfg.NP, device=self.device, dtype=F32)
                acts.g4b_adp = torch.empty(4, el // 2, device=self.device, dtype=F32)
            _lib.call("gwn_support_square", ptr(acts.adp), cfg.NP, cfg.NP, ptr(acts.adp2b), ptr(acts.adp2b_t), None, st)
            adp_t = acts.supT[-1] if getattr(acts, "supT", None) is not None and acts.training else None
            mats = [acts.adp, acts.adp2b] + ([adp_t, acts.adp2b_t] if adp_t is not None else [])
            arr = (ctypes.c_void_p * len(mats))(*[ptr(m) for m in mats])
            _lib.call("gwn_support_g4_bf16", ctypes.cast(arr, ctypes.POINTER(ctypes.c_void_p)), len(mats), cfg.N,
                      cfg.NP, ptr(acts.g4b_adp), el, st)
            fw += [acts.g4b_adp[0].data_ptr(), acts.g4b_adp[1].data_ptr()]
            bw = bw + [acts.g4b_adp[2].data_ptr(), acts.g4b_adp[3].data_ptr()] if adp_t is not None else []
        if len(fw) != 2 * cfg.nsup:
            return None
        if len(bw) == 2 * cfg.nsup:
            acts.g4bt_arr = (ctypes.c_void_p * len(bw))(*bw)
        return (ctypes.c_void_p * len(fw))(*fw)

    def _fixed_squares(self, fixed_sups):
        """(A_k^2, (A_k^2)^T) of the padded fixed supports, and the gwn_support_g4 copies of
        (A_k, A_k^2) and (A_k^T, (A_k^2)^T) for the 16-node tile kernels, cached while the supports
        stay the same tensors (the cache keeps them referenced, so their addresses cannot be reused
        meanwhile).  Returns (sq, sqt, g4f, g4b) with g4f / g4b [2 * nfixed][floats]."""
        fixed_sups = list(fixed_sups) if self.cfg.use_gcn else []
        key = tuple(s_.data_ptr() for s_ in fixed_sups)
        c = getattr(self, "_sq_cache", None)
        if c is None or c[0] != key:
            NP = self.cfg.NP
            sq, sqt, fw, bw = [], [], [], []
            for s_ in fixed_sups:
                a2 = torch.empty(NP, NP, device=self.device, dtype=F32)
                a2t = torch.empty(NP, NP, device=self.device, dtype=F32)
                at = torch.empty(NP, NP, device=self.device, dtype=F32)
                _lib.call("gwn_support_square", ptr(s_), NP, NP, ptr(a2), ptr(a2t), ptr(at), _lib.stream())
                sq.append(a2)
                sqt.append(a2t)
                fw += [s_, a2]
                bw += [at, a2t]
            g4f = self._g4(fw) if fw else None
            g4b = self._g4(bw) if bw else None
            c = (key, fixed_sups, sq, sqt, g4f, g4b, [bw[2 * k] for k in range(len(fixed_sups))])
            self._sq_cache = c
        return list(c[2]), list(c[3]), c[4], c[5]

    @staticmethod
    def ksplit_fields(scr):
        """gwn_gcn_args / gwn_gcn_bwd_args fields of the support split (auto policy in the library)."""
        if "kws" not in scr:
            return {}
        return {"ksplit": 0, "ksplit_ws": scr["kws"].data_ptr(), "ksplit_count": scr["kcnt"].data_ptr()}

    def _fused_gcn(self):
        """gwn_gcn_fwd takes the fused path (c == 32, n <= 512, nsup <= 8; include/gwn.h)."""
        cfg = self.cfg
        return cfg.C == 32 and cfg.square and cfg.N <= 512 and (not cfg.use_gcn or cfg.nsup <= 8)

    def _bn_fold_ok(self, sup_batch):
        """BatchNorm on load needs the fused gcn forward (its epilogue applies the residual affine)
        and C = 32 (the fold kernel); otherwise bn(z) is materialised."""
        return self._fused_gcn()

    def layer_input(self, acts, i):
        """(x, w_fg, b_fg, (mean, scale, shift)) of layer i's gated TCN / residual: the normalised
        activation X[i] with the layer's own weights, or -- BatchNorm folded -- the pre-BN z of
        layer i-1 with the folded weights and bn(z) = (z - mean) * scale + beta for the residual
        and the TCN weight gradient."""
        if i == 0 or not acts.bn_fold:
            return ptr(acts.X[i]), ptr(self.pk("fg_w%d" % i)), ptr(self.pk("fg_b%d" % i)), (None, None, None)
        return (ptr(acts.Z[i - 1]), acts.w_fold[i].data_ptr(), acts.b_fold[i].data_ptr(),
                (ptr(acts.mean[i - 1]), acts.bn_scale[i - 1].data_ptr(), ptr(self.pk("bn_b%d" % (i - 1)))))

    def _head_fwd(self, skipcat, skr, e1, y, rows_f, ws):
        """skip sum (relu'd) -> end_conv_1 (+relu) -> end_conv_2 (model.py:216-222, 238-240)."""
        cfg = self.cfg
        L, C = cfg.L, cfg.D  # the skip convs read the gated (dilation-channel) outputs
        acts = _HeadBufs(skipcat, skr, e1, y)
        if self._head_nt():
            hb = self.head_bf16()
            gemm_nt(acts.skipcat, L * C, self.pk("skip_w"), L * C, acts.skr, cfg.S, rows_f, cfg.S, L * C,
                    bias=self.pk("skip_bsum"), relu=1, bf16=hb)
            gemm_nt(acts.skr, cfg.S, self.pk("e1_w"), cfg.S, acts.e1, cfg.E, rows_f, cfg.E, cfg.S,
                    bias=self.pk("e1_b"), relu=1, bf16=hb)
            gemm_nt(acts.e1, cfg.E, self.pk("e2_w"), cfg.E, acts.y, cfg.O, rows_f, cfg.O, cfg.E,
                    bias=self.pk("e2_b"))
        else:
            gemm(acts.skipcat, L * C, 1, self.pk("skip_w"), 1, L * C, acts.skr, cfg.S, 1,
                 M=rows_f, N=cfg.S, K=L * C, bias=self.pk("skip_bsum"), relu=1)
            gemm(acts.skr, cfg.S, 1, self.pk("e1_w"), 1, cfg.S, acts.e1, cfg.E, 1,
                 M=rows_f, N=cfg.E, K=cfg.S, bias=self.pk("e1_b"), relu=1)
            gemm(acts.e1, cfg.E, 1, self.pk("e2_w"), 1, cfg.E, acts.y, cfg.O, 1,
                 M=rows_f, N=cfg.O, K=cfg.E, bias=self.pk("e2_b"),
                 ksplit=_ksplit_thin(rows_f, cfg.O, cfg.E), part=ws)

    # ---------------------------------------------------------------------------------------
    def infer_ok(self):
        """The lean inference schedule needs the fused GCN path and the NT head GEMMs."""
        cfg = self.cfg
        return (os.environ.get("GWN_LEAN_EVAL", "1") != "0" and cfg.C == 32 and cfg.square and cfg.N <= 512
                and cfg.nsup <= 8 and self._head_nt() and not cfg.per_sample)

    def _infer_bufs(self, B, ts):
        key = ("infer", B, tuple(ts))
        b = self._scratch.get(key)
        if b is not None:
            return b
        cfg = self.cfg
        C, L, P = cfg.C, cfg.L, B * cfg.N
        tf = ts[-1]
        e = lambda *s_: torch.empty(*s_, device=self.device, dtype=F32)  # noqa: E731
        maxrows = max(ts[i + 1] for i in range(L)) * P
        b = {"x0": e(ts[0] * P, C), "xa": e(maxrows, C), "xb": e(maxrows, C), "xg": e(maxrows, C),
             "skipcat": e(tf * P, L * C), "skr": e(tf * P, cfg.S), "e1": e(tf * P, cfg.E), "y": e(tf * P, cfg.O),
             "adp": torch.zeros(cfg.NP, cfg.NP, device=self.device, dtype=F32) if cfg.adp_params else None,
             "metrics": e(4),
             "ws": e(_lib.load().gwn_masked_loss_workspace_floats(B, cfg.O, cfg.N, tf) + 16)}
        self._scratch[key] = b
        return b

    def infer(self, flat, fixed_sups, x, bn_bufs, lead_pad=0):
        """Eval-mode forward when no backward follows (model.py:175-241 with the module in eval
        mode under torch.no_grad, as in train.py:385-386 / test.py:65-66): the schedule of
        forward() minus the state a backward needs -- no (tanh, sigmoid) pairs, no hop pieces in
        HBM, BatchNorm with running statistics folded into the fused GCN epilogue (no z), the
        layer activations in two ping-pong buffers.  Returns (out [B, O, N, T_f], buffers)."""
        cfg = self.cfg
        C, N, L = cfg.C, cfg.N, cfg.L
        if x.dim() != 4:
            raise RuntimeError("gwnet: expected a 4-D input [B, C, N, T], got %d-D" % x.dim())
        B, cin, n, t_in = x.shape
        if n != N or cin != cfg.Cin:
            raise RuntimeError("gwnet: expected input [B, %d, %d, T], got %s" % (cfg.Cin, N, tuple(x.shape)))
        if x.dtype != F32 or not x.is_cuda:
            raise RuntimeError("gwnet (gwn_amd): input must be a float32 CUDA/HIP tensor")
        ts = cfg.times(t_in + lead_pad)
        if ts[-1] < 1:
            raise RuntimeError("gwnet: input too short for the receptive field")
        st = _lib.stream()
        self.pack_params(flat)
        P = B * N
        tf = ts[-1]
        bf = self._infer_bufs(B, ts)
        sups = list(fixed_sups) if cfg.use_gcn else []
        if cfg.adp_params:
            _lib.call("gwn_adaptive_adj_fwd", ptr(self.pk("nv1")), ptr(self.pk("nv2")), N, 10, ptr(bf["adp"]),
                      cfg.NP, st)
            sups.append(bf["adp"])
        sup_arr = (ctypes.c_void_p * max(len(sups), 1))(*[s_.data_ptr() for s_ in sups])
        bf["sup2_arr"] = bf["g4f_arr"] = None
        if self._pow_ok(1):
            sq2, _, g4f, _ = self._fixed_squares(fixed_sups)
            g4f_p = [t_.data_ptr() for t_ in g4f] if g4f is not None else []
            if cfg.adp_params:
                if "adp2" not in bf:
                    bf["adp2"] = torch.empty(cfg.NP, cfg.NP, device=self.device, dtype=F32)
                    bf["adp2_t"] = torch.empty(cfg.NP, cfg.NP, device=self.device, dtype=F32)
                _lib.call("gwn_support_square", ptr(bf["adp"]), cfg.NP, cfg.NP, ptr(bf["adp2"]), ptr(bf["adp2_t"]),
                          None, st)
                sq2 = sq2 + [bf["adp2"]]
                if self._t16_ok():
                    if "g4_adp" not in bf:
                        bf["g4_adp"] = torch.empty(2, int(_lib.load().gwn_support_g4_floats(N)), device=self.device,
                                                   dtype=F32)
                    self._g4_into([bf["adp"], bf["adp2"]], bf["g4_adp"])
                    g4f_p += [bf["g4_adp"][0].data_ptr(), bf["g4_adp"][1].data_ptr()]
            bf["sup2_arr"] = (ctypes.c_void_p * len(sq2))(*[t_.data_ptr() for t_ in sq2])
            if self._t16_ok() and len(g4f_p) == 2 * len(sups):
                bf["g4f_arr"] = (ctypes.c_void_p * len(g4f_p))(*g4f_p)
        planes = self.split_planes()
        g4bf = None
        if planes and sups:
            # bf16 mode: the bf16 tile copies of (A_k, A_k^2), the adaptive one's rebuilt per call
            hold = bf.get("g4b_holder")
            if hold is None:
                hold = bf["g4b_holder"] = _G4Holder()
            hold.adp, hold.training, hold.supT = bf["adp"], False, None
            g4bf = self._g4_bf16(fixed_sups, hold, st)
        planes = planes if g4bf is not None else 0
        sx = x.stride()
        _lib.call("gwn_start_conv_fwd", ptr(x), sx[0], sx[1], sx[2], sx[3], B, cin, N, t_in, ts[0],
                  ptr(self.pk("start_w")), ptr(self.pk("start_b")), C, ptr(bf["x0"]), None, st)
        xcur = bf["x0"]
        for i in range(L):
            d = cfg.dilations[i]
            ta = _lib.TcnArgs(x=ptr(xcur), t_in=ts[i], P=P, c=C, dilation=d,
                              w_fg=ptr(self.pk("fg_w%d" % i)), b_fg=ptr(self.pk("fg_b%d" % i)),
                              xg=ptr(bf["xg"]), ld_xg=C, fg=None,
                              skipcat=bf["skipcat"].data_ptr() + 4 * i * C, ld_skip=L * C,
                              skip_row0=(ts[i + 1] - tf) * P, ntaps=cfg.K, c_out=cfg.D)
            _lib.call("gwn_gated_tcn_fwd", ctypes.byref(ta), st)
            if i == L - 1:
                break  # the last gcn / bn output never reaches the output
            xnext = bf["xa"] if xcur is not bf["xa"] else bf["xb"]
            rm, rv, _, eps, _ = bn_bufs[i]
            ga = _lib.GcnArgs(rows=ts[i + 1] * P, n=N, c=C, nsup=cfg.nsup if cfg.use_gcn else 0,
                              sup=ctypes.cast(sup_arr, ctypes.POINTER(ctypes.c_void_p)), ld_sup=cfg.NP,
                              h=ptr(bf["xg"]), ld_h=C,
                              w_mlp=ptr(self.pk("mlp_w%d" % i)), b_mlp=ptr(self.pk("mlp_b%d" % i)),
                              residual=xcur.data_ptr() + 4 * d * P * C, z=None,
                              seed_ptr=ptr(self.seed), salt=i, drop_p=0.0, bn_partials=None,
                              no_pieces=1, bn_running_mean=ptr(rm), bn_running_var=ptr(rv),
                              bn_weight=ptr(self.pk("bn_g%d" % i)), bn_bias=ptr(self.pk("bn_b%d" % i)),
                              bn_eps=eps, bn_out=ptr(xnext), sup2=self._arr_field(bf["sup2_arr"]),
                              sup_g4=self._arr_field(bf["g4f_arr"]),
                              w_mlp_t=ptr(self.pk("mlp_wT%d" % i)),
                              sup_g4b=self._arr_field(g4bf), split_planes=planes)
            _lib.call("gwn_gcn_fwd", ctypes.byref(ga), st)
            xcur = xnext
        self._head_fwd(bf["skipcat"], bf["skr"], bf["e1"], bf["y"], tf * P, None)
        out = torch.empty(B, cfg.O, N, tf, device=self.device, dtype=F32)
        _lib.call("gwn_to_nchw", ptr(bf["y"]), B, cfg.O, N, tf, ptr(out), st)
        return out, bf

    # ---------------------------------------------------------------------------------------
    def backward(self, acts, dout):
        """Gradients of every active parameter into self.gpacked (kernel layout).  dout: the output
        gradient [B, O, N, T_f], or None when scratch "dy" already holds it in row layout
        (gwn_masked_loss_rows)."""
        for _ in self.backward_stages(acts, dout):
            pass

    def early_grad_range(self):
        """The flat range [a, b) whose gradients are final after the head stage of the backward
        (backward_stages' first yield): end_conv_1's weight and bias (written at once by its
        weight-gradient GEMM, the largest single gradient: 131.6k of the ~300k floats at METR-LA).
        None when they are not contiguous or not active."""
        lay = self.layout
        w, b = lay.flat_off.get("end_conv_1.weight"), lay.flat_off.get("end_conv_1.bias")
        if w is None or b is None:
            return None
        a0, a1 = w[0], w[0] + int(torch.Size(w[1]).numel())
        if b[0] != a1:
            return None
        return a0, a1 + int(torch.Size(b[1]).numel())

    def unpack_grads_range(self, gflat, a, b):
        """unpack_grads for flat entries [a, b) only."""
        if b > a:
            _lib.call("gwn_gather", ptr(self.gpacked), self.uidx.data_ptr() + 4 * a, gflat.data_ptr() + 4 * a, b - a,
                      _lib.stream())

    def backward_stages(self, acts, dout):
        """backward as a generator: it yields once after the head (end_conv_2 / end_conv_1 / skip
        convs: early_grad_range is final then), so a data-parallel trainer can start that range's
        all-reduce while the layers' backward runs; the rest completes when the generator ends."""
        cfg = self.cfg
        C, D, N, L, S, E, O = cfg.C, cfg.D, cfg.N, cfg.L, cfg.S, cfg.E, cfg.O
        B, ts, P = acts.B, acts.ts, acts.P
        tf = ts[-1]
        rows_f = tf * P
        sc = self.scratch(B, ts)
        ws = sc["ws"]
        st = _lib.stream()
        lib = _lib
        OP = cfg.OP
        if dout is not None:
            dout = dout.contiguous()
            lib.call("gwn_from_nchw_ld", ptr(dout), B, O, N, tf, ptr(sc["dy"]), OP, st)
        # (Weight / adjacency gradients on a second stream beside the input gradients were measured
        # slower in rounds 1, 2 and 5 -- the co-running launches slow the data path more than they
        # hide, DESIGN.md section 4 -- and are not built.)
        # fused layer backward: BN backward in the gcn_bwd prologue, gate backward in its epilogue,
        # the next BN's statistics in the TCN input-gradient epilogue (3 launches fewer per layer)
        fuse = self._fuse_ok(acts)
        # weight / adjacency gradients as partials, one reduction launch for the whole backward
        defer = fuse and self._defer_ok(sc)
        if getattr(acts, "pieces_b", False) and not (defer and "dh_l" in sc):
            raise RuntimeError("gwn_amd: the forward stored bf16 hop pieces for the grouped weight gradient, "
                               "which this backward does not run")
        segs = []
        gram_now = None
        # the adaptive support's gradient of every layer in one gwn_gram_group launch at the end
        # (fp32 mode; the bf16 mode's tiled-operand gram stays per layer)
        gram_group = (defer and "tt_l" in sc and cfg.adp_live and not getattr(acts, "gram_g4", False)
                      and getattr(acts, "g4bt_arr", None) is None and L >= 2)
        # the bf16 mode's counterpart on the tiled operands (each layer's t1 / t2 in acts.TG4[i])
        gram_g4_group = (defer and getattr(acts, "gram_g4", False) and cfg.adp_live and L >= 2
                         and getattr(acts, "ws_g4g", None) is not None and acts.ws_g4g is not False
                         and len(acts.TG4) == L - 1)

        def head_wgrad(dY, J, X, Kc, w, b, ldy=None):
            # (the head's weight gradients on a second stream beside its input gradients, joined
            # before the deferred reduction, measured slower: 24.4-24.7k vs 25.0k samples/s,
            # profiles/r05/head_side)
            wgrad(dY, J, X, Kc, rows_f, w, ws, b, ldy=ldy)

        nt = self._head_nt()
        hb = nt and self.head_bf16()

        def head_wgrad_bf16(dY, J, X, Kc, w, b, key, now=False):
            # the bf16 mode: partials on bf16 operands over row chunks (gwn_wgrad_bf16_partials),
            # reduced with the deferred ones at the end of the backward, else (or now: end_conv_1,
            # final at the head stage's yield, early_grad_range) right away.  (An fp32 form of this
            # kernel for the fp32 head measured 94 + 58 us against the split-K GEMM's 57 + 38:
            # latency-bound at one workgroup per CU)
            n = _lib.load().gwn_wgrad_bf16_partial_count(rows_f, J, Kc)
            part = sc.get(key)
            if part is None or part.numel() < n * (J * Kc + J):
                part = sc[key] = torch.empty(n * (J * Kc + J), device=self.device, dtype=F32)
            lib.call("gwn_wgrad_bf16_partials", ptr(dY), J, J, ptr(X), Kc, Kc, rows_f, ptr(part), st)
            seg = _lib.ReduceSeg(part=ptr(part), nparts=n, part_stride=J * Kc + J, J=J, Kc=Kc, out=ptr(w), ld_out=Kc,
                                 out2=ptr(b), db_off=J * Kc)
            if defer and not now:
                segs.append(seg)
            else:
                lib.call("gwn_reduce_partials", (_lib.ReduceSeg * 1)(seg), 1, st)

        # end_conv_2: its weight gradient from the 32-column padded output gradient on the row
        # reduction kernel (deferred), else the split-K GEMM
        if defer and "part_e2g" in sc:  # one-problem gwn_wgrad_group (4 column groups per workgroup)
            part, nparts = sc["part_e2g"]
            pr = _lib.WgradProblem(dY=ptr(sc["dy"]), ldy=OP, X=ptr(acts.e1), ldx=E, x_rows=rows_f, shift=0,
                                   part=ptr(part), R=rows_f)
            lib.call("gwn_wgrad_group", (_lib.WgradProblem * 1)(pr), 1, OP, E, 1, st)
            segs.append(_lib.ReduceSeg(part=ptr(part), nparts=nparts, part_stride=OP * E + OP, J=O, Kc=E,
                                       out=ptr(self.gk("e2_w")), ld_out=E, out2=ptr(self.gk("e2_b")), db_off=OP * E))
        elif defer and "part_e2" in sc:
            part = sc["part_e2"]
            lib.call("gwn_wgrad_partials", ptr(sc["dy"]), OP, OP, ptr(acts.e1), E, rows_f, E, 1, 0, rows_f,
                     None, None, None, ptr(part), st)
            segs.append(_lib.ReduceSeg(part=ptr(part), nparts=_lib.load().gwn_wgrad_partial_count(rows_f, OP, E),
                                       part_stride=OP * E + OP, J=O, Kc=E, out=ptr(self.gk("e2_w")), ld_out=E,
                                       out2=ptr(self.gk("e2_b")), db_off=OP * E))
        else:
            head_wgrad(sc["dy"], O, acts.e1, E, self.gk("e2_w"), self.gk("e2_b"), ldy=OP)
        if nt:
            gemm_nt(sc["dy"], OP, self.pk("e2_wT"), O, sc["de1"], E, rows_f, E, O, mask=acts.e1, ldmask=E)
        else:
            gemm(sc["dy"], OP, 1, self.pk("e2_w"), E, 1, sc["de1"], E, 1, M=rows_f, N=E, K=O,
                 epi=2, mask=acts.e1, ldmask=E)
        # end_conv_1
        if hb:
            head_wgrad_bf16(sc["de1"], E, acts.skr, S, self.gk("e1_w"), self.gk("e1_b"), "part_hb_e1", now=True)
        else:
            head_wgrad(sc["de1"], E, acts.skr, S, self.gk("e1_w"), self.gk("e1_b"))
        if nt:
            gemm_nt(sc["de1"], E, self.pk("e1_wT"), E, sc["dsk"], S, rows_f, S, E, mask=acts.skr, ldmask=S, bf16=hb)
        else:
            gemm(sc["de1"], E, 1, self.pk("e1_w"), S, 1, sc["dsk"], S, 1, M=rows_f, N=S, K=E,
                 epi=2, mask=acts.skr, ldmask=S)
        # skip convs
        if hb:
            head_wgrad_bf16(sc["dsk"], S, acts.skipcat, L * D, self.gk("skip_w"), self.gk("skip_bsum"), "part_hb_skip")
        else:
            head_wgrad(sc["dsk"], S, acts.skipcat, L * D, self.gk("skip_w"), self.gk("skip_bsum"))
        if nt:
            gemm_nt(sc["dsk"], S, self.pk("skip_wT"), S, sc["dskipcat"], L * D, rows_f, L * D, S, bf16=hb)
        else:
            gemm(sc["dsk"], S, 1, self.pk("skip_w"), L * D, 1, sc["dskipcat"], L * D, 1, M=rows_f, N=L * D, K=S)
        yield "head"
        dnext = None
        bufs = [sc["dxa"], sc["dxb"]]
        first_adp = True
        adp_index = cfg.nsup - 1 if cfg.adp_params else -1
        for i in range(L - 1, -1, -1):
            d, sh = cfg.dilations[i], cfg.shift(i)
            rows = ts[i + 1] * P
            dx = bufs[i % 2]
            dh, dhc, dfg = sc["dh"], sc["dhc"], sc["dfg"]
            grouped = defer and "dh_l" in sc
            if grouped:  # this layer's own dh / dfg, read by the grouped weight gradients at the end
                dh, dfg = sc["dh_l"][i], sc["dfg_l"][i]
            ld_dhc = cfg.W
            if gram_group and i < L - 1:  # this layer's own t1 / t2 (grouped gram at the end)
                dhc, ld_dhc = sc["tt_l"][i], 3 * C
            dxg, ld_dxg, acc = None, 0, 0
            drop = float(self.dropout) if (acts.training and cfg.use_gcn) else 0.0
            if dnext is not None:
                if not fuse:
                    lib.call("gwn_batchnorm_bwd", ptr(dnext), ptr(acts.Z[i]), rows, C, ptr(self.pk("bn_g%d" % i)),
                             ptr(acts.mean[i]), ptr(acts.rstd[i]), ptr(self.gk("bn_g%d" % i)),
                             ptr(self.gk("bn_b%d" % i)), ptr(dx), sh * P, ptr(dh), ptr(acts.seed), i,
                             drop, 1 if acts.training else 0, ptr(ws), st)
                gb = _lib.GcnBwdArgs(rows=rows, n=N, c=D, c_out=C, nsup=cfg.nsup if cfg.use_gcn else 0,
                                     sup=ctypes.cast(acts.sup_arr, ctypes.POINTER(ctypes.c_void_p)),
                                     ld_sup=cfg.NP,
                                     h=ptr(acts.H[i]), ld_h=cfg.W, w_mlp=ptr(self.pk("mlp_w%d" % i)),
                                     dh=ptr(dh), dhcat=ptr(dhc), ld_dhcat=ld_dhc,
                                     dw_mlp=ptr(self.gk("mlp_w%d" % i)), db_mlp=ptr(self.gk("mlp_b%d" % i)),
                                     adp_index=adp_index, dadp=ptr(sc["dadp"]),
                                     accumulate_dadp=0 if first_adp else 1, workspace=ptr(ws),
                                     sup_t=ctypes.cast(acts.supT_arr, ctypes.POINTER(ctypes.c_void_p))
                                     if acts.supT_arr is not None else None,
                                     skip_weight_grads=1 if defer else 0,
                                     # power-schedule backward (the persistent 16-node tile
                                     # kernel: 750 vs 863 us per step for the chained one, 21.3k
                                     # vs 20.5k samples/s)
                                     sup2_t=self._arr_field(getattr(acts, "sup2t_arr", None)),
                                     sup_g4_t=self._arr_field(getattr(acts, "g4b_arr", None)),
                                     sup_g4b_t=self._arr_field(getattr(acts, "g4bt_arr", None)),
                                     tg4=(ptr(acts.TG4[i]) if gram_g4_group else ptr(sc["tg4"]))
                                     if (defer and getattr(acts, "gram_g4", False) and adp_index >= 0) else None,
                                     **self.ksplit_fields(sc))
                sb = getattr(acts, "sup_batch", 1)
                if sb > 1:
                    gb.sup_bstride, gb.sup_batch = cfg.NP * cfg.NP, sb
                if getattr(acts, "g4bt_arr", None) is not None:  # bf16 operands (fp32 accumulation)
                    gb.split_planes = getattr(acts, "planes", 1)
                if fuse:
                    gb.dh = None
                    gb.bn_dy, gb.bn_z = ptr(dnext), ptr(acts.Z[i])
                    gb.bn_gamma, gb.bn_mean, gb.bn_rstd = ptr(self.pk("bn_g%d" % i)), ptr(acts.mean[i]), ptr(acts.rstd[i])
                    gb.bn_sums, gb.bn_dgamma, gb.bn_dbeta = ptr(sc["bnsums"]), ptr(self.gk("bn_g%d" % i)), ptr(self.gk("bn_b%d" % i))
                    gb.dres, gb.dh_out = dx.data_ptr() + 4 * sh * P * C, ptr(dh)
                    gb.seed_ptr, gb.salt, gb.drop_p = ptr(acts.seed), i, drop
                    gb.fg, gb.dskip, gb.ld_dskip = ptr(acts.FG[i]), sc["dskipcat"].data_ptr() + 4 * i * D, L * D
                    gb.skip_row0, gb.dfg = (ts[i + 1] - tf) * P, ptr(dfg)
                lib.call("gwn_gcn_bwd", ctypes.byref(gb), st)
                if defer:
                    if not grouped:
                        self._defer_gcn_grads(acts, i, rows, dh, sc, segs, st)
                    if adp_index >= 0 and not (gram_group or gram_g4_group):  # after the layer's TCN backward
                        gram_now = (dhc, first_adp)
                if adp_index >= 0:
                    first_adp = False
                dxg, ld_dxg, acc = dhc, ld_dhc, 1
            xin, _, _, raff = self.layer_input(acts, i)
            tb = _lib.TcnBwdArgs(x=xin, x_mean=raff[0], x_scale=raff[1], x_shift=raff[2], t_in=ts[i], P=P, c=C,
                                 dilation=d, ntaps=cfg.K, c_out=D,
                                 w_fg=ptr(self.pk("fg_w%d" % i)), fg=ptr(acts.FG[i]),
                                 dxg=ptr(dxg), ld_dxg=ld_dxg,
                                 dskip=sc["dskipcat"].data_ptr() + 4 * i * D, ld_dskip=L * D,
                                 skip_row0=(ts[i + 1] - tf) * P, dfg=ptr(dfg),
                                 dw_fg=ptr(self.gk("fg_w%d" % i)), db_fg=ptr(self.gk("fg_b%d" % i)),
                                 dx=ptr(dx), accumulate_dx=acc, workspace=ptr(ws),
                                 skip_weight_grads=1 if defer else 0)
            if fuse:
                if dnext is not None:
                    tb.dfg_ready, tb.acc_row0 = 1, sh * P
                if i >= 1:  # statistics of bn[i-1], whose output gradient is this dx
                    tb.bn_z, tb.bn_mean, tb.bn_rstd = ptr(acts.Z[i - 1]), ptr(acts.mean[i - 1]), ptr(acts.rstd[i - 1])
                    tb.bn_sums = ptr(sc["bnsums"])
            lib.call("gwn_gated_tcn_bwd", ctypes.byref(tb), st)
            if defer:
                if not grouped:
                    part = sc["part_tcn"][i]
                    lib.call("gwn_wgrad_partials", ptr(dfg), 2 * C, 2 * C, xin, C, ts[i] * P, C, 2, d * P, rows,
                             raff[0], raff[1], raff[2], ptr(part), st)
                    segs.append(_lib.ReduceSeg(part=ptr(part),
                                               nparts=_lib.load().gwn_wgrad_partial_count(rows, 2 * C, 2 * C),
                                               part_stride=4 * C * C + 2 * C, J=2 * C, Kc=2 * C,
                                               out=ptr(self.gk("fg_w%d" % i)), ld_out=2 * C,
                                               out2=ptr(self.gk("fg_b%d" % i))))
                if gram_now is not None:
                    self._defer_gram(acts, i, rows, gram_now[0], adp_index, gram_now[1], sc, st)
                    gram_now = None
            dnext = dx
        # start conv
        rows0 = ts[0] * P
        if defer and "part_start" in sc:
            part = sc["part_start"]
            lib.call("gwn_wgrad_partials", ptr(dnext), C, C, ptr(acts.xin), cfg.Cin, rows0, cfg.Cin, 1, 0, rows0,
                     None, None, None, ptr(part), st)
            segs.append(_lib.ReduceSeg(part=ptr(part), nparts=_lib.load().gwn_wgrad_partial_count(rows0, C, cfg.Cin),
                                       part_stride=C * cfg.Cin + C, J=C, Kc=cfg.Cin, out=ptr(self.gk("start_w")),
                                       ld_out=cfg.Cin, out2=ptr(self.gk("start_b"))))
        else:
            wgrad(dnext, C, acts.xin, cfg.Cin, rows0, self.gk("start_w"), ws, self.gk("start_b"))
        if defer and "dh_l" in sc:
            self._group_wgrads(acts, sc, segs, st)
        if gram_group:
            lay = []
            for i in range(L - 1):
                h, t = acts.H[i].data_ptr(), sc["tt_l"][i].data_ptr()
                lay.append(_lib.GramLayer(x1=h, t1=t + 4 * C, x2=h + 4 * (1 + 2 * adp_index) * C, t2=t + 8 * C,
                                          slices=ts[i + 1] * P // N))
            for c, ch in enumerate(_layer_chunks(len(lay))):
                sub = [lay[i] for i in ch]
                lib.call("gwn_gram_group", (_lib.GramLayer * len(sub))(*sub), len(sub), cfg.W, 3 * C, N,
                         ptr(sc["dadp"]), cfg.NP, int(c > 0), ptr(sc["ws_gram_group"]), st)
        if gram_g4_group:
            lay = []
            for i in range(L - 1):
                S = ts[i + 1] * P // N
                half = S * ((N + 15) // 16) * 1024  # bytes of one bf16 operand
                x, t = acts.XG4[i].data_ptr(), acts.TG4[i].data_ptr()
                lay.append(_lib.GramLayer(x1=x, t1=t, x2=x + half, t2=t + half, slices=S))
            for c, ch in enumerate(_layer_chunks(len(lay))):
                sub = [lay[i] for i in ch]
                lib.call("gwn_gram_g4_group", (_lib.GramLayer * len(sub))(*sub), len(sub), N, ptr(sc["dadp"]),
                         cfg.NP, int(c > 0), ptr(acts.ws_g4g), st)
        if defer:
            for k in range(0, len(segs), 32):  # <= 32 segments per launch (include/gwn.h)
                chunk = segs[k:k + 32]
                lib.call("gwn_reduce_partials", (_lib.ReduceSeg * len(chunk))(*chunk), len(chunk), st)
        if cfg.adp_live:
            lib.call("gwn_adaptive_adj_bwd", ptr(self.pk("nv1")), ptr(self.pk("nv2")), ptr(acts.adp),
                     ptr(sc["dadp"]), N, 10, cfg.NP, ptr(self.gk("nv1")), ptr(self.gk("nv2")), ptr(ws), st)

    # ---------------------------------------------------------------------------------------
    def _head_nt(self):
        """Row-tile NT GEMMs for the head (K dims / leading dims multiples of 4)."""
        cfg = self.cfg
        return all(v % 4 == 0 for v in (cfg.O, cfg.S, cfg.E, cfg.L * cfg.D))

    def head_bf16(self):
        """The bf16 mode's head (split_planes 2, configs[2]): the skip convs' and end_conv_1's GEMMs,
        their input gradients (gwn_gemm_nt_bf16) and weight gradients (gwn_wgrad_bf16_partials) on
        bf16 operands, fp32 in and out, fp32 sums; end_conv_2 (12 outputs) and the bias gradients
        stay fp32."""
        cfg = self.cfg
        return (self._head_nt() and self.split_planes() == 2 and cfg.S % 128 == 0 and cfg.E % 128 == 0
                and (cfg.L * cfg.D) % 128 == 0)

    def _fuse_ok(self, acts):
        cfg = self.cfg
        return (os.environ.get("GWN_FUSE_BWD", "1") != "0" and cfg.use_gcn and cfg.C == 32 and cfg.square
                and cfg.W % 32 == 0 and cfg.N <= 512 and acts.supT_arr is not None)

    def _defer_ok(self, sc):
        """Deferred weight / adjacency gradients (the fused C = 32 shapes; otherwise each is
        reduced in its own launches right after its layer)."""
        return "part_mlp" in sc

    @staticmethod
    def _group_plan(rows, J, Kt, ntaps):
        """Partial slots per problem of a gwn_wgrad_group launch (None: shape not built)."""
        lib = _lib.load()
        if not rows or len(rows) > 8 or not lib.gwn_wgrad_group_supported(J, Kt, ntaps):
            return None
        R = (ctypes.c_int * len(rows))(*rows)
        nb = (ctypes.c_int * len(rows))()
        if lib.gwn_wgrad_group_plan(R, len(rows), J, Kt, ntaps, nb) <= 0:
            return None
        return list(nb)

    def _group_wgrads(self, acts, sc, segs, st):
        """Every layer's gcn-mlp dW / db and gated-TCN dW / db: two gwn_wgrad_group launches over the
        layers' own dh / dfg, their partials reduced with the rest by gwn_reduce_partials."""
        cfg = self.cfg
        C, W, L, P = cfg.C, cfg.W, cfg.L, acts.P
        ts = acts.ts
        gm, gt = sc["group_np"]
        probs = []
        for i in range(L - 1):
            rows = ts[i + 1] * P
            part = sc["group_mlp"][i]
            pr = _lib.WgradProblem(dY=ptr(sc["dh_l"][i]), ldy=C, X=ptr(acts.H[i]), ldx=W, x_rows=rows, shift=0,
                                   part=ptr(part), R=rows)
            if getattr(acts, "pieces_b", False):  # the hop pieces as bf16 (columns 32 .. W)
                pr.Xb, pr.ldxb = acts.HB[i].data_ptr(), W - C
            probs.append(pr)
            segs.append(_lib.ReduceSeg(part=ptr(part), nparts=gm[i], part_stride=C * W + C, J=C, Kc=W,
                                       out=ptr(self.gk("mlp_w%d" % i)), ld_out=W, out2=ptr(self.gk("mlp_b%d" % i))))
        _lib.call("gwn_wgrad_group", (_lib.WgradProblem * len(probs))(*probs), len(probs), C, W, 1, st)
        probs = []
        ida = sc["aff_id"].data_ptr()
        for i in range(L):
            rows = ts[i + 1] * P
            xin, _, _, raff = self.layer_input(acts, i)
            if raff[0] is None:  # identity affine: (x - 0) * 1 + 0, exact
                raff = (ida, ida + 4 * C, ida + 8 * C)
            part = sc["group_tcn"][i]
            probs.append(_lib.WgradProblem(dY=ptr(sc["dfg_l"][i]), ldy=2 * C, X=xin, ldx=C, x_rows=ts[i] * P,
                                           shift=cfg.dilations[i] * P, x_mean=raff[0], x_scale=raff[1],
                                           x_shift=raff[2], part=ptr(part), R=rows))
            segs.append(_lib.ReduceSeg(part=ptr(part), nparts=gt[i], part_stride=4 * C * C + 2 * C, J=2 * C,
                                       Kc=2 * C, out=ptr(self.gk("fg_w%d" % i)), ld_out=2 * C,
                                       out2=ptr(self.gk("fg_b%d" % i))))
        _lib.call("gwn_wgrad_group", (_lib.WgradProblem * len(probs))(*probs), len(probs), 2 * C, C, 2, st)

    def _defer_gcn_grads(self, acts, i, rows, dh, sc, segs, st):
        """Layer i's dW_mlp / db_mlp partials for the end-of-backward reduction."""
        cfg = self.cfg
        C, W = cfg.C, cfg.W
        part = sc["part_mlp"][i]
        _lib.call("gwn_wgrad_partials", ptr(dh), C, C, ptr(acts.H[i]), W, rows, W, 1, 0, rows, None, None, None,
                  ptr(part), st)
        segs.append(_lib.ReduceSeg(part=ptr(part), nparts=_lib.load().gwn_wgrad_partial_count(rows, C, W),
                                   part_stride=C * W + C, J=C, Kc=W, out=ptr(self.gk("mlp_w%d" % i)),
                                   ld_out=W, out2=ptr(self.gk("mlp_b%d" % i))))

    def _defer_gram(self, acts, i, rows, dhc, adp_index, first_adp, sc, st):
        """Layer i's share of the adaptive-support gradient (gwn_gram, reduced into dadp right away:
        deferring its partials too wrote 12.8 MB of fresh partial slots per layer and slowed every
        gram launch by 20-30 %, more than the 7 reduce launches it saved)."""
        cfg = self.cfg
        C, W = cfg.C, cfg.W
        if getattr(acts, "gram_g4", False):
            # bf16 mode, tiled operands: X / hop 1 from the forward (acts.XG4[i]), t1 / t2 from this backward
            S = rows // cfg.N
            half = S * ((cfg.N + 15) // 16) * 1024  # bytes of one bf16 operand
            x, t = acts.XG4[i].data_ptr(), sc["tg4"].data_ptr()
            _lib.call("gwn_gram_g4_bf16", x, t, x + half, t + half, cfg.N, S, ptr(sc["dadp"]), cfg.NP, 0 if first_adp else 1,
                      ptr(sc["ws"]), st)
            return
        h = acts.H[i].data_ptr()
        t = dhc.data_ptr()
        fn = "gwn_gram_bf16" if getattr(acts, "g4bt_arr", None) is not None else "gwn_gram"
        _lib.call(fn, h, t + 4 * C, h + 4 * (1 + 2 * adp_index) * C, t + 4 * 2 * C, W, W, cfg.N, rows // cfg.N,
                  ptr(sc["dadp"]), cfg.NP, 0 if first_adp else 1, ptr(sc["ws"]), st)

    def unpack_grads(self, gflat, norm_ws=None):
        """Kernel-layout gradients -> the flat buffer; with norm_ws also the clip-norm partials (the
        optimizer's workspace, gwn_gather_sqnorm)."""
        if norm_ws is not None:
            _lib.call("gwn_gather_sqnorm", ptr(self.gpacked), ptr(self.uidx), ptr(gflat), self.layout.flat_total,
                      ptr(norm_ws), _lib.stream())
        else:
            _lib.call("gwn_gather", ptr(self.gpacked), ptr(self.uidx), ptr(gflat), self.layout.flat_total,
                      _lib.stream())


def _ksplit_thin(M, N, K):
    """Split-K for a thin output (N <= 32, e.g. end_conv_2: 12 columns) with a long K: the
    256 x 32 tiles alone give too few workgroups to fill the chip."""
    blocks = (M + 255) // 256
    if N > 32 or K < 256 or blocks >= 512:
        return 1
    return max(1, min(512 // blocks, K // 64))


def _ksplit(M, N, K):
    """Split-K of the head weight gradients (K = positions): up to 1024 tiles x splits, chunks of
    >= 192 rows.  Measured (tools/bench_head.py, METR B=64, profiles/r04/head_gemm_sweep.txt):
    end_conv_1 dW 49 splits 63.9 us, 64 splits 53.0 us (128 x 128 tiles fill the chip); skip dW
    35.4 / 33.7 us."""
    tiles = ((M + 127) // 128) * ((N + 63) // 64)
    ks = max(1, min(1024 // max(tiles, 1), K // 192))
    return ks


def gemm(A, lda_m, lda_k, B, ldb_k, ldb_n, Cout, ldc_m, ldc_n, M, N, K, bias=None, relu=0, epi=0,
         mask=None, ldmask=0, C0=None, ldc0=0, beta=1.0, ksplit=1, part=None, ones_out=None):
    d = _lib.GemmDesc()
    d.A, d.lda_m, d.lda_k = ptr(A), lda_m, lda_k
    d.B, d.ldb_k, d.ldb_n = ptr(B), ldb_k, ldb_n
    d.C, d.ldc_m, d.ldc_n = ptr(Cout), ldc_m, ldc_n
    d.M, d.N, d.K = M, N, K
    d.alpha = 1.0
    d.beta = beta
    d.bias_n = ptr(bias)
    d.relu = relu
    d.epi = epi
    d.mask, d.ldmask_m = ptr(mask), ldmask
    if C0 is not None:
        d.C0, d.ldc0_m, d.ldc0_n = ptr(C0), ldc0, 1
    d.ksplit = ksplit
    d.part = ptr(part)
    d.ones_out = ptr(ones_out)
    _lib.call("gwn_gemm", ctypes.byref(d), _lib.stream())


def gemm_nt(A, lda, B, ldb, Cout, ldc, M, N, K, bias=None, relu=0, mask=None, ldmask=0, bf16=False):
    """Cout[m][n] = epi(sum_k A[m][k] B[n][k])  (gwn_gemm_nt; bf16: gwn_gemm_nt_bf16's bf16 operands)."""
    _lib.call("gwn_gemm_nt_bf16" if bf16 else "gwn_gemm_nt", ptr(A), lda, ptr(B), ldb, ptr(Cout), ldc, M, N, K,
              ptr(bias), relu, ptr(mask), ldmask, _lib.stream())


def wgrad(dY, J, X, Kc, rows, out, ws, bias_out=None, ldy=None):
    """out[j][k] = sum_r dY[r][j] * X[r][k]   (1x1 conv weight gradient, split over rows; dY rows
    ldy >= J floats apart); bias_out[j] = sum_r dY[r][j] from the same launch (the GEMM's ones
    column)."""
    ks = _ksplit(J, Kc, rows)
    gemm(dY, 1, ldy or J, X, Kc, 1, out, Kc, 1, M=J, N=Kc, K=rows, ksplit=ks, part=ws, ones_out=bias_out)


GRAM_GL = 8  # layers of one grouped gram launch (gram.hip GL)


def _layer_chunks(n):
    """Layer indices 0..n-1 cut into consecutive chunks of at most GRAM_GL (one grouped gram
    launch each; the later launches accumulate into the first's output)."""
    return [list(range(i, min(n, i + GRAM_GL))) for i in range(0, n, GRAM_GL)]
