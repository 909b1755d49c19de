"""ORACLE (test infrastructure only) — CPU restatement of Graph WaveNet's hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker / CPU baseline.  The product (graph-wavenet_amd/gwn_amd)
never imports it.

It restates, with plain torch-CPU tensor algebra written independently of the reference source,
the arithmetic of:
  * nconv               reference model.py:12-14     ('ncvl,vw->ncwl')
  * nconv2 / gcn2       reference model.py:16-22, 57-80  (per-sample supports 'ncvl,nvw->ncwl')
  * gcn                 reference model.py:41-55     (K supports x order 2, concat, 1x1, dropout)
  * gwnet.forward       reference model.py:175-241   (pad, start conv, 8 gated/dilated layers,
                                                      skip, residual, BN, head)
  * adaptive adjacency  reference model.py:185-188
  * SVD node-embedding init  reference model.py:123-127
  * trainer.train       reference engine.py:41-58    (pad, masked MAE, clip 5, Adam)
  * masked metrics      reference Utils/util.py:510-552
  * asym_adj            reference Utils/util.py:130-136

Parity is PINNED: tests/test_oracle.py checks this restatement against the golden vectors in
tests/golden/*.npz, which tests/golden/make_golden.py produced by running the reference itself.
Default dtype is float64 (the "truth" the fp32 HIP path is compared against).

bf16 emulation (``Cfg(..., gcn_bf16=True)``): the arithmetic of libgwn's bf16 mode
(gwnet.set_compute_dtype("bf16"), configs[2]) with everything else exact -- the diffusion products
of every gcn take bf16-rounded operands (node features, A and A^2 forward; the mlp output
gradient and A, A^2 in the backward) with exact accumulation, the adaptive support's gradient
takes bf16-rounded operands, and the mlp, its weight gradient and every other layer stay exact
(``gcn_bf16``, a custom autograd node); ``gcn_bf16_mlp=True`` also rounds the per-piece mlp's
operands (weights, pieces, backward inputs) as the default bf16 mode does; ``head_bf16=True`` the
head's skip convs and end_conv_1 (their inputs and weights, and the operands of their input and
weight gradients; end_conv_2 and the bias gradients stay exact: ``_HeadLin``) as that mode's head does.  The HIP path accumulates in fp32 instead, so a test can
hold it to the fp32 rounding floor around this reference rather than to the bf16 distance from
the exact model.

Branch pinning (gradient tests only): the head's two ReLUs and the masked MAE (|pred - real|) are
kinked.  An element within fp32 rounding of a kink takes either branch in two equally valid
evaluations, and its gradient jumps.  ``forward`` / ``masked_metrics`` therefore accept the
branch the fp32 run took (``masks``: ReLU masks of the skip sum and of end_conv_1, the sign of
pred - real).  The value on that branch equals the plain one up to rounding; its gradient is the
one-sided gradient of that branch.
"""
import math

import numpy as np
import torch

F64 = torch.float64


class Cfg:
    """Hyper-parameters of one gwnet (reference ctor, model.py:83-86)."""

    def __init__(self, num_nodes, nfixed=2, gcn_bool=True, addaptadj=True, in_dim=2, out_dim=12, nhid=32,
                 skip=None, end=None, blocks=4, layers=2, dropout=0.0, kernel_size=2, dilation_channels=None,
                 first_dilation=1, gcn_bf16=False, gcn_bf16_mlp=False, head_bf16=False):
        self.N, self.nfixed = num_nodes, nfixed
        self.gcn_bool, self.addaptadj = gcn_bool, addaptadj
        self.Cin, self.O, self.C = in_dim, out_dim, nhid
        self.D = dilation_channels if dilation_channels is not None else nhid  # gated-TCN / gcn width
        self.S = skip if skip is not None else 8 * nhid
        self.E = end if end is not None else 16 * nhid
        self.blocks, self.layers, self.dropout = blocks, layers, dropout
        self.kernel_size = kernel_size
        self.gcn_bf16 = gcn_bf16  # libgwn's bf16 mode (module docstring)
        self.gcn_bf16_mlp = gcn_bf16_mlp  # ... with the per-piece mlp on bf16 operands too (_GcnBf16)
        self.head_bf16 = head_bf16  # ... and the skip convs / end_conv_1 on bf16 operands (_HeadLin)
        # gwnet_diff_G starts every block at dilation 4 (model.py:291)
        self.dilations = [first_dilation * 2 ** j for _ in range(blocks) for j in range(layers)]
        # model.py:130-157: every layer adds (kernel_size - 1) * 2^j -- the reference counts from
        # dilation 1 in both models, so for gwnet_diff_G this under-counts (the input must then be
        # long enough by itself)
        self.receptive_field = 1 + (kernel_size - 1) * sum(2 ** j for _ in range(blocks) for j in range(layers))
        self.adaptive = gcn_bool and addaptadj
        # model.py:110-128 + 225: the gcn path runs iff gcn_bool and supports is not None (the
        # adaptive branch turns supports=None into [])
        self.use_gcn = gcn_bool and (nfixed > 0 or self.adaptive)

    @property
    def L(self):
        return self.blocks * self.layers


def asym_adj(adj):
    a = np.asarray(adj, dtype=np.float64)
    rs = a.sum(1)
    with np.errstate(divide="ignore"):
        inv = 1.0 / rs
    inv[~np.isfinite(inv)] = 0.0
    return (inv[:, None] * a).astype(np.float32)


def svd_embeddings(aptinit, rank=10):
    u, s, v = torch.svd(torch.as_tensor(aptinit, dtype=torch.float32))
    r = torch.diag(s[:rank].sqrt())
    return u[:, :rank] @ r, r @ v[:, :rank].t()


def adaptive_adjacency(e1, e2):
    """softmax over rows of relu(E1 E2)."""
    logits = torch.clamp(e1 @ e2, min=0.0)
    logits = logits - logits.max(dim=1, keepdim=True).values
    ex = torch.exp(logits)
    return ex / ex.sum(dim=1, keepdim=True)


def diffuse(x, a):
    """y[b,c,w,t] = sum_v x[b,c,v,t] a[v,w]   (nconv)."""
    b, c, n, t = x.shape
    xt = x.permute(0, 1, 3, 2).reshape(b * c * t, n)
    return (xt @ a).reshape(b, c, t, n).permute(0, 1, 3, 2)


def diffuse_per_sample(x, a):
    """y[b,c,w,t] = sum_v x[b,c,v,t] a[b,v,w]   (nconv2: one support per sample, model.py:16-22)."""
    b, c, n, t = x.shape
    xt = x.permute(0, 1, 3, 2).reshape(b, c * t, n)
    return torch.bmm(xt, a).reshape(b, c, t, n).permute(0, 1, 3, 2)


def gcn2(x, supports, w, bias, order=2):
    """gcn2.forward (model.py:64-80) in eval mode: per-sample supports [B,N,N], piece-major concat
    [x, A1 x, A1^2 x, A2 x, ...], then the 1x1 conv."""
    out = [x]
    for a in supports:
        x1 = diffuse_per_sample(x, a)
        out.append(x1)
        for _ in range(2, order + 1):
            x1 = diffuse_per_sample(x1, a)
            out.append(x1)
    return pointwise(torch.cat(out, dim=1), w, bias)


def bf16_round(t):
    """Round to bf16 (round to nearest even) and back to t's dtype."""
    return t.to(torch.bfloat16).to(t.dtype)


class Bf16Pins:
    """Rounding-boundary pinning of the bf16 emulation (gradient / forward gates of the bf16 mode).

    Rounding an fp32-computed value v = exact + err (|err| <= band) to bf16 and rounding exact itself
    differ when exact lies within band of a rounding boundary (the midpoint of two adjacent bf16
    numbers) -- or, for values so small that band exceeds their ulp, by a few ulps; the difference
    propagates as a ~2^-8 relative change of one operand.  Like the ReLU / |.| branch pinning
    (module docstring), the emulation can take the rounding the HIP run took, element by element,
    where it is such a tie: |hip - exact| <= half an ulp of hip + band (what rounding a value
    within band of exact can give):
      * supports: the HIP run's fp32 A_k and A_k^2 (``sup``: [(A, A2), ...] in support order) are
        checked against the exact ones (max-rel <= ``sup_tol``) and rounded to bf16 in their place;
      * the gcn input g (``g[i]``: the layer's fp32 g, NCHW): bf16(g_hip) is adopted as above with
        band = ``g_band`` * max|g| (the fp32 error the layers below leave in g);
      * the hop pieces (``pieces[i]``: the bf16 pieces the HIP run stored, NCHW [B, 2K*C, N, T]):
        adopted with band = ``piece_band`` * sum|terms| (the fp32 accumulation error bound of the
        diffusion sum, sum|terms| = |rnd(g)| diffused through |rnd(A)|).
    Every difference that is not such a tie is counted in ``report`` as a violation (the tests
    require none); adopted ties are counted too, with the element count of each operand
    (``<tag>_total``): the band is a bound per tensor (a fraction of max|g|), so for elements far
    below the maximum it spans several ulps -- the tests also require the adopted ties to stay a
    small fraction (1e-3) of the elements (``adopted_fraction``), so that a systematic rounding error
    cannot be absorbed as ties."""

    def __init__(self, sup=None, g=None, pieces=None, sup_tol=1e-5, g_band=2.0 ** -16, piece_band=2.0 ** -19,
                 skr=None, head_band=2.0 ** -19, head_dy=None, head_dband=2.0 ** -18):
        self.sup, self.g, self.pieces = sup, g or {}, pieces or {}
        self.sup_tol, self.g_band, self.piece_band = sup_tol, g_band, piece_band
        # the head (head_bf16): the HIP run's fp32 relu(skip) (end_conv_1's operand, NCHW [B, S, N, T_f]),
        # adopted with band = head_band * sum|terms| of the skip sum; its backward's bf16 operands
        # head_dy["de1"] (end_conv_1's output gradient) and head_dy["dsk"] (the skip sum's), adopted
        # with band = head_dband * max|dy| (the fp32 error of short sums, generously)
        self.skr, self.head_band = skr, head_band
        self.head_dy, self.head_dband = head_dy or {}, head_dband
        self.report = {"g_adopted": 0, "g_bad": 0, "piece_adopted": 0, "piece_bad": 0, "sup_err": 0.0,
                       "skr_adopted": 0, "skr_bad": 0, "de1_adopted": 0, "de1_bad": 0, "dsk_adopted": 0,
                       "dsk_bad": 0}

    def adopt(self, own_b, exact, hip_b, band, tag):
        """own_b = bf16(exact); hip_b = the HIP run's bf16 value: hip_b where it is a rounding tie."""
        diff = own_b != hip_b
        self.report[tag + "_total"] = self.report.get(tag + "_total", 0) + own_b.numel()
        if not bool(diff.any()):
            return own_b
        _, e = torch.frexp(hip_b)  # hip = m 2^e, 0.5 <= |m| < 1: a bf16 ulp there is 2^(e - 8)
        half_ulp = torch.ldexp(torch.ones_like(hip_b), e - 9)
        reach = (hip_b - exact).abs() / (half_ulp + band)  # <= 1: a rounding of some value within band of exact
        tie = reach <= 1.0
        ok = diff & tie
        bad = diff & ~tie
        self.report[tag + "_adopted"] += int(ok.sum())
        self.report[tag + "_bad"] += int(bad.sum())
        if bool(bad.any()):  # the first few, for the failure message: (exact, hip, reach)
            det = list(zip(exact[bad].tolist()[:4], hip_b[bad].tolist()[:4], reach[bad].tolist()[:4]))
            self.report.setdefault(tag + "_bad_detail", []).extend(det)
        return torch.where(ok, hip_b, own_b)

    def adopted_fraction(self):
        """{tag: adopted / elements} of every operand the pins saw."""
        return {k[:-len("_total")]: self.report[k[:-len("_total")] + "_adopted"] / max(v, 1)
                for k, v in self.report.items() if k.endswith("_total")}

    def supports(self, sups):
        """the bf16 operands [(rnd(A), rnd(A^2))] of the HIP run's supports (checked)."""
        out = []
        for a, (ha, ha2) in zip(sups, self.sup):
            a2 = a @ a
            for ex, h in ((a, ha), (a2, ha2)):
                e = float((h.to(ex.dtype) - ex).abs().max() / ex.abs().max())
                self.report["sup_err"] = max(self.report["sup_err"], e)
            out.append((bf16_round(ha.to(a.dtype)), bf16_round(ha2.to(a.dtype))))
        return out


class _GcnBf16(torch.autograd.Function):
    """sum_q W_q . piece_q of gcn.forward (model.py:41-55, without the bias) in libgwn's bf16 mode
    (csrc/gcn_fused.hip gcn_fwd_t16b_kernel / gcn_bwd_t16_kernel<., true>, gram.hip
    gwn_gram_g4_bf16): the power schedule, pieces [g, A_1 g, A_1^2 g, A_2 g, ...] with
    A_k^q g = einsum(rnd(g), rnd(A_k^q)) ('ncvl,vw->ncwl'); the backward of the power schedule:
      dg  = W_0^T dy + sum_k W_{1+2k}^T (rnd(A_k) rnd(dy)) + W_{2+2k}^T (rnd(A_k^2) rnd(dy)),
      dW  = dy (x) [g, rnd(pieces)] (exact products; the pieces are stored as bf16 for it),
      dA_k = sum rnd(g) (x) rnd(t1) + rnd(A_k g) (x) rnd(t2),
             t1 = W_{1+2k}^T dy + W_{2+2k}^T (rnd(A_k) rnd(dy)),  t2 = W_{2+2k}^T dy
    (the chained-hop gradient of x2 = (x A) A, as the HIP path forms it).  rnd = bf16_round, or the
    identity (then this equals plain autograd through the chained hops up to reassociation).
    mrnd: the rounding of the per-piece 1x1 mlp's operands (gwn.h GWN_DTYPE_BF16_MLP, the default
    bf16 mode; t16_mlp_b): forward W_q . piece_q -> mrnd(W_q) . mrnd(piece_q), every W_q^T y of the
    backward (dg, t1, t2) -> mrnd(W_q)^T mrnd(y); dW stays exact.  None = exact mlp (GWN_BF16_MLP=0)."""

    @staticmethod
    def forward(ctx, g, w, rnd, mrnd, pin, *sups):
        # pin: (Bf16Pins, layer) -- take the HIP run's roundings where they are ties (Bf16Pins)
        pins, layer = pin if pin is not None else (None, None)
        C = g.shape[1]
        if pins is not None and rnd is bf16_round:
            sr = pins.supports(sups)
            gb = rnd(g)
            if layer in pins.g:
                gb = pins.adopt(gb, g, bf16_round(pins.g[layer].to(g.dtype)), pins.g_band * float(g.abs().max()), "g")
        else:
            sr = [(rnd(a), rnd(a @ a)) for a in sups]
            gb = rnd(g)
        pieces = [g]
        for ra, ra2 in sr:
            pieces += [diffuse(gb, ra), diffuse(gb, ra2)]
        h = torch.cat(pieces, dim=1)
        hb = None  # the bf16-stored hop pieces (the mlp operand in mlp mode, dW's operand)
        if pins is not None and rnd is bf16_round and layer in pins.pieces:
            hp = pins.pieces[layer].to(g.dtype)
            parts = []
            for k, (ra, ra2) in enumerate(sr):
                for q, m in enumerate((ra, ra2)):
                    pi = 1 + 2 * k + q
                    ex = h[:, pi * C:(pi + 1) * C]
                    terms = diffuse(gb.abs(), m.abs())
                    parts.append(pins.adopt(bf16_round(ex), ex, hp[:, (pi - 1) * C:pi * C],
                                            pins.piece_band * terms, "piece"))
            hb = torch.cat(parts, dim=1)
        ctx.rnd, ctx.mrnd = rnd, mrnd
        ctx.sr, ctx.gb, ctx.hb = sr, gb, hb
        ctx.save_for_backward(g, w, h, *sups)
        if mrnd is None:
            return pointwise(h, w)
        hm = mrnd(h) if hb is None else torch.cat([gb if mrnd is bf16_round else mrnd(g), hb], dim=1)
        return pointwise(hm, mrnd(w))

    @staticmethod
    def backward(ctx, dy):
        g, w, h, *sups = ctx.saved_tensors
        rnd, mrnd = ctx.rnd, ctx.mrnd
        C = g.shape[1]
        wr = w.reshape(w.shape[0], -1)
        wm, mr = (wr, lambda t: t) if mrnd is None else (mrnd(wr), mrnd)

        def wt(q, y):  # W_q^T y over the channel axis (the mlp's operand rounding)
            return torch.einsum("oi,bont->bint", wm[:, q * C:(q + 1) * C], mr(y))

        pb = rnd(h[:, C:]) if ctx.hb is None else ctx.hb
        hb = torch.cat([h[:, :C], pb], dim=1)  # the bf16-stored hop pieces
        dw = torch.einsum("bont,bint->oi", dy, hb).reshape(w.shape)
        dyb = rnd(dy)
        dg = wt(0, dy)
        dsups = []
        for k, a in enumerate(sups):
            ra, ra2 = ctx.sr[k]
            # (A y)[v] = sum_w A[v][w] y[w] = diffuse(y, A^T)
            e1 = diffuse(dyb, ra.t())
            e2 = diffuse(dyb, ra2.t())
            dg = dg + wt(1 + 2 * k, e1) + wt(2 + 2 * k, e2)
            da = None
            if ctx.needs_input_grad[5 + k]:
                t1 = wt(1 + 2 * k, dy) + wt(2 + 2 * k, e1)
                t2 = wt(2 + 2 * k, dy)
                x1b = pb[:, 2 * k * C:(2 * k + 1) * C]
                da = torch.einsum("bcvt,bcwt->vw", ctx.gb, rnd(t1)) + torch.einsum("bcvt,bcwt->vw", x1b, rnd(t2))
            dsups.append(da)
        return (dg, dw, None, None, None, *dsups)


class _HeadLin(torch.autograd.Function):
    """pointwise(xb, rnd(w)): one of the bf16 mode's head GEMMs (csrc/gemm_nt.hip gwn_gemm_nt_bf16:
    a skip conv, end_conv_1; model.py:216-222, 238), xb = bf16(x) with the HIP run's ties (Bf16Pins).
    Backward on bf16 operands as well: the input gradient rnd(w)^T rnd(dy) (the transposed-weight
    gwn_gemm_nt_bf16), the weight gradient rnd(dy) (x) xb (gwn_wgrad_bf16_partials, the same bf16
    activations as the forward); the bias gradients (outside) stay exact sums."""

    @staticmethod
    def forward(ctx, x, w, xb, dpin=None):
        # dpin: (Bf16Pins, "de1" | "dsk") -- the HIP run's rounding ties of the output gradient
        ctx.save_for_backward(xb, w)
        ctx.dpin = dpin
        return pointwise(xb, bf16_round(w))

    @staticmethod
    def backward(ctx, dy):
        xb, w = ctx.saved_tensors
        wr = bf16_round(w.reshape(w.shape[0], -1))
        dyb = bf16_round(dy)
        if ctx.dpin is not None:
            pins, key = ctx.dpin
            if key in pins.head_dy:
                hip = bf16_round(pins.head_dy[key].to(dy.dtype))
                dyb = pins.adopt(dyb, dy, hip, pins.head_dband * float(dy.abs().max()), key)
        dx = torch.einsum("oi,bont->bint", wr, dyb)
        dw = torch.einsum("bont,bint->oi", dyb, xb).reshape(w.shape)
        return dx, dw, None, None


def _head_bf16(p, gs, tf, masks, pins):
    """skip sum -> relu -> end_conv_1 of the bf16 mode (Cfg.head_bf16): the skip convs over the
    layers' gated outputs at the last tf steps and end_conv_1 as _HeadLin (bf16 operands, exact
    sums), the bf16 roundings of g and of relu(skip) pinned to the HIP run's ties where given.
    Returns (skip, e1) pre-activations."""
    skip, terms = None, None
    for i, g in enumerate(gs):
        gl = g[..., -tf:]
        gb = bf16_round(gl)
        if pins is not None and i in pins.g:
            gb = pins.adopt(gb, gl, bf16_round(pins.g[i][..., -tf:].to(gl.dtype)), pins.g_band * float(g.abs().max()), "g")
        w = p["skip_convs.%d.weight" % i]
        s = _HeadLin.apply(gl, w, gb.detach(), (pins, "dsk") if pins is not None else None) \
            + p["skip_convs.%d.bias" % i].view(1, -1, 1, 1)
        skip = s if skip is None else skip + s
        t = pointwise(gb.abs(), bf16_round(w).abs())
        terms = t if terms is None else terms + t
    sk = _relu(skip, masks, "skip")
    skb = bf16_round(sk)
    if pins is not None and pins.skr is not None:
        skb = pins.adopt(skb, sk, bf16_round(pins.skr.to(sk.dtype)), pins.head_band * terms.detach(), "skr")
    e1 = _HeadLin.apply(sk, p["end_conv_1.weight"], skb.detach(), (pins, "de1") if pins is not None else None) \
        + p["end_conv_1.bias"].view(1, -1, 1, 1)
    return skip, e1


def gcn_bf16(g, w, sups, rnd=bf16_round, mrnd=None, pin=None):
    """libgwn's bf16-mode gcn products (_GcnBf16): sum_q W_q piece_q, no bias; mrnd = the mlp's
    operand rounding (None: exact mlp); pin = (Bf16Pins, layer index) or None."""
    return _GcnBf16.apply(g, w, rnd, mrnd, pin, *sups)


def pointwise(x, w, bias=None):
    """1x1 convolution over NCHW: y[b,o,n,t] = sum_i w[o,i] x[b,i,n,t] + bias[o]."""
    y = torch.einsum("oi,bint->bont", w.reshape(w.shape[0], -1), x)
    return y if bias is None else y + bias.view(1, -1, 1, 1)


def dilated_conv(x, w, bias, d):
    """Conv with kernel (1,k), dilation d, no padding (model.py:135-141): output step t reads taps
    t, t+d, ..., t+(k-1)d."""
    k = w.shape[-1]
    t_out = x.shape[-1] - (k - 1) * d
    y = bias.view(1, -1, 1, 1)
    for j in range(k):
        y = y + pointwise(x[..., j * d:j * d + t_out], w[:, :, 0, j])
    return y


def batchnorm(x, gamma, beta, rmean, rvar, training, momentum=0.1, eps=1e-5):
    if training:
        n = x.numel() // x.shape[1]
        mu = x.mean(dim=(0, 2, 3))
        var = ((x - mu.view(1, -1, 1, 1)) ** 2).mean(dim=(0, 2, 3))
        if rmean is not None:
            with torch.no_grad():
                rmean.mul_(1 - momentum).add_(momentum * mu.detach().to(rmean.dtype))
                rvar.mul_(1 - momentum).add_(momentum * (var.detach() * n / max(n - 1, 1)).to(rvar.dtype))
    else:
        mu, var = rmean.to(x.dtype), rvar.to(x.dtype)
    return (x - mu.view(1, -1, 1, 1)) / torch.sqrt(var.view(1, -1, 1, 1) + eps) * gamma.view(1, -1, 1, 1) \
        + beta.view(1, -1, 1, 1)


def _relu(x, masks, key):
    """relu, or -- branch pinned -- x * mask (masks[key]: the branch taken, 1 = positive side)."""
    if masks is None or key not in masks:
        return torch.relu(x)
    return x * masks[key].to(x.dtype)


def forward(p, supports, x, cfg, training, bn_state=None, dropout_masks=None, masks=None, record=None, pins=None):
    """gwnet forward.  p: dict of parameter tensors (state_dict names); supports: list of [N,N]
    fixed supports; x: [B, Cin, N, T]; bn_state: dict name->buffer updated in train mode;
    masks: optional ReLU branches {"skip": [B,S,N,T_f], "e1": [B,E,N,T_f]} (module docstring);
    record: optional dict that receives the head's pre-activations "skip" and "e1" (detached);
    pins: optional Bf16Pins (bf16 emulation only: the HIP run's rounding ties)."""
    t = x.shape[-1]
    if t < cfg.receptive_field:
        x = torch.nn.functional.pad(x, (cfg.receptive_field - t, 0, 0, 0))
    h = pointwise(x, p["start_conv.weight"], p["start_conv.bias"])
    sups = list(supports) if cfg.use_gcn else []
    if cfg.use_gcn and cfg.adaptive:
        sups.append(adaptive_adjacency(p["nodevec1"], p["nodevec2"]))
    skip = None
    head_b = getattr(cfg, "head_bf16", False)
    gs = []  # (head_bf16: the gated outputs, for _head_bf16)
    for i, d in enumerate(cfg.dilations):
        res = h
        filt = torch.tanh(dilated_conv(res, p["filter_convs.%d.weight" % i], p["filter_convs.%d.bias" % i], d))
        gate = torch.sigmoid(dilated_conv(res, p["gate_convs.%d.weight" % i], p["gate_convs.%d.bias" % i], d))
        g = filt * gate
        if head_b:
            gs.append(g)
        else:
            s = pointwise(g, p["skip_convs.%d.weight" % i], p["skip_convs.%d.bias" % i])
            skip = s if skip is None else s + skip[..., -s.shape[-1]:]
        if cfg.use_gcn and getattr(cfg, "gcn_bf16", False):
            h = gcn_bf16(g, p["gconv.%d.mlp.mlp.weight" % i], sups,
                         mrnd=bf16_round if getattr(cfg, "gcn_bf16_mlp", False) else None,
                         pin=(pins, i) if pins is not None else None) \
                + p["gconv.%d.mlp.mlp.bias" % i].view(1, -1, 1, 1)
            if training and cfg.dropout > 0:
                m = dropout_masks[i] if dropout_masks is not None else \
                    (torch.rand_like(h) >= cfg.dropout).to(h.dtype)
                h = h * m / (1 - cfg.dropout)
        elif cfg.use_gcn:
            pieces = [g]
            for a in sups:
                y1 = diffuse(g, a)
                y2 = diffuse(y1, a)
                pieces += [y1, y2]
            h = pointwise(torch.cat(pieces, dim=1), p["gconv.%d.mlp.mlp.weight" % i], p["gconv.%d.mlp.mlp.bias" % i])
            if training and cfg.dropout > 0:
                m = dropout_masks[i] if dropout_masks is not None else \
                    (torch.rand_like(h) >= cfg.dropout).to(h.dtype)
                h = h * m / (1 - cfg.dropout)
        else:
            h = pointwise(g, p["residual_convs.%d.weight" % i], p["residual_convs.%d.bias" % i])
        h = h + res[..., -h.shape[-1]:]
        rm = bn_state["bn.%d.running_mean" % i] if bn_state is not None else None
        rv = bn_state["bn.%d.running_var" % i] if bn_state is not None else None
        h = batchnorm(h, p["bn.%d.weight" % i], p["bn.%d.bias" % i], rm, rv, training)
    if head_b:
        skip, e1 = _head_bf16(p, gs, h.shape[-1], masks, pins)
    else:
        e1 = pointwise(_relu(skip, masks, "skip"), p["end_conv_1.weight"], p["end_conv_1.bias"])
    if record is not None:
        record["skip"], record["e1"] = skip.detach(), e1.detach()
    return pointwise(_relu(e1, masks, "e1"), p["end_conv_2.weight"], p["end_conv_2.bias"])


def masked_metrics(pred, real, null_val=0.0, sign=None):
    """(mae, mape, rmse) with the zero-label mask renormalised by its mean (util.py:510-552).
    sign: optional branch of |pred - real| (module docstring)."""
    mask = (real != null_val).float()          # the reference builds the mask in fp32 (.float())
    mask = mask / mask.mean()
    mask = torch.where(torch.isnan(mask), torch.zeros_like(mask), mask)

    def fin(v):
        return torch.where(torch.isnan(v), torch.zeros_like(v), v).mean()

    diff = pred - real
    adiff = diff.abs() if sign is None else diff * sign.to(diff.dtype)
    mae = fin(adiff * mask)
    mape = fin(adiff / real * mask)
    rmse = torch.sqrt(fin(diff * diff * mask))
    return mae, mape, rmse


def engine_loss(p, supports, x, real_val, cfg, scaler_mean, scaler_std, bn_state=None, training=True, masks=None,
                record=None, pins=None, dropout_masks=None):
    """engine.py:41-51 up to the loss: pad 1, forward, inverse scale, masked MAE.
    masks: optional branches (module docstring; "sign": [B,1,N,T_out] of pred - real);
    dropout_masks: optional per-layer keep masks [B,C,N,T_i] (forward's)."""
    x = torch.nn.functional.pad(x, (1, 0, 0, 0))
    out = forward(p, supports, x, cfg, training, bn_state, dropout_masks=dropout_masks, masks=masks, record=record,
                  pins=pins)
    pred = out.transpose(1, 3) * scaler_std + scaler_mean
    real = real_val.unsqueeze(1)
    mae, mape, rmse = masked_metrics(pred, real, sign=None if masks is None else masks.get("sign"))
    return out, mae, mape, rmse


def grads(sd, supports, x, real_val, cfg, scaler_mean, scaler_std, dtype=F64, masks=None, record=None, pins=None,
          dropout_masks=None):
    """Per-parameter gradients of the engine loss (train mode); params that do not reach the
    output get no entry (the reference leaves their .grad None).  masks: optional branch pinning
    (module docstring); dropout_masks: optional per-layer keep masks (``forward``)."""
    p = {k: torch.tensor(np.asarray(v), dtype=dtype, requires_grad=True) for k, v in sd.items()
         if not _is_buffer(k)}
    bn = {k: torch.tensor(np.asarray(v), dtype=dtype) for k, v in sd.items() if "running" in k}
    sups = [torch.tensor(np.asarray(a), dtype=dtype) for a in supports]
    out, mae, mape, rmse = engine_loss(p, sups, torch.tensor(x, dtype=dtype), torch.tensor(real_val, dtype=dtype),
                                       cfg, scaler_mean, scaler_std, bn, masks=masks, record=record, pins=pins,
                                       dropout_masks=dropout_masks)
    names = list(p.keys())
    gs = torch.autograd.grad(mae, [p[n] for n in names], allow_unused=True)
    g = {n: gi for n, gi in zip(names, gs) if gi is not None}
    return out.detach(), (mae.item(), mape.item(), rmse.item()), g, bn


def _is_buffer(k):
    return ("running_" in k) or ("num_batches_tracked" in k)


class Trainer:
    """engine.trainer restated (engine.py:41-58): clip_grad_norm_(5) + torch.optim.Adam math."""

    def __init__(self, sd, supports, cfg, lr=1e-3, wd=1e-4, clip=5.0, scaler=(54.4, 19.5), dtype=F64):
        self.cfg, self.lr, self.wd, self.clip = cfg, lr, wd, clip
        self.scaler = scaler
        self.dtype = dtype
        self.p = {k: torch.tensor(np.asarray(v), dtype=dtype) for k, v in sd.items() if not _is_buffer(k)}
        self.bn = {k: torch.tensor(np.asarray(v), dtype=dtype) for k, v in sd.items() if "running" in k}
        self.m = {k: torch.zeros_like(v) for k, v in self.p.items()}
        self.v = {k: torch.zeros_like(v) for k, v in self.p.items()}
        self.t = 0
        self.sups = [torch.tensor(np.asarray(a), dtype=dtype) for a in supports]

    def train(self, x, real_val):
        for v in self.p.values():
            v.requires_grad_(True)
        out, mae, mape, rmse = engine_loss(self.p, self.sups, torch.as_tensor(x, dtype=self.dtype),
                                           torch.as_tensor(real_val, dtype=self.dtype), self.cfg,
                                           self.scaler[0], self.scaler[1], self.bn)
        names = list(self.p.keys())
        gs = torch.autograd.grad(mae, [self.p[n] for n in names], allow_unused=True)
        g = {n: gi for n, gi in zip(names, gs) if gi is not None}
        with torch.no_grad():
            total = math.sqrt(sum(float((gi.double() ** 2).sum()) for gi in g.values()))
            coef = min(self.clip / (total + 1e-6), 1.0)
            self.t += 1
            b1, b2, eps = 0.9, 0.999, 1e-8
            for n, gi in g.items():
                gi = gi * coef + self.wd * self.p[n]
                self.m[n] = self.m[n] + (1 - b1) * (gi - self.m[n])
                self.v[n] = self.v[n] * b2 + (1 - b2) * gi * gi
                denom = self.v[n].sqrt() / math.sqrt(1 - b2 ** self.t) + eps
                self.p[n] = self.p[n] - (self.lr / (1 - b1 ** self.t)) * self.m[n] / denom
        for v in self.p.values():
            v.requires_grad_(False)
        return mae.item(), mape.item(), rmse.item()
