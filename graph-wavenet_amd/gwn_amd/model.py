"""Drop-in ``gwnet`` (reference model.py:82-241) whose forward/backward run on libgwn (HIP, gfx950).

Constructor signature, attributes (``nodevec1``, ``nodevec2``, ``supports``, ``receptive_field``,
``supports_len``), submodule tree and therefore ``state_dict`` keys / shapes are those of the
reference, and parameters are created in the reference's order with the same init functions, so
``torch.manual_seed(s); gwnet(...)`` yields the reference's initial weights bit for bit.

Below the module boundary nothing is PyTorch compute: every parameter lives in one flat fp32
device buffer (``_flat``), the forward is a fixed schedule of libgwn launches (executor.py) and
the backward is the matching hand-written gradient schedule, wrapped as ONE autograd node.
"""
import ctypes
import os

import torch
import torch.nn as nn

from . import _lib
from .executor import Executor, _ksplit, gemm  # noqa: F401  (gemm re-exported for the op-level modules)

F32 = torch.float32


class nconv(nn.Module):
    """``einsum('ncvl,vw->ncwl')`` (reference model.py:8-14) on libgwn's batched MFMA GEMM."""

    def forward(self, x, A):
        return _NconvFn.apply(x, A)


class _NconvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, A):
        _require_device(x, A)
        x = x.contiguous()
        A = A.contiguous()
        B, C, N, T = x.shape
        y = torch.empty_like(x)
        # NCHW slices: rows = nodes, "channels" = the T time steps of one (b, c) pair
        _lib.call("gwn_nconv", A.data_ptr(), N, 1, x.data_ptr(), T, y.data_ptr(), T, None, 0, N, T, B * C,
                  _lib.stream())
        ctx.save_for_backward(x, A)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, A = ctx.saved_tensors
        dy = dy.contiguous()
        B, C, N, T = x.shape
        dx = dA = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            _lib.call("gwn_nconv", A.data_ptr(), N, 0, dy.data_ptr(), T, dx.data_ptr(), T, None, 0, N, T,
                      B * C, _lib.stream())
        if ctx.needs_input_grad[1]:
            dA = torch.empty_like(A)
            lib = _lib.load()
            ws = torch.empty(max(1, lib.gwn_nconv_adj_grad_workspace_floats(N, T, B * C)), device=x.device,
                             dtype=F32)
            _lib.call("gwn_nconv_adj_grad", x.data_ptr(), T, dy.data_ptr(), T, N, T, B * C, dA.data_ptr(), N,
                      0, ws.data_ptr(), _lib.stream())
        return dx, dA


class nconv2(nn.Module):
    """``einsum('ncvl,nvw->ncwl')`` (reference model.py:16-22): diffusion with one support per
    sample (the per-sample-graph variant's operator), one batched MFMA GEMM launch per call."""

    def forward(self, x, A):
        return _Nconv2Fn.apply(x, A)


class _Nconv2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, A):
        _require_device(x, A)
        B, C, N, T = x.shape
        if tuple(A.shape) != (B, N, N):
            raise RuntimeError("nconv2: supports must be [B, N, N] = [%d, %d, %d], got %s" % (B, N, N, tuple(A.shape)))
        x = x.contiguous()
        A = A.contiguous()
        y = torch.empty_like(x)
        # NCHW: sample b holds C slices of [N][T] (rows = nodes, "channels" = time steps)
        _lib.call("gwn_nconv2", A.data_ptr(), N, N * N, 1, x.data_ptr(), T, y.data_ptr(), T, N, T, C, B,
                  _lib.stream())
        ctx.save_for_backward(x, A)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, A = ctx.saved_tensors
        dy = dy.contiguous()
        B, C, N, T = x.shape
        dx = dA = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            _lib.call("gwn_nconv2", A.data_ptr(), N, N * N, 0, dy.data_ptr(), T, dx.data_ptr(), T, N, T, C, B,
                      _lib.stream())
        if ctx.needs_input_grad[1]:
            dA = torch.empty_like(A)
            _lib.call("gwn_nconv2_adj_grad", x.data_ptr(), T, dy.data_ptr(), T, N, T, C, B, dA.data_ptr(), N, N * N,
                      0, _lib.stream())
        return dx, dA


def _gemm_desc(A, lda_m, lda_k, B, ldb_k, ldb_n, C, ldc_m, ldc_n, M, N, K, **kw):
    d = _lib.GemmDesc()
    d.A, d.lda_m, d.lda_k = A, lda_m, lda_k
    d.B, d.ldb_k, d.ldb_n = B, ldb_k, ldb_n
    d.C, d.ldc_m, d.ldc_n = C, ldc_m, ldc_n
    d.M, d.N, d.K = M, N, K
    d.alpha, d.beta = 1.0, 1.0
    for k, v in kw.items():
        setattr(d, k, v)
    return d


class _LinearFn(torch.autograd.Function):
    """1x1 conv over NCHW (``Conv2d(c_in, c_out, (1, 1))``): per sample b, with P = H*W pixels,
    Y_b[o][p] = sum_i W[o][i] X_b[i][p] + bias[o] -- one batched libgwn GEMM (blockIdx.z = b);
    backward: dX_b = W^T dY_b (batched), dW = sum_b dY_b X_b^T with db from the GEMM's ones
    column, K = B*P walked through the two-level index map (fixed-order split-K reduce)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        _require_device(x, weight, bias)
        x = x.contiguous()
        B, ci, H, W = x.shape
        co = weight.shape[0]
        if weight.shape[1] != ci:
            raise RuntimeError("linear: weight expects %d input channels, got %d" % (weight.shape[1], ci))
        w2 = weight.reshape(co, ci).contiguous()
        P = H * W
        y = torch.empty(B, co, H, W, device=x.device, dtype=F32)
        # rows m = pixels p, columns n = output channels o: C(p, o) = y_b[o][p]
        d = _gemm_desc(x.data_ptr(), 1, P, w2.data_ptr(), 1, ci, y.data_ptr(), 1, P, P, co, ci,
                       bias_n=bias.data_ptr(), batch=B, a_bstride=ci * P, b_bstride=0, c_bstride=co * P)
        _lib.call("gwn_gemm", ctypes.byref(d), _lib.stream())
        ctx.save_for_backward(x, w2)
        ctx.wshape = tuple(weight.shape)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w2 = ctx.saved_tensors
        dy = dy.contiguous()
        B, ci, H, W = x.shape
        co = w2.shape[0]
        P = H * W
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            d = _gemm_desc(dy.data_ptr(), 1, P, w2.data_ptr(), ci, 1, dx.data_ptr(), 1, P, P, ci, co,
                           batch=B, a_bstride=co * P, b_bstride=0, c_bstride=ci * P)
            _lib.call("gwn_gemm", ctypes.byref(d), _lib.stream())
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            dw2 = torch.empty(co, ci, device=x.device, dtype=F32)
            db = torch.empty(co, device=x.device, dtype=F32)
            K = B * P
            ks = _ksplit(co, ci, K)
            lib = _lib.load()
            ws = torch.empty(max(1, lib.gwn_gemm_workspace_floats(co, ci, ks)), device=x.device, dtype=F32)
            # dW(o, i) = sum_k dY(o, k) X(i, k),  k = b*P + p  ->  (k / P) * (c*P) + k % P
            d = _gemm_desc(dy.data_ptr(), P, 1, x.data_ptr(), 1, P, dw2.data_ptr(), ci, 1, co, ci, K,
                           a_kin=P, a_ko_stride=co * P, b_kin=P, b_ko_stride=ci * P, ksplit=ks,
                           part=ws.data_ptr(), ones_out=db.data_ptr())
            _lib.call("gwn_gemm", ctypes.byref(d), _lib.stream())
            dw = dw2.view(ctx.wshape)
        return dx, dw, db


class linear(nn.Module):
    """1x1 convolution (reference model.py:24-30): ``mlp`` is the reference's Conv2d (state_dict
    parity); the forward / backward run on libgwn (``_LinearFn``).  Inside ``gwnet`` the same
    arithmetic is fused into the diffusion kernel's epilogue instead."""

    def __init__(self, c_in, c_out):
        super().__init__()
        self.mlp = torch.nn.Conv2d(c_in, c_out, kernel_size=(1, 1), padding=(0, 0), stride=(1, 1), bias=True)

    def forward(self, x):
        return _LinearFn.apply(x, self.mlp.weight, self.mlp.bias)


class gcn(nn.Module):
    """Diffusion graph convolution (reference model.py:32-55): for every support A, order hops of
    nconv (libgwn MFMA GEMMs), the piece-major concat [x, A1 x, A1^2 x, A2 x, ...], the 1x1 conv
    (libgwn) and dropout.  Standalone use runs these per operator (the concat and the dropout mask
    are torch data movement around the HIP arithmetic); inside ``gwnet`` the whole block is ONE
    fused kernel (``gwn_gcn_fwd`` / ``gwn_gcn_bwd``) and this module only holds the parameters."""

    def __init__(self, c_in, c_out, dropout, support_len=3, order=2):
        super().__init__()
        self.nconv = nconv()
        self.mlp = linear((order * support_len + 1) * c_in, c_out)
        self.dropout = dropout
        self.order = order

    def forward(self, x, support):
        out = [x]
        for a in support:
            x1 = self.nconv(x, a)
            out.append(x1)
            for _ in range(2, self.order + 1):
                x2 = self.nconv(x1, a)
                out.append(x2)
                x1 = x2
        h = torch.cat(out, dim=1)
        h = self.mlp(h)
        return torch.nn.functional.dropout(h, self.dropout, training=self.training)


class gcn2(nn.Module):
    """Diffusion graph convolution with per-sample supports (reference model.py:57-80): as ``gcn``
    with ``nconv2`` ('ncvl,nvw->ncwl', one [N, N] support per sample).  Standalone it runs the libgwn
    per-sample GEMMs; inside ``gwnet_diff_G`` the fused kernel with per-sample supports runs instead."""

    def __init__(self, c_in, c_out, dropout, support_len=3, order=2):
        super().__init__()
        self.nconv = nconv2()
        self.mlp = linear((order * support_len + 1) * c_in, c_out)
        self.dropout = dropout
        self.order = order

    forward = gcn.forward


def _require_device(*ts):
    for t in ts:
        if not (t.is_cuda and t.dtype == F32):
            raise RuntimeError("gwn_amd: the HIP path needs float32 tensors on a GPU device "
                               "(there is no CPU fallback)")


class gwnet(nn.Module):
    def __init__(self, device, num_nodes, dropout=0.3, supports=None, gcn_bool=True, addaptadj=True,
                 aptinit=None, in_dim=2, out_dim=12, residual_channels=32, dilation_channels=32,
                 skip_channels=256, end_channels=512, kernel_size=2, blocks=4, layers=2):
        super().__init__()
        self.dropout = dropout
        self.blocks = blocks
        self.layers = layers
        self.gcn_bool = gcn_bool
        self.addaptadj = addaptadj
        self.num_nodes = num_nodes
        self.in_dim, self.out_dim = in_dim, out_dim
        self.residual_channels, self.dilation_channels = residual_channels, dilation_channels
        self.skip_channels, self.end_channels = skip_channels, end_channels
        self.kernel_size = kernel_size
        self.compute_dtype = "bf16" if os.environ.get("GWN_DTYPE", "fp32") in ("bf16", "bfloat16") else "fp32"

        # Submodule registration order == reference state_dict order (model.py:95-100).
        for name in ("filter_convs", "gate_convs", "residual_convs", "skip_convs", "bn", "gconv"):
            setattr(self, name, nn.ModuleList())
        # RNG consumption order == reference (model.py:102-169): start_conv, node embeddings,
        # then per layer filter, gate, residual, skip, bn, gcn-mlp; then the two end convs.
        self.start_conv = nn.Conv2d(in_channels=in_dim, out_channels=residual_channels, kernel_size=(1, 1))
        self.supports = supports
        self.supports_len = len(supports) if supports is not None else 0
        if gcn_bool and addaptadj:
            if self.supports is None:
                self.supports = []
            if aptinit is None:
                e1 = torch.randn(num_nodes, 10)
                e2 = torch.randn(10, num_nodes)
            else:
                # SVD initialisation (model.py:123-127): E1 = U_10 sqrt(S_10), E2 = sqrt(S_10) V_10^T
                u, s, v = torch.svd(aptinit.detach().to("cpu", F32))
                root = torch.diag(s[:10] ** 0.5)
                e1 = torch.mm(u[:, :10], root)
                e2 = torch.mm(root, v[:, :10].t())
            self.nodevec1 = nn.Parameter(e1, requires_grad=True)
            self.nodevec2 = nn.Parameter(e2, requires_grad=True)
            self.supports_len += 1

        receptive_field = 1
        for _ in range(blocks):
            scope, dilation = kernel_size - 1, 1
            for _ in range(layers):
                self._add_layer(dilation)
                dilation *= 2
                receptive_field += scope
                scope *= 2
        self.end_conv_1 = nn.Conv2d(in_channels=skip_channels, out_channels=end_channels, kernel_size=(1, 1),
                                    bias=True)
        self.end_conv_2 = nn.Conv2d(in_channels=end_channels, out_channels=out_dim, kernel_size=(1, 1), bias=True)
        self.receptive_field = receptive_field

        self._executor = None
        self._flat = None
        self._flat_ptrs = None
        self._nbt = None
        self._sup_cache = (None, None, None)
        self._place(device)

    def _add_layer(self, dilation):
        rc, dc, k = self.residual_channels, self.dilation_channels, self.kernel_size
        self.filter_convs.append(nn.Conv2d(in_channels=rc, out_channels=dc, kernel_size=(1, k), dilation=dilation))
        # legacy Conv1d with a 2-D kernel (model.py:139-151): weight [out, in, 1, k]
        self.gate_convs.append(nn.Conv1d(in_channels=rc, out_channels=dc, kernel_size=(1, k), dilation=dilation))
        self.residual_convs.append(nn.Conv1d(in_channels=dc, out_channels=rc, kernel_size=(1, 1)))
        self.skip_convs.append(nn.Conv1d(in_channels=dc, out_channels=self.skip_channels, kernel_size=(1, 1)))
        self.bn.append(nn.BatchNorm2d(rc))
        if self.gcn_bool:
            self.gconv.append(gcn(dc, rc, self.dropout, support_len=self.supports_len))

    # -----------------------------------------------------------------------------------------
    def _place(self, device):
        """Move to ``device`` and alias every parameter into one flat fp32 buffer."""
        device = torch.device(device)
        super().to(device)
        params = list(self.parameters())
        total = sum(p.numel() for p in params)
        flat = torch.empty(total, device=device, dtype=F32)
        off = 0
        with torch.no_grad():
            for p in params:
                n = p.numel()
                flat[off:off + n].copy_(p.data.reshape(-1))
                p.data = flat[off:off + n].view_as(p)
                off += n
            nbt = torch.zeros(len(self.bn), device=device, dtype=torch.long)
            for i, m in enumerate(self.bn):
                nbt[i] = m.num_batches_tracked
                m.num_batches_tracked = nbt[i]
        self._flat = flat
        self._nbt = nbt
        self._params_cache = params
        self._flat_ptrs = tuple(p.data_ptr() for p in params)

    def _ensure_flat(self):
        # the Parameter objects are fixed at construction (the reference never re-registers
        # them); only their storage can move (.to(), .data = ...), which the pointer check sees
        params = self._params_cache
        ptrs = tuple(p.data_ptr() for p in params)
        if ptrs != self._flat_ptrs or params[0].device != self._flat.device:
            if any(p.dtype != F32 for p in params):
                raise RuntimeError("gwn_amd: gwnet runs in float32 only")
            self._place(params[0].device)
            self._executor = None

    def executor(self):
        self._ensure_flat()
        if self._executor is None:
            self._executor = Executor(self)
        ex = self._executor
        ex.dropout = self.dropout
        ex.compute_dtype = self.compute_dtype
        ex.bind(self._flat.device)
        return ex

    def set_compute_dtype(self, dtype):
        """Arithmetic precision of the diffusion / mlp products (not part of the reference API):
        "fp32" (default, torch.float32: exact fp32 products, the reference's arithmetic) or "bf16"
        (torch.bfloat16: bf16 MFMA operands with fp32 accumulation in the fused gcn forward and
        backward -- mixed precision; parameters, activations, gradients and Adam state stay fp32).
        Shapes without a bf16 kernel (c != 32, n > 512) keep the fp32 kernels."""
        if dtype in (torch.bfloat16, "bf16", "bfloat16"):
            self.compute_dtype = "bf16"
        elif dtype in (torch.float32, "fp32", "float32", "f32"):
            self.compute_dtype = "fp32"
        else:
            raise ValueError("gwn_amd: compute dtype must be fp32 or bf16, got %r" % (dtype,))
        return self

    def _fixed_supports(self):
        """Device copies of the fixed supports, zero-padded to [NP][NP] (NP = 32*ceil(N/32)), the
        layout the fused diffusion kernel streams (include/gwn.h, gwn_gcn_fwd)."""
        if self.supports is None or len(self.supports) == 0:
            return []
        key = tuple((s.data_ptr(), s._version) for s in self.supports)
        if self._sup_cache[0] != key:
            dev = self._flat.device
            n = self.num_nodes
            np_ = (n + 31) // 32 * 32
            padded, padded_t = [], []
            for s in self.supports:
                src = s.detach().to(dev, F32).contiguous()
                if tuple(src.shape) != (n, n):
                    raise RuntimeError("gwnet: supports must be [%d, %d], got %s" % (n, n, tuple(src.shape)))
                dst = torch.empty(np_, np_, device=dev, dtype=F32)
                _lib.call("gwn_pad_square", src.data_ptr(), n, n, dst.data_ptr(), np_, np_, 0, _lib.stream())
                padded.append(dst)
                # and its padded transpose, for the fused backward (A x computed as (A^T)^T x)
                dst_t = torch.empty(np_, np_, device=dev, dtype=F32)
                _lib.call("gwn_pad_square", src.data_ptr(), n, n, dst_t.data_ptr(), np_, np_, 1, _lib.stream())
                padded_t.append(dst_t)
            # the source tensors stay referenced by the cache, so no other tensor can take their
            # addresses while the key is live; the generation tells captured graphs (engine.py) that
            # the padded buffers they baked in are gone
            self._sup_cache = (key, padded, padded_t, tuple(self.supports))
            self._sup_gen = getattr(self, "_sup_gen", 0) + 1
        return self._sup_cache[1]

    def _fixed_supports_t(self):
        """Padded transposes of the fixed supports (cached with them, see _fixed_supports)."""
        self._fixed_supports()
        return self._sup_cache[2] if self.supports else []

    def _call_supports(self):
        """(padded supports, sup_batch) of the forward being run: gwnet's fixed supports."""
        return self._fixed_supports(), 1

    def _bn_bufs(self):
        out = []
        for m in self.bn:
            mom = 0.1 if m.momentum is None else m.momentum
            # num_batches_tracked: a view into the model's counter vector, advanced on the device by
            # the train-mode BatchNorm launch itself
            out.append((m.running_mean, m.running_var, float(mom), float(m.eps), m.num_batches_tracked))
        return out

    def forward(self, input):
        ex = self.executor()
        if not self.training and not torch.is_grad_enabled() and ex.infer_ok():
            # inference (eval mode under no_grad, train.py:385-386 / test.py:65-66): the lean
            # schedule that keeps no state for a backward
            out, _ = ex.infer(self._flat, self._fixed_supports(), input, self._bn_bufs())
            return out
        return _GwnetFn.apply(self, input, *self.parameters())


class gwnet_diff_G(gwnet):
    """Graph WaveNet with a different graph per sample (reference model.py:244-407), drop-in:
    same ctor signature, submodule tree / state_dict and RNG consumption order as the reference
    (no node-embedding parameters; every block's dilations start at 4), and
    ``forward(input, supports, aptinit)`` with ``supports`` a list of [B, N, N] tensors.

    The reference's adaptive adjacency (model.py:324-329) draws fresh embeddings E1 [B, N, 10],
    E2 [B, 10, N] from the CPU generator on every call -- they are not registered parameters, so
    they are never trained and their gradient is discarded.  This is reproduced as it stands: the
    same two ``torch.randn`` draws in the same order (bit-identical under the same seed), the
    per-sample softmax(relu(E1_b E2_b)) on the GPU (gwn_adaptive_adj_fwd_batched), appended as the
    last support, and no gradient through it.  ``aptinit`` must be None: the reference stops at an
    ``ipdb.set_trace()`` there (model.py:331, "fix this").  The diffusion runs in the fused kernels
    with per-sample supports (sup_batch = B), so it needs residual_channels = 32 and N <= 512.
    Without a graph convolution (gcn_bool False, or supports None without addaptadj) every layer
    takes the residual_convs 1x1 branch (model.py:391-398), on a second executor whose packed
    layout maps residual_convs instead of the gcn mlps."""

    def __init__(self, device, num_nodes, dropout=0.3, supports_len=0, gcn_bool=True, addaptadj=True, in_dim=2,
                 out_dim=12, residual_channels=32, dilation_channels=32, skip_channels=256, end_channels=512,
                 kernel_size=2, blocks=4, layers=2):
        nn.Module.__init__(self)
        self.dropout = dropout
        self.blocks = blocks
        self.layers = layers
        self.gcn_bool = gcn_bool
        self.addaptadj = addaptadj
        self.device = device
        self.num_nodes = num_nodes
        self.in_dim, self.out_dim = in_dim, out_dim
        self.residual_channels, self.dilation_channels = residual_channels, dilation_channels
        self.skip_channels, self.end_channels = skip_channels, end_channels
        self.kernel_size = kernel_size
        self.compute_dtype = "fp32"
        self.supports = None
        self.supports_len = supports_len
        self.first_dilation = 4
        self.per_sample_graphs = True
        for name in ("filter_convs", "gate_convs", "residual_convs", "skip_convs", "bn", "gconv"):
            setattr(self, name, nn.ModuleList())
        self.start_conv = nn.Conv2d(in_channels=in_dim, out_channels=residual_channels, kernel_size=(1, 1))
        receptive_field = 1
        rc, dc, k = residual_channels, dilation_channels, kernel_size
        for _ in range(blocks):
            scope, dilation = kernel_size - 1, 4
            for _ in range(layers):
                self.filter_convs.append(nn.Conv2d(rc, dc, kernel_size=(1, k), dilation=dilation))
                self.gate_convs.append(nn.Conv2d(rc, dc, kernel_size=(1, k), dilation=dilation))
                self.residual_convs.append(nn.Conv2d(dc, rc, kernel_size=(1, 1)))
                self.skip_convs.append(nn.Conv2d(dc, skip_channels, kernel_size=(1, 1)))
                self.bn.append(nn.BatchNorm2d(rc))
                dilation *= 2
                receptive_field += scope
                scope *= 2
                if gcn_bool:
                    self.gconv.append(gcn2(dc, rc, dropout, support_len=supports_len))
        self.end_conv_1 = nn.Conv2d(skip_channels, end_channels, kernel_size=(1, 1), bias=True)
        self.end_conv_2 = nn.Conv2d(end_channels, out_dim, kernel_size=(1, 1), bias=True)
        self.receptive_field = receptive_field
        self._executor = None
        self._flat = None
        self._flat_ptrs = None
        self._nbt = None
        self._sup_cache = (None, None, None)
        self._call = None
        self._res_executor = None
        self._place(device)

    def _call_supports(self):
        return self._call[:2]

    def residual_executor(self):
        """Executor of the no-graph-convolution branch (model.py:391-398)."""
        self.executor()  # (re)places the flat buffer first
        if self._res_executor is None or self._res_executor.layout.flat_total != self._flat.numel():
            self._res_executor = Executor(self, residual_only=True)
        ex = self._res_executor
        ex.dropout = self.dropout
        ex.compute_dtype = self.compute_dtype
        ex.bind(self._flat.device)
        return ex

    def forward(self, input, supports, aptinit):
        ex = self.executor()
        B = input.shape[0]
        N = self.num_nodes
        sups = list(supports) if supports is not None else None
        adp = None
        if self.gcn_bool and self.addaptadj:
            if sups is None:
                sups = []
            if aptinit is not None:
                raise NotImplementedError("gwnet_diff_G: the reference's aptinit path stops at ipdb.set_trace() "
                                          "(model.py:331); pass aptinit=None")
            # model.py:324-329: two fresh CPU draws per call, in this order
            nv1 = torch.randn(B, N, 10)
            nv2 = torch.randn(B, 10, N)
            adp = (nv1, nv2)
        if not self.gcn_bool or sups is None:
            # model.py:391-398: x = residual_convs[i](x) in every layer; no supports are read
            self._call = ([], 1, self.residual_executor())
            try:
                return _GwnetFn.apply(self, input, *self.parameters())
            finally:
                self._call = None
        nsup = len(sups) + (1 if adp is not None else 0)
        if nsup != self.supports_len:
            raise RuntimeError("gwnet_diff_G: built for %d supports, got %d" % (self.supports_len, nsup))
        np_ = (N + 31) // 32 * 32
        sq = np_ * np_
        dev = self._flat.device
        st = _lib.stream()
        padded = []
        for a in sups:
            src = a.detach().to(dev, F32).contiguous()
            if tuple(src.shape) != (B, N, N):
                raise RuntimeError("gwnet_diff_G: supports must be [%d, %d, %d], got %s" % (B, N, N, tuple(src.shape)))
            dst = torch.empty(B * sq, device=dev, dtype=F32)
            _lib.call("gwn_pad_square_batched", src.data_ptr(), B, N * N, N, N, dst.data_ptr(), np_, np_, sq, 0, st)
            padded.append(dst)
        if adp is not None:
            e1 = adp[0].to(dev)
            e2 = adp[1].to(dev)
            dst = torch.zeros(B * sq, device=dev, dtype=F32)
            _lib.call("gwn_adaptive_adj_fwd_batched", e1.data_ptr(), e2.data_ptr(), B, N, 10, dst.data_ptr(), np_,
                      sq, st)
            padded.append(dst)
        self._call = (padded, B, ex)
        try:
            return _GwnetFn.apply(self, input, *self.parameters())
        finally:
            self._call = None


class _GwnetFn(torch.autograd.Function):
    """The whole gwnet forward as one autograd node; its backward is libgwn's gradient schedule.
    Parameters that never reach the output (``residual_convs`` on the gcn path, the last layer's
    gconv / bn, model.py:225-236) get ``None`` gradients, exactly as under reference autograd."""

    @staticmethod
    def forward(ctx, model, x, *params):
        call = getattr(model, "_call", None)
        ex = call[2] if call is not None else model._executor
        training = model.training
        seed = None
        if training and model.dropout > 0:
            # F.dropout draws a fresh mask on every call (model.py:54): this forward and its
            # backward use a snapshot of the counter, which then advances for the next forward
            seed = ex.seed.clone()
            _lib.call("gwn_increment_u64", _lib.ptr(ex.seed), 1, _lib.stream())
        sups, sup_batch = model._call_supports()
        fixed_t = model._fixed_supports_t() if sup_batch <= 1 else None
        out, acts = ex.forward(model._flat, sups, x, training, model._bn_bufs(), seed=seed, sup_batch=sup_batch,
                               fixed_t=fixed_t)
        ctx.model = model
        ctx.ex = ex
        ctx.acts = acts
        return out

    @staticmethod
    def backward(ctx, dout):
        model = ctx.model
        ex = ctx.ex
        ex.backward(ctx.acts, dout)
        gflat = torch.zeros_like(model._flat)
        ex.unpack_grads(gflat)
        ctx.acts = None
        grads = []
        lay = ex.layout
        active = set(lay.active)
        for name, p in model.named_parameters():
            if name in active:
                off, shape = lay.flat_off[name]
                grads.append(gflat[off:off + p.numel()].view(shape))
            else:
                grads.append(None)
        return (None, None, *grads)
