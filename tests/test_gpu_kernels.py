"""libgwn kernels vs fp64 CPU references (op level).  Tolerances are written per test."""
import ctypes

import numpy as np
import pytest
import torch

from conftest import load_golden, rel_err

pytestmark = pytest.mark.gpu


def _gemm(**kw):
    from gwn_amd import _lib
    d = _lib.GemmDesc()
    d.alpha, d.beta, d.ksplit = 1.0, 1.0, 1
    for k, v in kw.items():
        if isinstance(v, torch.Tensor):
            v = v.data_ptr()
        setattr(d, k, v)
    _lib.call("gwn_gemm", ctypes.byref(d), _lib.stream())


@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (37, 29, 53), (256, 32, 32), (207, 64, 207), (300, 200, 100),
                                   (1000, 512, 256), (13, 7, 1000)])
@pytest.mark.parametrize("akc,bkc", [(True, False), (False, False), (True, True), (False, True)])
def test_gemm_layouts(gpu, M, N, K, akc, bkc):
    torch.manual_seed(M * 7 + N + K)
    A = torch.randn(M, K, dtype=torch.float64)
    B = torch.randn(K, N, dtype=torch.float64)
    ref = A @ B
    Ad = (A if akc else A.t()).contiguous().float().to(gpu)   # akc: [M][K]; else [K][M]
    Bd = (B.t() if bkc else B).contiguous().float().to(gpu)   # bkc: [N][K]; else [K][N]
    C = torch.full((M, N), float("nan"), device=gpu)
    _gemm(A=Ad, lda_m=K if akc else 1, lda_k=1 if akc else M, B=Bd, ldb_k=1 if bkc else N, ldb_n=K if bkc else 1,
          C=C, ldc_m=N, ldc_n=1, M=M, N=N, K=K)
    torch.cuda.synchronize()
    got = C.double().cpu()
    # exact fp32 fma chain: |err| <= ~K * 2^-24 * sum|a||b|
    bound = 2.0 ** -22 * K * (A.abs() @ B.abs())
    assert torch.all((got - ref).abs() <= bound + 1e-30), float(((got - ref).abs() / (bound + 1e-30)).max())


@pytest.mark.parametrize("M,N,K", [(207, 207, 197), (61, 222, 99), (300, 30, 1001), (13, 5, 7), (33, 224, 513)])
@pytest.mark.parametrize("akc,bkc", [(True, False), (False, False), (True, True), (False, True)])
def test_gemm_vector_quads_ragged(gpu, M, N, K, akc, bkc):
    """Leading dims padded to multiples of 4 (16-B quad loads enabled) with ragged M, N, K:
    the edge quads fall back to guarded scalar loads."""
    def pad4(v):
        return (v + 3) // 4 * 4 + 4
    torch.manual_seed(M + 3 * N + 7 * K)
    A = torch.randn(M, K, dtype=torch.float64)
    B = torch.randn(K, N, dtype=torch.float64)
    ref = A @ B
    if akc:
        lda = pad4(K)
        Ad = torch.zeros(M, lda, device=gpu); Ad[:, :K] = A.float().to(gpu)
        a_kw = dict(lda_m=lda, lda_k=1)
    else:
        lda = pad4(M)
        Ad = torch.zeros(K, lda, device=gpu); Ad[:, :M] = A.t().float().to(gpu)
        a_kw = dict(lda_m=1, lda_k=lda)
    if bkc:
        ldb = pad4(K)
        Bd = torch.zeros(N, ldb, device=gpu); Bd[:, :K] = B.t().float().to(gpu)
        b_kw = dict(ldb_k=1, ldb_n=ldb)
    else:
        ldb = pad4(N)
        Bd = torch.zeros(K, ldb, device=gpu); Bd[:, :N] = B.float().to(gpu)
        b_kw = dict(ldb_k=ldb, ldb_n=1)
    C = torch.full((M, N), float("nan"), device=gpu)
    part = torch.empty(4 * M * N, device=gpu)
    _gemm(A=Ad, B=Bd, C=C, ldc_m=N, ldc_n=1, M=M, N=N, K=K, ksplit=4 if K > 500 else 1, part=part,
          **a_kw, **b_kw)
    torch.cuda.synchronize()
    got = C.double().cpu()
    bound = 2.0 ** -22 * K * (A.abs() @ B.abs())
    assert torch.all((got - ref).abs() <= bound + 1e-30)


def test_mfma_layout_identity_asymmetric(gpu):
    """A = I with an asymmetric B must reproduce B exactly (catches a transposed C write)."""
    n = 64
    A = torch.eye(n, device=gpu)
    B = torch.arange(n * n, dtype=torch.float32, device=gpu).reshape(n, n) * 0.5 + 3
    C = torch.zeros(n, n, device=gpu)
    _gemm(A=A, lda_m=n, lda_k=1, B=B, ldb_k=n, ldb_n=1, C=C, ldc_m=n, ldc_n=1, M=n, N=n, K=n)
    torch.cuda.synchronize()
    assert torch.equal(C, B)


def test_gemm_splitk_bias_relu_residual(gpu):
    M, N, K = 96, 160, 5000
    torch.manual_seed(3)
    A = torch.randn(M, K, device=gpu)
    B = torch.randn(K, N, device=gpu)
    bias = torch.randn(N, device=gpu)
    C0 = torch.randn(M, N, device=gpu)
    part = torch.empty(8 * M * N, device=gpu)
    C = torch.empty(M, N, device=gpu)
    _gemm(A=A, lda_m=K, lda_k=1, B=B, ldb_k=N, ldb_n=1, C=C, ldc_m=N, ldc_n=1, M=M, N=N, K=K, ksplit=8, part=part,
          bias_n=bias, relu=1, C0=C0, ldc0_m=N, ldc0_n=1, beta=0.5)
    ref = torch.relu(A.double() @ B.double() + bias.double()) + 0.5 * C0.double()
    torch.cuda.synchronize()
    assert rel_err(C.cpu().numpy(), ref.cpu().numpy()) < 1e-5


@pytest.mark.parametrize("M,N,K,ks", [(64, 224, 13248, 12), (32, 32, 700, 1), (300, 40, 2000, 4), (20, 96, 37, 1)])
def test_gemm_ones_column_bias_grad(gpu, M, N, K, ks):
    """Weight-gradient form dW = dY^T X with the bias gradient sum_r dY[r][m] from the ones column."""
    from gwn_amd import _lib
    torch.manual_seed(11)
    dY = torch.randn(K, M, device=gpu)
    X = torch.randn(K, N, device=gpu)
    ws = torch.empty(max(1, _lib.load().gwn_gemm_workspace_floats(M, N, ks)), device=gpu)
    dW = torch.empty(M, N, device=gpu)
    db = torch.full((M,), float("nan"), device=gpu)
    _gemm(A=dY, lda_m=1, lda_k=M, B=X, ldb_k=N, ldb_n=1, C=dW, ldc_m=N, ldc_n=1, M=M, N=N, K=K, ksplit=ks,
          part=ws, ones_out=db, alpha=0.5)
    torch.cuda.synchronize()
    assert rel_err(dW.cpu().numpy(), 0.5 * (dY.double().t() @ X.double()).cpu().numpy()) < 1e-5
    assert rel_err(db.cpu().numpy(), 0.5 * dY.double().sum(0).cpu().numpy()) < 1e-5


def test_gemm_two_level_taps_and_slices(gpu):
    """Dilated two-tap rows (a_kin / a_row_shift / a_rows) and strided slices (b_nin / c_nin)."""
    P, T, Cc, d = 10, 6, 16, 2
    torch.manual_seed(4)
    X = torch.randn(T * P, Cc, device=gpu)
    W = torch.randn(2 * Cc, 24, device=gpu)  # [k=tap*C+ci][n]
    rows = (T - d) * P
    Y = torch.empty(rows, 24, device=gpu)
    _gemm(A=X, lda_m=Cc, lda_k=1, a_kin=Cc, a_row_shift=d * P, a_rows=T * P, B=W, ldb_k=24, ldb_n=1,
          C=Y, ldc_m=24, ldc_n=1, M=rows, N=24, K=2 * Cc)
    Xd, Wd = X.double().cpu(), W.double().cpu()
    ref = Xd[:rows] @ Wd[:Cc] + Xd[d * P:] @ Wd[Cc:]
    torch.cuda.synchronize()
    assert rel_err(Y.cpu().numpy(), ref.numpy()) < 1e-5
    # backward-data form: negative shift with validity window
    dY = torch.randn(rows, 2 * Cc, device=gpu)
    Wt = torch.randn(2 * Cc, 2 * Cc, device=gpu)  # [j][tap*C+ci]
    dX = torch.empty(T * P, Cc, device=gpu)
    _gemm(A=dY, lda_m=2 * Cc, lda_k=1, a_kin=2 * Cc, a_row_shift=-d * P, a_rows=rows, B=Wt, ldb_k=2 * Cc, ldb_n=1,
          b_kin=2 * Cc, b_ko_stride=Cc, C=dX, ldc_m=Cc, ldc_n=1, M=T * P, N=Cc, K=4 * Cc)
    dYd, Wtd = dY.double().cpu(), Wt.double().cpu()
    ref = torch.zeros(T * P, Cc, dtype=torch.float64)
    ref[:rows] += dYd @ Wtd[:, :Cc]
    ref[d * P:] += dYd @ Wtd[:, Cc:]
    torch.cuda.synchronize()
    assert rel_err(dX.cpu().numpy(), ref.numpy()) < 1e-5


def test_nconv_matches_reference_golden(gpu):
    from gwn_amd.model import nconv
    g = load_golden("g6_ops_n207.npz")
    x = torch.tensor(g["x"], device=gpu)
    A = torch.tensor(g["A"], device=gpu)
    y = nconv()(x, A)
    torch.cuda.synchronize()
    assert rel_err(y.cpu().numpy(), g["nconv"]) < 1e-5


def test_nconv_backward(gpu):
    from gwn_amd.model import nconv
    torch.manual_seed(5)
    x = torch.randn(2, 3, 29, 12, device=gpu, requires_grad=True)
    A = torch.rand(29, 29, device=gpu, requires_grad=True)
    y = nconv()(x, A)
    gy = torch.randn_like(y)
    y.backward(gy)
    xc = x.detach().double().cpu().requires_grad_(True)
    Ac = A.detach().double().cpu().requires_grad_(True)
    torch.einsum("ncvl,vw->ncwl", xc, Ac).backward(gy.double().cpu())
    assert rel_err(x.grad.cpu().numpy(), xc.grad.numpy()) < 1e-5
    assert rel_err(A.grad.cpu().numpy(), Ac.grad.numpy()) < 1e-5


def test_adaptive_adjacency_fwd_bwd(gpu):
    from gwn_amd import _lib
    from oracle import gwnet_oracle as orc
    g = load_golden("g6_ops_n207.npz")
    n = 207
    e1 = torch.tensor(g["e1"], device=gpu)
    e2 = torch.tensor(g["e2"], device=gpu)
    adp = torch.empty(n, n, device=gpu)
    _lib.call("gwn_adaptive_adj_fwd", e1.data_ptr(), e2.data_ptr(), n, 10, adp.data_ptr(), n, _lib.stream())
    torch.cuda.synchronize()
    assert rel_err(adp.cpu().numpy(), g["adp"]) < 1e-5
    dadp = torch.randn(n, n, device=gpu)
    de1, de2 = torch.empty(n, 10, device=gpu), torch.empty(10, n, device=gpu)
    ws = torch.empty(n * n, device=gpu)
    _lib.call("gwn_adaptive_adj_bwd", e1.data_ptr(), e2.data_ptr(), adp.data_ptr(), dadp.data_ptr(), n, 10, n,
              de1.data_ptr(), de2.data_ptr(), ws.data_ptr(), _lib.stream())
    a = torch.tensor(g["e1"], dtype=torch.float64, requires_grad=True)
    b = torch.tensor(g["e2"], dtype=torch.float64, requires_grad=True)
    orc.adaptive_adjacency(a, b).backward(dadp.double().cpu())
    torch.cuda.synchronize()
    assert rel_err(de1.cpu().numpy(), a.grad.numpy()) < 1e-4
    assert rel_err(de2.cpu().numpy(), b.grad.numpy()) < 1e-4


def test_gated_tcn_matches_reference_golden(gpu):
    from gwn_amd import _lib
    g = load_golden("g6_ops_n207.npz")
    x = torch.tensor(g["x"])  # [1, 32, 207, 12] NCHW
    B, C, N, T = x.shape
    d = 2
    P = B * N
    xl = x.permute(3, 0, 2, 1).contiguous().to(gpu)  # [T][B][N][C]
    fw = torch.tensor(g["w/filter_convs.1.weight"]).reshape(C, C, 2)
    gw = torch.tensor(g["w/gate_convs.1.weight"]).reshape(C, C, 2)
    wfg = torch.stack([fw, gw], 1).permute(0, 1, 3, 2).reshape(2 * C, 2 * C).contiguous().to(gpu)
    bfg = torch.stack([torch.tensor(g["w/filter_convs.1.bias"]), torch.tensor(g["w/gate_convs.1.bias"])],
                      1).reshape(-1).contiguous().to(gpu)
    rows = (T - d) * P
    xg = torch.empty(rows, C, device=gpu)
    fg = torch.empty(rows, 2 * C, device=gpu)
    a = _lib.TcnArgs(x=xl.data_ptr(), t_in=T, P=P, c=C, dilation=d, w_fg=wfg.data_ptr(), b_fg=bfg.data_ptr(),
                     xg=xg.data_ptr(), ld_xg=C, fg=fg.data_ptr(), skipcat=None, ld_skip=0, skip_row0=0)
    _lib.call("gwn_gated_tcn_fwd", ctypes.byref(a), _lib.stream())
    torch.cuda.synchronize()
    got = xg.cpu().reshape(T - d, B, N, C).permute(1, 3, 2, 0).numpy()
    assert rel_err(got, g["tcn_d2"]) < 1e-5


def test_batchnorm_fold_vs_materialised(gpu):
    """gwn_batchnorm_fwd_fold (BatchNorm applied on load): from per-chunk partials of z with a large
    channel offset (|mean| ~ 20 sigma), the saved statistics and running stats against fp64, then
    the next gated TCN on z with the folded weights (x_mean = the batch mean) against the same TCN
    on bn(z) with the original weights, and the TCN weight gradient with the affine applied on
    load (gwn_tcn_bwd_args.x_mean / x_scale / x_shift) against the plain one on bn(z)."""
    from gwn_amd import _lib
    torch.manual_seed(16)
    C, P, T, d = 32, 40, 6, 2
    rows = T * P
    z64 = torch.randn(rows, C, dtype=torch.float64) * (0.5 + torch.rand(C, dtype=torch.float64)) \
        + 20.0 * torch.randn(C, dtype=torch.float64)
    z = z64.float()
    chunks = torch.split(z.double(), 37)  # ragged chunks, as the per-slice partials
    part = torch.stack([torch.stack([torch.full((C,), float(ch.shape[0]), dtype=torch.float64), ch.mean(0),
                                     ((ch - ch.mean(0)) ** 2).sum(0)]) for ch in chunks]).float().to(gpu)
    gamma, beta = torch.randn(C, device=gpu), torch.randn(C, device=gpu)
    rm, rv = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
    mean, rstd, scale = (torch.empty(C, device=gpu) for _ in range(3))
    wfg = torch.randn(2 * C, 2 * C, device=gpu) * 0.2
    bfg = torch.randn(2 * C, device=gpu)
    wfold, bfold = torch.empty_like(wfg), torch.empty_like(bfg)
    nbt = torch.full((1,), 41, device=gpu, dtype=torch.int64)
    _lib.call("gwn_batchnorm_fwd_fold", part.data_ptr(), len(chunks), C, gamma.data_ptr(), beta.data_ptr(),
              rm.data_ptr(), rv.data_ptr(), 0.1, 1e-5, mean.data_ptr(), rstd.data_ptr(), scale.data_ptr(),
              wfg.data_ptr(), bfg.data_ptr(), wfold.data_ptr(), bfold.data_ptr(), nbt.data_ptr(), _lib.stream())
    zd = z.double()
    mu, var = zd.mean(0), zd.var(0, unbiased=False)
    torch.cuda.synchronize()
    assert rel_err(mean.cpu().numpy(), mu.numpy()) < 1e-6
    assert rel_err(rstd.cpu().numpy(), (1 / torch.sqrt(var + 1e-5)).numpy()) < 1e-6
    assert rel_err(rm.cpu().numpy(), (0.1 * mu).numpy()) < 1e-6
    assert int(nbt.item()) == 42  # num_batches_tracked advanced by the same launch
    assert rel_err(rv.cpu().numpy(), (0.9 + 0.1 * zd.var(0, unbiased=True)).numpy()) < 1e-6
    assert rel_err(scale.cpu().numpy(), (gamma.double().cpu() * rstd.double().cpu()).numpy()) < 1e-6
    # the TCN on z (folded, centred) = the TCN on bn(z)
    zg = z.to(gpu)
    xn = ((zg - mean) * rstd * gamma + beta).contiguous()
    out = {}
    for tag, x, w, b, xm in (("plain", xn, wfg, bfg, None), ("fold", zg, wfold, bfold, mean.data_ptr())):
        xg = torch.empty((T - d) * P, C, device=gpu)
        fg = torch.empty((T - d) * P, 2 * C, device=gpu)
        a = _lib.TcnArgs(x=x.data_ptr(), t_in=T, P=P, c=C, dilation=d, w_fg=w.data_ptr(), b_fg=b.data_ptr(),
                         xg=xg.data_ptr(), ld_xg=C, fg=fg.data_ptr(), skipcat=None, ld_skip=0, skip_row0=0, x_mean=xm)
        _lib.call("gwn_gated_tcn_fwd", ctypes.byref(a), _lib.stream())
        out[tag] = (xg, fg)
    torch.cuda.synchronize()
    assert rel_err(out["fold"][0].cpu().numpy(), out["plain"][0].cpu().numpy()) < 5e-6
    assert rel_err(out["fold"][1].cpu().numpy(), out["plain"][1].cpu().numpy()) < 5e-6
    # TCN weight gradient with BatchNorm on load
    R = (T - d) * P
    dfg = torch.randn(R, 2 * C, device=gpu)
    lib = _lib.load()
    ws = torch.empty(lib.gwn_wgrad_workspace_floats(R, 2 * C, 2 * C) + 16, device=gpu)
    dw = {k: torch.empty(2 * C, 2 * C, device=gpu) for k in ("plain", "fold")}
    db = {k: torch.empty(2 * C, device=gpu) for k in ("plain", "fold")}
    _lib.call("gwn_wgrad", dfg.data_ptr(), 2 * C, 2 * C, xn.data_ptr(), C, rows, C, 2, d * P, R,
              dw["plain"].data_ptr(), 2 * C, db["plain"].data_ptr(), ws.data_ptr(), _lib.stream())
    _lib.call("gwn_wgrad_bn", dfg.data_ptr(), 2 * C, 2 * C, zg.data_ptr(), C, rows, C, 2, d * P, R,
              mean.data_ptr(), scale.data_ptr(), beta.data_ptr(), dw["fold"].data_ptr(), 2 * C,
              db["fold"].data_ptr(), ws.data_ptr(), _lib.stream())
    torch.cuda.synchronize()
    assert rel_err(dw["fold"].cpu().numpy(), dw["plain"].cpu().numpy()) < 5e-6
    assert torch.equal(db["fold"], db["plain"])


def test_deferred_wgrad_reduction_bitwise(gpu):
    """gwn_wgrad_partials + ONE gwn_reduce_partials over several problems (the deferred weight
    gradients of a backward) give exactly gwn_wgrad's / gwn_wgrad_bn's results: the same partials,
    summed in the same fixed order."""
    from gwn_amd import _lib
    lib = _lib.load()
    torch.manual_seed(21)
    C, P, T, d = 32, 207 * 4, 5, 2
    R = (T - d) * P
    probs = []
    # gcn mlp: dY [R][32], X = h [R][224]
    probs.append(dict(dY=torch.randn(R, C, device=gpu), J=C, X=torch.randn(R, 7 * C, device=gpu), ldx=7 * C,
                      x_rows=R, Kt=7 * C, ntaps=1, shift=0, aff=(None, None, None)))
    # gated TCN with BatchNorm on load: dY = dfg [R][64], X = z [T*P][32], two taps
    z = torch.randn(T * P, C, device=gpu) * 2 + 5
    aff = (torch.randn(C, device=gpu) + 5, torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu))
    probs.append(dict(dY=torch.randn(R, 2 * C, device=gpu), J=2 * C, X=z, ldx=C, x_rows=T * P, Kt=C, ntaps=2,
                      shift=d * P, aff=aff))
    segs, ref = [], []
    for pr in probs:
        J, Kc = pr["J"], pr["Kt"] * pr["ntaps"]
        a = [None if t is None else t.data_ptr() for t in pr["aff"]]
        ws = torch.empty(lib.gwn_wgrad_workspace_floats(R, J, Kc) + 16, device=gpu)
        dw, db = torch.empty(J, Kc, device=gpu), torch.empty(J, device=gpu)
        _lib.call("gwn_wgrad_bn", pr["dY"].data_ptr(), J, J, pr["X"].data_ptr(), pr["ldx"], pr["x_rows"], pr["Kt"],
                  pr["ntaps"], pr["shift"], R, a[0], a[1], a[2], dw.data_ptr(), Kc, db.data_ptr(), ws.data_ptr(),
                  _lib.stream())
        ref.append((dw, db))
        cnt = lib.gwn_wgrad_partial_count(R, J, Kc)
        part = torch.empty(cnt * (J * Kc + J), device=gpu)
        _lib.call("gwn_wgrad_partials", pr["dY"].data_ptr(), J, J, pr["X"].data_ptr(), pr["ldx"], pr["x_rows"],
                  pr["Kt"], pr["ntaps"], pr["shift"], R, a[0], a[1], a[2], part.data_ptr(), _lib.stream())
        dw2, db2 = torch.full((J, Kc + 3), 7.0, device=gpu), torch.empty(J, device=gpu)
        segs.append((_lib.ReduceSeg(part=part.data_ptr(), nparts=cnt, part_stride=J * Kc + J, J=J, Kc=Kc,
                                    out=dw2.data_ptr(), ld_out=Kc + 3, out2=db2.data_ptr()), part, dw2, db2))
    arr = (_lib.ReduceSeg * len(segs))(*[sg[0] for sg in segs])
    _lib.call("gwn_reduce_partials", arr, len(segs), _lib.stream())
    torch.cuda.synchronize()
    for (dw, db), (_, _, dw2, db2) in zip(ref, segs):
        assert torch.equal(dw2[:, :dw.shape[1]], dw)
        assert torch.equal(db2, db)
        assert torch.all(dw2[:, dw.shape[1]:] == 7.0)


def test_narrow_wgrad_partials_vs_fp64(gpu):
    """The narrow form of gwn_wgrad_partials (Kc <= 4: the start conv's dW [32][2] and db over all
    positions) through gwn_reduce_partials, against fp64; ragged row counts."""
    from gwn_amd import _lib
    lib = _lib.load()
    for R, J, Kc in ((172224, 32, 2), (1001, 32, 3), (37, 64, 1)):
        torch.manual_seed(R + Kc)
        dY = torch.randn(R, J, dtype=torch.float64)
        X = torch.randn(R, Kc, dtype=torch.float64)
        cnt = lib.gwn_wgrad_partial_count(R, J, Kc)
        part = torch.empty(cnt * (J * Kc + J), device=gpu)
        dYd, Xd = dY.float().to(gpu), X.float().to(gpu)
        _lib.call("gwn_wgrad_partials", dYd.data_ptr(), J, J, Xd.data_ptr(), Kc, R, Kc, 1, 0, R, None, None, None,
                  part.data_ptr(), _lib.stream())
        dw, db = torch.empty(J, Kc, device=gpu), torch.empty(J, device=gpu)
        seg = (_lib.ReduceSeg * 1)(_lib.ReduceSeg(part=part.data_ptr(), nparts=cnt, part_stride=J * Kc + J, J=J, Kc=Kc,
                                                  out=dw.data_ptr(), ld_out=Kc, out2=db.data_ptr()))
        _lib.call("gwn_reduce_partials", seg, 1, _lib.stream())
        torch.cuda.synchronize()
        ref_w, ref_b = dY.t() @ X, dY.sum(0)
        bound_w = 2.0 ** -22 * R * (dY.abs().t() @ X.abs()) + 1e-30
        bound_b = 2.0 ** -22 * R * dY.abs().sum(0) + 1e-30
        assert torch.all((dw.double().cpu() - ref_w).abs() <= bound_w)
        assert torch.all((db.double().cpu() - ref_b).abs() <= bound_b)


def test_batchnorm_fwd_bwd(gpu):
    from gwn_amd import _lib
    torch.manual_seed(6)
    rows, c = 5000, 32
    z = (torch.randn(rows, c) * 3 + 1).to(gpu)
    gamma, beta = torch.randn(c, device=gpu), torch.randn(c, device=gpu)
    rm, rv = torch.zeros(c, device=gpu), torch.ones(c, device=gpu)
    out = torch.empty_like(z)
    mean, rstd = torch.empty(c, device=gpu), torch.empty(c, device=gpu)
    ws = torch.empty(_lib.load().gwn_batchnorm_workspace_floats(rows, c), device=gpu)
    _lib.call("gwn_batchnorm_fwd", z.data_ptr(), rows, c, gamma.data_ptr(), beta.data_ptr(), rm.data_ptr(),
              rv.data_ptr(), 0.1, 1e-5, 1, out.data_ptr(), mean.data_ptr(), rstd.data_ptr(), ws.data_ptr(),
              _lib.stream())
    zc = z.double().cpu().requires_grad_(True)
    bn = torch.nn.BatchNorm1d(c).double()
    with torch.no_grad():
        bn.weight.copy_(gamma.double().cpu())
        bn.bias.copy_(beta.double().cpu())
    ref = bn(zc)
    torch.cuda.synchronize()
    assert rel_err(out.cpu().numpy(), ref.detach().numpy()) < 1e-5
    assert rel_err(rm.cpu().numpy(), bn.running_mean.numpy()) < 1e-5
    assert rel_err(rv.cpu().numpy(), bn.running_var.numpy()) < 1e-5
    dy = torch.randn(rows, c, device=gpu)
    ref.backward(dy.double().cpu())
    dg, db = torch.empty(c, device=gpu), torch.empty(c, device=gpu)
    dres = torch.full((rows + 7, c), float("nan"), device=gpu)
    dh = torch.empty(rows, c, device=gpu)
    _lib.call("gwn_batchnorm_bwd", dy.data_ptr(), z.data_ptr(), rows, c, gamma.data_ptr(), mean.data_ptr(),
              rstd.data_ptr(), dg.data_ptr(), db.data_ptr(), dres.data_ptr(), 7, dh.data_ptr(), None, 0, 0.0, 1,
              ws.data_ptr(), _lib.stream())
    torch.cuda.synchronize()
    assert rel_err(dh.cpu().numpy(), zc.grad.numpy()) < 1e-4
    assert torch.all(dres[:7] == 0)
    assert torch.equal(dres[7:], dh)
    assert rel_err(dg.cpu().numpy(), bn.weight.grad.numpy()) < 1e-5
    assert rel_err(db.cpu().numpy(), bn.bias.grad.numpy()) < 1e-5


def test_masked_loss_and_grad(gpu):
    from gwn_amd import _lib
    from oracle import gwnet_oracle as orc
    torch.manual_seed(7)
    B, O, N, tf = 8, 12, 50, 3
    out = torch.randn(B, O, N, tf, device=gpu)
    real = torch.clamp(54.4 + 19.5 * torch.randn(B, O, N), 0, 80)
    real[torch.rand_like(real) < 0.1] = 0
    real_t = real.permute(0, 2, 1).contiguous().to(gpu).transpose(1, 2)  # non-contiguous [B][N][O] view... 
    real_v = real.permute(0, 2, 1).contiguous().to(gpu)  # [B][N][O]
    metrics = torch.empty(4, device=gpu)
    dout = torch.empty_like(out)
    ws = torch.empty(_lib.load().gwn_masked_loss_workspace_floats(B, O, N, tf), device=gpu)
    rs = real_v.stride()
    _lib.call("gwn_masked_loss", out.data_ptr(), real_v.data_ptr(), rs[0], rs[1], rs[2], B, O, N, tf, 54.4, 19.5,
              metrics.data_ptr(), dout.data_ptr(), ws.data_ptr(), _lib.stream())
    oc = out.double().cpu().requires_grad_(True)
    pred = oc.transpose(1, 3) * 19.5 + 54.4
    mae, mape, rmse = orc.masked_metrics(pred, real_v.double().cpu().unsqueeze(1))
    mae.backward()
    torch.cuda.synchronize()
    m = metrics.cpu().numpy()
    np.testing.assert_allclose(m[:3], [mae.item(), mape.item(), rmse.item()], rtol=2e-5)
    assert rel_err(dout.cpu().numpy(), oc.grad.numpy()) < 1e-5
    del real_t


@pytest.mark.parametrize("M,N,K", [(1, 12, 512), (1000, 12, 512), (1000, 512, 12), (777, 256, 256),
                                   (13248, 512, 256), (300, 200, 36), (129, 64, 4)])
@pytest.mark.parametrize("epi", ["plain", "bias_relu", "mask"])
def test_gemm_nt(gpu, M, N, K, epi):
    """gwn_gemm_nt (head convs and their input gradients) vs fp64: C = epi(A B^T), ragged tiles,
    K < one LDS tile, N < one MFMA tile; columns of C beyond N untouched."""
    from gwn_amd import _lib
    torch.manual_seed(M + 3 * N + 7 * K)
    A = torch.randn(M, K, dtype=torch.float64)
    Bm = torch.randn(N, K, dtype=torch.float64)
    bias = torch.randn(N, dtype=torch.float64)
    mask = torch.randn(M, N, dtype=torch.float64)
    ref = A @ Bm.t()
    if epi == "bias_relu":
        ref = torch.clamp(ref + bias, min=0.0)
    elif epi == "mask":
        ref = torch.where(mask > 0, ref, torch.zeros_like(ref))
    ldc = N + 4
    Cd = torch.full((M, ldc), 7.0, device=gpu)
    Ad, Bd = A.float().to(gpu), Bm.float().to(gpu)
    bd, md = bias.float().to(gpu), mask.float().to(gpu)
    _lib.call("gwn_gemm_nt", Ad.data_ptr(), K, Bd.data_ptr(), K, Cd.data_ptr(), ldc, M, N, K,
              bd.data_ptr() if epi == "bias_relu" else None, 1 if epi == "bias_relu" else 0,
              md.data_ptr() if epi == "mask" else None, N, _lib.stream())
    torch.cuda.synchronize()
    got = Cd.cpu().double()
    assert torch.all(got[:, N:] == 7.0)
    scale = float(ref.abs().max()) + 1e-30
    assert float((got[:, :N] - ref).abs().max()) / scale <= 2e-6


@pytest.mark.parametrize("M,N,K", [(1, 64, 256), (777, 256, 256), (20800, 512, 256), (20800, 256, 512),
                                   (300, 192, 36), (129, 64, 4)])
@pytest.mark.parametrize("epi", ["plain", "bias_relu", "mask"])
def test_gemm_nt_bf16(gpu, M, N, K, epi):
    """gwn_gemm_nt_bf16 (the bf16 mode's head GEMMs) vs fp64 of the bf16-rounded (RNE) operands:
    the fp32 accumulation floor; ragged row tiles, K < one LDS tile, column tiles of 64 and 128;
    columns of C beyond N untouched."""
    from gwn_amd import _lib
    torch.manual_seed(M + 5 * N + 11 * K)
    A = torch.randn(M, K) * 3
    Bm = torch.randn(N, K)
    bias = torch.randn(N, dtype=torch.float64)
    mask = torch.randn(M, N, dtype=torch.float64)
    rb = lambda t: t.to(torch.bfloat16).double()  # noqa: E731
    ref = rb(A) @ rb(Bm).t()
    if epi == "bias_relu":
        ref = torch.clamp(ref + bias, min=0.0)
    elif epi == "mask":
        ref = torch.where(mask > 0, ref, torch.zeros_like(ref))
    ldc = N + 4
    Cd = torch.full((M, ldc), 7.0, device=gpu)
    Ad, Bd = A.to(gpu), Bm.to(gpu)
    bd, md = bias.float().to(gpu), mask.float().to(gpu)
    _lib.call("gwn_gemm_nt_bf16", Ad.data_ptr(), K, Bd.data_ptr(), K, Cd.data_ptr(), ldc, M, N, K,
              bd.data_ptr() if epi == "bias_relu" else None, 1 if epi == "bias_relu" else 0,
              md.data_ptr() if epi == "mask" else None, N, _lib.stream())
    torch.cuda.synchronize()
    got = Cd.cpu().double()
    assert torch.all(got[:, N:] == 7.0)
    terms = rb(A).abs() @ rb(Bm).abs().t()  # fp32 accumulation error ~ 2^-24 sqrt(K) sum|terms|
    assert float(((got[:, :N] - ref).abs() / (terms + 1e-30)).max()) <= 2e-6
    # not the fp32 product: the operands really were rounded
    if epi == "plain" and K >= 36:
        assert float((got[:, :N] - A.double() @ Bm.double().t()).abs().max()) > 1e-4


@pytest.mark.parametrize("R,J,Kc,pad", [(20800, 512, 256, 0), (13248, 256, 256, 4), (777, 256, 128, 0),
                                        (100, 128, 128, 8)])
def test_wgrad_bf16_partials(gpu, R, J, Kc, pad):
    """gwn_wgrad_bf16_partials + gwn_reduce_partials (the bf16 mode's end_conv_1 and skip-conv weight
    gradients) vs fp64 of the bf16-rounded operands: dW = bf16(dY)^T bf16(X) at the fp32
    accumulation floor, db = the unrounded column sums of dY; ragged row chunks, padded leading
    dimensions."""
    from gwn_amd import _lib
    torch.manual_seed(R + J + Kc)
    dY = torch.randn(R, J + pad) * 2
    X = torch.rand(R, Kc + pad)
    rb = lambda t: t.to(torch.bfloat16).double()  # noqa: E731
    ref = rb(dY[:, :J]).t() @ rb(X[:, :Kc])
    terms = rb(dY[:, :J]).abs().t() @ rb(X[:, :Kc]).abs()
    dbr = dY[:, :J].double().sum(0)
    n = int(_lib.load().gwn_wgrad_bf16_partial_count(R, J, Kc))
    assert n >= 1
    part = torch.full((n * (J * Kc + J),), float("nan"), device=gpu)
    dYd, Xd = dY.to(gpu), X.to(gpu)
    out = torch.full((J, Kc + 3), 7.0, device=gpu)
    db = torch.empty(J, device=gpu)
    _lib.call("gwn_wgrad_bf16_partials", dYd.data_ptr(), J + pad, J, Xd.data_ptr(), Kc + pad, Kc, R, part.data_ptr(),
              _lib.stream())
    seg = _lib.ReduceSeg(part=part.data_ptr(), nparts=n, part_stride=J * Kc + J, J=J, Kc=Kc, out=out.data_ptr(),
                         ld_out=Kc + 3, out2=db.data_ptr(), db_off=J * Kc)
    _lib.call("gwn_reduce_partials", (_lib.ReduceSeg * 1)(seg), 1, _lib.stream())
    torch.cuda.synchronize()
    got = out.cpu().double()
    assert torch.all(got[:, Kc:] == 7.0)
    assert float(((got[:, :Kc] - ref).abs() / terms).max()) <= 2e-6
    assert float((db.cpu().double() - dbr).abs().max() / dY[:, :J].double().abs().sum(0).max()) <= 2e-6
    assert float((got[:, :Kc] - dY[:, :J].double().t() @ X[:, :Kc].double()).abs().max()) > 1e-4  # bf16 really


def _merge_bn(bnp, S, nkb, C):
    """Per-slice (count, mean, M2) [S][3][C] (fp64) from BN partial slots [S][nkb][3][C] (count-0
    slots carry nothing), Chan's merge; the fused forward writes one slot per slice (nkb = 1)."""
    p = bnp.double().cpu()[:S * nkb * 3 * C].view(S, nkb, 3, C)
    n = torch.zeros(S, C, dtype=torch.float64)
    mean = torch.zeros(S, C, dtype=torch.float64)
    m2 = torch.zeros(S, C, dtype=torch.float64)
    for t in range(nkb):
        nb, mb, qb = p[:, t, 0], p[:, t, 1], p[:, t, 2]
        nn = n + nb
        safe = torch.where(nn > 0, nn, torch.ones_like(nn))
        d = mb - mean
        mean = torch.where(nb > 0, mean + d * nb / safe, mean)
        m2 = torch.where(nb > 0, m2 + qb + d * d * n * nb / safe, m2)
        n = nn
    return torch.stack([n, mean, m2], dim=1)


def _bn_all(bnp, rows, n, C, K, NP):
    """(count, mean, M2) [1][3][C] of all rows from the gwn_gcn_bn_partial_count slots gwn_gcn_fwd
    writes (per slice or per workgroup tile range, by kernel; count-0 slots carry nothing)."""
    from gwn_amd import _lib
    return _merge_bn(bnp, 1, int(_lib.load().gwn_gcn_bn_partial_count(rows, n, C, K, NP)), C)


def _squares(gpu, sups, transposes=False):
    """gwn_support_square of each padded support: (A^2, (A^2)^T[, A^T])."""
    from gwn_amd import _lib
    out = []
    for s_ in sups:
        NP = s_.shape[0]
        a2 = torch.full_like(s_, float("nan"))
        a2t = torch.full_like(s_, float("nan"))
        at = torch.full_like(s_, float("nan")) if transposes else None
        _lib.call("gwn_support_square", s_.data_ptr(), NP, NP, a2.data_ptr(), a2t.data_ptr(),
                  at.data_ptr() if at is not None else None, _lib.stream())
        out.append((a2, a2t, at))
    return out


def _g4s(gpu, n, sups, sq, supT):
    """gwn_support_g4 copies for the 16-node tile kernels: forward [A_k, A_k^2] and backward
    [A_k^T, (A_k^2)^T], each as (buffer, pointer-array field, array) -- keep the tuple alive."""
    import ctypes
    from gwn_amd import _lib
    NP = sups[0].shape[0]
    P = ctypes.POINTER(ctypes.c_void_p)
    fl = _lib.load().gwn_support_g4_floats(n)
    out = []
    for mats in ([m for s_, q in zip(sups, sq) for m in (s_, q[0])],
                 [m for t_, q in zip(supT, sq) for m in (t_, q[1])]):
        buf = torch.full((len(mats), fl), float("nan"), device=gpu)
        src = (ctypes.c_void_p * len(mats))(*[m.data_ptr() for m in mats])
        _lib.call("gwn_support_g4", ctypes.cast(src, P), len(mats), n, NP, buf.data_ptr(), fl, _lib.stream())
        arr = (ctypes.c_void_p * len(mats))(*[buf[i].data_ptr() for i in range(len(mats))])
        out.append((buf, ctypes.cast(arr, P), arr))
    return out


@pytest.mark.parametrize("n", [16, 37, 207, 325])
def test_support_g4_layout(gpu, n):
    """gwn_support_g4: the 16-node k-interleaved copy of a padded support, element for element
    (include/gwn.h), against a host restatement of the layout."""
    import ctypes
    from gwn_amd import _lib
    torch.manual_seed(n + 7)
    NP = (n + 31) // 32 * 32
    mats = []
    for _ in range(3):
        s_ = torch.zeros(NP, NP, device=gpu)
        s_[:n, :n] = torch.rand(n, n, device=gpu)
        mats.append(s_)
    fl = _lib.load().gwn_support_g4_floats(n)
    nt = (n + 15) // 16
    assert fl == nt * nt * 256
    dst = torch.full((3, fl + 5), float("nan"), device=gpu)
    src = (ctypes.c_void_p * 3)(*[m.data_ptr() for m in mats])
    _lib.call("gwn_support_g4", ctypes.cast(src, ctypes.POINTER(ctypes.c_void_p)), 3, n, NP, dst.data_ptr(), fl + 5,
              _lib.stream())
    torch.cuda.synchronize()
    d = dst.cpu().numpy()
    for c, m in enumerate(mats):
        A = m.cpu().numpy()
        kg, t, g, j, i = np.meshgrid(np.arange(nt), np.arange(nt), np.arange(4), np.arange(16), np.arange(4),
                                     indexing="ij")
        idx = ((kg * nt + t) * 64 + 16 * g + j) * 4 + i
        ref = A[16 * kg + 4 * i + g, 16 * t + j]
        assert np.array_equal(d[c][idx.ravel()], ref.ravel())
        assert np.all(np.isnan(d[c][fl:]))  # nothing written past one copy


@pytest.mark.parametrize("n", [16, 37, 207, 325])
@pytest.mark.parametrize("count", [2, 4])
def test_support_square_g4(gpu, n, count):
    """gwn_support_square_g4: the square / transposes as gwn_support_square, and the 16-node tile
    copies of A, A^2 (, A^T, (A^2)^T) bit-identical to gwn_support_g4 of those matrices."""
    import ctypes
    from gwn_amd import _lib
    lib = _lib.load()
    torch.manual_seed(n + count)
    NP = (n + 31) // 32 * 32
    a = torch.zeros(NP, NP, device=gpu)
    a[:n, :n] = torch.rand(n, n, device=gpu)
    fl = lib.gwn_support_g4_floats(n)
    outs = [torch.full((NP, NP), float("nan"), device=gpu) for _ in range(3)]
    g4 = torch.full((4, fl), float("nan"), device=gpu)
    _lib.call("gwn_support_square_g4", a.data_ptr(), NP, NP, outs[0].data_ptr(), outs[1].data_ptr(),
              outs[2].data_ptr(), n, g4.data_ptr(), fl, count, _lib.stream())
    ref_sq = [torch.full((NP, NP), float("nan"), device=gpu) for _ in range(3)]
    _lib.call("gwn_support_square", a.data_ptr(), NP, NP, ref_sq[0].data_ptr(), ref_sq[1].data_ptr(),
              ref_sq[2].data_ptr(), _lib.stream())
    mats = [a, ref_sq[0], ref_sq[2], ref_sq[1]][:count]
    ref = torch.full((count, fl), float("nan"), device=gpu)
    src = (ctypes.c_void_p * count)(*[m.data_ptr() for m in mats])
    _lib.call("gwn_support_g4", ctypes.cast(src, ctypes.POINTER(ctypes.c_void_p)), count, n, NP, ref.data_ptr(), fl,
              _lib.stream())
    torch.cuda.synchronize()
    for o, r in zip(outs, ref_sq):
        assert torch.equal(o, r)
    assert torch.equal(g4[:count], ref)
    if count == 2:
        assert torch.all(torch.isnan(g4[2:]))


@pytest.mark.parametrize("n", [16, 37, 207, 325])
def test_support_square(gpu, n):
    """gwn_support_square: A^2 and its transpose (and A^T) of a padded support against fp64; the
    padding stays zero.  Bound: fp32 FMA chain over K = np terms."""
    torch.manual_seed(n)
    NP = (n + 31) // 32 * 32
    s_ = torch.zeros(NP, NP, device=gpu)
    s_[:n, :n] = torch.rand(n, n, device=gpu)
    ((a2, a2t, at),) = _squares(gpu, [s_], transposes=True)
    torch.cuda.synchronize()
    A = s_.double().cpu()
    ref = A @ A
    bound = 2.0 ** -22 * NP * (A.abs() @ A.abs()) + 1e-30
    assert torch.all((a2.double().cpu() - ref).abs() <= bound)
    assert torch.equal(a2t.cpu(), a2.cpu().t())
    assert torch.equal(at.cpu(), s_.cpu().t())
    assert torch.all(a2[n:, :] == 0) and torch.all(a2[:, n:] == 0)


@pytest.mark.parametrize("n", [16, 96, 207, 256, 325])
def test_gcn_fused_schedules_agree(gpu, n, monkeypatch):
    """The two schedules of the fused gcn forward / backward -- chained hops (hop 2 diffuses hop 1
    through LDS) and the power schedule (A and A^2 against the node features in one pass, backward
    W^T-after-diffusion) -- each whole-slice and with the support split (one workgroup per (slice,
    support), partial sums combined by the slice's last workgroup), the power forward on 16-node
    tiles (default) and on 32-node tiles (GWN_GCN_T16=0), against fp64 (model.py:41-55): hop
    pieces, z, BN partials, dxg and the adaptive-support pieces t1 / t2."""
    import ctypes
    from gwn_amd import _lib
    torch.manual_seed(n)
    C, K, S = 32, 3, 11
    NP = (n + 31) // 32 * 32
    W = (2 * K + 1) * C
    rows = S * n
    sups = []
    for _ in range(K):
        s = torch.zeros(NP, NP, device=gpu)
        s[:n, :n] = torch.rand(n, n, device=gpu) / n
        sups.append(s)
    supT = [s.t().contiguous() for s in sups]
    sq = _squares(gpu, sups)
    arr = (ctypes.c_void_p * K)(*[s.data_ptr() for s in sups])
    arrT = (ctypes.c_void_p * K)(*[s.data_ptr() for s in supT])
    arr2 = (ctypes.c_void_p * K)(*[q[0].data_ptr() for q in sq])
    arr2T = (ctypes.c_void_p * K)(*[q[1].data_ptr() for q in sq])
    g4f, g4b = _g4s(gpu, n, sups, sq, supT)
    P = ctypes.POINTER(ctypes.c_void_p)
    wm = torch.randn(C, W, device=gpu) * 0.1
    wmt = wm.t().contiguous()
    bm = torch.randn(C, device=gpu)
    res = torch.randn(rows, C, device=gpu)
    xg = torch.randn(rows, C, device=gpu)
    dh = torch.randn(rows, C, device=gpu)
    seed = torch.zeros(1, device=gpu, dtype=torch.int64)
    outs = []
    kws = torch.empty(_lib.load().gwn_gcn_ksplit_ws_floats(rows, n, K), device=gpu)
    kcnt = torch.zeros(S, device=gpu, dtype=torch.int32)
    for pw, ksplit, t16 in ((False, 1, "1"), (False, K, "1"), (True, 1, "1"), (True, K, "1"), (True, 1, "0")):
        monkeypatch.setenv("GWN_GCN_T16", t16)
        kf = dict(ksplit=ksplit, ksplit_ws=kws.data_ptr(), ksplit_count=kcnt.data_ptr())
        h = torch.zeros(rows, W, device=gpu)
        h[:, :C] = xg
        z = torch.empty(rows, C, device=gpu)
        bnp = torch.full((_lib.load().gwn_gcn_bn_partial_count(rows, n, C, K, NP) * 3 * C,), float("nan"), device=gpu)
        ga = _lib.GcnArgs(rows=rows, n=n, c=C, nsup=K, sup=ctypes.cast(arr, P),
                          ld_sup=NP, h=h.data_ptr(), ld_h=W, w_mlp=wm.data_ptr(), b_mlp=bm.data_ptr(),
                          residual=res.data_ptr(), z=z.data_ptr(), seed_ptr=seed.data_ptr(), salt=0, drop_p=0.0,
                          bn_partials=bnp.data_ptr(), sup2=ctypes.cast(arr2, P) if pw else None, w_mlp_t=wmt.data_ptr(),
                          sup_g4=g4f[1] if pw and t16 == "1" else None, **kf)
        _lib.call("gwn_gcn_fwd", ctypes.byref(ga), _lib.stream())
        dhc = torch.zeros(rows, W, device=gpu)
        gb = _lib.GcnBwdArgs(rows=rows, n=n, c=C, nsup=K, sup=ctypes.cast(arr, P),
                             ld_sup=NP, h=h.data_ptr(), ld_h=W, w_mlp=wm.data_ptr(), dh=dh.data_ptr(),
                             dhcat=dhc.data_ptr(), ld_dhcat=W, adp_index=K - 1, accumulate_dadp=0,
                             sup_t=ctypes.cast(arrT, P), skip_weight_grads=1,
                             sup2_t=ctypes.cast(arr2T, P) if pw else None,
                             sup_g4_t=g4b[1] if pw and t16 == "1" else None, **kf)
        _lib.call("gwn_gcn_bwd", ctypes.byref(gb), _lib.stream())
        torch.cuda.synchronize()
        outs.append((h.clone(), z.clone(), _bn_all(bnp, rows, n, C, K, NP), dhc.clone()))
        assert int(kcnt.abs().sum()) == 0  # the split leaves its counters zero
    # fp64 truth
    X = xg.double().cpu().view(S, n, C)
    A = [s[:n, :n].double().cpu() for s in sups]
    pieces = [X]
    for a in A:
        x1 = torch.einsum("svc,vw->swc", X, a)
        x2 = torch.einsum("svc,vw->swc", x1, a)
        pieces += [x1, x2]
    H = torch.cat(pieces, dim=2).reshape(rows, W)
    Z = H @ wm.double().cpu().t() + bm.double().cpu() + res.double().cpu()
    dP = (dh.double().cpu() @ wm.double().cpu()).view(S, n, W)
    dxg = dP[:, :, :C].clone()
    t1 = t2 = None
    for k, a in enumerate(A):
        dx2 = dP[:, :, (2 + 2 * k) * C:(3 + 2 * k) * C]
        dx1 = dP[:, :, (1 + 2 * k) * C:(2 + 2 * k) * C] + torch.einsum("swc,vw->svc", dx2, a)
        dxg = dxg + torch.einsum("swc,vw->svc", dx1, a)
        t1, t2 = dx1, dx2
    # fp32 rounding floor (max-abs error / max-abs value): the support split adds the partial
    # sums in another order than the MFMA chains (measured 2.02e-6 on dxg at n = 207)
    for h, z, st, dhc in outs:
        assert rel_err(h.cpu().numpy(), H.numpy()) <= 4e-6
        assert rel_err(z.cpu().numpy(), Z.numpy()) <= 4e-6
        assert rel_err(dhc[:, :C].cpu().numpy(), dxg.reshape(rows, C).numpy()) <= 4e-6
        assert rel_err(dhc[:, C:2 * C].cpu().numpy(), t1.reshape(rows, C).numpy()) <= 4e-6
        assert rel_err(dhc[:, 2 * C:3 * C].cpu().numpy(), t2.reshape(rows, C).numpy()) <= 4e-6
        assert torch.all(st[:, 0] == rows)
        assert rel_err(st[:, 1].numpy(), Z.mean(0, keepdim=True).numpy()) <= 1e-5
        m2 = ((Z - Z.mean(0, keepdim=True)) ** 2).sum(0, keepdim=True)
        assert rel_err(st[:, 2].numpy(), m2.numpy()) <= 1e-5
    # the split against the whole slice, per schedule: the same products, summed in another order
    for a_i, b_i in ((0, 1), (2, 3)):
        for a_, b_ in zip(outs[a_i], outs[b_i]):
            assert rel_err(a_.cpu().numpy(), b_.cpu().numpy()) <= 2e-6


@pytest.mark.parametrize("bn", [False, True])
@pytest.mark.parametrize("n,B,t_out,d,planes", [(207, 32, 8, 2, 0), (37, 64, 5, 1, 0), (207, 8, 3, 1, 0),
                                                (325, 32, 8, 1, 2), (207, 64, 10, 1, 0)])
# (planes 2: the bf16-mlp pair forward, where the TCN stays a separate launch -- fused there it was
#  7.5 % slower per PEMS step, profiles/r05/tcn_fused -- so both sides of the comparison are the
#  two-launch path and must agree bitwise)
def test_gcn_fwd_fused_tcn(gpu, n, B, t_out, d, bn, planes):
    """gwn_gcn_args.tcn: the gated TCN (model.py:206-212) computed inside the f32 16-node tile
    forward's staging (>= a slice per CU) against the same layer as two calls (gwn_gated_tcn_fwd,
    then gwn_gcn_fwd): xg (piece 0 of h), the (tanh, sigmoid) pairs, the skip rows, the hop pieces,
    z and the BN statistics agree to the fp32 floor (the products summed in another order), and xg
    matches fp64.  The last case has fewer slices than CUs: the TCN is then its own launch inside
    gwn_gcn_fwd and everything is bitwise the two-call result.  x is a pre-BN z (model.py:234-236,
    train mode): plain, its BatchNorm applied on load (x_mean, folded weights); with bn, that
    BatchNorm finalized by the TCN itself from [nparts][3][c] partials (gwn_tcn_args.bn: in every
    workgroup of the fused launch, or gwn_batchnorm_fwd_fold first): its outputs (mean, rstd,
    scale, running statistics, num_batches_tracked, w_fold, b_fold) against fp64 as well.  planes 2:
    the bf16-mlp pair forward (configs[2]), which takes the TCN as its own launch.  The fused call
    also carries gwn_gcn_args.clock (bench.py's timing): every workgroup's (start, end) stamped.
    (207, 64, 10): 640 slices, 2.5 per CU -- the tile ranges straddle slices, the pipelined staging's
    ranges touch 3-4 slices (items of several slices interleaved, boundary slices' TCN in two CUs)."""
    import ctypes
    from gwn_amd import _lib
    lib = _lib.load()
    torch.manual_seed(n + B + d + bn)
    C, K = 32, 3
    NP = (n + 31) // 32 * 32
    W = (2 * K + 1) * C
    P = B * n
    t_in = t_out + d
    S = t_out * B
    rows = S * n
    sups = []
    for _ in range(K):
        s_ = torch.zeros(NP, NP, device=gpu)
        s_[:n, :n] = torch.rand(n, n, device=gpu) / n
        sups.append(s_)
    supT = [s_.t().contiguous() for s_ in sups]
    sq = _squares(gpu, sups)
    arr = (ctypes.c_void_p * K)(*[s_.data_ptr() for s_ in sups])
    arr2 = (ctypes.c_void_p * K)(*[q[0].data_ptr() for q in sq])
    g4f, _ = _g4s(gpu, n, sups, sq, supT)
    PP = ctypes.POINTER(ctypes.c_void_p)
    extra = dict(sup_g4=g4f[1])
    if planes:
        el = lib.gwn_support_g4_bf16_elems(n)
        mats = [m for s_, q in zip(sups, sq) for m in (s_, q[0])]
        g4bf = torch.zeros(len(mats), el // 2, device=gpu)
        srcb = (ctypes.c_void_p * len(mats))(*[m.data_ptr() for m in mats])
        _lib.call("gwn_support_g4_bf16", ctypes.cast(srcb, PP), len(mats), n, NP, g4bf.data_ptr(), el, _lib.stream())
        arrb = (ctypes.c_void_p * len(mats))(*[g4bf[i].data_ptr() for i in range(len(mats))])
        extra = dict(split_planes=planes, sup_g4b=ctypes.cast(arrb, PP))
    x = torch.randn(t_in * P, C, device=gpu) * 2 + 3 + torch.randn(C, device=gpu)
    xmean = torch.randn(C, device=gpu) + 3
    wfg = torch.randn(2 * C, 2 * C, device=gpu) * 0.15
    bfg = torch.randn(2 * C, device=gpu) * 0.1
    wm = torch.randn(C, W, device=gpu) * 0.1
    wmt = wm.t().contiguous()
    bm = torch.randn(C, device=gpu)
    seed = torch.zeros(1, device=gpu, dtype=torch.int64)
    ld_skip = 3 * C
    skip_row0 = (t_out - 1) * P
    nparts = int(lib.gwn_gcn_bn_partial_count(rows, n, C, K, NP))
    # the layer below's BatchNorm partials over x's rows: 300 ragged chunks, some empty
    xr = x.double().cpu()
    cuts = sorted(set([0, xr.shape[0]] + torch.randint(0, xr.shape[0], (297,)).tolist()))
    bpl = torch.zeros(len(cuts) - 1 + 3, 3, C, dtype=torch.float64)
    for q, (lo, hi) in enumerate(zip(cuts[:-1], cuts[1:])):
        if hi > lo:
            blk = xr[lo:hi]
            bpl[q, 0], bpl[q, 1] = hi - lo, blk.mean(0)
            bpl[q, 2] = ((blk - blk.mean(0)) ** 2).sum(0)
    bparts = bpl.float().to(gpu).contiguous()
    gamma, beta = torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu)
    outs = {}
    for fused in (False, True):
        h = torch.full((rows, W), float("nan"), device=gpu)
        fg = torch.full((rows, 2 * C), float("nan"), device=gpu)
        skip = torch.full((rows - skip_row0, ld_skip), float("nan"), device=gpu)
        z = torch.empty(rows, C, device=gpu)
        bnp = torch.full((nparts * 3 * C,), float("nan"), device=gpu)
        ta = _lib.TcnArgs(x=x.data_ptr(), t_in=t_in, P=P, c=C, dilation=d, w_fg=wfg.data_ptr(), b_fg=bfg.data_ptr(),
                          xg=h.data_ptr(), ld_xg=W, fg=fg.data_ptr(), skipcat=skip.data_ptr(), ld_skip=ld_skip,
                          skip_row0=skip_row0, x_mean=xmean.data_ptr())
        res_aff = {}
        bo = None
        if bn:
            bo = dict(mean=torch.full((C,), float("nan"), device=gpu), rstd=torch.full((C,), float("nan"), device=gpu),
                      scale=torch.full((C,), float("nan"), device=gpu), rm=torch.zeros(C, device=gpu) + 0.5,
                      rv=torch.ones(C, device=gpu), nbt=torch.full((1,), 3, device=gpu, dtype=torch.int64),
                      wf=torch.full_like(wfg, float("nan")), bf=torch.full_like(bfg, float("nan")))
            bfp = _lib.BnFold(gamma=gamma.data_ptr(), beta=beta.data_ptr(), running_mean=bo["rm"].data_ptr(),
                              running_var=bo["rv"].data_ptr(), momentum=0.1, eps=1e-5, save_mean=bo["mean"].data_ptr(),
                              save_rstd=bo["rstd"].data_ptr(), scale=bo["scale"].data_ptr(), w_next=wfg.data_ptr(),
                              b_next=bfg.data_ptr(), w_fold=bo["wf"].data_ptr(), b_fold=bo["bf"].data_ptr(),
                              num_batches_tracked=bo["nbt"].data_ptr())
            ta.bn, ta.bn_partials, ta.bn_nparts = ctypes.addressof(bfp), bparts.data_ptr(), bparts.shape[0]
            ta.x_mean = None
            res_aff = dict(residual_mean=bo["mean"].data_ptr(), residual_scale=bo["scale"].data_ptr(),
                           residual_shift=beta.data_ptr())
        ga = _lib.GcnArgs(rows=rows, n=n, c=C, nsup=K, sup=ctypes.cast(arr, PP), ld_sup=NP, h=h.data_ptr(), ld_h=W,
                          w_mlp=wm.data_ptr(), b_mlp=bm.data_ptr(), residual=x.data_ptr() + 4 * d * P * C,
                          z=z.data_ptr(), seed_ptr=seed.data_ptr(), salt=0, drop_p=0.0, bn_partials=bnp.data_ptr(),
                          sup2=ctypes.cast(arr2, PP), w_mlp_t=wmt.data_ptr(), **extra, **res_aff)
        if fused:
            ga.tcn = ctypes.pointer(ta)
            clk = torch.zeros(2 * _cus(), device=gpu, dtype=torch.int64)
            ga.clock = clk.data_ptr()  # the instrumentation rides along (results compared as ever)
            used = ctypes.c_int(-1)
            ga.bn_slots_used = ctypes.pointer(used)
        else:
            _lib.call("gwn_gated_tcn_fwd", ctypes.byref(ta), _lib.stream())
        _lib.call("gwn_gcn_fwd", ctypes.byref(ga), _lib.stream())
        torch.cuda.synchronize()
        outs[fused] = (h, fg, skip[:, :C], z, _bn_all(bnp, rows, n, C, K, NP)) + (
            tuple(bo[k] for k in ("mean", "rstd", "scale", "rm", "rv", "nbt", "wf", "bf")) if bn else ())
    (h0, fg0, sk0, z0, st0), (h1, fg1, sk1, z1, st1) = outs[False][:5], outs[True][:5]
    # gwn_gcn_args.bn_slots_used: the leading slots that can hold rows (the tile grid); the rest
    # zero-count, so a consumer merging only those gets the same statistics
    assert 1 <= used.value <= min(nparts, _cus())
    assert torch.all(bnp.view(nparts, 3, C)[used.value:, 0] == 0)
    assert int(bnp.view(nparts, 3, C)[:used.value, 0].sum(0)[0]) == rows
    # gwn_gcn_args.clock: every workgroup of the tile launch stamped (start, end), slots [0, grid)
    c = clk.cpu().reshape(-1, 2)
    g = int((c[:, 1] > 0).sum())
    assert g == used.value
    assert 0 < g <= _cus() and bool((c[:g] > 0).all()) and bool((c[g:] == 0).all())
    assert bool((c[:g, 1] >= c[:g, 0]).all())
    span_ms = float(c[:g, 1].max() - c[:g, 0].min()) / lib.gwn_wall_clock_khz()
    assert 0 < span_ms < 1000
    if S < _cus() or planes:
        for a_, b_ in zip(outs[False], outs[True]):
            assert torch.equal(a_, b_)
        return
    # fp64 truth of xg (and of the BatchNorm the TCN finalized)
    if bn:
        mu, var = xr.mean(0), xr.var(0, unbiased=False)
        rstd = 1.0 / torch.sqrt(var + 1e-5)
        sc = rstd * gamma.double().cpu()
        for k, (mean_, rstd_, scale_, rm_, rv_, nbt_, wf_, bf_) in ((k, outs[k][5:]) for k in (False, True)):
            assert rel_err(mean_.cpu().numpy(), mu.numpy()) <= 1e-6
            assert rel_err(rstd_.cpu().numpy(), rstd.numpy()) <= 1e-6
            assert rel_err(scale_.cpu().numpy(), sc.numpy()) <= 1e-6
            assert rel_err(rm_.cpu().numpy(), (0.45 + 0.1 * mu).numpy()) <= 1e-6
            assert rel_err(rv_.cpu().numpy(), (0.9 + 0.1 * xr.var(0, unbiased=True)).numpy()) <= 1e-6
            assert int(nbt_.item()) == 4
            assert rel_err(wf_.cpu().numpy(), (wfg.double().cpu() * sc.repeat(2)[None, :]).numpy()) <= 1e-6
            bref = bfg.double().cpu() + wfg.double().cpu() @ beta.double().cpu().repeat(2)
            assert rel_err(bf_.cpu().numpy(), bref.numpy()) <= 1e-6
        xd = ((xr - mu) * sc + beta.double().cpu())
        W_ = wfg.double().cpu()
        f = torch.cat([xd[:rows], xd[d * P:d * P + rows]], dim=1) @ W_.t() + bfg.double().cpu()
    else:
        xd = (xr - xmean.double().cpu())
        f = torch.cat([xd[:rows], xd[d * P:d * P + rows]], dim=1) @ wfg.double().cpu().t() + bfg.double().cpu()
    xg_ref = torch.tanh(f[:, 0::2]) * torch.sigmoid(f[:, 1::2])
    # (the fp32 floor of 64-term sums of ~5-magnitude products, as the row-GEMM TCN's tests: 5e-6)
    assert rel_err(h0[:, :C].cpu().numpy(), xg_ref.numpy()) <= 5e-6
    assert rel_err(h1[:, :C].cpu().numpy(), xg_ref.numpy()) <= 5e-6
    assert rel_err(h1[:, :C].cpu().numpy(), h0[:, :C].cpu().numpy()) <= 5e-6
    assert rel_err(fg1.cpu().numpy(), fg0.cpu().numpy()) <= 5e-6
    assert torch.equal(sk1, h1[skip_row0:, :C])
    floor = 5e-6 if not planes else 1e-2  # (bf16: a tie rounded the other way moves a piece by 1 ulp)
    assert rel_err(h1.cpu().numpy(), h0.cpu().numpy()) <= max(floor, 5e-6)
    assert rel_err(z1.cpu().numpy(), z0.cpu().numpy()) <= floor
    assert torch.equal(st1[:, 0], st0[:, 0])
    assert rel_err(st1[:, 1].numpy(), st0[:, 1].numpy()) <= max(floor, 1e-5)
    assert rel_err(st1[:, 2].numpy(), st0[:, 2].numpy()) <= max(floor, 1e-5)


def _cus():
    return torch.cuda.get_device_properties(0).multi_processor_count


@pytest.mark.parametrize("pw", [False, True])
def test_gcn_split_many_slices_bn_prologue_gate_epilogue(gpu, pw):
    """The support split at scale: 80 slices (10 groups of 8 workgroups per support)
    with the fused extras of the training step -- BatchNorm on load of the residual in the forward,
    the BN-backward prologue and the gate-backward epilogue in the backward -- split (ksplit = nsup)
    against whole slices (ksplit = 1): z, BN partials, dres, dh, dfg and t1 / t2 agree to the fp32
    reassociation floor, and the per-slice counters are left zero."""
    import ctypes
    from gwn_amd import _lib
    torch.manual_seed(80 + pw)
    n, C, K, S = 207, 32, 3, 80
    NP = (n + 31) // 32 * 32
    W = (2 * K + 1) * C
    rows = S * n
    sups = []
    for _ in range(K):
        s = torch.zeros(NP, NP, device=gpu)
        s[:n, :n] = torch.rand(n, n, device=gpu) / n
        sups.append(s)
    supT = [s.t().contiguous() for s in sups]
    sq = _squares(gpu, sups)
    P = ctypes.POINTER(ctypes.c_void_p)
    arr = (ctypes.c_void_p * K)(*[s.data_ptr() for s in sups])
    arrT = (ctypes.c_void_p * K)(*[s.data_ptr() for s in supT])
    arr2 = (ctypes.c_void_p * K)(*[q[0].data_ptr() for q in sq])
    arr2T = (ctypes.c_void_p * K)(*[q[1].data_ptr() for q in sq])
    g4f, g4b = _g4s(gpu, n, sups, sq, supT)
    wm = torch.randn(C, W, device=gpu) * 0.1
    wmt = wm.t().contiguous()
    bm = torch.randn(C, device=gpu)
    res = torch.randn(rows, C, device=gpu) * 2 + 1
    rmean, rscale, rshift = torch.randn(C, device=gpu), torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu)
    xg = torch.randn(rows, C, device=gpu)
    seed = torch.full((1,), 5, device=gpu, dtype=torch.int64)
    bn_dy = torch.randn(rows, C, device=gpu)
    bn_z = torch.randn(rows, C, device=gpu)
    gamma, bmean, brstd = torch.randn(C, device=gpu), torch.randn(C, device=gpu), torch.rand(C, device=gpu) + 0.5
    sums = torch.randn(2 * C, device=gpu) * 100
    fg = torch.rand(rows, 2 * C, device=gpu)
    dskip = torch.randn(rows, C, device=gpu)
    kws = torch.empty(_lib.load().gwn_gcn_ksplit_ws_floats(rows, n, K), device=gpu)
    kcnt = torch.zeros(S, device=gpu, dtype=torch.int32)
    outs = []
    for ksplit in (1, K):
        kf = dict(ksplit=ksplit, ksplit_ws=kws.data_ptr(), ksplit_count=kcnt.data_ptr())
        h = torch.zeros(rows, W, device=gpu)
        h[:, :C] = xg
        z = torch.empty(rows, C, device=gpu)
        bnp = torch.full((_lib.load().gwn_gcn_bn_partial_count(rows, n, C, K, NP) * 3 * C,), float("nan"), device=gpu)
        ga = _lib.GcnArgs(rows=rows, n=n, c=C, nsup=K, sup=ctypes.cast(arr, P), ld_sup=NP, h=h.data_ptr(), ld_h=W,
                          w_mlp=wm.data_ptr(), b_mlp=bm.data_ptr(), residual=res.data_ptr(), z=z.data_ptr(),
                          seed_ptr=seed.data_ptr(), salt=2, drop_p=0.3, bn_partials=bnp.data_ptr(),
                          residual_mean=rmean.data_ptr(), residual_scale=rscale.data_ptr(),
                          residual_shift=rshift.data_ptr(), sup2=ctypes.cast(arr2, P) if pw else None, w_mlp_t=wmt.data_ptr(),
                          sup_g4=g4f[1] if pw and ksplit == 1 else None, **kf)
        _lib.call("gwn_gcn_fwd", ctypes.byref(ga), _lib.stream())
        dhc = torch.zeros(rows, W, device=gpu)
        dres = torch.zeros(rows, C, device=gpu)
        dh_out = torch.zeros(rows, C, device=gpu)
        dfg = torch.zeros(rows, 2 * C, device=gpu)
        dg, db = torch.zeros(C, device=gpu), torch.zeros(C, device=gpu)
        gb = _lib.GcnBwdArgs(rows=rows, n=n, c=C, nsup=K, sup=ctypes.cast(arr, P), ld_sup=NP, h=h.data_ptr(),
                             ld_h=W, w_mlp=wm.data_ptr(), dh=None, dhcat=dhc.data_ptr(), ld_dhcat=W,
                             adp_index=K - 1, accumulate_dadp=0, sup_t=ctypes.cast(arrT, P), skip_weight_grads=1,
                             bn_dy=bn_dy.data_ptr(), bn_z=bn_z.data_ptr(), bn_gamma=gamma.data_ptr(),
                             bn_mean=bmean.data_ptr(), bn_rstd=brstd.data_ptr(), bn_sums=sums.data_ptr(),
                             bn_dgamma=dg.data_ptr(), bn_dbeta=db.data_ptr(), dres=dres.data_ptr(),
                             dh_out=dh_out.data_ptr(), seed_ptr=seed.data_ptr(), salt=4, drop_p=0.3,
                             fg=fg.data_ptr(), dskip=dskip.data_ptr(), ld_dskip=C, skip_row0=0, dfg=dfg.data_ptr(),
                             sup2_t=ctypes.cast(arr2T, P) if pw else None,
                             sup_g4_t=g4b[1] if pw and ksplit == 1 else None, **kf)
        _lib.call("gwn_gcn_bwd", ctypes.byref(gb), _lib.stream())
        torch.cuda.synchronize()
        assert int(kcnt.abs().sum()) == 0
        outs.append((h.clone(), z.clone(), _bn_all(bnp, rows, n, C, K, NP), dres.clone(), dh_out.clone(), dfg.clone(),
                     dhc[:, C:3 * C].clone(), dg.clone(), db.clone()))
    # against fp64 with the host-rebuilt masks: the forward's dropout (salt 2) on the mlp output
    # of the kernel's own pieces plus the BN-on-load residual; the backward's BN-backward prologue
    # and its dropout (salt 4): dres = dz, dh_out = dz * keep / (1 - p)
    from test_gpu_model import _np_uniform
    for o in outs:
        keep_f = torch.tensor(_np_uniform(5, 2, np.arange(rows * C, dtype=np.int64)).reshape(rows, C) >= 0.3,
                              dtype=torch.float64)
        zr = (o[0].double().cpu() @ wm.double().cpu().t() + bm.double().cpu()) * keep_f / 0.7 \
            + (res.double().cpu() - rmean.double().cpu()) * rscale.double().cpu() + rshift.double().cpu()
        assert rel_err(o[1].cpu().numpy(), zr.numpy()) <= 4e-6
        zb, dyb = bn_z.double().cpu(), bn_dy.double().cpu()
        k1, k2 = sums[:C].double().cpu() / rows, sums[C:].double().cpu() / rows
        rs_, gm_ = brstd.double().cpu(), gamma.double().cpu()
        dz = gm_ * rs_ * (dyb - k1 - (zb - bmean.double().cpu()) * rs_ * k2)
        keep_b = torch.tensor(_np_uniform(5, 4, np.arange(rows * C, dtype=np.int64)).reshape(rows, C) >= 0.3,
                              dtype=torch.float64)
        assert rel_err(o[3].cpu().numpy(), dz.numpy()) <= 2e-6
        assert rel_err(o[4].cpu().numpy(), (dz * keep_b / 0.7).numpy()) <= 2e-6
        assert np.array_equal((o[4] == 0).cpu().numpy(), keep_b.numpy() == 0)
    # (pw: the whole slices run the 16-node tile kernels, the split the 32-node ones -- products
    # and BN merges in other orders than the split's)
    for a_, b_ in zip(*outs):
        assert rel_err(b_.cpu().numpy(), a_.cpu().numpy()) <= (4e-6 if pw else 2e-6)
    # dfg really is the gate backward of dxg + dskip (fp64 from the whole-slice run's pieces)
    assert float(outs[0][5].abs().max()) > 0


@pytest.mark.parametrize("n", [16, 207, 325])
def test_gcn_pow_forward_modes(gpu, n):
    """The power-schedule forward (16-node tile kernel) in the inference / dropout modes the chained
    one has: the dropout
    mask is the same counter hash (identical zero pattern), eval BatchNorm folded into the epilogue
    with no hop pieces stored (gwn_gcn_args.bn_out / no_pieces) matches fp64."""
    import ctypes
    from gwn_amd import _lib
    torch.manual_seed(n + 1)
    C, K, S = 32, 3, 6
    NP = (n + 31) // 32 * 32
    W = (2 * K + 1) * C
    rows = S * n
    sups = []
    for k in range(K):
        s = torch.zeros(NP, NP, device=gpu)
        a = torch.rand(n, n, device=gpu) * (torch.rand(n, n, device=gpu) < (0.05 if k < 2 else 1.0))
        a = a + torch.eye(n, device=gpu)
        s[:n, :n] = a / a.sum(1, keepdim=True)
        sups.append(s)
    sq = _squares(gpu, sups)
    P = ctypes.POINTER(ctypes.c_void_p)
    arr = (ctypes.c_void_p * K)(*[s.data_ptr() for s in sups])
    arr2 = (ctypes.c_void_p * K)(*[q[0].data_ptr() for q in sq])
    g4f, _ = _g4s(gpu, n, sups, sq, [q[1] for q in sq])
    wm = torch.randn(C, W, device=gpu) * 0.1
    wmt = wm.t().contiguous()
    bm = torch.randn(C, device=gpu)
    res = torch.randn(rows, C, device=gpu)
    xg = torch.randn(rows, C, device=gpu)
    seed = torch.full((1,), 99, device=gpu, dtype=torch.int64)

    def run(pw, drop=0.0, eval_bn=None):
        h = torch.zeros(rows, W, device=gpu)
        h[:, :C] = xg
        z = torch.full((rows, C), 7.0, device=gpu)
        bnp = torch.empty(_lib.load().gwn_gcn_bn_partial_count(rows, n, C, K, NP) * 3 * C, device=gpu)
        kw = {}
        if eval_bn is not None:
            rm, rv, g_, b_, xo = eval_bn
            kw.update(no_pieces=1, bn_running_mean=rm.data_ptr(), bn_running_var=rv.data_ptr(),
                      bn_weight=g_.data_ptr(), bn_bias=b_.data_ptr(), bn_eps=1e-5, bn_out=xo.data_ptr())
        ga = _lib.GcnArgs(rows=rows, n=n, c=C, nsup=K, sup=ctypes.cast(arr, P),
                          ld_sup=NP, h=h.data_ptr(), ld_h=W, w_mlp=wm.data_ptr(), b_mlp=bm.data_ptr(),
                          residual=res.data_ptr(), z=None if eval_bn is not None else z.data_ptr(),
                          seed_ptr=seed.data_ptr(), salt=3, drop_p=drop,
                          bn_partials=None if eval_bn is not None else bnp.data_ptr(),
                          sup2=ctypes.cast(arr2, P) if pw else None, w_mlp_t=wmt.data_ptr(),
                          sup_g4=g4f[1] if pw else None, **kw)
        _lib.call("gwn_gcn_fwd", ctypes.byref(ga), _lib.stream())
        torch.cuda.synchronize()
        return h, z, bnp

    h, z, bnp = run(True)
    X = xg.double().cpu().view(S, n, C)
    pieces = [X]
    for s in sups:
        a = s[:n, :n].double().cpu()
        x1 = torch.einsum("svc,vw->swc", X, a)
        x2 = torch.einsum("svc,vw->swc", x1, a)
        pieces += [x1, x2]
    H = torch.cat(pieces, dim=2).reshape(rows, W)
    Z = H @ wm.double().cpu().t() + bm.double().cpu() + res.double().cpu()
    assert rel_err(h.cpu().numpy(), H.numpy()) <= 4e-6
    assert rel_err(z.cpu().numpy(), Z.numpy()) <= 4e-6
    _, zp, _ = run(True, drop=0.3)
    _, zc, _ = run(False, drop=0.3)
    # the dropped set is gwn_uniform(seed 99, salt 3, row*C + c) < p rebuilt on the host, and the
    # kept values carry the 1/(1-p) scale (fp64 of the same pieces)
    from test_gpu_model import _np_uniform
    keep = _np_uniform(99, 3, np.arange(rows * C, dtype=np.int64)).reshape(rows, C) >= np.float32(0.3)
    assert 0.28 < 1.0 - keep.mean() < 0.32
    zd = (H @ wm.double().cpu().t() + bm.double().cpu()) * torch.tensor(keep, dtype=torch.float64) / 0.7 \
        + res.double().cpu()
    for zz in (zp, zc):
        assert np.array_equal((zz == res).cpu().numpy(), ~keep)
        assert rel_err(zz.cpu().numpy(), zd.numpy()) <= 4e-6
    assert rel_err(zp.cpu().numpy(), zc.cpu().numpy()) <= 1e-5
    rm, rv = torch.randn(C, device=gpu), torch.rand(C, device=gpu) + 0.5
    g_, b_ = torch.randn(C, device=gpu), torch.randn(C, device=gpu)
    xo = torch.empty(rows, C, device=gpu)
    run(True, eval_bn=(rm, rv, g_, b_, xo))
    ref = (Z - rm.double().cpu()) / torch.sqrt(rv.double().cpu() + 1e-5) * g_.double().cpu() + b_.double().cpu()
    assert rel_err(xo.cpu().numpy(), ref.numpy()) <= 2e-5


@pytest.mark.parametrize("n,slices,pairs,ld", [(207, 50, 2, 32), (16, 3, 1, 32), (325, 7, 2, 40), (33, 1, 2, 224),
                                               (207, 768, 2, 32)])
@pytest.mark.parametrize("accumulate", [0, 1])
def test_gram_vs_fp64(gpu, n, slices, pairs, ld, accumulate):
    """gwn_gram (the adaptive-support gradient, the backward of model.py:13 w.r.t. A over all slices of
    a layer, both hop pairs) against an fp64 einsum: odd tile counts (n = 207: 7 tiles, 325: 11), a
    single tile, one slice, padded row strides, accumulation into dA.  Bound: an fp32 FMA chain over K = slices*32*pairs terms, |err| <= 2^-22 K sum|x||t|."""
    from gwn_amd import _lib
    lib = _lib.load()
    torch.manual_seed(n + slices)
    X = [torch.randn(slices * n, ld, dtype=torch.float64) for _ in range(pairs)]
    T = [torch.randn(slices * n, ld, dtype=torch.float64) for _ in range(pairs)]
    ref = torch.zeros(n, n, dtype=torch.float64)
    absb = torch.zeros(n, n, dtype=torch.float64)
    for p in range(pairs):
        xs = X[p][:, :32].reshape(slices, n, 32)
        ts = T[p][:, :32].reshape(slices, n, 32)
        ref += torch.einsum("svc,swc->vw", xs, ts)
        absb += torch.einsum("svc,swc->vw", xs.abs(), ts.abs())
    ldA = n + 3
    init = torch.randn(n, ldA, dtype=torch.float64)
    dA = init.float().to(gpu)
    if accumulate:
        ref = ref + init[:, :n].float().double()
        absb = absb + init[:, :n].abs()
    Xd = [x.float().to(gpu) for x in X]
    Td = [t.float().to(gpu) for t in T]
    ws = torch.empty(lib.gwn_gram_workspace_floats(n, slices) + 16, device=gpu)
    x2 = Xd[1].data_ptr() if pairs == 2 else None
    t2 = Td[1].data_ptr() if pairs == 2 else None
    _lib.call("gwn_gram", Xd[0].data_ptr(), Td[0].data_ptr(), x2, t2, ld, ld, n, slices, dA.data_ptr(), ldA,
              accumulate, ws.data_ptr(), _lib.stream())
    torch.cuda.synchronize()
    got = dA.double().cpu()[:, :n]
    bound = 2.0 ** -22 * (slices * 32 * pairs + 8) * absb
    assert torch.all((got - ref).abs() <= bound + 1e-30), float(((got - ref).abs() / (bound + 1e-30)).max())
    # columns beyond n untouched
    assert torch.equal(dA.cpu()[:, n:], init.float()[:, n:])


def _to_g4(a, slices, n):
    """[slices*n][32] -> gwn_gram_g4_bf16's bf16 tiled activation layout (include/gwn.h): lane (g, j)
    of a (slice, tile) KiB holds node 16 vt + j, channels 4g .. 4g+3 then 16+4g .. 16+4g+3."""
    nt = (n + 15) // 16
    x = torch.zeros(slices, nt * 16, 32, dtype=a.dtype)
    x[:, :n] = a.reshape(slices, n, 32)
    # [s][vt][j][oh][g][r] -> [s][vt][g][j][oh][r]
    x = x.reshape(slices, nt, 16, 2, 4, 4).permute(0, 1, 4, 2, 3, 5)
    return x.reshape(-1).contiguous().bfloat16()


@pytest.mark.parametrize("n,slices,pairs", [(207, 50, 2), (16, 3, 1), (325, 7, 2), (33, 1, 2), (207, 768, 2),
                                            (883, 13, 2)])
@pytest.mark.parametrize("accumulate", [0, 1])
def test_gram_g4_vs_fp64(gpu, n, slices, pairs, accumulate):
    """gwn_gram_g4_bf16 (the bf16 mode's adaptive-support gram on the 16-node tiled operands the bf16
    tile kernels write) against an fp64 einsum of the bf16-rounded operands: odd and single tiles,
    one slice, many splits, accumulation.  The products are exact in fp32, so the bound is the fp32
    accumulation chain's, as test_gram_vs_fp64."""
    from gwn_amd import _lib
    lib = _lib.load()
    torch.manual_seed(n + slices + 1)
    X = [torch.randn(slices * n, 32, dtype=torch.float64).bfloat16().double() for _ in range(pairs)]
    T = [torch.randn(slices * n, 32, dtype=torch.float64).bfloat16().double() for _ in range(pairs)]
    ref = torch.zeros(n, n, dtype=torch.float64)
    absb = torch.zeros(n, n, dtype=torch.float64)
    for p in range(pairs):
        xs, ts = X[p].reshape(slices, n, 32), T[p].reshape(slices, n, 32)
        ref += torch.einsum("svc,swc->vw", xs, ts)
        absb += torch.einsum("svc,swc->vw", xs.abs(), ts.abs())
    ldA = n + 3
    init = torch.randn(n, ldA, dtype=torch.float64)
    dA = init.float().to(gpu)
    if accumulate:
        ref = ref + init[:, :n].float().double()
        absb = absb + init[:, :n].abs()
    Xd = [_to_g4(x.float(), slices, n).to(gpu) for x in X]
    Td = [_to_g4(t.float(), slices, n).to(gpu) for t in T]
    ws = torch.empty(lib.gwn_gram_g4_workspace_floats(n, slices) + 16, device=gpu)
    x2 = Xd[1].data_ptr() if pairs == 2 else None
    t2 = Td[1].data_ptr() if pairs == 2 else None
    _lib.call("gwn_gram_g4_bf16", Xd[0].data_ptr(), Td[0].data_ptr(), x2, t2, n, slices, dA.data_ptr(), ldA,
              accumulate, ws.data_ptr(), _lib.stream())
    torch.cuda.synchronize()
    got = dA.double().cpu()[:, :n]
    bound = 2.0 ** -22 * (slices * 32 * pairs + 8) * absb
    assert torch.all((got - ref).abs() <= bound + 1e-30), float(((got - ref).abs() / (bound + 1e-30)).max())
    assert torch.equal(dA.cpu()[:, n:], init.float()[:, n:])


@pytest.mark.parametrize("n,slices", [(325, [36, 30, 9, 3]), (207, [48, 7]), (16, [5, 1, 2]), (33, [1])])
@pytest.mark.parametrize("accumulate", [0, 1])
def test_gram_g4_group_vs_fp64(gpu, n, slices, accumulate):
    """gwn_gram_g4_group (the bf16 mode's adaptive-support gram of several layers in one launch: two
    half-output workgroups per CU pair, each over an equal share of every layer's (slice, pair)
    steps) against an fp64 einsum of the bf16-rounded operands, both pairs per layer in the xg4 /
    tg4 layout (x2 / t2 right after x1 / t1); odd tile counts, a single slice.  Bound: the fp32
    accumulation chain, as test_gram_g4_vs_fp64."""
    from gwn_amd import _lib
    lib = _lib.load()
    torch.manual_seed(n + sum(slices))
    ref = torch.zeros(n, n, dtype=torch.float64)
    absb = torch.zeros(n, n, dtype=torch.float64)
    bufs, lays = [], []
    for S in slices:
        X = [torch.randn(S * n, 32, dtype=torch.float64).bfloat16().double() for _ in range(2)]
        T = [torch.randn(S * n, 32, dtype=torch.float64).bfloat16().double() for _ in range(2)]
        for p in range(2):
            xs, ts = X[p].reshape(S, n, 32), T[p].reshape(S, n, 32)
            ref += torch.einsum("svc,swc->vw", xs, ts)
            absb += torch.einsum("svc,swc->vw", xs.abs(), ts.abs())
        xb = torch.cat([_to_g4(x.float(), S, n) for x in X]).to(gpu)
        tb = torch.cat([_to_g4(t.float(), S, n) for t in T]).to(gpu)
        half = S * ((n + 15) // 16) * 1024
        bufs += [xb, tb]
        lays.append(_lib.GramLayer(x1=xb.data_ptr(), t1=tb.data_ptr(), x2=xb.data_ptr() + half,
                                   t2=tb.data_ptr() + half, slices=S))
    ldA = n + 3
    init = torch.randn(n, ldA, dtype=torch.float64)
    dA = init.float().to(gpu)
    if accumulate:
        ref = ref + init[:, :n].float().double()
        absb = absb + init[:, :n].abs()
    sl = (ctypes.c_int * len(slices))(*slices)
    ws = torch.empty(lib.gwn_gram_g4_group_workspace_floats(n, sl, len(slices)) + 16, device=gpu)
    _lib.call("gwn_gram_g4_group", (_lib.GramLayer * len(lays))(*lays), len(lays), n, dA.data_ptr(), ldA,
              accumulate, ws.data_ptr(), _lib.stream())
    torch.cuda.synchronize()
    got = dA.double().cpu()[:, :n]
    bound = 2.0 ** -22 * (sum(slices) * 32 * 2 + 8) * absb
    assert torch.all((got - ref).abs() <= bound + 1e-30), float(((got - ref).abs() / (bound + 1e-30)).max())
    assert torch.equal(dA.cpu()[:, n:], init.float()[:, n:])


def test_nconv2_vs_reference_golden(gpu):
    """nconv2 (model.py:16-22, per-sample supports) on the batched MFMA GEMM against the reference's
    own output and fp64 autograd gradients (tests/golden/make_golden_nconv2.py).  fp32 MFMA chain
    over K = N = 37 terms: max-rel 1e-5."""
    from gwn_amd.model import nconv2
    g = load_golden("g9_nconv2_n37.npz")
    x = torch.tensor(g["x"], dtype=torch.float32, device=gpu, requires_grad=True)
    A = torch.tensor(g["A"], dtype=torch.float32, device=gpu, requires_grad=True)
    y = nconv2()(x, A)
    (y * torch.tensor(g["g"], dtype=torch.float32, device=gpu)).sum().backward()
    torch.cuda.synchronize()
    assert rel_err(y.detach().cpu().numpy(), g["y"]) < 1e-5
    assert rel_err(x.grad.cpu().numpy(), g["dx"]) < 1e-5
    assert rel_err(A.grad.cpu().numpy(), g["dA"]) < 1e-5


@pytest.mark.parametrize("B,C,N,T", [(1, 1, 1, 1), (2, 3, 33, 7), (64, 32, 207, 12), (5, 2, 325, 13)])
def test_nconv2_vs_fp64(gpu, B, C, N, T):
    """nconv2 forward and both gradients against an fp64 einsum at METR-LA / PEMS-BAY shapes and
    ragged edges (16-B quad loads off when strides are not multiples of 4).  Bound: fp32 FMA chain,
    |err| <= 2^-22 K sum|a||b| per element."""
    from gwn_amd.model import nconv2
    torch.manual_seed(B * 1000 + N)
    x = torch.randn(B, C, N, T, dtype=torch.float64)
    A = torch.rand(B, N, N, dtype=torch.float64) / N
    gy = torch.randn(B, C, N, T, dtype=torch.float64)
    ref = torch.einsum("ncvl,nvw->ncwl", x, A)
    dx_ref = torch.einsum("ncwl,nvw->ncvl", gy, A)
    dA_ref = torch.einsum("ncvl,ncwl->nvw", x, gy)
    xd = x.float().to(gpu).requires_grad_(True)
    Ad = A.float().to(gpu).requires_grad_(True)
    y = nconv2()(xd, Ad)
    y.backward(gy.float().to(gpu))
    torch.cuda.synchronize()
    b_y = 2.0 ** -22 * N * torch.einsum("ncvl,nvw->ncwl", x.abs(), A.abs()) + 1e-30
    b_dx = 2.0 ** -22 * N * torch.einsum("ncwl,nvw->ncvl", gy.abs(), A.abs()) + 1e-30
    b_dA = 2.0 ** -22 * C * T * torch.einsum("ncvl,ncwl->nvw", x.abs(), gy.abs()) + 1e-30
    for got, want, bound in ((y.detach(), ref, b_y), (xd.grad, dx_ref, b_dx), (Ad.grad, dA_ref, b_dA)):
        err = (got.double().cpu() - want).abs()
        assert torch.all(err <= bound), float((err / bound).max())


@pytest.mark.parametrize("n,layout", [(16, 0), (207, 0), (207, 1), (40, 1)])
def test_gcn_fused_per_sample_supports(gpu, n, layout):
    """Fused gcn forward / backward with one support set per sample (gcn2, model.py:57-80: the
    per-sample-graph variant's 'ncvl,nvw->ncwl' diffusions): slice s = t*Bs + b diffuses with
    sample b's supports (the chained schedule).  Against fp64: hop pieces, z, dxg."""
    import ctypes
    from gwn_amd import _lib
    torch.manual_seed(n + layout)
    C, K, Bs, T = 32, 2, 3, 2
    S = T * Bs
    NP = (n + 31) // 32 * 32
    W = (2 * K + 1) * C
    rows = S * n
    sup = torch.zeros(K, Bs, NP, NP, device=gpu)
    sup[:, :, :n, :n] = torch.rand(K, Bs, n, n, device=gpu) / n
    supT = sup.transpose(2, 3).contiguous()
    arr = (ctypes.c_void_p * K)(*[sup[k].data_ptr() for k in range(K)])
    arrT = (ctypes.c_void_p * K)(*[supT[k].data_ptr() for k in range(K)])
    wm = torch.randn(C, W, device=gpu) * 0.1
    wmt = wm.t().contiguous()
    bm = torch.randn(C, device=gpu)
    res = torch.randn(rows, C, device=gpu)
    xg = torch.randn(rows, C, device=gpu)
    dh = torch.randn(rows, C, device=gpu)
    seed = torch.zeros(1, device=gpu, dtype=torch.int64)
    h = torch.zeros(rows, W, device=gpu)
    h[:, :C] = xg
    z = torch.empty(rows, C, device=gpu)
    ga = _lib.GcnArgs(rows=rows, n=n, c=C, nsup=K, sup=ctypes.cast(arr, ctypes.POINTER(ctypes.c_void_p)),
                      ld_sup=NP, h=h.data_ptr(), ld_h=W, w_mlp=wm.data_ptr(), b_mlp=bm.data_ptr(),
                      residual=res.data_ptr(), z=z.data_ptr(), seed_ptr=seed.data_ptr(), salt=0, drop_p=0.0,
                      layout=layout, sup_bstride=NP * NP, sup_batch=Bs)
    _lib.call("gwn_gcn_fwd", ctypes.byref(ga), _lib.stream())
    dhc = torch.zeros(rows, W, device=gpu)
    gb = _lib.GcnBwdArgs(rows=rows, n=n, c=C, nsup=K, sup=ctypes.cast(arr, ctypes.POINTER(ctypes.c_void_p)),
                         ld_sup=NP, h=h.data_ptr(), ld_h=W, w_mlp=wm.data_ptr(), dh=dh.data_ptr(),
                         dhcat=dhc.data_ptr(), ld_dhcat=W, adp_index=-1, accumulate_dadp=0,
                         sup_t=ctypes.cast(arrT, ctypes.POINTER(ctypes.c_void_p)), skip_weight_grads=1,
                         layout=layout, sup_bstride=NP * NP, sup_batch=Bs)
    _lib.call("gwn_gcn_bwd", ctypes.byref(gb), _lib.stream())
    torch.cuda.synchronize()
    # fp64 truth, slice s -> sample s % Bs
    X = xg.double().cpu().view(S, n, C)
    A = sup[:, :, :n, :n].double().cpu()                        # [K][Bs][n][n]
    Aslice = A[:, torch.arange(S) % Bs]                          # [K][S][n][n]
    pieces = [X]
    for k in range(K):
        x1 = torch.einsum("svc,svw->swc", X, Aslice[k])
        x2 = torch.einsum("svc,svw->swc", x1, Aslice[k])
        pieces += [x1, x2]
    H = torch.cat(pieces, dim=2).reshape(rows, W)
    Z = H @ wm.double().cpu().t() + bm.double().cpu() + res.double().cpu()
    dP = (dh.double().cpu() @ wm.double().cpu()).view(S, n, W)
    dxg = dP[:, :, :C].clone()
    for k in range(K):
        dx2 = dP[:, :, (2 + 2 * k) * C:(3 + 2 * k) * C]
        dx1 = dP[:, :, (1 + 2 * k) * C:(2 + 2 * k) * C] + torch.einsum("swc,svw->svc", dx2, Aslice[k])
        dxg = dxg + torch.einsum("swc,svw->svc", dx1, Aslice[k])
    assert rel_err(h.cpu().numpy(), H.numpy()) <= 2e-6
    assert rel_err(z.cpu().numpy(), Z.numpy()) <= 2e-6
    assert rel_err(dhc[:, :C].cpu().numpy(), dxg.reshape(rows, C).numpy()) <= 2e-6


def test_nconv2_errors_and_strided_input(gpu):
    """nconv2 raises like the reference on a support batch that does not match x (einsum shape
    error), refuses CPU tensors (no fallback), and accepts non-contiguous x (a transpose view)."""
    from gwn_amd.model import nconv2
    x = torch.randn(2, 3, 16, 5, device=gpu)
    with pytest.raises(RuntimeError):
        nconv2()(x, torch.rand(3, 16, 16, device=gpu))
    with pytest.raises(RuntimeError):
        nconv2()(x.cpu(), torch.rand(2, 16, 16))
    A = torch.rand(2, 16, 16, device=gpu)
    xt = torch.randn(2, 3, 5, 16, device=gpu).transpose(2, 3)  # [2, 3, 16, 5], non-contiguous
    y = nconv2()(xt, A)
    ref = torch.einsum("ncvl,nvw->ncwl", xt.double().cpu(), A.double().cpu())
    assert rel_err(y.cpu().numpy(), ref.numpy()) < 1e-5


@pytest.mark.parametrize("planes", [1, 2])
@pytest.mark.parametrize("n", [16, 207, 325])
def test_gcn_t16_bf16_forward(gpu, n, planes):
    """The bf16 16-node tile forward (gwn_gcn_args.sup_g4b, split_planes 1 / 2): the diffusion on
    bf16 MFMA operands with fp32 accumulation, the mlp in fp32 (1) or on bf16 MFMA operands (2,
    GWN_DTYPE_BF16_MLP), z / BN partials in fp32, against fp64 (model.py:41-55 + residual).  Bound:
    bf16 rounding of the node features and supports (2^-9 relative each) over K = n terms of
    positive weights -- hop pieces and z within 1e-2 of their max magnitude; the BN statistics of z
    within 1e-2.  planes 2 also against an fp64 evaluation of z from the bf16-rounded pieces and
    weights (the arithmetic of t16_mlp_b, fp32 accumulation the only difference): 1e-5."""
    import ctypes
    from gwn_amd import _lib
    torch.manual_seed(n + 3)
    C, K, S = 32, 3, 21
    NP = (n + 31) // 32 * 32
    W = (2 * K + 1) * C
    rows = S * n
    sups = []
    for _ in range(K):
        s_ = torch.zeros(NP, NP, device=gpu)
        a = torch.rand(n, n, device=gpu)
        s_[:n, :n] = a / a.sum(1, keepdim=True)
        sups.append(s_)
    sq = _squares(gpu, sups)
    P = ctypes.POINTER(ctypes.c_void_p)
    el = _lib.load().gwn_support_g4_bf16_elems(n)
    mats = [m for s_, q in zip(sups, sq) for m in (s_, q[0])]
    g4b = torch.zeros(len(mats), el // 2, device=gpu)
    src = (ctypes.c_void_p * len(mats))(*[m.data_ptr() for m in mats])
    _lib.call("gwn_support_g4_bf16", ctypes.cast(src, P), len(mats), n, NP, g4b.data_ptr(), el, _lib.stream())
    arrb = (ctypes.c_void_p * len(mats))(*[g4b[i].data_ptr() for i in range(len(mats))])
    arr = (ctypes.c_void_p * K)(*[s_.data_ptr() for s_ in sups])
    wm = torch.randn(C, W, device=gpu) * 0.1
    wmt = wm.t().contiguous()
    bm = torch.randn(C, device=gpu)
    res = torch.randn(rows, C, device=gpu)
    xg = torch.randn(rows, C, device=gpu)
    seed = torch.zeros(1, device=gpu, dtype=torch.int64)
    h = torch.zeros(rows, W, device=gpu)
    h[:, :C] = xg
    z = torch.empty(rows, C, device=gpu)
    bnp = torch.full((_lib.load().gwn_gcn_bn_partial_count(rows, n, C, K, NP) * 3 * C,), float("nan"), device=gpu)
    ga = _lib.GcnArgs(rows=rows, n=n, c=C, nsup=K, sup=ctypes.cast(arr, P), ld_sup=NP, h=h.data_ptr(), ld_h=W,
                      w_mlp=wm.data_ptr(), b_mlp=bm.data_ptr(), residual=res.data_ptr(), z=z.data_ptr(),
                      seed_ptr=seed.data_ptr(), salt=0, drop_p=0.0, bn_partials=bnp.data_ptr(), w_mlp_t=wmt.data_ptr(),
                      split_planes=planes, sup_g4b=ctypes.cast(arrb, P))
    _lib.call("gwn_gcn_fwd", ctypes.byref(ga), _lib.stream())
    torch.cuda.synchronize()
    if planes == 2:
        bf = lambda t: t.to(torch.bfloat16).double()  # noqa: E731
        hb = torch.cat([bf(xg.double().cpu()), bf(h[:, C:].double().cpu())], dim=1)  # the stored pieces
        zm = hb @ bf(wm.double().cpu()).t() + bm.double().cpu() + res.double().cpu()
        assert rel_err(z.cpu().numpy(), zm.numpy()) <= 1e-5
    X = xg.double().cpu().view(S, n, C)
    pieces = [X]
    for s_ in sups:
        a = s_[:n, :n].double().cpu()
        x1 = torch.einsum("svc,vw->swc", X, a)
        x2 = torch.einsum("svc,vw->swc", x1, a)
        pieces += [x1, x2]
    H = torch.cat(pieces, dim=2).reshape(rows, W)
    Z = H @ wm.double().cpu().t() + bm.double().cpu() + res.double().cpu()
    for p_ in range(1, W // C):
        assert rel_err(h[:, p_ * C:(p_ + 1) * C].cpu().numpy(), H[:, p_ * C:(p_ + 1) * C].numpy()) <= 1e-2, p_
    assert torch.equal(h[:, :C], xg)
    assert rel_err(z.cpu().numpy(), Z.numpy()) <= 1e-2
    st = _bn_all(bnp, rows, n, C, K, NP)
    assert torch.all(st[:, 0] == rows)
    assert rel_err(st[:, 1].numpy(), Z.mean(0, keepdim=True).numpy()) <= 1e-2


@pytest.mark.parametrize("n", [16, 207, 325])
@pytest.mark.parametrize("path", ["t16", "t16b", "t32"])
def test_gcn_fwd_bn_fold(gpu, n, path, monkeypatch):
    """gwn_gcn_args.bn_fold: the BatchNorm finalize + fold into the next gated TCN issued by
    gwn_gcn_fwd (a second launch; t32 = GWN_GCN_T16=0, the 32-node kernels).  Against fp64
    statistics of the z the launch wrote (model.py:236, train mode): mean / rstd / running stats
    within 1e-5, scale = gamma * rstd, w_fold = w_next * scale (same fp32 product), b_fold within
    1e-5, num_batches_tracked advanced once per launch (two launches back to back)."""
    from gwn_amd import _lib
    monkeypatch.setenv("GWN_GCN_T16", "0" if path == "t32" else "1")
    torch.manual_seed(n + 11)
    C, K, S = 32, 3, 23
    NP = (n + 31) // 32 * 32
    W = (2 * K + 1) * C
    rows = S * n
    sups = []
    for _ in range(K):
        s_ = torch.zeros(NP, NP, device=gpu)
        a = torch.rand(n, n, device=gpu)
        s_[:n, :n] = a / a.sum(1, keepdim=True)
        sups.append(s_)
    supT = [s_.t().contiguous() for s_ in sups]
    sq = _squares(gpu, sups)
    P = ctypes.POINTER(ctypes.c_void_p)
    arr = (ctypes.c_void_p * K)(*[s_.data_ptr() for s_ in sups])
    arr2 = (ctypes.c_void_p * K)(*[q[0].data_ptr() for q in sq])
    g4f, _ = _g4s(gpu, n, sups, sq, supT)
    extra = {}
    if path == "t16b":
        el = _lib.load().gwn_support_g4_bf16_elems(n)
        mats = [m for s_, q in zip(sups, sq) for m in (s_, q[0])]
        g4bf = torch.zeros(len(mats), el // 2, device=gpu)
        src = (ctypes.c_void_p * len(mats))(*[m.data_ptr() for m in mats])
        _lib.call("gwn_support_g4_bf16", ctypes.cast(src, P), len(mats), n, NP, g4bf.data_ptr(), el, _lib.stream())
        arrb = (ctypes.c_void_p * len(mats))(*[g4bf[i].data_ptr() for i in range(len(mats))])
        extra = dict(split_planes=1, sup_g4b=ctypes.cast(arrb, P))
    elif path == "t16":
        extra = dict(sup_g4=g4f[1])
    wm = torch.randn(C, W, device=gpu) * 0.1
    wmt = wm.t().contiguous()
    bm = torch.randn(C, device=gpu)
    res = torch.randn(rows, C, device=gpu) + 5.0 * torch.randn(C, device=gpu)  # channel offsets
    h = torch.zeros(rows, W, device=gpu)
    h[:, :C] = torch.randn(rows, C, device=gpu)
    z = torch.empty(rows, C, device=gpu)
    seed = torch.zeros(1, device=gpu, dtype=torch.int64)
    bnp = torch.full((_lib.load().gwn_gcn_bn_partial_count(rows, n, C, K, NP) * 3 * C,), float("nan"), device=gpu)
    gamma, beta = torch.randn(C, device=gpu), torch.randn(C, device=gpu)
    rm, rv = torch.randn(C, device=gpu), torch.rand(C, device=gpu) + 0.5
    rm0, rv0 = rm.clone(), rv.clone()
    mean, rstd, scale = (torch.full((C,), float("nan"), device=gpu) for _ in range(3))
    wfg = torch.randn(2 * C, 2 * C, device=gpu) * 0.2
    bfg = torch.randn(2 * C, device=gpu)
    wfold, bfold = torch.full_like(wfg, float("nan")), torch.full_like(bfg, float("nan"))
    nbt = torch.full((1,), 7, device=gpu, dtype=torch.int64)
    bf = _lib.BnFold(gamma=gamma.data_ptr(), beta=beta.data_ptr(), running_mean=rm.data_ptr(),
                     running_var=rv.data_ptr(), momentum=0.1, eps=1e-5, save_mean=mean.data_ptr(),
                     save_rstd=rstd.data_ptr(), scale=scale.data_ptr(), w_next=wfg.data_ptr(), b_next=bfg.data_ptr(),
                     w_fold=wfold.data_ptr(), b_fold=bfold.data_ptr(), num_batches_tracked=nbt.data_ptr())
    ga = _lib.GcnArgs(rows=rows, n=n, c=C, nsup=K, sup=ctypes.cast(arr, P), ld_sup=NP, h=h.data_ptr(), ld_h=W,
                      w_mlp=wm.data_ptr(), b_mlp=bm.data_ptr(), residual=res.data_ptr(), z=z.data_ptr(),
                      seed_ptr=seed.data_ptr(), salt=0, drop_p=0.0, bn_partials=bnp.data_ptr(), w_mlp_t=wmt.data_ptr(),
                      sup2=ctypes.cast(arr2, P), bn_fold=ctypes.pointer(bf), **extra)
    for launch in range(2):
        rm.copy_(rm0)
        rv.copy_(rv0)
        _lib.call("gwn_gcn_fwd", ctypes.byref(ga), _lib.stream())
        torch.cuda.synchronize()
        assert int(nbt.item()) == 8 + launch
        zd = z.double().cpu()
        mu, var = zd.mean(0), zd.var(0, unbiased=False)
        assert rel_err(mean.cpu().numpy(), mu.numpy()) < 1e-5
        assert rel_err(rstd.cpu().numpy(), (1 / torch.sqrt(var + 1e-5)).numpy()) < 1e-5
        assert rel_err(rm.cpu().numpy(), (0.9 * rm0.double().cpu() + 0.1 * mu).numpy()) < 1e-5
        assert rel_err(rv.cpu().numpy(), (0.9 * rv0.double().cpu() + 0.1 * zd.var(0, unbiased=True)).numpy()) < 1e-5
        assert torch.equal(scale, rstd * gamma)
        assert torch.equal(wfold, wfg * scale.repeat(2)[None, :])
        ref_b = bfg.double().cpu() + wfg.double().cpu() @ beta.double().cpu().repeat(2)
        assert rel_err(bfold.cpu().numpy(), ref_b.numpy()) < 1e-5


def _from_g4(buf, which, slices, n):
    """Inverse of _to_g4 for operand `which` of a tiled bf16 buffer: [slices*nt*16][32] fp64
    (rows >= n are the tiles' padding nodes)."""
    nt = (n + 15) // 16
    x = buf.view(torch.bfloat16)[which * slices * nt * 512:(which + 1) * slices * nt * 512].double().cpu()
    # [s][vt][g][j][oh][r] -> [s][vt][j][oh][g][r]
    x = x.reshape(slices, nt, 4, 16, 2, 4).permute(0, 1, 3, 4, 2, 5)
    return x.reshape(slices, nt * 16, 32)


@pytest.mark.parametrize("n, mode", [(n, m) for n in (16, 207, 325)
                                     for m in ("bn_gate", "bn_gate_tg4", "plain", "bn_gate_tg4_mlp", "plain_mlp")]
                         + [(207, "bn_gate_tg4_mlp_pairs"), (207, "plain_mlp_pairs")])
def test_gcn_t16_bf16_backward(gpu, n, mode):
    """The bf16 16-node tile backward (gcn_bwd_t16_kernel<1024, true>: gwn_gcn_bwd_args.sup_g4b_t,
    split_planes 1) against fp64, kernel level (model.py:41-55 backward): the BN-backward prologue
    (dres, dh_out with the dropout mask rebuilt on the host), the diffusion of bf16(dh) through
    bf16(A_k^T), bf16((A_k^2)^T), the channel maps W^T in fp32, t1 / t2 of the adaptive support
    (dhcat columns, or bf16 in gwn_gram_g4_bf16's tiled layout with tg4), and the gate-backward
    epilogue (dfg from dxg + dskip and the saved (tanh f, sigmoid s)) or the plain dxg store.
    Bounds: against an fp64 evaluation of the same bf16-rounded operands (the arithmetic the kernel
    implements, fp32 accumulation the only difference) 2e-5 of each output's max magnitude (tg4: one
    bf16 rounding, 2^-8); against the exact fp64 gradient 1e-2 (the forward test's bound).
    *_mlp: split_planes 2 (GWN_DTYPE_BF16_MLP), the channel maps on bf16 MFMA: every W_q^T y of the
    emulation takes bf16(W_q), bf16(y), with y = dh the kernel's own fp32 dh (dh_out, itself checked
    against fp64 at 2e-6: the bf16 image holds exactly bf16 of it).  An fp32 intermediate e1 / e2 (a
    diffusion of dh) within its accumulation error (2^-19 of the sum of |terms|) of a bf16 rounding
    boundary may round the other way in the kernel: each such tie is allowed its one bf16 ulp times
    |bf16(W_q)| in the outputs it feeds (_tie_allow), on top of the same 2e-5 -- per element, so a
    wrong operand or product still fails (a fixed 3e-4 of the max had to grow with every new draw).
    *_pairs (n = 207): 2 * ceil(10 * CUs / 13) + 1 slices (395), so the launch takes
    gcn_bwd_t16b2_kernel (two slices per wave from ~10 pair units per CU), with an odd last slice."""
    import ctypes
    from gwn_amd import _lib
    from test_gpu_model import _np_uniform
    pairs = mode.endswith("_pairs")  # (the pair kernel's cases run at the bench's n = 207 only)
    mode = mode.replace("_pairs", "")
    planes = 2 if mode.endswith("_mlp") else 1
    mode = mode.replace("_mlp", "")
    torch.manual_seed(n + 11)
    nt_ = (n + 15) // 16  # pairs: the fewest slices that give ~10 pair units per CU, odd
    C, K, S = 32, 3, (2 * -(-10 * torch.cuda.get_device_properties(0).multi_processor_count // nt_) + 1 if pairs else 21)
    NP = (n + 31) // 32 * 32
    W = (2 * K + 1) * C
    rows = S * n
    nt = (n + 15) // 16
    sups = []
    for _ in range(K):
        s_ = torch.zeros(NP, NP, device=gpu)
        a = torch.rand(n, n, device=gpu)
        s_[:n, :n] = a / a.sum(1, keepdim=True)
        sups.append(s_)
    supT = [s_.t().contiguous() for s_ in sups]
    sq = _squares(gpu, sups)
    P = ctypes.POINTER(ctypes.c_void_p)
    el = _lib.load().gwn_support_g4_bf16_elems(n)
    mats = [m for t_, q in zip(supT, sq) for m in (t_, q[1])]  # A_k^T, (A_k^2)^T
    g4bt = torch.zeros(len(mats), el // 2, device=gpu)
    src = (ctypes.c_void_p * len(mats))(*[m.data_ptr() for m in mats])
    _lib.call("gwn_support_g4_bf16", ctypes.cast(src, P), len(mats), n, NP, g4bt.data_ptr(), el, _lib.stream())
    arrb = (ctypes.c_void_p * len(mats))(*[g4bt[i].data_ptr() for i in range(len(mats))])
    arr = (ctypes.c_void_p * K)(*[s_.data_ptr() for s_ in sups])
    arrT = (ctypes.c_void_p * K)(*[s_.data_ptr() for s_ in supT])
    wm = torch.randn(C, W, device=gpu) * 0.1
    h = torch.zeros(rows, W, device=gpu)
    dhc = torch.zeros(rows, W, device=gpu)
    bn = mode != "plain"
    kw = {}
    drop, salt, seedv = 0.3, 4, 77
    seed = torch.full((1,), seedv, device=gpu, dtype=torch.int64)
    if bn:
        bn_dy, bn_z = torch.randn(rows, C, device=gpu), torch.randn(rows, C, device=gpu) * 2 + 0.5
        gamma, bmean, brstd = torch.randn(C, device=gpu), torch.randn(C, device=gpu), torch.rand(C, device=gpu) + 0.5
        sums = torch.randn(2 * C, device=gpu) * 50
        fg = torch.rand(rows, 2 * C, device=gpu)
        fg[:, 0::2] = fg[:, 0::2] * 2 - 1  # tanh f in (-1, 1), sigmoid s in (0, 1)
        dskip = torch.randn(rows, C, device=gpu)
        skip_row0 = (S - 3) * n
        dres, dh_out = torch.zeros(rows, C, device=gpu), torch.zeros(rows, C, device=gpu)
        dfg = torch.zeros(rows, 2 * C, device=gpu)
        dg, db = torch.zeros(C, device=gpu), torch.zeros(C, device=gpu)
        kw = dict(dh=None, bn_dy=bn_dy.data_ptr(), bn_z=bn_z.data_ptr(), bn_gamma=gamma.data_ptr(),
                  bn_mean=bmean.data_ptr(), bn_rstd=brstd.data_ptr(), bn_sums=sums.data_ptr(),
                  bn_dgamma=dg.data_ptr(), bn_dbeta=db.data_ptr(), dres=dres.data_ptr(), dh_out=dh_out.data_ptr(),
                  seed_ptr=seed.data_ptr(), salt=salt, drop_p=drop, fg=fg.data_ptr(), dskip=dskip.data_ptr(),
                  ld_dskip=C, skip_row0=skip_row0, dfg=dfg.data_ptr())
    else:
        dh = torch.randn(rows, C, device=gpu)
        kw = dict(dh=dh.data_ptr())
    tg4 = None
    if mode == "bn_gate_tg4":
        tg4 = torch.full((2 * S * nt * 512,), -1, device=gpu, dtype=torch.int16)
        kw["tg4"] = tg4.data_ptr()
    gb = _lib.GcnBwdArgs(rows=rows, n=n, c=C, nsup=K, sup=ctypes.cast(arr, P), ld_sup=NP, h=h.data_ptr(), ld_h=W,
                         w_mlp=wm.data_ptr(), dhcat=dhc.data_ptr(), ld_dhcat=W, adp_index=K - 1, accumulate_dadp=0,
                         sup_t=ctypes.cast(arrT, P), skip_weight_grads=1, split_planes=planes, sup_g4b_t=ctypes.cast(arrb, P),
                         **kw)
    _lib.call("gwn_gcn_bwd", ctypes.byref(gb), _lib.stream())
    torch.cuda.synchronize()
    if pairs:  # bitwise the same on a second launch (build.sh: the packed-fp32 hazard it avoids)
        keep_out = [t.clone() for t in (dhc, dfg if bn else dhc, tg4 if tg4 is not None else dhc)]
        for _ in range(2):
            _lib.call("gwn_gcn_bwd", ctypes.byref(gb), _lib.stream())
            torch.cuda.synchronize()
            for a_, b_ in zip(keep_out, (dhc, dfg if bn else dhc, tg4 if tg4 is not None else dhc)):
                assert torch.equal(a_, b_)
    # fp64: the BN-backward prologue and dropout (gwn_uniform rebuilt on the host)
    if bn:
        z, dy = bn_z.double().cpu(), bn_dy.double().cpu()
        mu, rs, gm = bmean.double().cpu(), brstd.double().cpu(), gamma.double().cpu()
        k1, k2 = sums[:C].double().cpu() / rows, sums[C:].double().cpu() / rows
        dz = gm * rs * (dy - k1 - (z - mu) * rs * k2)
        keep = _np_uniform(seedv, salt, np.arange(rows * C, dtype=np.int64)).reshape(rows, C) >= drop
        dhr = dz * torch.tensor(keep, dtype=torch.float64) / (1 - drop)
        assert rel_err(dres.cpu().numpy(), dz.numpy()) <= 2e-6
        assert rel_err(dh_out.cpu().numpy(), dhr.numpy()) <= 2e-6
        assert torch.equal(db.cpu(), sums[:C].cpu()) and torch.equal(dg.cpu(), sums[C:].cpu())
    else:
        dhr = dh.double().cpu()
    bf = lambda t: t.to(torch.bfloat16).double()  # noqa: E731
    Wd = wm.double().cpu()
    # the kernel's own dh (fp32, checked above) is what its bf16 image and mlp operands round
    dh_k = dh_out.double().cpu() if bn else dhr

    def grads(rnd):
        mr = rnd if planes == 2 else (lambda t: t)
        Wm = mr(Wd)
        wq = lambda y, q: mr(y) @ Wm[:, q * C:(q + 1) * C]  # noqa: E731  (W_q^T applied to rows)
        dsrc = dhr if rnd is not bf else dh_k
        Db = rnd(dsrc.view(S, n, C))
        dxg = wq(dsrc, 0)
        t1 = t2 = None
        allow = torch.zeros(rows, C, dtype=torch.float64)  # _tie_allow of dxg (mlp mode)
        a_t1 = torch.zeros(rows, C, dtype=torch.float64)
        for k in range(K):
            a = rnd(sups[k][:n, :n].double().cpu())
            a2 = rnd(sq[k][0][:n, :n].double().cpu())
            e1 = torch.einsum("vw,swc->svc", a, Db).reshape(rows, C)
            e2 = torch.einsum("vw,swc->svc", a2, Db).reshape(rows, C)
            dxg = dxg + wq(e1, 1 + 2 * k) + wq(e2, 2 + 2 * k)
            if planes == 2 and rnd is bf:
                band1 = 2.0 ** -19 * torch.einsum("vw,swc->svc", a.abs(), Db.abs()).reshape(rows, C)
                band2 = 2.0 ** -19 * torch.einsum("vw,swc->svc", a2.abs(), Db.abs()).reshape(rows, C)
                u1, u2 = _tie_allow(e1, band1), _tie_allow(e2, band2)
                allow = allow + u1 @ Wm[:, (1 + 2 * k) * C:(2 + 2 * k) * C].abs() \
                    + u2 @ Wm[:, (2 + 2 * k) * C:(3 + 2 * k) * C].abs()
                if k == K - 1:
                    a_t1 = u1 @ Wm[:, (2 + 2 * k) * C:(3 + 2 * k) * C].abs()
            if k == K - 1:
                t1 = wq(dsrc, 1 + 2 * k) + wq(e1, 2 + 2 * k)
                t2 = wq(dsrc, 2 + 2 * k)
        return dxg, t1, t2, allow, a_t1

    exact, emul = grads(lambda t: t), grads(bf)
    if bn:
        f, s = fg[:, 0::2].double().cpu(), fg[:, 1::2].double().cpu()
        sk = torch.zeros(rows, C, dtype=torch.float64)
        sk[skip_row0:] = dskip.double().cpu()[:rows - skip_row0]  # dskip row m - skip_row0 (include/gwn.h)

        def gate(dxg):
            gv = dxg + sk
            out = torch.empty(rows, 2 * C, dtype=torch.float64)
            out[:, 0::2] = gv * s * (1 - f * f)
            out[:, 1::2] = gv * f * s * (1 - s)
            return out
        got_main, want_main, want_exact = dfg.cpu().numpy(), gate(emul[0]).numpy(), gate(exact[0]).numpy()
        al = torch.empty(rows, 2 * C, dtype=torch.float64)  # the tie allowance through the gate
        al[:, 0::2] = emul[3] * (s * (1 - f * f)).abs()
        al[:, 1::2] = emul[3] * (f * s * (1 - s)).abs()
        allow_main = al.numpy()
    else:
        got_main, want_main, want_exact = dhc[:, :C].cpu().numpy(), emul[0].numpy(), exact[0].numpy()
        allow_main = emul[3].numpy()
    tol = 2e-5
    _assert_tie_close(got_main, want_main, allow_main, tol)
    assert rel_err(got_main, want_exact) <= 1e-2
    if tg4 is not None:
        for which, (em, ex) in enumerate(((emul[1], exact[1]), (emul[2], exact[2]))):
            got = _from_g4(tg4, which, S, n)
            assert torch.all(got[:, n:] == 0)  # the tiles' padding nodes
            got = got[:, :n].reshape(rows, C).numpy()
            _assert_tie_close(got, em.numpy(), (emul[4] if which == 0 else 0 * emul[4]).numpy(), 2 ** -8 + tol)
            assert rel_err(got, ex.numpy()) <= 1e-2
        assert torch.all(dhc[:, C:3 * C] == 0)  # t1 / t2 went to tg4 only
    else:
        for j, (em, ex) in enumerate(((emul[1], exact[1]), (emul[2], exact[2]))):
            got = dhc[:, (1 + j) * C:(2 + j) * C].cpu().numpy()
            _assert_tie_close(got, em.numpy(), (emul[4] if j == 0 else 0 * emul[4]).numpy(), tol)
            assert rel_err(got, ex.numpy()) <= 1e-2


def _tie_allow(y, band):
    """Per element of an fp64 value y that an fp32 computation carries within +-band: one bf16 ulp
    where y lies within band of a bf16 rounding boundary (the fp32 value may round to the other
    neighbour), else 0."""
    yb = y.to(torch.bfloat16).double()
    _, e = torch.frexp(yb)
    ulp = torch.ldexp(torch.ones_like(yb), e - 8)  # a bf16 ulp at |yb| (the larger side of a binade)
    mid = yb + torch.sign(y - yb) * ulp / 2
    return torch.where((y - mid).abs() <= band, ulp, torch.zeros_like(yb))


def _assert_tie_close(got, want, allow, tol):
    """|got - want| <= tol * max|want| + allow, per element (allow: the rounding-tie allowance)."""
    err = np.abs(got.astype(np.float64) - want)
    bound = tol * np.max(np.abs(want)) + allow
    worst = float(np.max(err / bound))
    assert worst <= 1.0, (worst, float(np.max(err) / np.max(np.abs(want))), int((allow > 0).sum()))


@pytest.mark.parametrize("shape", ["mlp", "mlp_xb", "tcn", "e2"])
def test_wgrad_group_vs_fp64(gpu, shape):
    """gwn_wgrad_group (the deferred weight gradients of several layers in one launch, then
    gwn_reduce_partials) against fp64, per problem: the gcn mlp of 7 layers (J = 32, Kc = 224,
    the METR-LA row counts scaled down, ragged), the gated TCN of 8 layers (J = 64, two taps
    d*P apart, BatchNorm affine on load, identity affine for the first), end_conv_2 on its 32-row
    padded gradient (J = 32, Kc = 512, one problem).  mlp_xb: the bf16 mode's mlp form
    -- columns 0..31 fp32 from X, the hop pieces (columns 32..223) from a bf16 matrix Xb with
    ldxb = 200 (> 192: the row pitch is exercised) -- against fp64 on the same bf16 values.  Bound
    per element: an fp32 FMA chain over the rows, |err| <= 2^-22 R sum|dY||X|.  A second launch is
    bitwise identical (fixed-order sums)."""
    import ctypes
    from gwn_amd import _lib
    lib = _lib.load()
    torch.manual_seed({"mlp": 1, "mlp_xb": 4, "tcn": 2, "e2": 3}[shape])
    P = 207 * 3
    xb = shape == "mlp_xb"
    ldxb = 200
    if shape in ("mlp", "mlp_xb"):
        J, Kt, ntaps, Ts = 32, 224, 1, [12, 10, 9, 7, 6, 4, 3]
    elif shape == "tcn":
        J, Kt, ntaps, Ts = 64, 32, 2, [12, 10, 9, 7, 6, 4, 3, 1]
    else:
        J, Kt, ntaps, Ts = 32, 512, 1, [1]
    dil = [1, 2, 1, 2, 1, 2, 1, 2]
    probs, host = [], []
    for p, t in enumerate(Ts):
        R = t * P + (p % 3)  # ragged
        shift = dil[p] * P if ntaps == 2 else 0
        x_rows = R + (ntaps - 1) * shift
        dY = torch.randn(R, J, dtype=torch.float64)
        if shape == "e2":
            dY[:, 12:] = 0.0  # the padded output gradient
        X = torch.randn(x_rows, Kt, dtype=torch.float64) * 2 + 1
        if xb:  # the pieces as the kernel sees them: bf16 values
            X[:, 32:] = X[:, 32:].to(torch.bfloat16).double()
        aff = None
        if shape == "tcn":
            aff = (torch.zeros(Kt), torch.ones(Kt), torch.zeros(Kt)) if p == 0 else \
                (torch.randn(Kt) + 1, torch.rand(Kt) + 0.5, torch.randn(Kt))
        host.append((dY, X, aff, R, shift))
    nb = (ctypes.c_int * len(Ts))()
    total = lib.gwn_wgrad_group_plan((ctypes.c_int * len(Ts))(*[h[3] for h in host]), len(Ts), J, Kt, ntaps, nb)
    assert total > 0 and sum(nb) == total
    keep = []
    for p, (dY, X, aff, R, shift) in enumerate(host):
        dYd, Xd = dY.float().to(gpu), X.float().to(gpu)
        affd = [a.float().to(gpu) for a in aff] if aff is not None else [None] * 3
        part = torch.full((nb[p] * (J * Kt * ntaps + J),), float("nan"), device=gpu)
        Xbd = None
        if xb:  # Xb[r][k - 32] = X[r][k] (bf16), the fp32 X keeps garbage past column 32
            Xbd = torch.zeros(X.shape[0], ldxb, dtype=torch.bfloat16)
            Xbd[:, :Kt - 32] = X[:, 32:].to(torch.bfloat16)
            Xbd = Xbd.to(gpu)
            Xd[:, 32:] = float("nan")
        keep.append((dYd, Xd, affd, part, Xbd))
        probs.append(_lib.WgradProblem(dY=dYd.data_ptr(), ldy=J, X=Xd.data_ptr(), ldx=Kt, x_rows=X.shape[0], shift=shift,
                                       x_mean=affd[0].data_ptr() if aff is not None else None,
                                       x_scale=affd[1].data_ptr() if aff is not None else None,
                                       x_shift=affd[2].data_ptr() if aff is not None else None,
                                       part=part.data_ptr(), R=R,
                                       Xb=Xbd.data_ptr() if xb else None, ldxb=ldxb if xb else 0))
    arr = (_lib.WgradProblem * len(probs))(*probs)
    Kc = Kt * ntaps
    outs = []
    for rep in range(2):
        _lib.call("gwn_wgrad_group", arr, len(probs), J, Kt, ntaps, _lib.stream())
        res = []
        segs = []
        for p in range(len(probs)):
            dw, db = torch.empty(J, Kc, device=gpu), torch.empty(J, device=gpu)
            res.append((dw, db))
            segs.append(_lib.ReduceSeg(part=keep[p][3].data_ptr(), nparts=nb[p], part_stride=J * Kc + J, J=J, Kc=Kc,
                                       out=dw.data_ptr(), ld_out=Kc, out2=db.data_ptr()))
        _lib.call("gwn_reduce_partials", (_lib.ReduceSeg * len(segs))(*segs), len(segs), _lib.stream())
        torch.cuda.synchronize()
        outs.append(res)
    for p, (dY, X, aff, R, shift) in enumerate(host):
        Xf = X.float().double()
        if aff is not None:
            Xf = ((X.float() - aff[0].float()) * aff[1].float() + aff[2].float()).double()
        Xk = torch.cat([Xf[tap * shift:tap * shift + R] for tap in range(ntaps)], dim=1)
        dYf = dY.float().double()
        ref_w, ref_b = dYf.t() @ Xk, dYf.sum(0)
        bw = 2.0 ** -22 * R * (dYf.abs().t() @ Xk.abs()) + 1e-30
        bb = 2.0 ** -22 * R * dYf.abs().sum(0) + 1e-30
        dw, db = outs[0][p]
        assert torch.all((dw.double().cpu() - ref_w).abs() <= bw), (p, float(((dw.double().cpu() - ref_w).abs() / bw).max()))
        assert torch.all((db.double().cpu() - ref_b).abs() <= bb), p
        assert torch.equal(outs[1][p][0], dw) and torch.equal(outs[1][p][1], db)


@pytest.mark.parametrize("n", [207, 16, 325])
@pytest.mark.parametrize("cu", ["1", "0"])
def test_gram_group_vs_fp64(gpu, n, cu, monkeypatch):
    """gwn_gram_group (the adaptive-support gradient of several layers in one launch) against fp64:
    layers of 36 / 30 / 9 / 3 slices with the training step's operand layout (x in h [rows][224]
    columns 0 and 160, t1 / t2 in [rows][96] columns 32 and 64), accumulating into dA, on both
    kernels: the CU-resident one (n <= 256: one workgroup per CU over an equal range of (layer,
    slice, pair) steps, the whole output in its accumulators) and, GWN_GRAM_CU=0 or n > 256,
    gram_kernel (splits dealt to the layers by slice count).  Bound: the fp32 FMA chain."""
    import ctypes
    from gwn_amd import _lib
    monkeypatch.setenv("GWN_GRAM_CU", cu)
    lib = _lib.load()
    torch.manual_seed(n + 5)
    slices = [36, 30, 9, 3] if n != 325 else [12, 5]
    ldx, ldt = 224, 96
    ref = torch.zeros(n, n, dtype=torch.float64)
    absb = torch.zeros(n, n, dtype=torch.float64)
    keep, lay = [], []
    for S in slices:
        H = torch.randn(S * n, ldx, dtype=torch.float64)
        Tt = torch.randn(S * n, ldt, dtype=torch.float64)
        X1, X2 = H[:, :32].reshape(S, n, 32), H[:, 160:192].reshape(S, n, 32)
        T1, T2 = Tt[:, 32:64].reshape(S, n, 32), Tt[:, 64:96].reshape(S, n, 32)
        for x, t in ((X1, T1), (X2, T2)):
            xf, tf_ = x.float().double(), t.float().double()
            ref += torch.einsum("svc,swc->vw", xf, tf_)
            absb += torch.einsum("svc,swc->vw", xf.abs(), tf_.abs())
        Hd, Td = H.float().to(gpu), Tt.float().to(gpu)
        keep += [Hd, Td]
        lay.append(_lib.GramLayer(x1=Hd.data_ptr(), t1=Td.data_ptr() + 4 * 32, x2=Hd.data_ptr() + 4 * 160,
                                  t2=Td.data_ptr() + 4 * 64, slices=S))
    ldA = n + 3
    init = torch.randn(n, ldA, dtype=torch.float64)
    dA = init.float().to(gpu)
    ref = ref + init[:, :n].float().double()
    absb = absb + init[:, :n].abs()
    sl = (ctypes.c_int * len(slices))(*slices)
    ws = torch.empty(lib.gwn_gram_group_workspace_floats(n, sl, len(slices)) + 16, device=gpu)
    _lib.call("gwn_gram_group", (_lib.GramLayer * len(lay))(*lay), len(lay), ldx, ldt, n, dA.data_ptr(), ldA, 1,
              ws.data_ptr(), _lib.stream())
    torch.cuda.synchronize()
    got = dA.double().cpu()[:, :n]
    bound = 2.0 ** -22 * (sum(slices) * 64 + 8) * absb
    assert torch.all((got - ref).abs() <= bound + 1e-30), float(((got - ref).abs() / (bound + 1e-30)).max())
    assert torch.equal(dA.cpu()[:, n:], init.float()[:, n:])
