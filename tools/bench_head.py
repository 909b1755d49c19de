"""Head-GEMM shapes (skip / end_conv_1 / end_conv_2 and their backward at T_f = 1, B = 64, N = 207):
libgwn's gwn_gemm vs the vendor BLAS libraries behind torch.mm (rocBLAS and hipBLASLt), HIP-event timed.  Usage: python tools/bench_head.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-wavenet_amd"))

import torch  # noqa: E402

from gwn_amd import _lib  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return 1000.0 * e0.elapsed_time(e1) / reps


def gwn_mm(A, B, C, ksplit=1, ws=None):
    """C[M,N] = A[M,K] @ B[K,N] (row-major) through gwn_gemm."""
    M, K = A.shape
    N = B.shape[1]
    d = _lib.GemmDesc()
    d.A, d.lda_m, d.lda_k = A.data_ptr(), A.stride(0), A.stride(1)
    d.B, d.ldb_k, d.ldb_n = B.data_ptr(), B.stride(0), B.stride(1)
    d.C, d.ldc_m, d.ldc_n = C.data_ptr(), C.stride(0), C.stride(1)
    d.M, d.N, d.K = M, N, K
    d.alpha, d.beta, d.ksplit = 1.0, 1.0, ksplit
    d.part = ws.data_ptr() if ws is not None else None
    _lib.call("gwn_gemm", ctypes.byref(d), _lib.stream())


def main():
    dev = torch.device("cuda:0")
    R = 64 * 207
    shapes = [("skip fwd", R, 256, 256), ("end1 fwd", R, 512, 256), ("end2 fwd", R, 12, 512),
              ("end2 dX", R, 512, 12), ("end1 dX", R, 256, 512), ("skip dX", R, 256, 256),
              ("end1 dW", 512, 256, R), ("skip dW", 256, 256, R), ("end2 dW", 12, 512, R),
              ("mlp dW", 32, 224, 768 * 207), ("tcn dW", 64, 64, 768 * 207)]
    torch.manual_seed(0)
    for name, M, N, K in shapes:
        flop = 2.0 * M * N * K
        if K > 4 * max(M, N):  # weight-gradient form: A^T stored [K][M]
            At = torch.randn(K, M, device=dev)
            A = At.t()
        else:
            A = torch.randn(M, K, device=dev)
        B = torch.randn(K, N, device=dev)
        C = torch.empty(M, N, device=dev)
        torch.backends.cuda.preferred_blas_library("cublaslt")
        t_lt = timeit(lambda: torch.mm(A, B, out=C))
        torch.backends.cuda.preferred_blas_library("cublas")
        t_torch = timeit(lambda: torch.mm(A, B, out=C))
        ks = 1
        if K > 4 * max(M, N):
            tiles = ((M + 127) // 128) * ((N + 63) // 64)
            ks = max(1, min(1024 // tiles, K // 256))
        ws = torch.empty(max(1, _lib.load().gwn_gemm_workspace_floats(M, N, ks)), device=dev)
        t_gwn = timeit(lambda: gwn_mm(A, B, C, ks, ws))
        if K > 4 * max(M, N) and M >= 256:  # split-K sweep of the head weight gradients
            sweep = []
            for k2 in (4, 8, 12, 16, 24, 32, 48, 64, 96):
                ws2 = torch.empty(max(1, _lib.load().gwn_gemm_workspace_floats(M, N, k2)), device=dev)
                sweep.append("ks%d %.1f" % (k2, timeit(lambda: gwn_mm(A, B, C, k2, ws2))))
            print("   ", name, "split-K sweep (us):", ", ".join(sweep), flush=True)
        print("%-9s M=%6d N=%4d K=%6d  rocBLAS %7.1f us (%5.1f TF)  hipBLASLt %7.1f us (%5.1f TF)  "
              "gwn_gemm %7.1f us (%5.1f TF)"
              % (name, M, N, K, t_torch, flop / t_torch / 1e6, t_lt, flop / t_lt / 1e6, t_gwn, flop / t_gwn / 1e6),
              flush=True)


if __name__ == "__main__":
    main()
