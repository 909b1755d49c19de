"""Probe: the head's GEMM shapes (METR M = 64*207, PEMS M = 64*325 rows) on gwn_gemm_nt, gwn_gemm_nt_bf16
and the library fp32 GEMM (torch.mm -> hipBLASLt / rocBLAS), HIP events over 50 back-to-back calls
each.  GWN_LIB selects an experiment build of the library (tools/exp_build.sh)."""
import sys

import torch

sys.path.insert(0, "graph-wavenet_amd")
from gwn_amd import _lib  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False


def timed(f, reps=50):
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / reps


for M in (64 * 207, 64 * 325):
    for name, N, K, relu, mask in (("skip", 256, 256, 1, 0), ("e1", 512, 256, 1, 0), ("dsk", 256, 512, 0, 1),
                                   ("dskipcat", 256, 256, 0, 0)):
        A = torch.randn(M, K, device="cuda")
        B = torch.randn(N, K, device="cuda")
        C = torch.empty(M, N, device="cuda")
        bias = torch.randn(N, device="cuda")
        mk = torch.randn(M, N, device="cuda")
        res = []
        for fn in ("gwn_gemm_nt", "gwn_gemm_nt_bf16"):
            res.append(timed(lambda: _lib.call(fn, A.data_ptr(), K, B.data_ptr(), K, C.data_ptr(), N, M, N, K,
                                               bias.data_ptr() if relu else None, relu,
                                               mk.data_ptr() if mask else None, N, _lib.stream())))
        res.append(timed(lambda: A @ B.t()))
        mb = (M * K + M * N * (2 if mask else 1)) * 4 / 1e6
        print("M=%5d %-9s N=%3d K=%3d  f32 %6.1f us  bf16 %6.1f us (%5.2f TB/s of %5.1f MB)  torch.mm %6.1f us"
              % (M, name, N, K, res[0], res[1], mb / res[1], mb, res[2]), flush=True)
