"""Library reference for the head GEMMs (fp32): torch.mm (hipBLASLt / rocBLAS) on the shapes of the
output head at METR-LA (rows 64*207) and PEMS-BAY (rows 64*325): end_conv_1 forward
[rows, 256] x [256, 512], its data gradient [rows, 512] x [512, 256], its weight gradient
[512, rows] x [rows, 256].  Prints microseconds per call (HIP events over 50 calls) and TFLOP/s,
to set against libgwn's gemm_nt / gemm kernels in profiles/r04/*_step.txt.

    python tools/exp/head_gemm_torch.py
"""
import torch


def main():
    dev = torch.device("cuda:0")
    for name, rows in (("metr", 64 * 207), ("pems", 64 * 325)):
        shapes = {"e1_fwd": ((rows, 256), (256, 512)), "dskip": ((rows, 512), (512, 256)),
                  "dW1": ((512, rows), (rows, 256))}
        for k, (sa, sb) in shapes.items():
            a = torch.randn(*sa, device=dev)
            b = torch.randn(*sb, device=dev)
            if k == "dW1":  # the weight gradient reads both operands row-major over rows
                a = torch.randn(rows, 512, device=dev).t()
            for _ in range(5):
                torch.mm(a, b)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                torch.mm(a, b)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 50
            fl = 2.0 * sa[0] * sa[1] * sb[1]
            print("%s %-7s %5d x %4d x %4d: %7.1f us  %6.1f TFLOP/s" % (name, k, sa[0], sa[1], sb[1], us, fl / us / 1e6),
                  flush=True)


if __name__ == "__main__":
    main()
