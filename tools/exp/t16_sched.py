"""Experiment transforms of gcn_fused.hip's fp32 tile forward (wave scheduling; timing + parity
both valid): python tools/exp/t16_sched.py <file> <desync|prio_diff|prio_epi>
  desync     waves of odd SIMD-quads (wave >> 2 odd) take the supports in reverse order, so the
             four waves of a SIMD are not all in the same phase of their tiles
  prio_diff  s_setprio 1 around each diffusion loop (the MFMA-dense phase issues first)
  prio_epi   s_setprio 1 around the mlps + epilogue (the latency phases issue first)"""
import sys

p = sys.argv[1]
mode = sys.argv[2] if len(sys.argv) > 2 else __import__("os").environ["T16_SCHED"]
s = open(p).read()
k0 = s.index("__global__ __launch_bounds__(MAXT) void gcn_fwd_t16_kernel(")
k1 = s.index("bf16 operands (configs[2]'s mixed precision)", k0)
body = s[k0:k1]
if mode == "desync":
    old = """      for (int k = 0; k < a.nsup; ++k) {
        f32x4v acc[2][2];  // [power][channel half]"""
    new = """      for (int kk = 0; kk < a.nsup; ++kk) {
        const int k = ((wave >> 2) & 1) ? a.nsup - 1 - kk : kk;
        f32x4v acc[2][2];  // [power][channel half]"""
    assert old in body
    body = body.replace(old, new)
elif mode == "prio_diff":
    old = "        t16_diffuse(xs, hs, p.g4[2 * k], p.g4[2 * k + 1], n, tile, lane, acc);\n"
    assert old in body
    body = body.replace(old, "        __builtin_amdgcn_s_setprio(1);\n" + old + "        __builtin_amdgcn_s_setprio(0);\n")
elif mode == "prio_epi":
    old = "      t16_epilogue(a, hacc, row0, w0, lane, n, bn);\n"
    assert old in body
    body = body.replace(old, "      __builtin_amdgcn_s_setprio(1);\n" + old + "      __builtin_amdgcn_s_setprio(0);\n")
    old = "          t16_mlp(ws + (1 + 2 * k + q) * CH * LDW16, LDW16, acc[q], lane, hacc);\n"
    assert old in body
    body = body.replace(old, "          __builtin_amdgcn_s_setprio(1);\n" + old + "          __builtin_amdgcn_s_setprio(0);\n")
else:
    raise SystemExit("mode?")
s = s[:k0] + body + s[k1:]
open(p, "w").write(s)
