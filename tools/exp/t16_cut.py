"""Experiment transforms of gcn_fused.hip (timing only, wrong results): remove one part of the t16
kernels' per-tile work.   python tools/exp/t16_cut.py <file> <nomlp|nodiff|noepi>"""
import sys

p, mode = sys.argv[1], sys.argv[2]
s = open(p).read()
if mode == "nomlp":  # every channel map becomes a no-op
    a = s.index("__device__ __forceinline__ void t16_mlp(")
    b = s.index("{", a)
    s = s[:b + 1] + "\n  if (lane >= 0) return;\n" + s[b + 1:]
elif mode == "nodiff":  # the diffusion loop is skipped (accumulators zero)
    a = s.index("__device__ __forceinline__ void t16_diffuse(")
    b = s.index("  int ks0 = 0;", a)
    s = s[:b] + "  if (lane >= 0) return;\n" + s[b:]
elif mode == "noepi":  # no epilogue (z, residual, dropout, BN)
    a = s.index("__device__ __forceinline__ void t16_epilogue(")
    b = s.index("{", a)
    s = s[:b + 1] + "\n  if (lane >= 0) return;\n" + s[b + 1:]
elif mode == "noload":  # the ring's support fragments are not fetched in the loop
    s = s.replace("      s1[nx] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r1, off(ks + T16_RING - 1), 0, 0));",
                  "      s1[nx] = s1[r] * 0.5f;", 1)
    s = s.replace("      s2[nx] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r2, off(ks + T16_RING - 1), 0, 0));",
                  "      s2[nx] = s2[r] * 0.5f;", 1)
elif mode == "nolds":  # the image operands are not read in the loop
    s = s.replace("    const float na = xp[4 * (ks + 1) * 16], nb = xp[hs + 4 * (ks + 1) * 16];",
                  "    const float na = xa * 0.5f, nb = xb * 0.5f;", 1)
elif mode == "nozst":  # the forward epilogue computes z but does not store it
    old = "    if (valid) *(float4*)(dst + m * CH + c0) = make_float4(v[4 * oh], v[4 * oh + 1], v[4 * oh + 2], v[4 * oh + 3]);"
    assert old in s
    s = s.replace(old, "", 1)
elif mode == "nores":  # no residual load in the forward epilogue
    old = "    const float4 rq = *(const float4*)(a.residual + m * CH + c0);"
    assert old in s
    s = s.replace(old, "    const float4 rq = make_float4(bq.x, bq.y, 0.0f, 1.0f);", 1)
elif mode == "ntplain":  # hop pieces with plain stores instead of non-temporal ones
    old = "              if (nt_ok) __builtin_nontemporal_store(acc[q][hf], (f32x4v*)(dp + 16 * hf));"
    assert old in s
    s = s.replace(old, "              if (nt_ok) *(f32x4v*)(dp + 16 * hf) = acc[q][hf];", 1)
else:
    raise SystemExit("mode?")
open(p, "w").write(s)
