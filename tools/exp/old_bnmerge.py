"""Experiment transform (tools/exp_build.sh): the in-kernel BN merge's partial loads as before round 6
(the count load under the slot test, which compiled to a branch around it)."""
import sys

p = sys.argv[1]
s = open(p).read()
old = """#pragma unroll
    for (int u = 0; u < U; ++u) {  // unconditional loads (a slot past nparts reads slot 0, then counts 0)
      const int i = i0 + u * nsub;
      const float* pp = f.part + (long)(i < f.nparts ? i : 0) * 3 * CH;
      nb[u] = pp[c];
      mb[u] = pp[CH + c];
      qb[u] = pp[2 * CH + c];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + u * nsub >= f.nparts) nb[u] = 0.0f;"""
assert old in s
s = s.replace(old, """#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * nsub;
      const float* pp = f.part + (long)(i < f.nparts ? i : 0) * 3 * CH;
      nb[u] = i < f.nparts ? pp[c] : 0.0f;
      mb[u] = pp[CH + c];
      qb[u] = pp[2 * CH + c];
    }""")
open(p, "w").write(s)
