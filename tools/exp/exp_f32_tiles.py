"""Experiment transform (tools/exp_build.sh): the fp32 NT GEMM's tile choice, from the EXP_F32_TILE
environment variable of the build: 'a' = 64x64 tiles always, 'b' = 64x128 for N % 128 == 0 else
64x64, 'c' = 128x128 for N % 128 == 0 else 128x64 (no workgroup-count threshold)."""
import os
import sys

p = sys.argv[1].replace("gcn_fused.hip", "gemm_nt.hip")
s = open(p).read()
old = """  else if (N % 128 == 0 && (long)((M + 127) / 128) * (N / 128) >= 384) launch<128, 128, 2, 2>(p, s);
  else launch<128, 64, 2, 2>(p, s);"""
assert old in s
v = os.environ["EXP_F32_TILE"]
new = {"a": "  else launch<64, 64, 2, 2>(p, s);",
       "b": "  else if (N % 128 == 0) launch<64, 128, 2, 2>(p, s);\n  else launch<64, 64, 2, 2>(p, s);",
       "c": "  else if (N % 128 == 0) launch<128, 128, 2, 2>(p, s);\n  else launch<128, 64, 2, 2>(p, s);"}[v]
s = s.replace(old, new)
open(p, "w").write(s)
