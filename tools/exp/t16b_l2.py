"""Experiment transforms (timing only, wrong results) of the bf16 tile kernels' support fragment
stream: python tools/exp/t16b_l2.py <file> [col0]   (mode also from env T16B_L2)
  col0   every tile reads node column 0's support blocks (the same ~66 KB: L1/L2 hits, no L2
         bandwidth) -- if the kernels speed up, the fragment stream's L2 bandwidth bounds them"""
import os
import sys

p = sys.argv[1]
mode = sys.argv[2] if len(sys.argv) > 2 else os.environ["T16B_L2"]
s = open(p).read()
a = s.index("__device__ __forceinline__ void t16b_diffuse(")
b = s.index("auto off = [&](int kg) { return ((kg * nt + tile) * 64 + lane) * 16; };", a)
if mode == "col0":
    s = s[:b] + "auto off = [&](int kg) { return ((kg * nt + 0) * 64 + lane) * 16; };" + \
        s[b + len("auto off = [&](int kg) { return ((kg * nt + tile) * 64 + lane) * 16; };"):]
else:
    raise SystemExit("mode?")
open(p, "w").write(s)
