import sys
p = sys.argv[1].replace("gcn_fused.hip", "gemm_nt.hip")
s = open(p).read()
old = """  if (N % 128 == 0 && (long)((M + 127) / 128) * (N / 128) >= 384) launch_bf16<128, 128, 2, 2>(p, s);
  else launch_bf16<128, 64, 2, 2>(p, s);"""
assert old in s
s = s.replace(old, """  if (N % 128 == 0) launch_bf16<64, 128, 2, 2>(p, s);
  else launch_bf16<64, 64, 2, 2>(p, s);""")
open(p, "w").write(s)
