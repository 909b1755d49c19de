"""Experiment transform (tools/exp_build.sh): the f32 16-node tile forward stamps five points per
workgroup into gwn_gcn_args.clock ([CUs][8] u64 instead of [CUs][2]): 0 start, 1 after the
channel-map / TCN-weight staging (and the in-kernel BN finalize) issue, 2 after the first phase's
staging barrier, 3 after the last phase's tiles, 4 after the BN flush.  For tools/t16_phases.py."""
import sys

p = sys.argv[1]
s = open(p).read()
old_start = "  if (a.clk != nullptr && threadIdx.x == 0) a.clk[2 * blockIdx.x] = wall_clock64();"
assert old_start in s
s = s.replace(old_start, "  if (a.clk != nullptr && threadIdx.x == 0) a.clk[8 * blockIdx.x] = wall_clock64();")
old_end = "  if (threadIdx.x == 0) a.clk[2 * blockIdx.x + 1] = wall_clock64();"
assert old_end in s
s = s.replace(old_end, "  if (threadIdx.x == 0) a.clk[8 * blockIdx.x + 4] = wall_clock64();")
s = s.replace("__device__ __forceinline__ void t16_clock_end(const FusedFwd& a) {",
              "__device__ __forceinline__ void t16_stamp(const FusedFwd& a, int k) {\n"
              "  if (a.clk != nullptr && threadIdx.x == 0) a.clk[8 * blockIdx.x + k] = wall_clock64();\n}\n"
              "__device__ __forceinline__ void t16_clock_end(const FusedFwd& a) {", 1)
# the f32 t16 forward only (the first kernel that follows the helpers)
k0 = s.index("void gcn_fwd_t16_kernel(")
k1 = s.index("void gcn_fwd_t16b_kernel(")
body = s[k0:k1]
old = "  if (tcn) t16_tcn_stage_weights(a, wpart, imgs);  // (the finalize's scratch: the free image space)\n"
assert old in body
body = body.replace(old, old + "  t16_stamp(a, 1);\n", 1)
old = "    __syncthreads();\n    const int span = (int)(p1 - p0);\n"
assert old in body
body = body.replace(old, "    __syncthreads();\n    if (p0 == rg.tb) t16_stamp(a, 2);\n    const int span = (int)(p1 - p0);\n", 1)
old = "  t16_bn_flush(a, bn, wpart);\n  t16_clock_end(a);\n"
assert old in body
body = body.replace(old, "  t16_stamp(a, 3);\n" + old, 1)
s = s[:k0] + body + s[k1:]
open(p, "w").write(s)
