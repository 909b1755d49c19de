"""Experiment transform (tools/exp_build.sh): t16_stage_maps as before round 6's batching (one
element per iteration: load -> wait -> LDS write)."""
import sys

p = sys.argv[1]
s = open(p).read()
i = s.index("__device__ __forceinline__ void t16_stage_maps(")
j = s.index("// rows [0, rows) of a slice's node features")
s = s[:i] + '''__device__ __forceinline__ void t16_stage_maps(const float* w, int ld_w, bool backward, int npieces, float* dst) {
  if (backward) {
    const int total = npieces * CH * 8;
    for (int e = threadIdx.x; e < total; e += blockDim.x) {
      const int r = e >> 3, q = e & 7;
      *(float4*)(dst + r * LDW16 + 4 * q) = *(const float4*)(w + (long)(r & 31) * ld_w + (r >> 5) * CH + 4 * q);
    }
  } else {
    const int total = npieces * CH * CH;
    for (int e = threadIdx.x; e < total; e += blockDim.x) {
      const int r = e >> 5, o = e & 31;
      dst[r * LDW16 + o] = w[(long)o * ld_w + (r >> 5) * CH + (r & 31)];
    }
  }
}

''' + s[j:]
open(p, "w").write(s)
