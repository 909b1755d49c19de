// Probe: placement of a workgroup's waves on the 4 SIMDs (HW_ID) and the MFMA time of 4..16-wave
// workgroups of one f32 accumulator chain each.  Build: hipcc --offload-arch=gfx950 -O3 tools/wave_placement_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));
__global__ void probe(float* out, int iters, float a, float b, unsigned* simd) {
  f32x16 acc;
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  const float av = a + threadIdx.x * 1e-7f, bv = b - threadIdx.x * 1e-7f;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 8; ++u) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
  }
  float s = 0.0f;
  for (int r = 0; r < 16; ++r) s += acc[r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) {
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    simd[blockIdx.x * 16 + threadIdx.x / 64] = hw;
  }
}
int main() {
  float* out; unsigned* simd;
  hipMalloc(&out, 1024 * 1024 * sizeof(float));
  hipMalloc(&simd, 4096 * 16 * 4);
  for (int waves : {4, 7, 8, 14, 16}) {
    for (int grid : {64, 256}) {
      const int iters = 2048;
      hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
      probe<<<grid, 64 * waves>>>(out, 16, 1.f, 1.f, simd);
      hipEventRecord(e0);
      probe<<<grid, 64 * waves>>>(out, iters, 1.f, 1.f, simd);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      const double per_wave_cycles = (double)iters * 8 * 64;  // if alone on a SIMD
      unsigned h[16]; hipMemcpy(h, simd + 16 * 0, 64, hipMemcpyDeviceToHost);
      printf("waves/WG=%2d grid=%3d: %.3f ms = %.2f x one-wave-per-SIMD time (at 2.4 GHz); SIMD ids of block 0:", waves, grid, ms,
             ms * 1e-3 * 2.4e9 / per_wave_cycles);
      for (int w = 0; w < waves; ++w) printf(" %u", (h[w] >> 4) & 3);
      printf("\n");
    }
  }
  return 0;
}
