// Probe: issue rate of v_mfma_f32_32x32x2_f32 with 1, 2 or 4 independent accumulator chains per
// wave and 1 or 2 waves per SIMD.  Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_probe.hip -o /tmp/mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int CHAINS>
__global__ void probe(float* out, int iters, float a, float b) {
  f32x16 acc[CHAINS];
  for (int c = 0; c < CHAINS; ++c)
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.0f;
  const float av = a + threadIdx.x * 1e-7f, bv = b - threadIdx.x * 1e-7f;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 8 / CHAINS; ++u)
#pragma unroll
      for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[c], 0, 0, 0);
  }
  float s = 0.0f;
  for (int c = 0; c < CHAINS; ++c)
    for (int r = 0; r < 16; ++r) s += acc[c][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int CHAINS>
void run(int waves_per_cu, float* out) {
  const int iters = 4096;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  probe<CHAINS><<<256, 64 * waves_per_cu>>>(out, 16, 1.0f, 1.0f);
  hipEventRecord(e0);
  probe<CHAINS><<<256, 64 * waves_per_cu>>>(out, iters, 1.0f, 1.0f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double mfma = 256.0 * waves_per_cu * iters * 8;
  const double tf = mfma * 4096.0 / (ms * 1e-3) / 1e12;
  printf("chains=%d waves/CU=%2d: %.3f ms  %.1f TFLOP/s  (%.1f cyc/MFMA/SIMD at 2.4 GHz)\n", CHAINS, waves_per_cu,
         ms, tf, (ms * 1e-3 * 2.4e9) / (mfma / 1024.0));
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 1024 * sizeof(float));
  for (int w : {4, 8, 12, 16}) {
    run<1>(w, out);
    run<2>(w, out);
    run<4>(w, out);
  }
  hipFree(out);
  return 0;
}
