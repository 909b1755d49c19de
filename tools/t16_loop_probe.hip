// Microbenchmark of the t16 diffusion inner loop (tools only, never the product): MFMA utilisation
// of v_mfma_f32_16x16x4_f32 k-steps against what each k-step also issues.
//   NACC  independent accumulators per k-step (4: the product's 2 powers x 2 channel halves;
//         8: two 16-node sub-tiles per wave sharing the image operands)
//   LDSRD image operands read from LDS every k-step (as the product) or kept in registers
//   GLD   support fragments fetched every k-step through a 4-step ring (as the product)
// One workgroup per CU (256), WAVES waves each, STEPS k-steps per wave.  Prints us and the MFMA
// busy fraction at the measured clock-free count: mfma cycles / (SIMDs x wall x 2.4 GHz).
// Build: hipcc --offload-arch=gfx950 -O3 -o t16_loop_probe tools/t16_loop_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f32x4v __attribute__((ext_vector_type(4)));

template <int NACC, bool LDSRD, bool GLD>
__global__ __launch_bounds__(1024) void loop_kernel(const float* G, int ld, int steps, float* out) {
  __shared__ float img[4096 * 2];
  for (int e = threadIdx.x; e < 8192; e += blockDim.x) img[e] = 0.001f * (e & 255);
  __syncthreads();
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  const int wave = threadIdx.x >> 6;
  f32x4v acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)G, (short)0, 224 * ld * 4, 0x00020000);
  const int w0 = (wave * 16) % 208;
  auto off = [&](int ks) { return (((4 * ks + g) % 224) * ld + w0 + j) * 4; };
  float s1[4], s2[4];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    s1[q] = GLD ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off(q), 0, 0)) : 0.5f + q;
    s2[q] = GLD ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off(q) + 4 * 16, 0, 0)) : 0.25f + q;
    __builtin_amdgcn_sched_barrier(0);
  }
  const float* xp = img + g * 16 + j;
  float xa = xp[0], xb = xp[4096];
  for (int ks0 = 0; ks0 < steps; ks0 += 4) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ks = ks0 + q;
      const int nx = (q + 3) & 3;
      if (GLD) {
        s1[nx] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off(ks + 3), 0, 0));
        s2[nx] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off(ks + 3) + 4 * 16, 0, 0));
      }
      float na = xa, nb = xb;
      if (LDSRD) {
        na = xp[((4 * (ks + 1)) & 255) * 16];
        nb = xp[4096 + ((4 * (ks + 1)) & 255) * 16];
      }
      __builtin_amdgcn_sched_barrier(0);
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa, s1[q], acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(xb, s1[q], acc[1], 0, 0, 0);
      acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa, s2[q], acc[2], 0, 0, 0);
      acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(xb, s2[q], acc[3], 0, 0, 0);
      if (NACC == 8) {
        acc[4 % NACC] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa, s1[(q + 1) & 3], acc[4 % NACC], 0, 0, 0);
        acc[5 % NACC] = __builtin_amdgcn_mfma_f32_16x16x4f32(xb, s1[(q + 1) & 3], acc[5 % NACC], 0, 0, 0);
        acc[6 % NACC] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa, s2[(q + 1) & 3], acc[6 % NACC], 0, 0, 0);
        acc[7 % NACC] = __builtin_amdgcn_mfma_f32_16x16x4f32(xb, s2[(q + 1) & 3], acc[7 % NACC], 0, 0, 0);
      }
      if (LDSRD) {
        xa = na;
        xb = nb;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  float sum = 0.0f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) sum += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = sum;
}

// support fragments of 4 k-steps per 16-B load (k-interleaved tiled layout), two groups in flight
template <bool LDSRD>
__global__ __launch_bounds__(1024) void loop128_kernel(const float* G, int ld, int steps, float* out) {
  __shared__ float img[4096 * 2];
  for (int e = threadIdx.x; e < 8192; e += blockDim.x) img[e] = 0.001f * (e & 255);
  __syncthreads();
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  const int wave = threadIdx.x >> 6;
  f32x4v acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
  // two powers x 52 k-step groups x 13 tiles x 1 KiB (the k-interleaved copies of A and A^2)
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)G, (short)0, 2 * 52 * 13 * 1024, 0x00020000);
  const int tile = wave % 13;
  // group kg of tile t: 1 KiB at ((kg % 48) * 13 + t) * 1024, lane l's 16 B at l * 16
  auto off = [&](int kg) { return (((kg % 52) * 13 + tile) * 256 + lane * 4) * 4; };
  f32x4v a1[2], a2[2];
  a1[0] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(r, off(0), 0, 0));
  a2[0] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(r, off(0) + 52 * 13 * 1024, 0, 0));
  __builtin_amdgcn_sched_barrier(0);
  const float* xp = img + g * 16 + j;
  float xa = xp[0], xb = xp[4096];
  for (int ks0 = 0; ks0 < steps; ks0 += 8) {
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
      a1[1 - hb] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(r, off(ks0 / 4 + hb + 1), 0, 0));
      a2[1 - hb] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(r, off(ks0 / 4 + hb + 1) + 52 * 13 * 1024, 0, 0));
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int ks = ks0 + 4 * hb + q;
        float na = xa, nb = xb;
        if (LDSRD) {
          na = xp[((4 * (ks + 1)) & 255) * 16];
          nb = xp[4096 + ((4 * (ks + 1)) & 255) * 16];
        }
        __builtin_amdgcn_sched_barrier(0);
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa, a1[hb][q], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(xb, a1[hb][q], acc[1], 0, 0, 0);
        acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa, a2[hb][q], acc[2], 0, 0, 0);
        acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(xb, a2[hb][q], acc[3], 0, 0, 0);
        if (LDSRD) {
          xa = na;
          xb = nb;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  float sum = 0.0f;
#pragma unroll
  for (int i = 0; i < 4; ++i) sum += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = sum;
}

void run128(const char* tag, int waves, const float* G, float* out) {
  const int steps = 4096;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) loop128_kernel<true><<<256, 64 * waves>>>(G, 224, steps, out);
  hipEventRecord(e0);
  const int reps = 10;
  for (int i = 0; i < reps; ++i) loop128_kernel<true><<<256, 64 * waves>>>(G, 224, steps, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.0f;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = 1000.0 * ms / reps;
  const double mfma_cyc = (double)steps * 4 * 32.0 * waves / 4.0;
  printf("%-22s waves/CU %2d  %8.1f us  MFMA busy @2.4GHz %.3f\n", tag, waves, us, mfma_cyc / (us * 2400.0));
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

template <int NACC, bool LDSRD, bool GLD>
void run(const char* tag, int waves, const float* G, float* out) {
  const int steps = 4096;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) loop_kernel<NACC, LDSRD, GLD><<<256, 64 * waves>>>(G, 224, steps, out);
  hipEventRecord(e0);
  const int reps = 10;
  for (int i = 0; i < reps; ++i) loop_kernel<NACC, LDSRD, GLD><<<256, 64 * waves>>>(G, 224, steps, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.0f;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = 1000.0 * ms / reps;
  const double mfma_cyc = (double)steps * NACC * 32.0 * waves / 4.0;  // per SIMD
  printf("%-22s waves/CU %2d  %8.1f us  MFMA busy @2.4GHz %.3f\n", tag, waves, us, mfma_cyc / (us * 2400.0));
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  float *G, *out;
  hipMalloc(&G, 2 * 52 * 13 * 1024);
  hipMalloc(&out, 256 * 1024 * 4);
  std::vector<float> h(2 * 52 * 13 * 256);
  for (size_t i = 0; i < h.size(); ++i) h[i] = 0.001f * (i % 97);
  hipMemcpy(G, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  for (int w : {4, 8, 16}) {
    run128("acc4 lds+gld128", w, G, out);
    run<4, false, false>("acc4 regs", w, G, out);
    run<4, true, false>("acc4 lds", w, G, out);
    run<4, true, true>("acc4 lds+gld", w, G, out);
    run<8, true, true>("acc8 lds+gld", w, G, out);
    run<8, false, false>("acc8 regs", w, G, out);
  }
  hipFree(G);
  hipFree(out);
  return 0;
}
