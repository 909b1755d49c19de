// Support preparation for the fused diffusion kernels (model.py:41-55's A_k, held padded): the
// squares A^2 / (A^2)^T (the power schedule's second hop in one pass), transposes, zero-padded copies
// and the 16-node k-interleaved copies of gwn_support_g4 / gwn_support_g4_bf16 (one 16-B load per
// lane fetches four k-steps of a support fragment in gcn_fused.hip's tile kernels).
#include "gwn_internal.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

__device__ __forceinline__ int crow(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }
__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.0f;
  return z;
}

// C = A A and C^T for a padded support A [np][ld] (zero outside [n][n], so C is too): one
// 4-wave workgroup per 32 x 32 output tile on v_mfma_f32_32x32x2_f32, each wave a quarter of K
// (np / 2 k-steps, a multiple of 16) with its operands loaded four k-steps ahead; the four partial
// tiles are added in wave order through LDS.  Also A^T when at != nullptr.
// element (r, c) of a padded support into its gwn_support_g4 copy (r, c < 16 * nt)
__device__ __forceinline__ void g4_put(float* dst, int nt, int r, int c, float v) {
  if (r < 16 * nt && c < 16 * nt)
    dst[((long)((r >> 4) * nt + (c >> 4)) * 64 + 16 * (r & 3) + (c & 15)) * 4 + ((r & 15) >> 2)] = v;
}

// A^2, (A^2)^T and optionally A^T of a padded support; with g4, also the gwn_support_g4 copies of
// A and A^2 (g4 + 0 / 1 * g4_stride) and, with g4_count == 4, of A^T and (A^2)^T (2 / 3) -- the
// adaptive support's per-step preparation in one launch
__global__ __launch_bounds__(256) void support_square_kernel(const float* A, int np, int ld, float* C, float* CT,
                                                             float* AT, float* g4, long g4_stride, int g4_nt,
                                                             int g4_count) {
  __shared__ float red[4][32][33];
  const int ti = blockIdx.y * 32, tj = blockIdx.x * 32;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, half = lane >> 5, col = lane & 31;
  const int per = np / 8;  // k-steps per wave (np / 2 in all), a multiple of 4
  f32x16 acc = zero16();
  // D[i][j] = sum_k A[ti + i][k] A[k][tj + j]: A operand lane (half, col) = A[ti + col][2 ks + half]
  const float* ar = A + (long)(ti + col) * ld + half;
  const float* br = A + (long)half * ld + tj + col;
  for (int ks = wave * per; ks < (wave + 1) * per; ks += 4) {
    float a[4], b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a[j] = ar[2 * (ks + j)];
      b[j] = br[(long)2 * (ks + j) * ld];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j], b[j], acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) red[wave][crow(r, half)][col] = acc[r];
  __syncthreads();
  for (int e = threadIdx.x; e < 1024; e += 256) {
    const int i = e >> 5, j = e & 31;  // C row-major: coalesced rows
    C[(long)(ti + i) * ld + tj + j] = ((red[0][i][j] + red[1][i][j]) + red[2][i][j]) + red[3][i][j];
    const int jt = e >> 5, it = e & 31;  // C^T rows: C[. ][jt] down the column
    CT[(long)(tj + jt) * ld + ti + it] = ((red[0][it][jt] + red[1][it][jt]) + red[2][it][jt]) + red[3][it][jt];
    if (g4) {
      const float v = ((red[0][i][j] + red[1][i][j]) + red[2][i][j]) + red[3][i][j];
      g4_put(g4 + g4_stride, g4_nt, ti + i, tj + j, v);
      if (g4_count == 4) g4_put(g4 + 3 * g4_stride, g4_nt, tj + j, ti + i, v);
    }
  }
  if (AT || g4) {
    __syncthreads();
    for (int e = threadIdx.x; e < 1024; e += 256) red[0][e >> 5][e & 31] = A[(long)(ti + (e >> 5)) * ld + tj + (e & 31)];
    __syncthreads();
    for (int e = threadIdx.x; e < 1024; e += 256) {
      if (AT) AT[(long)(tj + (e >> 5)) * ld + ti + (e & 31)] = red[0][e & 31][e >> 5];
      if (g4) {
        const int i = e >> 5, j = e & 31;
        g4_put(g4, g4_nt, ti + i, tj + j, red[0][i][j]);
        if (g4_count == 4) g4_put(g4 + 2 * g4_stride, g4_nt, tj + j, ti + i, red[0][i][j]);
      }
    }
  }
}

__global__ void pad_copy_kernel(const float* src, int n, int ld_src, float* dst, int ld_dst, int np,
                                int transpose, long src_bstride = 0, long dst_bstride = 0) {
  __shared__ float tile[32][33];
  src += blockIdx.z * src_bstride;  // batched: blockIdx.z walks the matrices
  dst += blockIdx.z * dst_bstride;
  const int bx = blockIdx.x * 32, by = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 8 rows per pass
  for (int r = ty; r < 32; r += 8) {
    const int i = by + r, j = bx + tx;
    tile[r][tx] = (i < n && j < n) ? src[(long)i * ld_src + j] : 0.0f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    if (transpose) {
      const int i = bx + r, j = by + tx;
      if (i < np && j < np) dst[(long)i * ld_dst + j] = tile[tx][r];
    } else {
      const int i = by + r, j = bx + tx;
      if (i < np && j < np) dst[(long)i * ld_dst + j] = tile[r][tx];
    }
  }
}

}  // namespace

extern "C" int gwn_support_square(const float* a, int np, int ld, float* a2, float* a2_t, float* a_t, hipStream_t s) {
  return gwn_support_square_g4(a, np, ld, a2, a2_t, a_t, 0, nullptr, 0, 0, s);
}

extern "C" int gwn_support_square_g4(const float* a, int np, int ld, float* a2, float* a2_t, float* a_t, int n,
                                     float* g4, long g4_stride, int g4_count, hipStream_t s) {
  GWN_REQUIRE(a && a2 && a2_t && np > 0 && np % 32 == 0 && ld >= np, "support_square: np must be a multiple of 32");
  GWN_REQUIRE(!g4 || (n > 0 && (n + 31) / 32 * 32 <= np && (g4_count == 2 || g4_count == 4) &&
                      g4_stride >= gwn_support_g4_floats(n)),
              "support_square_g4: needs n <= np, g4_count 2 or 4 and g4_stride >= gwn_support_g4_floats(n)");
  dim3 grid(np / 32, np / 32);
  support_square_kernel<<<grid, 256, 0, s>>>(a, np, ld, a2, a2_t, a_t, g4, g4_stride, g4 ? (n + 15) / 16 : 0,
                                             g4_count);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

namespace {
struct G4Src {
  const float* src[32];
};
// one 256-thread block per (1-KiB block = (k-group, tile), copy): thread e writes float e of the block
__global__ __launch_bounds__(256) void support_g4_kernel(G4Src gs, int nt, int ld, float* dst, long dst_stride) {
  const int blk = blockIdx.x, c = blockIdx.y;
  const int kg = blk / nt, t = blk - kg * nt;
  const int e = threadIdx.x, lane = e >> 2, i = e & 3, g = lane >> 4, j = lane & 15;
  dst[(long)c * dst_stride + (long)blk * 256 + e] = gs.src[c][(long)(16 * kg + 4 * i + g) * ld + 16 * t + j];
}
}  // namespace

extern "C" long gwn_support_g4_floats(int n) {
  const long nt = (n + 15) / 16;
  return n > 0 ? nt * nt * 256 : 0;
}

extern "C" int gwn_support_g4(const float* const* src, int count, int n, int ld, float* dst, long dst_stride,
                              hipStream_t s) {
  GWN_REQUIRE(src && dst && n > 0 && count > 0 && count <= 32 && ld >= (n + 31) / 32 * 32 &&
                  dst_stride >= gwn_support_g4_floats(n),
              "support_g4: needs 1..32 padded [np][ld] supports (ld >= 32*ceil(n/32)) and dst_stride >= "
              "gwn_support_g4_floats(n)");
  G4Src gs = {};
  for (int c = 0; c < count; ++c) gs.src[c] = src[c];
  const int nt = (n + 15) / 16;
  support_g4_kernel<<<dim3(nt * nt, count), 256, 0, s>>>(gs, nt, ld, dst, dst_stride);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

namespace {
// bf16 copy: one 512-thread block per (32-row k-group, 16-column tile, copy): thread e writes element
// e of the block, lane e >> 3's k-step row 8 (lane >> 4) + (e & 7)
__global__ __launch_bounds__(512) void support_g4_bf16_kernel(G4Src gs, int nt, int ld, __bf16* dst, long dst_stride) {
  const int blk = blockIdx.x, c = blockIdx.y;
  const int kg = blk / nt, t = blk - kg * nt;
  const int e = threadIdx.x, lane = e >> 3, i = e & 7;
  dst[(long)c * dst_stride + (long)blk * 512 + e] =
      (__bf16)gs.src[c][(long)(32 * kg + 8 * (lane >> 4) + i) * ld + 16 * t + (lane & 15)];
}
}  // namespace

extern "C" long gwn_support_g4_bf16_elems(int n) {
  const long nt = (n + 15) / 16, nkg = (n + 31) / 32;
  return n > 0 ? nkg * nt * 512 : 0;
}

extern "C" int gwn_support_g4_bf16(const float* const* src, int count, int n, int ld, void* dst, long dst_stride,
                                   hipStream_t s) {
  GWN_REQUIRE(src && dst && n > 0 && count > 0 && count <= 32 && ld >= (n + 31) / 32 * 32 &&
                  dst_stride >= gwn_support_g4_bf16_elems(n) && dst_stride % 8 == 0,
              "support_g4_bf16: needs 1..32 padded [np][ld] supports (ld >= 32*ceil(n/32)) and dst_stride >= "
              "gwn_support_g4_bf16_elems(n), a multiple of 8");
  G4Src gs = {};
  for (int c = 0; c < count; ++c) gs.src[c] = src[c];
  const int nt = (n + 15) / 16, nkg = (n + 31) / 32;
  support_g4_bf16_kernel<<<dim3(nkg * nt, count), 512, 0, s>>>(gs, nt, ld, (__bf16*)dst, dst_stride);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

extern "C" int gwn_transpose(const float* src, int n, int ld_src, float* dst, int ld_dst, hipStream_t s) {
  GWN_REQUIRE(n > 0, "transpose: bad shape");
  dim3 grid((n + 31) / 32, (n + 31) / 32);
  pad_copy_kernel<<<grid, 256, 0, s>>>(src, n, ld_src, dst, ld_dst, n, 1);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

extern "C" int gwn_pad_square(const float* src, int n, int ld_src, float* dst, int np, int ld_dst, int transpose,
                              hipStream_t s) {
  GWN_REQUIRE(n > 0 && np >= n && ld_dst >= np, "pad_square: bad shape");
  dim3 grid((np + 31) / 32, (np + 31) / 32);
  pad_copy_kernel<<<grid, 256, 0, s>>>(src, n, ld_src, dst, ld_dst, np, transpose);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

extern "C" int gwn_pad_square_batched(const float* src, int batch, long src_bstride, int n, int ld_src, float* dst,
                                      int np, int ld_dst, long dst_bstride, int transpose, hipStream_t s) {
  GWN_REQUIRE(n > 0 && np >= n && ld_dst >= np && batch > 0 && batch <= 65535 && src_bstride >= (long)n * ld_src &&
                  dst_bstride >= (long)np * ld_dst,
              "pad_square_batched: bad shape");
  dim3 grid((np + 31) / 32, (np + 31) / 32, batch);
  pad_copy_kernel<<<grid, 256, 0, s>>>(src, n, ld_src, dst, ld_dst, np, transpose, src_bstride, dst_bstride);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

