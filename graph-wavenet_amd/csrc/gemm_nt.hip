// Row-tile "NT" GEMM for the output head of Graph WaveNet (model.py:216-222, 238-240):
//     C[m][n] = epi( sum_k A[m][k] * B[n][k] )        A [M][lda], B [N][ldb], both K-contiguous
// i.e. a 1x1 conv over channels-last activations (B = the conv weight [out][in]) and, with the
// transposed weight, its input gradient.  M = positions (~10^4), N, K in {12, 256, 512}.
//
// 256 threads = 4 waves; each wave owns a (BM/WGM) x (BN/WGN) block of 32x32 MFMA tiles
// (v_mfma_f32_32x32x2_f32, exact fp32).  K runs in BK = 32 tiles staged through LDS by coalesced
// 16-B loads (rows of 128 B, double buffered, one barrier per tile, the next tile's global loads in
// flight during the MFMAs).  The MFMA K order is permuted within a tile — step j takes
// k = 16*half + j in lane half `half` — so every lane reads its 16 A (and B) values of a tile as
// four conflict-free ds_read_b128 (rows padded to 36 floats).  Out-of-range rows / columns / k are
// buffer loads past the resource end (zeros) and dropped stores: no predicated loads.
#include "gwn_internal.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int BK = 32;
constexpr int LDK = BK + 4;      // LDS row stride (floats)
constexpr int OOR = 0x7ffffff0;  // out-of-range byte offset

struct NtArgs {
  const float* A; long lda;
  const float* B; long ldb;
  float* C; long ldc;
  int M, N, K;
  const float* bias; int relu;
  const float* mask; long ldmask;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ int crow(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }

template <int BM, int BN, int WGM, int WGN>
__global__ __launch_bounds__(256) void gemm_nt_kernel(const NtArgs p) {
  static_assert(WGM * WGN == 4, "4 waves");
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1, "wave tile >= 32x32");
  constexpr int AQ = BM * BK / 4 / 256;  // float4 per thread per tile
  constexpr int BQ = (BN * BK / 4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) float As[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN * LDK];

  const int tid = threadIdx.x, lane = tid & 63, half = lane >> 5, col = lane & 31;
  const int wave = tid >> 6, wm = wave % WGM, wn = wave / WGM;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const __amdgpu_buffer_rsrc_t ra = rsrc(p.A, ((long)(p.M - 1) * p.lda + p.K) * 4);
  const __amdgpu_buffer_rsrc_t rb = rsrc(p.B, ((long)(p.N - 1) * p.ldb + p.K) * 4);

  float4 pa[AQ], pb[BQ];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < AQ; ++i) {
      const int q = tid + 256 * i, r = q >> 3, k = k0 + 4 * (q & 7);
      const int off = (m0 + r < p.M && k < p.K) ? (int)(((long)(m0 + r) * p.lda + k) * 4) : OOR;
      pa[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < BQ; ++i) {
      const int q = tid + 256 * i, r = q >> 3, k = k0 + 4 * (q & 7);
      const int off = (q < BN * BK / 4 && n0 + r < p.N && k < p.K) ? (int)(((long)(n0 + r) * p.ldb + k) * 4) : OOR;
      pb[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rb, off, 0, 0));
    }
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < AQ; ++i) {
      const int q = tid + 256 * i;
      *(float4*)&As[buf][(q >> 3) * LDK + 4 * (q & 7)] = pa[i];
    }
#pragma unroll
    for (int i = 0; i < BQ; ++i) {
      const int q = tid + 256 * i;
      if (q < BN * BK / 4) *(float4*)&Bs[buf][(q >> 3) * LDK + 4 * (q & 7)] = pb[i];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  const int nk = (p.K + BK - 1) / BK;
  gload(0);
  swrite(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * BK);
    float af[TM][16], bf[TN][16];
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      const float* s = &As[buf][(wm * WTM + 32 * t + col) * LDK + 16 * half];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = *(const float4*)(s + 4 * q);
        af[t][4 * q] = v.x; af[t][4 * q + 1] = v.y; af[t][4 * q + 2] = v.z; af[t][4 * q + 3] = v.w;
      }
    }
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const float* s = &Bs[buf][(wn * WTN + 32 * t + col) * LDK + 16 * half];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = *(const float4*)(s + 4 * q);
        bf[t][4 * q] = v.x; bf[t][4 * q + 1] = v.y; bf[t][4 * q + 2] = v.z; bf[t][4 * q + 3] = v.w;
      }
    }
#pragma unroll
    for (int j = 0; j < 16; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int t = 0; t < TN; ++t)
          acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][j], bf[t][j], acc[i][t], 0, 0, 0);
    if (kt + 1 < nk) swrite(buf ^ 1);
    __syncthreads();
  }

  // epilogue: bias, relu, relu-backward mask; 32 lanes of a half write one 128-B row segment
  const __amdgpu_buffer_rsrc_t rc = rsrc(p.C, ((long)(p.M - 1) * p.ldc + p.N) * 4);
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    const int n = n0 + wn * WTN + 32 * t + col;
    const bool nok = n < p.N;
    const float bn = (p.bias && nok) ? p.bias[n] : 0.0f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * WTM + 32 * i + crow(r, half);
        const bool ok = nok && m < p.M;
        float v = acc[i][t][r] + bn;
        if (p.relu) v = fmaxf(v, 0.0f);
        if (p.mask) v = (ok && p.mask[(long)m * p.ldmask + n] > 0.0f) ? v : 0.0f;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rc,
                                              ok ? (int)(((long)m * p.ldc + n) * 4) : OOR, 0, 0);
      }
  }
}

template <int BM, int BN, int WGM, int WGN>
void launch(const NtArgs& p, hipStream_t s) {
  dim3 grid((p.M + BM - 1) / BM, (p.N + BN - 1) / BN);
  gemm_nt_kernel<BM, BN, WGM, WGN><<<grid, 256, 0, s>>>(p);
}

inline bool al16(const void* q) { return ((uintptr_t)q & 15u) == 0; }

}  // namespace

extern "C" int gwn_gemm_nt(const float* A, long lda, const float* B, long ldb, float* C, long ldc, int M, int N,
                           int K, const float* bias, int relu, const float* mask, long ldmask, hipStream_t s) {
  GWN_REQUIRE(A && B && C && M > 0 && N > 0 && K > 0, "gemm_nt: bad shape");
  GWN_REQUIRE(K % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 && al16(A) && al16(B),
              "gemm_nt: K, lda, ldb must be multiples of 4 and A, B 16-B aligned");
  GWN_REQUIRE(lda >= K && ldb >= K && ldc >= N && (!mask || ldmask >= N), "gemm_nt: leading dimensions");
  GWN_REQUIRE(((long)M * lda + K) * 4 < 0x7fff0000L && ((long)N * ldb + K) * 4 < 0x7fff0000L &&
                  ((long)M * ldc + N) * 4 < 0x7fff0000L,
              "gemm_nt: operand beyond a 2 GB buffer window");
  NtArgs p = {A, lda, B, ldb, C, ldc, M, N, K, bias, relu, mask, ldmask};
  // tile choice: enough workgroups for 256 CUs (two resident per CU), wide N tiles when N allows
  if (N <= 32) launch<128, 32, 4, 1>(p, s);
  else if (N % 128 == 0 && (long)((M + 127) / 128) * (N / 128) >= 384) launch<128, 128, 2, 2>(p, s);
  else launch<128, 64, 2, 2>(p, s);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}
