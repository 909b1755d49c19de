// Row-tile "NT" GEMM for the output head of Graph WaveNet (model.py:216-222, 238-240), fp32 MFMA
// or (gwn_gemm_nt_bf16) bf16 MFMA operands:
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
constexpr int NT_STORE_AUX = 2;  // output stores non-temporal (head GEMMs 128.4 -> 123.0 us per METR step)

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

// epilogue of a wave's TM x TN 32x32 tiles at (mb, nb): bias, relu, relu-backward mask; 32 lanes
// of a half write one 128-B row segment
template <int TM, int TN>
__device__ __forceinline__ void nt_epilogue(const NtArgs& p, const f32x16 (&acc)[TM][TN], int mb, int nb, int half,
                                            int col) {
  const __amdgpu_buffer_rsrc_t rc = rsrc(p.C, ((long)(p.M - 1) * p.ldc + p.N) * 4);
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    const int n = nb + 32 * t + col;
    const bool nok = n < p.N;
    const float bn = (p.bias && nok) ? p.bias[n] : 0.0f;
    // the column's mask values, all loaded before the first store (a load after a store to a
    // possibly aliasing C would wait for it: one memory round trip per element)
    float mk[TM][16];
    if (p.mask) {
      const __amdgpu_buffer_rsrc_t rm = rsrc(p.mask, ((long)(p.M - 1) * p.ldmask + p.N) * 4);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = mb + 32 * i + crow(r, half);
          mk[i][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                   rm, (nok && m < p.M) ? (int)(((long)m * p.ldmask + n) * 4) : OOR, 0, 0));
        }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mb + 32 * i + crow(r, half);
        const bool ok = nok && m < p.M;
        float v = acc[i][t][r] + bn;
        if (p.relu) v = fmaxf(v, 0.0f);
        if (p.mask) v = mk[i][r] > 0.0f ? v : 0.0f;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rc,
                                              ok ? (int)(((long)m * p.ldc + n) * 4) : OOR, 0, NT_STORE_AUX);
      }
  }
}

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

  nt_epilogue<TM, TN>(p, acc, m0 + wm * WTM, n0 + wn * WTN, half, col);
}

// bf16 operands (gwn_gemm_nt_bf16, the bf16 mode's head): the same tiles and epilogue, A and B
// rounded to bf16 (RNE) as they are staged -- fp32 in memory, one cvt per element per tile -- and
// v_mfma_f32_32x32x16_bf16 with fp32 accumulation: lane (col, half) of a 32x32 tile takes k = 16s +
// 8 half .. +7 of its row for k-step s (one conflict-free ds_read_b128 per tile and step: 80-B rows).
// The tile order keeps the column tiles of a row block on one XCD (id % 8 is the XCD): their A rows
// come from that XCD's L2 after the first.
typedef __bf16 bf16x8n __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4n __attribute__((ext_vector_type(4)));
constexpr int LDH = BK + 8;  // bf16 LDS row stride: 80 B

template <int BM, int BN, int WGM, int WGN>
__global__ __launch_bounds__(256) void gemm_nt_bf16_kernel(const NtArgs p, const int nrow, const int ncol) {
  static_assert(WGM * WGN == 4, "4 waves");
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int AQ = BM * BK / 4 / 256;
  constexpr int BQ = (BN * BK / 4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) __bf16 As[2][BM * LDH];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[2][BN * LDH];

  const int id = blockIdx.x, xcd = id & 7, j = id >> 3;
  const int row_tile = (j / ncol) * 8 + xcd, col_tile = j - (j / ncol) * ncol;
  if (row_tile >= nrow) return;  // (the grid rounds the row tiles up to a multiple of 8)
  const int tid = threadIdx.x, lane = tid & 63, half = lane >> 5, col = lane & 31;
  const int wave = tid >> 6, wm = wave % WGM, wn = wave / WGM;
  const int m0 = row_tile * BM, n0 = col_tile * BN;
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
  auto cvt4 = [](float4 v) { return bf16x4n{(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w}; };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < AQ; ++i) {
      const int q = tid + 256 * i;
      *(bf16x4n*)&As[buf][(q >> 3) * LDH + 4 * (q & 7)] = cvt4(pa[i]);
    }
#pragma unroll
    for (int i = 0; i < BQ; ++i) {
      const int q = tid + 256 * i;
      if (q < BN * BK / 4) *(bf16x4n*)&Bs[buf][(q >> 3) * LDH + 4 * (q & 7)] = cvt4(pb[i]);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int t = 0; t < TN; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][t][r] = 0.0f;

  const int nk = (p.K + BK - 1) / BK;
  gload(0);
  swrite(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * BK);
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8n af[TM], bf[TN];
#pragma unroll
      for (int t = 0; t < TM; ++t) af[t] = *(const bf16x8n*)&As[buf][(wm * WTM + 32 * t + col) * LDH + 16 * ks + 8 * half];
#pragma unroll
      for (int t = 0; t < TN; ++t) bf[t] = *(const bf16x8n*)&Bs[buf][(wn * WTN + 32 * t + col) * LDH + 16 * ks + 8 * half];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int t = 0; t < TN; ++t) acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bf[t], acc[i][t], 0, 0, 0);
    }
    if (kt + 1 < nk) swrite(buf ^ 1);
    __syncthreads();
  }
  nt_epilogue<TM, TN>(p, acc, m0 + wm * WTM, n0 + wn * WTN, half, col);
}


// Weight-gradient partials on bf16 operands (gwn_wgrad_bf16_partials, the bf16 mode's head: end_conv_1
// and the skip convs): part[c][j*Kc + k] = sum_{r in chunk c} bf16(dY[r][j]) bf16(X[r][k]) on
// v_mfma_f32_32x32x16_bf16 (fp32 sums), part[c][J*Kc + j] = sum_r dY[r][j] (fp32, unrounded).
// A workgroup owns one 128 x 128 output tile and one row chunk; 32 rows per step, staged as bf16
// [column][row] images (80-B rows: the MFMA's 8 consecutive rows per lane are one ds_read_b128):
// thread (col, rh) loads rows 16 rh .. 16 rh + 15 of its column with coalesced 4-B loads (a wave
// reads 64 consecutive floats of a row) and writes them as two 16-B bf16 octets.  The next step's
// loads are in flight during the current step's MFMAs.  Deterministic: the chunks' partials are
// summed by gwn_reduce_partials.
struct WgB {
  const float* dY; long ldy;
  const float* X; long ldx;
  float* part;
  int J, Kc, R, nsplit;
};
constexpr int WBR = 32;       // rows per step
constexpr int WLD = WBR + 8;  // bf16 image row stride (80 B)

__global__ __launch_bounds__(256) void wgrad_bf16_kernel(const WgB p) {
  __shared__ __attribute__((aligned(16))) __bf16 Ys[2][128 * WLD];
  __shared__ __attribute__((aligned(16))) __bf16 Xs[2][128 * WLD];
  __shared__ float bred[128];
  const int nkt = p.Kc / 128, ntiles = (p.J / 128) * nkt;
  // the tiles of a row chunk on one XCD (workgroups are dealt to the 8 XCDs round-robin): its dY
  // and X rows come from that XCD's L2 after the first tile's reads
  const int xcd = blockIdx.x & 7, q = blockIdx.x >> 3;
  const int tile = q % ntiles, c = (q / ntiles) * 8 + xcd;
  if (c >= p.nsplit) return;
  const int jt = tile / nkt, kt = tile - jt * nkt;
  const int j0 = 128 * jt, k0 = 128 * kt;
  const int r0 = (int)((long)p.R * c / p.nsplit), r1 = (int)((long)p.R * (c + 1) / p.nsplit);
  const int tid = threadIdx.x, lane = tid & 63, half = lane >> 5, col = lane & 31;
  const int wave = tid >> 6, wm = wave & 1, wn = wave >> 1;
  const int scol = tid & 127, rh = tid >> 7;  // staging: column and row half
  const __amdgpu_buffer_rsrc_t ry = rsrc(p.dY, (long)r1 * p.ldy * 4);
  const __amdgpu_buffer_rsrc_t rx = rsrc(p.X, (long)r1 * p.ldx * 4);
  const bool bias = kt == 0;

  float yv[16], xv[16];
  auto gload = [&](int rs) {
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = rs + 16 * rh + e;
      const bool ok = row < r1;
      yv[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                            ry, ok ? (int)(((long)row * p.ldy + j0 + scol) * 4) : OOR, 0, 0));
      xv[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                            rx, ok ? (int)(((long)row * p.ldx + k0 + scol) * 4) : OOR, 0, 0));
    }
  };
  float bsum = 0.0f;
  auto swrite = [&](int buf) {
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      bf16x8n y8, x8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        y8[e] = (__bf16)yv[8 * g + e];
        x8[e] = (__bf16)xv[8 * g + e];
      }
      *(bf16x8n*)&Ys[buf][scol * WLD + 16 * rh + 8 * g] = y8;
      *(bf16x8n*)&Xs[buf][scol * WLD + 16 * rh + 8 * g] = x8;
    }
    if (bias) {
#pragma unroll
      for (int e = 0; e < 16; ++e) bsum += yv[e];
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][t][r] = 0.0f;

  const int nst = (r1 - r0 + WBR - 1) / WBR;
  if (nst > 0) {
    gload(r0);
    swrite(0);
  }
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const int buf = st & 1;
    if (st + 1 < nst) gload(r0 + (st + 1) * WBR);
#pragma unroll
    for (int ks = 0; ks < WBR / 16; ++ks) {
      bf16x8n af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = *(const bf16x8n*)&Ys[buf][(64 * wm + 32 * i + col) * WLD + 16 * ks + 8 * half];
#pragma unroll
      for (int t = 0; t < 2; ++t) bf[t] = *(const bf16x8n*)&Xs[buf][(64 * wn + 32 * t + col) * WLD + 16 * ks + 8 * half];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bf[t], acc[i][t], 0, 0, 0);
    }
    if (st + 1 < nst) swrite(buf ^ 1);
    __syncthreads();
  }
  float* out = p.part + (long)c * ((long)p.J * p.Kc + p.J);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        out[(long)(j0 + 64 * wm + 32 * i + crow(r, half)) * p.Kc + k0 + 64 * wn + 32 * t + col] = acc[i][t][r];
  if (bias) {  // the two row halves of a column, summed in a fixed order
    if (rh == 1) bred[scol] = bsum;
    __syncthreads();
    if (rh == 0) out[(long)p.J * p.Kc + j0 + scol] = bsum + bred[scol];
  }
}

// Thin N (N <= 32, the head's end_conv_2 forward: N = 12 outputs over K = 512 channels): one
// 32-row block per workgroup, the K tiles dealt round-robin to its 4 waves (k-split, so 4x as many
// loads in flight as a 128-row block), straight from global memory: lane (i, h) reads the 16
// contiguous floats k0 + 16h .. of row i of A and of B (the MFMA's permuted K, as above).  The
// waves' partial tiles are summed through LDS in a fixed order (wave 0 + 1 + 2 + 3), then the
// epilogue.  HBM-bound: 414 workgroups at M = 13248 instead of 104.
__global__ __launch_bounds__(256) void gemm_nt_thin_kernel(const NtArgs p) {
  __shared__ float red[3][16][64];
  const int tid = threadIdx.x, lane = tid & 63, half = lane >> 5, col = lane & 31, wave = tid >> 6;
  const int m0 = blockIdx.x * 32;
  const __amdgpu_buffer_rsrc_t ra = rsrc(p.A, ((long)(p.M - 1) * p.lda + p.K) * 4);
  const __amdgpu_buffer_rsrc_t rb = rsrc(p.B, ((long)(p.N - 1) * p.ldb + p.K) * 4);
  const int nk = (p.K + BK - 1) / BK;
  float4 a[4], b[4];
  auto load = [&](int kt) {
    const int k = kt * BK + 16 * half;
    const bool kin = kt < nk;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int kq = k + 4 * q;
      const int oa = (kin && m0 + col < p.M && kq < p.K) ? (int)(((long)(m0 + col) * p.lda + kq) * 4) : OOR;
      const int ob = (kin && col < p.N && kq < p.K) ? (int)(((long)col * p.ldb + kq) * 4) : OOR;
      a[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ra, oa, 0, 0));
      b[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rb, ob, 0, 0));
    }
  };
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  load(wave);
  for (int kt = wave; kt < nk; kt += 4) {
    float af[16], bf[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      af[4 * q] = a[q].x; af[4 * q + 1] = a[q].y; af[4 * q + 2] = a[q].z; af[4 * q + 3] = a[q].w;
      bf[4 * q] = b[q].x; bf[4 * q + 1] = b[q].y; bf[4 * q + 2] = b[q].z; bf[4 * q + 3] = b[q].w;
    }
    load(kt + 4);
#pragma unroll
    for (int j = 0; j < 16; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[j], bf[j], acc, 0, 0, 0);
  }
  if (wave > 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wave - 1][r][lane] = acc[r];
  }
  __syncthreads();
  if (wave > 0) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = ((acc[r] + red[0][r][lane]) + red[1][r][lane]) + red[2][r][lane];
  const __amdgpu_buffer_rsrc_t rc = rsrc(p.C, ((long)(p.M - 1) * p.ldc + p.N) * 4);
  const int n = col;
  const bool nok = n < p.N;
  const float bn = (p.bias && nok) ? p.bias[n] : 0.0f;
  float mk[16];
  if (p.mask) {
    const __amdgpu_buffer_rsrc_t rm = rsrc(p.mask, ((long)(p.M - 1) * p.ldmask + p.N) * 4);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + crow(r, half);
      mk[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                            rm, (nok && m < p.M) ? (int)(((long)m * p.ldmask + n) * 4) : OOR, 0, 0));
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + crow(r, half);
    const bool ok = nok && m < p.M;
    float v = acc[r] + bn;
    if (p.relu) v = fmaxf(v, 0.0f);
    if (p.mask) v = mk[r] > 0.0f ? v : 0.0f;
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rc, ok ? (int)(((long)m * p.ldc + n) * 4) : OOR,
                                          0, NT_STORE_AUX);
  }
}

// Small K (K <= 32, 16-B aligned rows: the head's end_conv_2 input gradient, K = 12): an
// element-wise streaming kernel.  Thread t owns output columns 4t .. 4t+3 and keeps their B rows
// (K x 4 floats) in registers; workgroups stride over the rows: per row one broadcast read of
// A's K values, one float4 of the mask, K x 4 FMAs, one float4 store.  HBM-bound (mask in, C out).
template <int KQ>
__global__ __launch_bounds__(256) void gemm_nt_smallk_kernel(const NtArgs p) {
  const int n4 = blockIdx.y * blockDim.x + threadIdx.x;  // column quad
  const int n = 4 * n4;
  const bool nok = n < p.N;
  float4 w[4][KQ];  // w[c][q] = B[n + c][4q .. 4q+3]
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int q = 0; q < KQ; ++q)
      w[c][q] = (nok && 4 * q < p.K) ? *(const float4*)(p.B + (long)(n + c) * p.ldb + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
  float4 bias = make_float4(0.f, 0.f, 0.f, 0.f);
  if (p.bias && nok) bias = *(const float4*)(p.bias + n);
  if (!nok) return;
  for (int m = blockIdx.x; m < p.M; m += gridDim.x) {
    const float* ar = p.A + (long)m * p.lda;
    float4 av[KQ];
#pragma unroll
    for (int q = 0; q < KQ; ++q) av[q] = (4 * q < p.K) ? *(const float4*)(ar + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 mk = make_float4(1.f, 1.f, 1.f, 1.f);
    if (p.mask) mk = *(const float4*)(p.mask + (long)m * p.ldmask + n);
    float o[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float v = 0.0f;
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        v = fmaf(av[q].x, w[c][q].x, v);
        v = fmaf(av[q].y, w[c][q].y, v);
        v = fmaf(av[q].z, w[c][q].z, v);
        v = fmaf(av[q].w, w[c][q].w, v);
      }
      o[c] = v;
    }
    const float bb[4] = {bias.x, bias.y, bias.z, bias.w};
    const float mm[4] = {mk.x, mk.y, mk.z, mk.w};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      o[c] += bb[c];
      if (p.relu) o[c] = fmaxf(o[c], 0.0f);
      if (p.mask) o[c] = mm[c] > 0.0f ? o[c] : 0.0f;
    }
    *(float4*)(p.C + (long)m * p.ldc + n) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

template <int BM, int BN, int WGM, int WGN>
void launch(const NtArgs& p, hipStream_t s) {
  dim3 grid((p.M + BM - 1) / BM, (p.N + BN - 1) / BN);
  gemm_nt_kernel<BM, BN, WGM, WGN><<<grid, 256, 0, s>>>(p);
}

inline bool al16(const void* q) { return ((uintptr_t)q & 15u) == 0; }

template <int BM, int BN, int WGM, int WGN>
void launch_bf16(const NtArgs& p, hipStream_t s) {
  const int nrow = (p.M + BM - 1) / BM, ncol = (p.N + BN - 1) / BN;
  gemm_nt_bf16_kernel<BM, BN, WGM, WGN><<<(nrow + 7) / 8 * 8 * ncol, 256, 0, s>>>(p, nrow, ncol);
}

}  // namespace

extern "C" int gwn_gemm_nt_bf16(const float* A, long lda, const float* B, long ldb, float* C, long ldc, int M,
                                int N, int K, const float* bias, int relu, const float* mask, long ldmask,
                                hipStream_t s) {
  GWN_REQUIRE(A && B && C && M > 0 && K > 0 && N >= 64 && N % 64 == 0, "gemm_nt_bf16: bad shape (N a multiple of 64)");
  GWN_REQUIRE(K % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 && al16(A) && al16(B),
              "gemm_nt_bf16: K, lda, ldb must be multiples of 4 and A, B 16-B aligned");
  GWN_REQUIRE(lda >= K && ldb >= K && ldc >= N && (!mask || ldmask >= N), "gemm_nt_bf16: leading dimensions");
  GWN_REQUIRE(((long)M * lda + K) * 4 < 0x7fff0000L && ((long)N * ldb + K) * 4 < 0x7fff0000L &&
                  ((long)M * ldc + N) * 4 < 0x7fff0000L,
              "gemm_nt_bf16: operand beyond a 2 GB buffer window");
  NtArgs p = {A, lda, B, ldb, C, ldc, M, N, K, bias, relu, mask, ldmask};
  if (N % 128 == 0 && (long)((M + 127) / 128) * (N / 128) >= 384) launch_bf16<128, 128, 2, 2>(p, s);
  else launch_bf16<128, 64, 2, 2>(p, s);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

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
  // small K (the K x 4 B values per thread fit in registers) and 16-B aligned rows everywhere
  const bool quads = N % 4 == 0 && K % 4 == 0 && ldc % 4 == 0 && al16(C) && (!bias || al16(bias)) &&
                     (!mask || (ldmask % 4 == 0 && al16(mask)));
  if (K <= 32 && N >= 64 && quads) {
    const int kq = K / 4;
    const int threads = N / 4 < 256 ? N / 4 : 256;
    dim3 grid(M < 2048 ? M : 2048, (N / 4 + threads - 1) / threads);
    switch (kq) {
      case 1: gemm_nt_smallk_kernel<1><<<grid, threads, 0, s>>>(p); break;
      case 2: gemm_nt_smallk_kernel<2><<<grid, threads, 0, s>>>(p); break;
      case 3: gemm_nt_smallk_kernel<3><<<grid, threads, 0, s>>>(p); break;
      case 4: gemm_nt_smallk_kernel<4><<<grid, threads, 0, s>>>(p); break;
      case 5: gemm_nt_smallk_kernel<5><<<grid, threads, 0, s>>>(p); break;
      case 6: gemm_nt_smallk_kernel<6><<<grid, threads, 0, s>>>(p); break;
      case 7: gemm_nt_smallk_kernel<7><<<grid, threads, 0, s>>>(p); break;
      default: gemm_nt_smallk_kernel<8><<<grid, threads, 0, s>>>(p); break;
    }
    GWN_CHECK_LAUNCH();
    return GWN_OK;
  }
  // tile choice: enough workgroups for 256 CUs (two resident per CU), wide N tiles when N allows
  if (N <= 32) gemm_nt_thin_kernel<<<(M + 31) / 32, 256, 0, s>>>(p);
  else if (N % 128 == 0 && (long)((M + 127) / 128) * (N / 128) >= 384) launch<128, 128, 2, 2>(p, s);
  else launch<128, 64, 2, 2>(p, s);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

extern "C" int gwn_wgrad_bf16_partial_count(int R, int J, int Kc) {
  if (R <= 0 || J <= 0 || Kc <= 0 || J % 128 || Kc % 128) return 0;
  const int ntiles = (J / 128) * (Kc / 128);
  // about two workgroups per CU, but at least 12 row steps (384 rows) per workgroup
  int ns = (2 * gwn_device_cus() + ntiles - 1) / ntiles;
  const int cap = R / 384 > 1 ? R / 384 : 1;
  ns = ns < cap ? ns : cap;
  return ns < 1 ? 1 : ns;
}

extern "C" int gwn_wgrad_bf16_partials(const float* dY, long ldy, int J, const float* X, long ldx, int Kc, int R,
                                       float* part, hipStream_t s) {
  GWN_REQUIRE(dY && X && part && R > 0 && J > 0 && Kc > 0 && J % 128 == 0 && Kc % 128 == 0,
              "wgrad_bf16: J and Kc multiples of 128, R > 0");
  GWN_REQUIRE(ldy >= J && ldx >= Kc, "wgrad_bf16: leading dimensions");
  GWN_REQUIRE((long)R * ldy * 4 < 0x7fff0000L && (long)R * ldx * 4 < 0x7fff0000L,
              "wgrad_bf16: operand beyond a 2 GB buffer window");
  const int ns = gwn_wgrad_bf16_partial_count(R, J, Kc);
  WgB p = {dY, ldy, X, ldx, part, J, Kc, R, ns};
  wgrad_bf16_kernel<<<(ns + 7) / 8 * 8 * (J / 128) * (Kc / 128), 256, 0, s>>>(p);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}
