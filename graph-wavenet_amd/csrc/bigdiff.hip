// Large-graph diffusion (nconv, model.py:12-14, for n > 512: the N = 2048 dense-graph config):
//     Y_s[w][c] (+)= sum_v G[v][w] X_s[v][c]        for every slice s (c = 32 channels)
// as ONE GEMM over all slices: M = n (w), N = slices * 32 ((s, c) two-level), K = n (v), with the
// support G streamed through LDS in 32-row K tiles (the 16 MB support of N = 2048 is L2 / MALL
// resident and read once per column block of 256 outputs), shared by 8 slices per workgroup.
//
// Workgroup tile 256 (w) x 256 (8 slices x 32 channels), 8 waves, each 2 x 4 accumulator tiles of
// v_mfma_f32_32x32x2_f32 (exact fp32 FMA chains; 8 independent chains per wave, so the 64-cycle
// dependent latency never stalls the matrix pipe).  Both operands are staged k-major in LDS
// (G rows = v, contiguous w; X rows = v, contiguous (s, c)), double buffered, the next tile's
// 16-B global loads in flight while the current tile's 128 MFMAs per wave run.  XCD-aware block
// order: the 8 column blocks (w) of one slice group run on one XCD, so the slice group's X tiles
// are shared in that XCD's L2.
#include "gwn_internal.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int BM = 256, BN = 256, BK = 32;
constexpr int WM = 2, WN = 4;          // wave grid (m, n)
constexpr int TM = 4, TN = 2;          // 32x32 tiles per wave: 128 x 64
constexpr int NT = 64 * WM * WN;       // 512 threads
constexpr int LDA = BM + 4, LDB = BN + 4;
constexpr int NXCD = 8;

struct BigDiff {
  const float* G; int ldg, np;          // G [np][ldg], zero outside [n][n]
  const float* X; long ldx;             // X [slices * n][ldx], channels 0..31
  float* Y; long ldy;                   // Y [slices * n][ldy]
  const float* Y0; long ldy0;           // optional addend (may alias Y)
  int n, slices;
};

__device__ __forceinline__ int crow(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }

__global__ __launch_bounds__(NT, 1) void bigdiff_kernel(const BigDiff p) {
  __shared__ __attribute__((aligned(16))) float As[2][BK * LDA];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK * LDB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int mblocks = (p.n + BM - 1) / BM;
  const int sgroups = (p.slices + 7) / 8;
  // XCD-aware order: blocks b and b + 8 share an XCD; the column blocks of one slice group take
  // consecutive j = b / 8 on the same XCD
  const int b = blockIdx.x, xcd = b % NXCD, j = b / NXCD;
  const int mb = j % mblocks, sg = (j / mblocks) * NXCD + xcd;
  if (sg >= sgroups) return;
  const int m0 = mb * BM, s0 = sg * 8;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int jj = 0; jj < TN; ++jj)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][jj][r] = 0.0f;

  // per thread: 4 float4 of the G tile (row k, 4 consecutive w) and 4 of the X tile (slice, row k, 4 channels)
  float4 ra[4], rb[4];
  auto load = [&](int k0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + q * NT;            // 0 .. 2047
      const int kk = e >> 6, mq = (e & 63) * 4;
      const int v = k0 + kk, w = m0 + mq;
      ra[q] = (v < p.np && w + 3 < p.np) ? *(const float4*)(p.G + (long)v * p.ldg + w) : make_float4(0.f, 0.f, 0.f, 0.f);
      const int sl = e >> 8, rem = e & 255, kk2 = rem >> 3, cq = (rem & 7) * 4;
      const int s = s0 + sl, v2 = k0 + kk2;
      rb[q] = (s < p.slices && v2 < p.n) ? *(const float4*)(p.X + ((long)s * p.n + v2) * p.ldx + cq)
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + q * NT;
      const int kk = e >> 6, mq = (e & 63) * 4;
      *(float4*)&As[buf][kk * LDA + mq] = ra[q];
      const int sl = e >> 8, rem = e & 255, kk2 = rem >> 3, cq = (rem & 7) * 4;
      *(float4*)&Bs[buf][kk2 * LDB + sl * 32 + cq] = rb[q];
    }
  };

  const int nkt = (p.n + BK - 1) / BK;
  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nkt) load((kt + 1) * BK);
    const float* as = &As[buf][0];
    const float* bs = &Bs[buf][0];
#pragma unroll
    for (int kp = 0; kp < BK / 2; ++kp) {
      const int krow = 2 * kp + (lane >> 5);
      float a[TM], bv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = as[krow * LDA + (wm * TM + i) * 32 + (lane & 31)];
#pragma unroll
      for (int jj = 0; jj < TN; ++jj) bv[jj] = bs[krow * LDB + (wn * TN + jj) * 32 + (lane & 31)];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int jj = 0; jj < TN; ++jj)
          acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], bv[jj], acc[i][jj], 0, 0, 0);
    }
    if (kt + 1 < nkt) store(buf ^ 1);
    __syncthreads();
  }
  // epilogue: D[w][(s, c)] -> Y[s*n + w][c]; lanes = c (32 consecutive floats per row segment)
  const int c = lane & 31, half = lane >> 5;
#pragma unroll
  for (int jj = 0; jj < TN; ++jj) {
    const int s = s0 + wn * TN + jj;
    if (s >= p.slices) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int w = m0 + (wm * TM + i) * 32 + crow(r, half);
        if (w >= p.n) continue;
        const long row = (long)s * p.n + w;
        float v = acc[i][jj][r];
        if (p.Y0) v += p.Y0[row * p.ldy0 + c];
        p.Y[row * p.ldy + c] = v;
      }
    }
  }
}

inline bool al16(const void* q) { return ((uintptr_t)q & 15u) == 0; }

}  // namespace

bool gwn_bigdiff_eligible(int n, int c, const float* G, int ldg, const float* x, long ldx, const float* y, long ldy,
                          const float* y0, long ldy0) {
  return n > 512 && c == 32 && al16(G) && (ldg & 3) == 0 && ldg >= n && al16(x) && (ldx & 3) == 0 && al16(y) &&
         (ldy & 3) == 0 && (!y0 || (al16(y0) && (ldy0 & 3) == 0));
}

// y_s = G^T x_s (+ y0) for every slice, G = the padded support [np][ldg] (np = 32*ceil(n/32))
int gwn_bigdiff(const float* G, int ldg, const float* x, long ldx, float* y, long ldy, const float* y0, long ldy0,
                int n, int slices, hipStream_t s) {
  GWN_REQUIRE(n > 0 && slices > 0, "bigdiff: bad shape");
  BigDiff p;
  p.G = G; p.ldg = ldg; p.np = (n + 31) / 32 * 32;
  p.X = x; p.ldx = ldx; p.Y = y; p.ldy = ldy; p.Y0 = y0; p.ldy0 = ldy0;
  p.n = n; p.slices = slices;
  GWN_REQUIRE(p.np <= ldg, "bigdiff: support rows shorter than 32*ceil(n/32)");
  const int mblocks = (n + BM - 1) / BM;
  const int sgroups = (slices + 7) / 8;
  const int blocks = ((sgroups + NXCD - 1) / NXCD) * NXCD * mblocks;
  GWN_DEBUG_RANGE(G, ((long)(p.np - 1) * ldg + p.np) * 4, "bigdiff G");
  GWN_DEBUG_RANGE(x, (((long)slices * n - 1) * ldx + 32) * 4, "bigdiff x");
  GWN_DEBUG_RANGE(y, (((long)slices * n - 1) * ldy + 32) * 4, "bigdiff y");
  bigdiff_kernel<<<blocks, NT, 0, s>>>(p);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}
