// Generic fp32 GEMM on the CDNA4 f32-input MFMA (v_mfma_f32_32x32x2_f32, exact fp32 fma chain).
//
// One kernel template serves every matrix-shaped step of the Graph WaveNet hot path:
//   * diffusion  y_s = A^T x_s   (nconv, model.py:12-14)   M = nodes, N = slices*C, K = nodes
//   * 1x1 / dilated convs        (model.py:135-151, 161-169) M = positions, N = C_out, K = C_in*taps
//   * weight / adjacency grads   (their backward)           K = positions or slices*C, split-K
// Tiles are staged k-major through LDS (double buffered, register prefetch of the next k-tile,
// one barrier per k-tile); every wave owns TM x TN 32x32 accumulator tiles (16 VGPRs each).
#include "gwn_internal.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int BK = 16;

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// Shared epilogue for EPI_STORE / EPI_MASKGRAD (also used by the split-K reduction).
__device__ __forceinline__ void epi_store(const GemmParams& p, int m, int n, float v,
                                          unsigned long long seed, long cofs = 0) {
  if (p.epi == EPI_MASKGRAD) {
    v = (p.mask[(long)m * p.ldmask_m + n] > 0.0f) ? v : 0.0f;
  } else {
    if (p.bias_n) v += p.bias_n[n];
    if (p.relu) v = fmaxf(v, 0.0f);
    if (p.drop_p > 0.0f) {
      float u = gwn_uniform(seed, p.seed_salt, (unsigned long long)m * (unsigned)p.N + n);
      v = (u >= p.drop_p) ? v * (1.0f / (1.0f - p.drop_p)) : 0.0f;
    }
  }
  const int no = n / p.c_nin, ni = n - no * p.c_nin;  // C0 shares the column map of C
  if (p.C0) v += p.beta * p.C0[cofs + (long)m * p.ldc0_m + (long)ni * p.ldc0_n + (long)no * p.c0_no_stride];
  p.C[cofs + (long)m * p.ldc_m + (long)ni * p.ldc_n + (long)no * p.c_no_stride] = v;
}

// Operands are staged as "quads": 4 consecutive elements along the operand's contiguous
// dimension (k for AKC/BKC, m or n otherwise).  vec_a / vec_b (host-checked alignment) turn a
// quad into one 16-B global load; otherwise the quad is 4 guarded scalar loads.
template <int WM, int WN, int TM, int TN, bool AKC, bool BKC>
__global__ __launch_bounds__(64 * WM * WN) void gemm_kernel(const GemmParams p, const int vec_a,
                                                           const int vec_b) {
  constexpr int NT = 64 * WM * WN;
  constexpr int BM = WM * TM * 32;
  constexpr int BN = WN * TN * 32;
  constexpr int LDA = BM + 4;
  constexpr int LDB = BN + 4;
  constexpr int AQ = BM * BK / 4, BQ = BN * BK / 4;
  constexpr int A_PER = (AQ + NT - 1) / NT;
  constexpr int B_PER = (BQ + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) float As[2][BK * LDA];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK * LDB];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  // blockIdx.z: the split-K index, or the batch index of a batched launch (ksplit == 1 then)
  const bool batched = p.batch > 1;
  const int split = batched ? 0 : (int)blockIdx.z;
  const long bz = batched ? (long)blockIdx.z : 0;
  const float* __restrict__ Ap = p.A + bz * p.a_bstride;
  const float* __restrict__ Bp = p.B + bz * p.b_bstride;
  const long cofs = bz * p.c_bstride;
  const int kbeg = split * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);

  const bool a_tiled = (p.a_kin % BK == 0) || (p.a_kin >= p.K);
  const bool b_tiled = (p.b_kin % BK == 0) || (p.b_kin >= p.K);
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  float4 ra[A_PER], rb[B_PER];

  // scalar element loads (any layout; per-element two-level index when the tile straddles)
  auto a_elem = [&](int m, int k, int ko0) -> float {
    if (m >= p.M || k >= kend) return 0.0f;
    const int ko = a_tiled ? ko0 : (int)((unsigned)k / (unsigned)p.a_kin);
    const int ki = k - ko * p.a_kin;
    const int srow = m + ko * p.a_row_shift;
    if (srow < 0 || srow >= p.a_rows) return 0.0f;
    return Ap[(long)srow * p.lda_m + (long)ki * p.lda_k + (long)ko * p.a_ko_stride];
  };
  auto b_elem = [&](int k, int n, int kb0) -> float {
    if (n >= p.N || k >= kend) return 0.0f;
    const int kb = b_tiled ? kb0 : (int)((unsigned)k / (unsigned)p.b_kin);
    const int kj = k - kb * p.b_kin;
    const int no = (unsigned)n / (unsigned)p.b_nin, ni = n - no * p.b_nin;
    return Bp[(long)kj * p.ldb_k + (long)kb * p.b_ko_stride + (long)ni * p.ldb_n + (long)no * p.b_no_stride];
  };

  auto load = [&](int k0) {
    // k-tiles never straddle an a_kin block when a_kin % BK == 0 (the hot configurations);
    // otherwise (e.g. NCHW slices with T = 12 inner steps) the block is resolved per element.
    const int ko0 = k0 / p.a_kin;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int q = tid + i * NT;
      float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      if (q < AQ) {
        if (AKC) {  // quad = 4 consecutive k of row m
          const int m = m0 + q / (BK / 4), k = k0 + (q % (BK / 4)) * 4;
          const int srow = m + ko0 * p.a_row_shift;
          if (vec_a && m < p.M && k + 3 < kend && srow >= 0 && srow < p.a_rows) {
            v = *(const float4*)(Ap + (long)srow * p.lda_m + (k - ko0 * p.a_kin) + (long)ko0 * p.a_ko_stride);
          } else {
            v.x = a_elem(m, k, ko0); v.y = a_elem(m, k + 1, ko0);
            v.z = a_elem(m, k + 2, ko0); v.w = a_elem(m, k + 3, ko0);
          }
        } else {  // quad = 4 consecutive m at one k
          const int k = k0 + q / (BM / 4), m = m0 + (q % (BM / 4)) * 4;
          const int srow = m + ko0 * p.a_row_shift;
          if (vec_a && k < kend && m + 3 < p.M && srow >= 0 && srow + 3 < p.a_rows) {
            v = *(const float4*)(Ap + srow + (long)(k - ko0 * p.a_kin) * p.lda_k + (long)ko0 * p.a_ko_stride);
          } else {
            v.x = a_elem(m, k, ko0); v.y = a_elem(m + 1, k, ko0);
            v.z = a_elem(m + 2, k, ko0); v.w = a_elem(m + 3, k, ko0);
          }
        }
      }
      ra[i] = v;
    }
    const int kb0 = k0 / p.b_kin;
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int q = tid + i * NT;
      float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      if (q < BQ) {
        if (BKC) {  // quad = 4 consecutive k of column n
          const int n = n0 + q / (BK / 4), k = k0 + (q % (BK / 4)) * 4;
          if (vec_b && n < p.N && k + 3 < kend) {
            const int no = (unsigned)n / (unsigned)p.b_nin, ni = n - no * p.b_nin;
            v = *(const float4*)(Bp + (k - kb0 * p.b_kin) + (long)kb0 * p.b_ko_stride + (long)ni * p.ldb_n +
                                 (long)no * p.b_no_stride);
          } else {
            v.x = b_elem(k, n, kb0); v.y = b_elem(k + 1, n, kb0);
            v.z = b_elem(k + 2, n, kb0); v.w = b_elem(k + 3, n, kb0);
          }
        } else {  // quad = 4 consecutive n at one k
          const int k = k0 + q / (BN / 4), n = n0 + (q % (BN / 4)) * 4;
          if (vec_b && k < kend && n + 3 < p.N) {
            const int no = (unsigned)n / (unsigned)p.b_nin, ni = n - no * p.b_nin;
            v = *(const float4*)(Bp + (long)(k - kb0 * p.b_kin) * p.ldb_k + (long)kb0 * p.b_ko_stride + ni +
                                 (long)no * p.b_no_stride);
          } else {
            v.x = b_elem(k, n, kb0); v.y = b_elem(k, n + 1, kb0);
            v.z = b_elem(k, n + 2, kb0); v.w = b_elem(k, n + 3, kb0);
          }
        }
      }
      rb[i] = v;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int q = tid + i * NT;
      if (q >= AQ) continue;
      if (AKC) {
        const int mm = q / (BK / 4), kk = (q % (BK / 4)) * 4;
        As[buf][kk * LDA + mm] = ra[i].x;
        As[buf][(kk + 1) * LDA + mm] = ra[i].y;
        As[buf][(kk + 2) * LDA + mm] = ra[i].z;
        As[buf][(kk + 3) * LDA + mm] = ra[i].w;
      } else {
        const int kk = q / (BM / 4), mm = (q % (BM / 4)) * 4;
        *(float4*)&As[buf][kk * LDA + mm] = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int q = tid + i * NT;
      if (q >= BQ) continue;
      if (BKC) {
        const int nn = q / (BK / 4), kk = (q % (BK / 4)) * 4;
        Bs[buf][kk * LDB + nn] = rb[i].x;
        Bs[buf][(kk + 1) * LDB + nn] = rb[i].y;
        Bs[buf][(kk + 2) * LDB + nn] = rb[i].z;
        Bs[buf][(kk + 3) * LDB + nn] = rb[i].w;
      } else {
        const int kk = q / (BN / 4), nn = (q % (BN / 4)) * 4;
        *(float4*)&Bs[buf][kk * LDB + nn] = rb[i];
      }
    }
  };

  const int nkt = (kend > kbeg) ? (kend - kbeg + BK - 1) / BK : 0;
  // ones column: the first column-tile's threads tid < BM also sum the staged A tile along k
  const bool do_ones = p.ones_out != nullptr && blockIdx.y == 0;
  float rsum = 0.0f;
  if (nkt > 0) {
    load(kbeg);
    store(0);
    __syncthreads();
  }
  for (int kt = 0; kt < nkt; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nkt) load(kbeg + (kt + 1) * BK);
    const float* as = &As[buf][0];
    const float* bs = &Bs[buf][0];
    if (do_ones && tid < BM) {
#pragma unroll
      for (int kk = 0; kk < BK; ++kk) rsum += as[kk * LDA + tid];
    }
#pragma unroll
    for (int kp = 0; kp < BK / 2; ++kp) {
      const int krow = 2 * kp + (lane >> 5);
      float a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = as[krow * LDA + (wm * TM + i) * 32 + (lane & 31)];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = bs[krow * LDB + (wn * TN + j) * 32 + (lane & 31)];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nkt) store(buf ^ 1);
    __syncthreads();
  }

  if (do_ones && tid < BM && m0 + tid < p.M) {
    const float v = p.alpha * rsum;
    if (p.ksplit > 1) p.part[(long)p.ksplit * p.M * p.N + (long)split * p.M + m0 + tid] = v;
    else p.ones_out[m0 + tid] = v;
  }
  // epilogue: the mode branch is hoisted out of the (fully unrolled) accumulator walk
  auto walk = [&](auto&& f) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + (wn * TN + j) * 32 + (lane & 31);
#pragma unroll
        for (int r = 0; r < 16; ++r)
          f(m0 + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5), n, p.alpha * acc[i][j][r]);
      }
  };
  if (p.ksplit > 1) {
    float* part = p.part + (long)split * p.M * p.N;
    walk([&](int m, int n, float v) {
      if (m < p.M && n < p.N) part[(long)m * p.N + n] = v;
    });
  } else if (p.epi == EPI_GATE) {
    // column n = 2c + g: g=0 filter (tanh), g=1 gate (sigmoid); partner lives in lane^1
    walk([&](int m, int n, float v) {
      v += (n < p.N) ? p.bias_n[n] : 0.0f;
      const float other = __shfl_xor(v, 1);
      if (((lane & 1) == 0) && m < p.M && n < p.N) {
        const float f = tanhf(v), g = sigmoidf_(other);
        const float xg = f * g;
        const int c = n >> 1;
        p.C[(long)m * p.ldc_m + c] = xg;
        p.aux[(long)m * p.ld_aux + n] = f;
        p.aux[(long)m * p.ld_aux + n + 1] = g;
        if (p.aux2 && m >= p.aux2_row0) p.aux2[(long)(m - p.aux2_row0) * p.ld_aux2 + c] = xg;
      }
    });
  } else {
    const unsigned long long seed = p.seed_ptr ? *p.seed_ptr : 0ull;
    walk([&](int m, int n, float v) {
      if (m < p.M && n < p.N) epi_store(p, m, n, v, seed, cofs);
    });
  }
}

// 32 consecutive outputs per block x 8 split lanes (lane l sums splits l, l+8, ...; each wave-load
// covers two 128-B segments), then a fixed-order tree over the 8 lanes.
// Outputs [M*N, M*N + M) are the ones column (partials stored after all [ksplit][M][N] tiles).
__global__ void splitk_reduce_kernel(const GemmParams p) {
  __shared__ float sh[256];
  const long mn = (long)p.M * p.N;
  const long total = mn + (p.ones_out ? p.M : 0);
  const int ej = threadIdx.x & 31, lane = threadIdx.x >> 5;
  const long idx = blockIdx.x * 32L + ej;
  // four independent chains per lane keep four loads in flight; merged in a fixed order
  float v0 = 0.0f, v1 = 0.0f, v2 = 0.0f, v3 = 0.0f;
  if (idx < total) {
    const float* q = idx < mn ? p.part + idx : p.part + (long)p.ksplit * mn + (idx - mn);
    const long st = idx < mn ? mn : p.M;
    int s = lane;
    for (; s + 24 < p.ksplit; s += 32) {
      v0 += q[(long)s * st];
      v1 += q[(long)(s + 8) * st];
      v2 += q[(long)(s + 16) * st];
      v3 += q[(long)(s + 24) * st];
    }
    for (; s < p.ksplit; s += 8) v0 += q[(long)s * st];
  }
  sh[threadIdx.x] = (v0 + v1) + (v2 + v3);
  __syncthreads();
#pragma unroll
  for (int w = 4; w > 0; w >>= 1) {
    if (lane < w) sh[threadIdx.x] += sh[threadIdx.x + 32 * w];
    __syncthreads();
  }
  if (lane == 0 && idx >= mn && idx < total) {
    p.ones_out[idx - mn] = sh[ej];
  } else if (lane == 0 && idx < mn) {
    const unsigned long long seed = p.seed_ptr ? *p.seed_ptr : 0ull;
    const int m = (int)(idx / p.N), n = (int)(idx - (long)m * p.N);
    epi_store(p, m, n, sh[ej], seed);
  }
}

template <int WM, int WN, int TM, int TN>
int launch_cfg(const GemmParams& p, bool akc, bool bkc, int va, int vb, hipStream_t s) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  dim3 grid((p.M + BM - 1) / BM, (p.N + BN - 1) / BN, p.batch > 1 ? p.batch : p.ksplit);
  dim3 block(64 * WM * WN);
  if (akc && bkc) gemm_kernel<WM, WN, TM, TN, true, true><<<grid, block, 0, s>>>(p, va, vb);
  else if (akc) gemm_kernel<WM, WN, TM, TN, true, false><<<grid, block, 0, s>>>(p, va, vb);
  else if (bkc) gemm_kernel<WM, WN, TM, TN, false, true><<<grid, block, 0, s>>>(p, va, vb);
  else gemm_kernel<WM, WN, TM, TN, false, false><<<grid, block, 0, s>>>(p, va, vb);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

inline bool al16(const void* ptr) { return ((uintptr_t)ptr & 15u) == 0; }
inline bool m4(long v) { return (v & 3) == 0; }

}  // namespace

int gwn_gemm_launch(const GemmParams& pin, hipStream_t s) {
  GemmParams p = pin;
  GWN_REQUIRE(p.M > 0 && p.N > 0 && p.K >= 0, "gemm: bad shape");
  if (p.a_kin <= 0 || p.a_kin > p.K) p.a_kin = (p.K > 0 ? p.K : 1);
  if (p.b_kin <= 0 || p.b_kin > p.K) p.b_kin = (p.K > 0 ? p.K : 1);
  if (p.b_nin <= 0 || p.b_nin > p.N) p.b_nin = p.N;
  if (p.c_nin <= 0 || p.c_nin > p.N) p.c_nin = p.N;
  if (p.a_rows <= 0) p.a_rows = 0x7fffffff;
  GWN_REQUIRE(p.C != nullptr && p.A != nullptr && p.B != nullptr, "gemm: null operand");
  GWN_REQUIRE(p.epi != EPI_GATE || (p.ksplit <= 1 && p.aux && p.bias_n && (p.N % 2) == 0),
              "gemm: gate epilogue needs aux, bias, even N and no split-K");
  GWN_REQUIRE(p.epi != EPI_MASKGRAD || p.mask, "gemm: mask-grad epilogue needs a mask");
  GWN_REQUIRE(p.ones_out == nullptr || p.epi != EPI_GATE, "gemm: ones column is not combined with the gate epilogue");
  if (p.ksplit < 1) p.ksplit = 1;
  if (p.batch > 1)
    GWN_REQUIRE(p.ksplit == 1 && p.epi == EPI_STORE && !p.ones_out && !p.mask && !p.aux && p.batch <= 65535,
                "gemm: a batched launch needs ksplit 1, the store epilogue, no ones column / mask / aux");
  if (p.ksplit > 1) {
    GWN_REQUIRE(p.part != nullptr, "gemm: split-K needs a partial buffer");
    int chunk = (p.K + p.ksplit - 1) / p.ksplit;
    chunk = (chunk + BK - 1) / BK * BK;
    p.kchunk = chunk;
    p.ksplit = (p.K + chunk - 1) / chunk;
    if (p.ksplit < 1) p.ksplit = 1;
  } else {
    p.kchunk = p.K > 0 ? (p.K + BK - 1) / BK * BK : BK;
  }
  const bool akc = (p.lda_k == 1 && p.lda_m != 1);
  const bool bkc = (p.ldb_k == 1 && p.ldb_n != 1);
  const bool a_tiled = (p.a_kin % BK == 0) || (p.a_kin >= p.K);
  const bool b_tiled = (p.b_kin % BK == 0) || (p.b_kin >= p.K);
  // 16-B quads are legal when the quad never straddles an index block and every stride that
  // moves between quads is a multiple of 4 floats
  const bool bat = p.batch > 1;
  const int va = al16(p.A) && (!bat || m4(p.a_bstride)) && a_tiled && m4(p.a_ko_stride) && m4(p.a_kin) &&
                 (akc ? m4(p.lda_m) : (p.lda_m == 1 && m4(p.lda_k) && m4(p.a_row_shift)));
  const int vb = al16(p.B) && (!bat || m4(p.b_bstride)) && b_tiled && m4(p.b_ko_stride) && m4(p.b_no_stride) && m4(p.b_kin) &&
                 (bkc ? m4(p.ldb_n) : (p.ldb_n == 1 && m4(p.ldb_k) && m4(p.b_nin)));
  // tile choice: the largest tile that still gives >= 2 workgroups per CU (512), else the one with
  // the most workgroups; thin dimensions get thin tiles
  auto nblk = [&](int bm, int bn) {
    return (long)((p.M + bm - 1) / bm) * ((p.N + bn - 1) / bn) * (p.batch > 1 ? p.batch : p.ksplit);
  };
  constexpr long FILL = 512;
  int rc;
  if (p.M <= 32 && p.N <= 32) rc = launch_cfg<1, 1, 1, 1>(p, akc, bkc, va, vb, s);        // 32 x 32
  else if (p.M <= 32 && p.N <= 224) rc = launch_cfg<1, 7, 1, 1>(p, akc, bkc, va, vb, s);  // 32 x 224
  else if (p.N <= 32)
    rc = nblk(256, 32) >= FILL ? launch_cfg<4, 1, 2, 1>(p, akc, bkc, va, vb, s)          // 256 x 32
                               : launch_cfg<1, 1, 1, 1>(p, akc, bkc, va, vb, s);         // 32 x 32
  else if (p.N <= 64 && p.M <= 64) rc = launch_cfg<2, 2, 1, 1>(p, akc, bkc, va, vb, s);   // 64 x 64
  else if (p.N <= 64 && p.M > 128 && p.M <= 224) rc = launch_cfg<7, 1, 1, 2>(p, akc, bkc, va, vb, s);  // 224 x 64
  else if (p.N <= 64)
    rc = nblk(128, 64) >= FILL ? launch_cfg<4, 1, 1, 2>(p, akc, bkc, va, vb, s)          // 128 x 64
                               : launch_cfg<2, 2, 1, 1>(p, akc, bkc, va, vb, s);
  else if (p.M > 160 && p.M <= 224) rc = launch_cfg<7, 1, 1, 2>(p, akc, bkc, va, vb, s);
  else if (p.M >= 128 && nblk(128, 128) >= FILL) rc = launch_cfg<2, 2, 2, 2>(p, akc, bkc, va, vb, s);  // 128 x 128
  else rc = launch_cfg<2, 2, 1, 1>(p, akc, bkc, va, vb, s);                               // 64 x 64
  if (rc != GWN_OK || p.ksplit <= 1) return rc;
  const long total = (long)p.M * p.N + (p.ones_out ? p.M : 0);
  splitk_reduce_kernel<<<(unsigned)((total + 31) / 32), 256, 0, s>>>(p);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}
