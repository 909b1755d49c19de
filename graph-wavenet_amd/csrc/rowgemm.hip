// Weight-stationary row GEMM for the gated TCN (model.py:206-212) and its input gradient:
//     Y[m][n] = epi( sum_{h<2} sum_{j<KH} A[m + h*shift][h*a_tap + j] * B(h*KH + j, n) )
// i.e. a K = 2*KH contraction whose two halves are the two taps of the dilated (1 x 2) kernel
// (rows m and m + shift).  M is large (all positions), K and N are small (<= 128, <= 64).
//
// The K dimension is laid onto v_mfma_f32_32x32x2_f32 PERMUTED: MFMA step j takes, in lane half h,
// k = h*KH + j (instead of 2j + h).  Then lane (i, h) needs the KH contiguous floats
// A[m0 + i + h*shift][h*a_tap .. +KH) — one row segment, read with 16-B loads straight into the
// A-operand registers — and the weights B(h*KH + j, n) sit in registers for the whole kernel.
// LDS only stages the weights once per block; after that each wave streams 32-row chunks with no
// barrier, the next chunk's loads in flight while the current chunk's MFMAs run.  The accumulator layout (col = lane&31 = n, rows on
// registers) writes two 128-B row segments per store instruction.
#include "gwn_internal.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

struct RowGemm {
  const float* A; long lda; int a_rows; long shift; int a_tap;  // tap h reads row m + h*shift, col h*a_tap
  const float* B; long ldb_k, ldb_tap, ldb_n;                   // B(h*KH + j, n) = B[j*ldb_k + h*ldb_tap + n*ldb_n]
  float* C; long ldc;                                            // STORE: C[m][n] (+= C0 if accumulate)
  int accumulate;
  const float* bias;                                             // GATE: bias[n]
  float* aux; long ld_aux;                                       // GATE: aux[m][n] = tanh f / sigmoid g
  float* aux2; long ld_aux2; int aux2_row0;                      // GATE: skip copy of xg for m >= row0
  int M, ntiles;                                                 // N = 32 * ntiles
  long acc_row0;                                                 // STORE + accumulate: rows < acc_row0 not accumulated
  const float* bn_z; const float* bn_mean; const float* bn_rstd; // BNSTAT: per-wave partials of sum C and
  float* bn_part;                                                //   sum C*xhat(bn_z), [wave][2][32]
  const float* center;                                           // CENTER: A[.][h*a_tap + j] - center[j]
};

// gate nonlinearities: gwn_gate_sigmoid / gwn_gate_tanh (gwn_internal.h)
__device__ __forceinline__ float sigmoidf_(float x) { return gwn_gate_sigmoid(x); }
__device__ __forceinline__ float tanhf_(float x) { return gwn_gate_tanh(x); }
__device__ __forceinline__ int crow(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }

// Each wave walks 32-row chunks (grid stride).  Every global access goes through a buffer
// resource: rows outside the operand give an out-of-range offset, which the hardware turns into
// a zero load or a dropped store — no branches, no exec masking, and the waits stay counted
// (the next chunk's loads remain in flight across the epilogue).
constexpr int OOR = 0x7ffffff0;  // out-of-range byte offset

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}
// output stores non-temporal (cache policy 2): gated forward 133 -> 122 us per METR step
constexpr int ST_AUX = 2;
__device__ __forceinline__ void st32(__amdgpu_buffer_rsrc_t r, int off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, off, 0, ST_AUX);
}
__device__ __forceinline__ float ld32(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}

// GATE: one wave computes both column tiles of a chunk — filter f = cols 2c (tile 0) and gate
// g = cols 2c+1 (tile 1) — so every lane owns channel c = col of both and writes full rows:
// xg[m][c] = tanh(f) * sigmoid(g) (128 B per row) and fg[m][2c .. 2c+1] = (tanh f, sigmoid g).
// STORE: ntiles waves share a chunk, one 32-column tile each.
// The stationary weights stay in LDS ([row][2 KH + 4]: 2 KH + 4 = 4 mod 64, so the 16 lanes of a
// ds_read_b128 pass hit distinct banks) and are read four k-steps at a time next to the MFMAs,
// instead of 2 KH registers per lane (228-288 registers, one wave per SIMD) -> two waves per SIMD.
template <int KH, bool GATE, bool BNSTAT, bool CENTER = false>
__global__ __launch_bounds__(256) void rowgemm_kernel(const RowGemm p) {
  constexpr int NQ = KH / 4;  // float4 per lane per chunk
  constexpr int NT = GATE ? 2 : 1;
  const int lane = threadIdx.x & 63, half = lane >> 5, col = lane & 31;
  const int nchunks = (p.M + 31) >> 5;
  const int ntiles = GATE ? 1 : p.ntiles;
  const int gw = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  const int tile = gw % ntiles;
  const int wave = gw / ntiles;
  const int nwaves = (gridDim.x * (blockDim.x >> 6)) / ntiles;

  const int n = 32 * tile + col;  // STORE column
  const __amdgpu_buffer_rsrc_t ra = rsrc(p.A, (long)p.a_rows * p.lda * 4);
  const __amdgpu_buffer_rsrc_t rc = rsrc(p.C, (long)p.M * p.ldc * 4);
  const __amdgpu_buffer_rsrc_t rx = rsrc(GATE ? p.aux : p.C, GATE ? (long)p.M * p.ld_aux * 4 : 0);
  const long skip_rows = (GATE && p.aux2) ? (long)p.M - p.aux2_row0 : 0;
  const __amdgpu_buffer_rsrc_t rk = rsrc(GATE && p.aux2 ? p.aux2 : p.C, skip_rows > 0 ? skip_rows * p.ld_aux2 * 4 : 0);

  auto load = [&](int chunk, float4* a) {
    const long row = (long)chunk * 32 + col + half * p.shift;
    const int voff = (row >= 0 && row < p.a_rows) ? (int)((row * p.lda + half * p.a_tap) * 4) : OOR;
#pragma unroll
    for (int q = 0; q < NQ; ++q) a[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ra, voff, 16 * q, 0));
  };

  // the first chunk's loads go out before the weight staging (they do not depend on it)
  float4 a[NQ];
  int chunk = wave;
  load(chunk, a);
  // stationary weights w[t][j] = B(half*KH + j, column of (t, col)), staged once per block in LDS
  // (rows: GATE (t, col) -> t*32 + col holds output column 2 col + t; STORE: row n)
  constexpr int K = 2 * KH, LDT = K + 4;
  float bn[NT];
  extern __shared__ float4 bt4[];
  const float* wrow[NT];  // this lane's weight rows in LDS
  {
    float* bt = (float*)bt4;
    const int N = GATE ? 64 : 32 * p.ntiles;
    for (int e = threadIdx.x; e < K * N; e += blockDim.x) {
      const int k = e % K, nn = e / K;
      const int row = GATE ? (nn & 1) * 32 + (nn >> 1) : nn;
      bt[row * LDT + k] = p.B[(k % KH) * p.ldb_k + (k / KH) * p.ldb_tap + (long)nn * p.ldb_n];
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      wrow[t] = bt + (GATE ? t * 32 + col : 32 * tile + col) * LDT + half * KH;
      bn[t] = GATE ? p.bias[2 * col + t] : 0.0f;
    }
  }
  if (wave >= nwaves) return;  // after the block-wide staging barrier
  // CENTER (BatchNorm on load, gwn_batchnorm_fwd_fold): the column means are wave-uniform
  float cmu[KH];
#pragma unroll
  for (int j = 0; j < KH; ++j) cmu[j] = CENTER ? p.center[j] : 0.0f;
  // BNSTAT (N = 32: channel n = col): running sums of the final C and C*xhat over this wave's rows
  const __amdgpu_buffer_rsrc_t rz = rsrc(BNSTAT ? p.bn_z : p.C, BNSTAT ? (long)p.M * 32 * 4 : 0);
  const float bmu = BNSTAT ? p.bn_mean[col] : 0.0f, brs = BNSTAT ? p.bn_rstd[col] : 0.0f;
  float bs0 = 0.0f, bs1 = 0.0f;
  for (; chunk < nchunks; chunk += nwaves) {
    const long m0 = (long)chunk * 32;
    // C0 of this chunk first, then the next chunk's A: the epilogue waits only for the former
    float c0[16], zz[16];
    if (!GATE && p.accumulate) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long m = m0 + crow(r, half);
        c0[r] = ld32(rc, (m < p.M && m >= p.acc_row0) ? (int)((m * p.ldc + n) * 4) : OOR);
      }
    }
    if (BNSTAT) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long m = m0 + crow(r, half);
        zz[r] = ld32(rz, m < p.M ? (int)((m * 32 + n) * 4) : OOR);
      }
    }
    float4 an[NQ];
    load(chunk + nwaves, an);
    __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of the MFMAs
    f32x16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      float av[4] = {a[q].x, a[q].y, a[q].z, a[q].w};
      if (CENTER) {
#pragma unroll
        for (int e = 0; e < 4; ++e) av[e] -= cmu[4 * q + e];
      }
      float wq[NT][4];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const float4 v = *(const float4*)(wrow[t] + 4 * q);
        wq[t][0] = v.x; wq[t][1] = v.y; wq[t][2] = v.z; wq[t][3] = v.w;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[e], wq[t][e], acc[t], 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const long m = m0 + crow(r, half);
      const bool ok = m < p.M;
      if (GATE) {
        const float f = tanhf_(acc[0][r] + bn[0]), g = sigmoidf_(acc[NT - 1][r] + bn[NT - 1]);
        const float xg = f * g;
        st32(rc, ok ? (int)((m * p.ldc + col) * 4) : OOR, xg);
        typedef unsigned v2u __attribute__((ext_vector_type(2)));
        const v2u fgv = {__builtin_bit_cast(unsigned, f), __builtin_bit_cast(unsigned, g)};
        __builtin_amdgcn_raw_buffer_store_b64(fgv, rx, ok ? (int)((m * p.ld_aux + 2 * col) * 4) : OOR, 0,
                                              ST_AUX);
        if (skip_rows > 0)
          st32(rk, ok && m >= p.aux2_row0 ? (int)(((m - p.aux2_row0) * p.ld_aux2 + col) * 4) : OOR, xg);
      } else {
        float v = acc[0][r];
        if (p.accumulate) v += c0[r];
        st32(rc, ok ? (int)((m * p.ldc + n) * 4) : OOR, v);
        if (BNSTAT && ok) {
          bs0 += v;
          bs1 += v * ((zz[r] - bmu) * brs);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) a[q] = an[q];
  }
  if (BNSTAT) {
    // lane halves hold disjoint rows of the same channel: fold half 1 onto half 0 (fixed order)
    bs0 += __shfl_xor(bs0, 32);
    bs1 += __shfl_xor(bs1, 32);
    if (half == 0) {
      p.bn_part[(long)gw * 64 + col] = bs0;
      p.bn_part[(long)gw * 64 + 32 + col] = bs1;
    }
  }
}

// 8 waves per CU (12 for the gated forward, which its 168 registers allow, measured no faster)
inline int rowgemm_grid(int M, int ntiles, bool gate) {
  const int nchunks = (M + 31) / 32;
  int waves = nchunks * (gate ? 1 : ntiles);
  const int cap = 256 * 8;
  if (waves > cap) waves = cap;
  return (waves + 3) / 4;  // 4 | 4*grid, so every tile gets grid*4/ntiles waves
}

template <int KH, bool GATE, bool BNSTAT = false, bool CENTER = false>
int launch(const RowGemm& p, hipStream_t s) {
  GWN_REQUIRE((long)p.a_rows * p.lda * 4 < 0x7fff0000L && (long)p.M * p.ldc * 4 < 0x7fff0000L &&
                  (long)p.M * p.ld_aux * 4 < 0x7fff0000L && (long)p.M * p.ld_aux2 * 4 < 0x7fff0000L,
              "rowgemm: operand larger than a 2 GB buffer window");
  const int nchunks = (p.M + 31) / 32;
  // 8 waves per CU (2 per SIMD at ~200 VGPRs), grid-stride over the chunks; the wave count is
  // a multiple of ntiles so every tile gets the same number of waves
  GWN_REQUIRE(p.ntiles == 1 || p.ntiles == 2 || p.ntiles == 4, "rowgemm: N must be 32, 64 or 128");
  GWN_REQUIRE(!BNSTAT || (p.ntiles == 1 && p.ldc == 32), "rowgemm: BN statistics need N = ldc = 32");
  (void)nchunks;
  const int grid = rowgemm_grid(p.M, p.ntiles, GATE);
  const size_t lds = (size_t)(GATE ? 64 : 32 * p.ntiles) * (2 * KH + 4) * sizeof(float);
  rowgemm_kernel<KH, GATE, BNSTAT, CENTER><<<grid, 256, lds, s>>>(p);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

inline bool al16(const void* ptr) { return ((uintptr_t)ptr & 15u) == 0; }

}  // namespace

// xg / fg / skip <- gated dilated conv of x (gwn_gated_tcn_fwd)
int gwn_rowgemm_tcn_fwd(const gwn_tcn_args* a, hipStream_t s) {
  const int c = a->c, P = a->P, t_out = a->t_in - a->dilation;
  GWN_REQUIRE(c == 32 && al16(a->x) && al16(a->fg), "rowgemm tcn_fwd: needs c = 32 and 16-B aligned x / fg");
  RowGemm p = {};
  p.A = a->x; p.lda = c; p.a_rows = a->t_in * P; p.shift = (long)a->dilation * P; p.a_tap = 0;
  // B(k = tap*c + ci, n) = w_fg[n][tap*c + ci]
  p.B = a->w_fg; p.ldb_k = 1; p.ldb_tap = c; p.ldb_n = 2 * c;
  p.C = a->xg; p.ldc = a->ld_xg;
  p.bias = a->b_fg;
  p.aux = a->fg; p.ld_aux = a->fg ? 2 * c : 0;  // no fg: an empty window drops the stores
  p.aux2 = a->skipcat; p.ld_aux2 = a->ld_skip; p.aux2_row0 = a->skip_row0;
  p.M = t_out * P; p.ntiles = 2;
  p.center = a->x_mean;
  if (p.center) return launch<32, true, false, true>(p, s);
  return launch<32, true>(p, s);
}

// dx[r'][ci] (+)= sum_tap sum_j dfg[r' - tap*d*P][j] * w_fg[j][tap*c + ci]
int gwn_rowgemm_tcn_bwd_data(const gwn_tcn_bwd_args* a, hipStream_t s) {
  const int c = a->c, P = a->P, t_out = a->t_in - a->dilation;
  GWN_REQUIRE(c == 32 && al16(a->dfg) && al16(a->dx), "rowgemm tcn_bwd: needs c = 32 and 16-B aligned dfg / dx");
  RowGemm p = {};
  p.A = a->dfg; p.lda = 2 * c; p.a_rows = t_out * P; p.shift = -(long)a->dilation * P; p.a_tap = 0;
  // B(k = tap*2c + j, n = ci) = w_fg[j][tap*c + ci]
  p.B = a->w_fg; p.ldb_k = 2 * c; p.ldb_tap = c; p.ldb_n = 1;
  p.C = a->dx; p.ldc = c; p.accumulate = a->accumulate_dx; p.acc_row0 = a->acc_row0;
  p.M = a->t_in * P; p.ntiles = 1;
  if (a->bn_sums) {
    p.bn_z = a->bn_z; p.bn_mean = a->bn_mean; p.bn_rstd = a->bn_rstd; p.bn_part = a->workspace;
    return launch<64, false, true>(p, s);
  }
  return launch<64, false>(p, s);
}

// partial count of gwn_rowgemm_tcn_bwd_data's BN statistics ([n][2][32] in the workspace)
int gwn_rowgemm_tcn_bwd_nparts(const gwn_tcn_bwd_args* a) { return 4 * rowgemm_grid(a->t_in * a->P, 1, false); }
