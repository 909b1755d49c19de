// Op-level C-ABI of libgwn: the Graph WaveNet hot-path operators (reference model.py /
// engine.py / Utils/util.py) built from the MFMA GEMM (gemm.hip) and the reduction /
// element-wise kernels below.  All reductions use a fixed order (per-block partials, then an
// in-order merge), so every result is bitwise reproducible.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "gwn_internal.h"

namespace {
thread_local char g_err[512] = "";

constexpr int RED_BLOCKS = 512;  // partial-reduction blocks (fixed -> fixed summation order)

inline bool aligned16(const void* ptr) { return ((uintptr_t)ptr & 15u) == 0; }

gwn_gemm_desc gemm_zero() {
  gwn_gemm_desc d;
  memset(&d, 0, sizeof(d));
  d.alpha = 1.0f;
  d.beta = 1.0f;
  d.ksplit = 1;
  return d;
}

int pick_ksplit(int M, int N, int K) {
  // aim for ~1024 blocks over the output tiles (see gemm.hip launch configs: >= 64x64 tiles),
  // K-slices of >= 256 rows; the split reduction is a parallel fixed-order tree (gemm.hip)
  long tiles = ((M + 127) / 128) * (long)((N + 63) / 64);
  if (tiles < 1) tiles = 1;
  long ks = 1024 / tiles;
  long maxks = K / 256;
  if (ks > maxks) ks = maxks;
  if (ks < 1) ks = 1;
  return (int)ks;
}

// ---------------------------------------------------------------------------------------------
// block-level fixed-order sum over blockDim.x (power of two) threads
template <int NT>
__device__ float block_sum(float v, float* sh) {
  sh[threadIdx.x] = v;
  __syncthreads();
#pragma unroll
  for (int s = NT / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) sh[threadIdx.x] += sh[threadIdx.x + s];
    __syncthreads();
  }
  float r = sh[0];
  __syncthreads();
  return r;
}

template <int NT>
__device__ float block_max(float v, float* sh) {
  sh[threadIdx.x] = v;
  __syncthreads();
#pragma unroll
  for (int s = NT / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) sh[threadIdx.x] = fmaxf(sh[threadIdx.x], sh[threadIdx.x + s]);
    __syncthreads();
  }
  float r = sh[0];
  __syncthreads();
  return r;
}

// ---------------------------------------------------------------------------------------------
// adaptive adjacency: one block per row v.  logits l[w] = relu(sum_k e1[v][k] e2[k][w])
__global__ void adp_fwd_kernel(const float* e1, const float* e2, int n, int d, float* adp, int ld,
                               long adp_bstride = 0) {
  __shared__ float sh[256];
  const int v = blockIdx.x;
  // batched (blockIdx.y = sample): embeddings [B][n][d] / [B][d][n], outputs adp_bstride apart
  e1 += (long)blockIdx.y * n * d;
  e2 += (long)blockIdx.y * d * n;
  adp += (long)blockIdx.y * adp_bstride;
  if (n <= 256 && d <= 16) {
    // one column per thread: its d embedding loads issued together, the logit kept in a register
    // (the loop form below re-derived it per pass with a memory round trip per k); the same fma
    // order, exp and scaling, so the same values
    const int w = threadIdx.x;
    const bool on = w < n;
    float e1v[16], e2v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      e1v[k] = k < d ? e1[(long)v * d + k] : 0.0f;
      e2v[k] = (k < d && on) ? e2[(long)k * n + w] : 0.0f;
    }
    float l = 0.0f;
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k < d) l = fmaf(e1v[k], e2v[k], l);
    l = fmaxf(l, 0.0f);
    const float mx = block_max<256>(on ? l : -INFINITY, sh);
    const float ex = on ? expf(l - mx) : 0.0f;
    const float sum = block_sum<256>(ex, sh);
    const float inv = 1.0f / sum;
    for (int c = threadIdx.x; c < ld; c += 256) adp[(long)v * ld + c] = (c < n) ? ex * inv : 0.0f;
    return;
  }
  float mx = -INFINITY;
  for (int w = threadIdx.x; w < n; w += 256) {
    float l = 0.0f;
    for (int k = 0; k < d; ++k) l = fmaf(e1[(long)v * d + k], e2[(long)k * n + w], l);
    l = fmaxf(l, 0.0f);
    mx = fmaxf(mx, l);
  }
  mx = block_max<256>(mx, sh);
  float sum = 0.0f;
  for (int w = threadIdx.x; w < n; w += 256) {
    float l = 0.0f;
    for (int k = 0; k < d; ++k) l = fmaf(e1[(long)v * d + k], e2[(long)k * n + w], l);
    l = fmaxf(l, 0.0f);
    const float ex = expf(l - mx);
    adp[(long)v * ld + w] = ex;
    sum += ex;
  }
  sum = block_sum<256>(sum, sh);
  const float inv = 1.0f / sum;
  for (int w = threadIdx.x; w < ld; w += 256)
    adp[(long)v * ld + w] = (w < n) ? adp[(long)v * ld + w] * inv : 0.0f;
}

// dlogit[v][w] = adp*(dadp - sum_w' adp*dadp) * [pre > 0]
// row v of dL = relu'(E1 E2) * softmax'(dadp) and, from the same block, row v of dE1 = dL E2^T
// (the embedding rank d <= ADP_MAXD: per-thread partials over its w, fixed-order block sums)
constexpr int ADP_MAXD = 16;
__global__ void adp_bwd_kernel(const float* e1, const float* e2, const float* adp, const float* dadp,
                               int n, int d, int ld, float* dl, float* de1) {
  __shared__ float sh[256];
  const int v = blockIdx.x;
  float dot = 0.0f;
  for (int w = threadIdx.x; w < n; w += 256) dot += adp[(long)v * ld + w] * dadp[(long)v * ld + w];
  dot = block_sum<256>(dot, sh);
  float pe[ADP_MAXD], ev[ADP_MAXD];
#pragma unroll
  for (int k = 0; k < ADP_MAXD; ++k) {
    pe[k] = 0.0f;
    ev[k] = e1[(long)v * d + min(k, d - 1)];
  }
  for (int w = threadIdx.x; w < ld; w += 256) {
    // the column's embedding values and the row's adp / dadp all requested before the first use
    // (the k loop loaded e2 one value per memory round trip)
    const int wc = min(w, n - 1);
    float e2v[ADP_MAXD];
#pragma unroll
    for (int k = 0; k < ADP_MAXD; ++k) e2v[k] = e2[(long)min(k, d - 1) * n + wc];
    const float a = adp[(long)v * ld + wc], da = dadp[(long)v * ld + wc];
    float g = 0.0f;
    if (w < n) {
      float l = 0.0f;
#pragma unroll
      for (int k = 0; k < ADP_MAXD; ++k)
        if (k < d) l = fmaf(ev[k], e2v[k], l);
      g = (l > 0.0f) ? a * (da - dot) : 0.0f;
#pragma unroll
      for (int k = 0; k < ADP_MAXD; ++k)
        if (k < d) pe[k] = fmaf(g, e2v[k], pe[k]);
    }
    dl[(long)v * ld + w] = g;
  }
  // all d sums in one fixed-order tree (8 barriers, not 8 per value)
  __shared__ float shk[ADP_MAXD][256];
#pragma unroll
  for (int k = 0; k < ADP_MAXD; ++k)
    if (k < d) shk[k][threadIdx.x] = pe[k];
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) {
#pragma unroll
      for (int k = 0; k < ADP_MAXD; ++k)
        if (k < d) shk[k][threadIdx.x] += shk[k][threadIdx.x + st];
    }
    __syncthreads();
  }
  if ((int)threadIdx.x < d) de1[(long)v * d + threadIdx.x] = shk[threadIdx.x][0];
}

// dE2[k][w] = sum_v e1[v][k] dL[v][w]: 16 columns w per 1024-thread block, 64 lanes over v
// (v mod 64) each holding all d partial sums, folded by a fixed-order tree over the lanes
__global__ __launch_bounds__(1024) void adp_bwd_e2_kernel(const float* e1, const float* dl, int n, int d, int ld,
                                                          float* de2) {
  __shared__ float sh[64][ADP_MAXD][16];
  const int tw = threadIdx.x & 15, tv = threadIdx.x >> 4;
  const int w = blockIdx.x * 16 + tw;
  float acc[ADP_MAXD];
#pragma unroll
  for (int k = 0; k < ADP_MAXD; ++k) acc[k] = 0.0f;
  if (w < n) {
    // four rows' loads in flight per round (the same v order of the sums)
    for (int v0 = tv; v0 < n; v0 += 4 * 64) {
      float gq[4], eq[4][ADP_MAXD];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int v = min(v0 + 64 * u, n - 1);
        gq[u] = dl[(long)v * ld + w];
#pragma unroll
        for (int k = 0; k < ADP_MAXD; ++k) eq[u][k] = e1[(long)v * d + min(k, d - 1)];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (v0 + 64 * u >= n) break;
#pragma unroll
        for (int k = 0; k < ADP_MAXD; ++k)
          if (k < d) acc[k] = fmaf(eq[u][k], gq[u], acc[k]);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < ADP_MAXD; ++k) sh[tv][k][tw] = acc[k];
  __syncthreads();
  for (int st = 32; st > 0; st >>= 1) {
    if (tv < st) {
#pragma unroll
      for (int k = 0; k < ADP_MAXD; ++k) sh[tv][k][tw] += sh[tv + st][k][tw];
    }
    __syncthreads();
  }
  if (tv != 0 || w >= n) return;
#pragma unroll
  for (int k = 0; k < ADP_MAXD; ++k)
    if (k < d) de2[(long)k * n + w] = sh[0][k][tw];
}

// ---------------------------------------------------------------------------------------------
__global__ void start_conv_kernel(const float* x, long sb, long sc, long sn, long st, int B, int cin,
                                  int n, int t, int t0, const float* W, const float* bias, int c,
                                  float* out, float* xin) {
  const long rows = (long)t0 * B * n;
  const long total = rows * c;
  const int pad = t0 - t;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const long row = idx / c;
    const int co = (int)(idx - row * c);
    const int v = (int)(row % n);
    const long tb = row / n;
    const int b = (int)(tb % B);
    const int tt = (int)(tb / B);
    const int ts = tt - pad;
    float acc = bias[co];
    for (int ci = 0; ci < cin; ++ci) {
      const float xv = (ts >= 0) ? x[b * sb + ci * sc + v * sn + (long)ts * st] : 0.0f;
      acc = fmaf(W[co * cin + ci], xv, acc);
      if (co == 0 && xin) xin[row * cin + ci] = xv;
    }
    out[idx] = acc;
  }
}

// c == 32, cin <= 4: eight lanes per row, four output channels each (one 16-B store per lane, a
// row's 128 B per eight lanes), 32-bit row arithmetic (the generic kernel's per-element 64-bit
// divisions made a 22 MB write take 23 us); the cin input values of a row are one broadcast load
// each, lane q < cin also copies value q to xin.  (One lane per channel with 4-B stores: 15.5 us
// per METR step.)  Per channel the same fma order as the generic kernel.
template <int CIN>
__global__ __launch_bounds__(256) void start_conv32_kernel(const float* x, long sb, long sc, long sn, long st, int B,
                                                           int n, int t, int t0, const float* W, const float* bias,
                                                           float* out, float* xin) {
  const int rows = t0 * B * n;
  const int q = threadIdx.x & 7, co = 4 * q;
  float bco[4], w[4][CIN];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    bco[e] = bias[co + e];
#pragma unroll
    for (int ci = 0; ci < CIN; ++ci) w[e][ci] = W[(co + e) * CIN + ci];
  }
  const int pad = t0 - t;
  for (int row = blockIdx.x * 32 + (threadIdx.x >> 3); row < rows; row += gridDim.x * 32) {
    const int v = row % n, tb = row / n, b = tb % B, ts = tb / B - pad;
    float xv[CIN];
#pragma unroll
    for (int ci = 0; ci < CIN; ++ci)
      xv[ci] = ts >= 0 ? x[b * sb + ci * sc + v * sn + (long)ts * st] : 0.0f;
    float acc[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc[e] = bco[e];
#pragma unroll
      for (int ci = 0; ci < CIN; ++ci) acc[e] = fmaf(w[e][ci], xv[ci], acc[e]);
    }
    if (q < CIN && xin) {
      float mine = xv[0];
#pragma unroll
      for (int ci = 1; ci < CIN; ++ci) mine = (q == ci) ? xv[ci] : mine;
      xin[(long)row * CIN + q] = mine;
    }
    *(float4*)(out + (long)row * 32 + co) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  }
}

// ---------------------------------------------------------------------------------------------
// gated TCN backward element-wise part: dfg from dxg (+ skip grad) and the saved tanh/sigmoid.
__global__ void gate_bwd_kernel(const float* dxg, long ld_dxg, const float* dskip, long ld_dskip,
                                int skip_row0, const float* fg, long rows, int c, float* dfg) {
  const long total = rows * c;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const long r = idx / c;
    const int ch = (int)(idx - r * c);
    float g = dxg ? dxg[r * ld_dxg + ch] : 0.0f;
    if (dskip && r >= skip_row0) g += dskip[(r - skip_row0) * ld_dskip + ch];
    const float f = fg[r * 2 * c + 2 * ch], s = fg[r * 2 * c + 2 * ch + 1];
    dfg[r * 2 * c + 2 * ch] = g * s * (1.0f - f * f);
    dfg[r * 2 * c + 2 * ch + 1] = g * f * s * (1.0f - s);
  }
}

// ---------------------------------------------------------------------------------------------
// column partial sums: partial[blk][j] = sum over the block's row chunk of f(a[r][j])
//   mode 0: a;  mode 1: a * ((b - mean[j]) * rstd[j])
template <int MODE>
__global__ void colsum_partial_kernel(const float* a, long lda, const float* b, long ldb,
                                      const float* mean, const float* rstd, long rows, int ncol,
                                      float* partial) {
  __shared__ float sh[256];
  const long chunk = (rows + gridDim.x - 1) / gridDim.x;
  const long r0 = blockIdx.x * chunk;
  const long r1 = (r0 + chunk < rows) ? r0 + chunk : rows;
  if (ncol <= 256) {
    const int lanes = 256 / ncol;  // row lanes per column
    const int col = threadIdx.x % ncol, rl = threadIdx.x / ncol;
    float acc = 0.0f;
    if (rl < lanes) {
      for (long r = r0 + rl; r < r1; r += lanes) {
        float v = a[r * lda + col];
        if (MODE == 1) v *= (b[r * ldb + col] - mean[col]) * rstd[col];
        acc += v;
      }
    }
    sh[threadIdx.x] = (rl < lanes) ? acc : 0.0f;
    __syncthreads();
    if ((int)threadIdx.x < ncol) {
      float s = 0.0f;
      for (int i = 0; i < lanes; ++i) s += sh[i * ncol + threadIdx.x];
      partial[(long)blockIdx.x * ncol + threadIdx.x] = s;
    }
  } else {
    for (int col = threadIdx.x; col < ncol; col += 256) {
      float acc = 0.0f;
      for (long r = r0; r < r1; ++r) {
        float v = a[r * lda + col];
        if (MODE == 1) v *= (b[r * ldb + col] - mean[col]) * rstd[col];
        acc += v;
      }
      partial[(long)blockIdx.x * ncol + col] = acc;
    }
  }
}

// BatchNorm backward statistics in one pass: partial[blk][j] = sum dy, partial[blk][c + j] =
// sum dy * xhat over the block's row chunk (c | 256)
__global__ void bn_bwd_partial_kernel(const float* dy, const float* z, const float* mean, const float* rstd,
                                      long rows, int c, float* partial) {
  __shared__ float sh[2][256];
  const long chunk = (rows + gridDim.x - 1) / gridDim.x;
  const long r0 = blockIdx.x * chunk;
  const long r1 = (r0 + chunk < rows) ? r0 + chunk : rows;
  const int lanes = 256 / c;
  const int col = threadIdx.x % c, rl = threadIdx.x / c;
  float s0 = 0.0f, s1 = 0.0f;
  if (rl < lanes) {
    const float mu = mean[col], rs = rstd[col];
    for (long r = r0 + rl; r < r1; r += lanes) {
      const float g = dy[r * c + col];
      s0 += g;
      s1 += g * ((z[r * c + col] - mu) * rs);
    }
  }
  sh[0][threadIdx.x] = (rl < lanes) ? s0 : 0.0f;
  sh[1][threadIdx.x] = (rl < lanes) ? s1 : 0.0f;
  __syncthreads();
  for (int t = threadIdx.x; t < 2 * c; t += 256) {
    const int h = t / c, j = t - h * c;
    float s = 0.0f;
    for (int i = 0; i < lanes; ++i) s += sh[h][i * c + j];
    partial[(long)blockIdx.x * 2 * c + t] = s;
  }
}

// Many partials (e.g. one per wave of a rowgemm launch): one block per column, 256 lanes each
// summing a strided subset, then a fixed-order tree.
__global__ void colsum_final_wide_kernel(const float* partial, int nparts, int ncol, float* out,
                                         int accumulate) {
  __shared__ float sh[256];
  const int j = blockIdx.x;
  float s0 = 0.0f, s1 = 0.0f;
  int i = threadIdx.x;
  for (; i + 256 < nparts; i += 512) {
    s0 += partial[(long)i * ncol + j];
    s1 += partial[(long)(i + 256) * ncol + j];
  }
  if (i < nparts) s0 += partial[(long)i * ncol + j];
  sh[threadIdx.x] = s0 + s1;
  __syncthreads();
#pragma unroll
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[j] = accumulate ? out[j] + sh[0] : sh[0];
}

// ---------------------------------------------------------------------------------------------
// BatchNorm statistics: per block (count, mean, M2) over its row chunk (two passes over the chunk),
// merged in block order with Chan's formula.
__global__ void bn_partial_kernel(const float* z, long rows, int c, float* part) {
  __shared__ float sh[256];
  const long chunk = (rows + gridDim.x - 1) / gridDim.x;
  const long r0 = blockIdx.x * chunk;
  const long r1 = (r0 + chunk < rows) ? r0 + chunk : rows;
  const long cnt = (r1 > r0) ? r1 - r0 : 0;
  const int lanes = 256 / c;
  const int col = threadIdx.x % c, rl = threadIdx.x / c;
  float s = 0.0f;
  if (rl < lanes)
    for (long r = r0 + rl; r < r1; r += lanes) s += z[r * c + col];
  sh[threadIdx.x] = (rl < lanes) ? s : 0.0f;
  __syncthreads();
  float mean = 0.0f;
  if (cnt > 0) {
    float t = 0.0f;
    for (int i = 0; i < lanes; ++i) t += sh[i * c + col];
    mean = t / (float)cnt;
  }
  __syncthreads();
  float q = 0.0f;
  if (rl < lanes)
    for (long r = r0 + rl; r < r1; r += lanes) {
      const float dlt = z[r * c + col] - mean;
      q += dlt * dlt;
    }
  sh[threadIdx.x] = (rl < lanes) ? q : 0.0f;
  __syncthreads();
  if ((int)threadIdx.x < c) {
    float m2 = 0.0f;
    for (int i = 0; i < lanes; ++i) m2 += sh[i * c + threadIdx.x];
    float* pp = part + (long)blockIdx.x * 3 * c;
    pp[threadIdx.x] = (float)cnt;
    pp[c + threadIdx.x] = mean;
    pp[2 * c + threadIdx.x] = m2;
  }
}

// The per-chunk BatchNorm partials [nparts][3][c] (count, mean, M2) of channel j merged over one
// 256-thread block as fp64 sums n, S = sum n_b mean_b, Q = sum (M2_b + n_b mean_b^2) (strided subsets
// per thread, then a fixed-order tree; no division per merge); thread 0 returns n, mean = S / n and
// M2 = Q - S mean (fp32 inputs: the fp64 cancellation costs ~1e-16 (1 + mean^2 / var) of the variance)
__device__ void bn_merge_channel(const float* part, int nparts, int c, int j, double& n_out, double& mean_out,
                                 double& m2_out) {
  __shared__ double sn[256], sm[256], sq[256];
  double n = 0.0, s1 = 0.0, s2 = 0.0;
  // a thread's partials (i = tid, tid + 256, ...) are loaded four at a time before they are added
  constexpr int U = 4;
  for (int i0 = 0; i0 < nparts; i0 += 256 * U) {
    float nbv[U], mbv[U], m2v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + (int)threadIdx.x + 256 * u;
      const float* pp = part + (long)i * 3 * c;
      const bool ok = i < nparts;
      nbv[u] = ok ? pp[j] : 0.0f;
      mbv[u] = ok ? pp[c + j] : 0.0f;
      m2v[u] = ok ? pp[2 * c + j] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (nbv[u] <= 0.0f) continue;
      const double nm = (double)nbv[u] * (double)mbv[u];
      n += nbv[u];
      s1 += nm;
      s2 += (double)m2v[u] + nm * (double)mbv[u];
    }
  }
  sn[threadIdx.x] = n; sm[threadIdx.x] = s1; sq[threadIdx.x] = s2;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      sn[threadIdx.x] += sn[threadIdx.x + w];
      sm[threadIdx.x] += sm[threadIdx.x + w];
      sq[threadIdx.x] += sq[threadIdx.x + w];
    }
    __syncthreads();
  }
  n_out = sn[0];
  mean_out = n_out > 0.0 ? sm[0] / n_out : 0.0;
  const double m2 = sq[0] - sm[0] * mean_out;
  m2_out = m2 > 0.0 ? m2 : 0.0;
}

__global__ void bn_finalize_kernel(const float* part, int nparts, int c, float momentum, float eps,
                                   float* running_mean, float* running_var, float* save_mean,
                                   float* save_rstd, long long* nbt) {
  // one block per channel
  const int j = blockIdx.x;
  if (nbt && j == 0 && threadIdx.x == 0) *nbt += 1;  // BatchNorm2d.num_batches_tracked
  double n, mean, m2;
  bn_merge_channel(part, nparts, c, j, n, mean, m2);
  if (threadIdx.x != 0) return;
  const double var = (n > 0.0) ? m2 / n : 0.0;
  save_mean[j] = (float)mean;
  save_rstd[j] = (float)(1.0 / sqrt(var + (double)eps));
  if (running_mean) {
    const double unbiased = (n > 1.0) ? m2 / (n - 1.0) : var;
    running_mean[j] = (float)((1.0 - momentum) * running_mean[j] + momentum * mean);
    running_var[j] = (float)((1.0 - momentum) * running_var[j] + momentum * unbiased);
  }
}

__global__ void bn_apply_kernel(const float* z, long rows, int c, const float* mean,
                                const float* rstd, const float* rvar, float eps,
                                const float* gamma, const float* beta, float* out) {
  const long total = rows * c;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int j = (int)(idx % c);
    const float rs = rstd ? rstd[j] : 1.0f / sqrtf(rvar[j] + eps);
    out[idx] = (z[idx] - mean[j]) * rs * gamma[j] + beta[j];
  }
}

// bn_finalize_kernel + the scale of the normalisation folded into the next gated TCN
// (gwn_batchnorm_fwd_fold), one block per channel j: the merge, then column j of both taps of the
// next layer's weights (w_next [2c][2c]: row = output channel, column = tap*c + ci) scaled by
// scale[j]; block 0 also folds beta into the bias (independent of the statistics)
__global__ void bn_finalize_fold_kernel(const float* part, int nparts, int c, float momentum, float eps,
                                        const float* gamma, const float* beta, float* running_mean,
                                        float* running_var, float* save_mean, float* save_rstd, float* scale,
                                        const float* w_next, const float* b_next, float* w_fold, float* b_fold,
                                        long long* nbt) {
  __shared__ float ssc;
  __shared__ float bp[256];
  const int j = blockIdx.x;
  if (nbt && j == 0 && threadIdx.x == 0) *nbt += 1;  // BatchNorm2d.num_batches_tracked
  // the weight operands do not depend on the statistics: loaded before the merge (latency hidden)
  const bool wcol = w_next && (int)threadIdx.x < 4 * c;  // (row, tap) pairs of column j
  const long we = (long)(threadIdx.x >> 1) * 2 * c + (threadIdx.x & 1) * c + j;
  const float wv = wcol ? w_next[we] : 0.0f;
  // b_fold[row] = b_next[row] + sum_k w_next[row][k] * beta[k % c]: block j folds rows j and j + c,
  // one product per thread, fixed-order tree per row
  const int half = threadIdx.x / (2 * c), k = threadIdx.x % (2 * c);
  const int row = j + half * c;
  const bool brow = w_next && half < 2;
  const float bv = brow ? w_next[(long)row * 2 * c + k] * beta[k % c] : 0.0f;
  double n, mean, m2;
  bn_merge_channel(part, nparts, c, j, n, mean, m2);
  if (threadIdx.x == 0) {
    const double var = (n > 0.0) ? m2 / n : 0.0;
    const float rs = (float)(1.0 / sqrt(var + (double)eps));
    save_mean[j] = (float)mean;
    save_rstd[j] = rs;
    if (running_mean) {
      const double unbiased = (n > 1.0) ? m2 / (n - 1.0) : var;
      running_mean[j] = (float)((1.0 - momentum) * running_mean[j] + momentum * mean);
      running_var[j] = (float)((1.0 - momentum) * running_var[j] + momentum * unbiased);
    }
    const float sc = rs * gamma[j];  // bn(z) = (z - mean) * sc + beta
    scale[j] = sc;
    ssc = sc;
  }
  if (!w_next) return;
  bp[threadIdx.x] = bv;
  __syncthreads();
  if (wcol) w_fold[we] = wv * ssc;
  for (int w = c; w > 0; w >>= 1) {
    if (brow && k < w) bp[threadIdx.x] += bp[threadIdx.x + w];
    __syncthreads();
  }
  if (brow && k == 0) b_fold[row] = b_next[row] + bp[threadIdx.x];
}

// eval-mode BatchNorm: the running statistics as (mean, rstd) for the backward
__global__ void bn_running_stats_kernel(const float* rmean, const float* rvar, int c, float eps,
                                        float* mean, float* rstd) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < c) {
    mean[j] = rmean[j];
    rstd[j] = 1.0f / sqrtf(rvar[j] + eps);
  }
}

// dz = gamma*rstd*(dy - k1 - xhat*k2); dres[r + row0] = dz; dres rows < row0 zeroed; dh = dropout'(dz)
__global__ void bn_bwd_apply_kernel(const float* dy, const float* z, long rows, int c,
                                    const float* gamma, const float* mean, const float* rstd,
                                    const float* sums, float inv_n, float* dres, int res_row0, float* dh,
                                    const unsigned long long* seed_ptr, unsigned long long salt,
                                    float drop_p, float* dgamma, float* dbeta) {
  const long total = rows * c;
  const unsigned long long seed = seed_ptr ? *seed_ptr : 0ull;
  const long zero_total = (long)res_row0 * c;
  if (blockIdx.x == 0)
    for (int j = threadIdx.x; j < c; j += blockDim.x) {
      if (dbeta) dbeta[j] = sums[j];
      if (dgamma) dgamma[j] = sums[c + j];
    }
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total + zero_total;
       idx += (long)gridDim.x * blockDim.x) {
    if (idx >= total) {
      if (dres) dres[idx - total] = 0.0f;
      continue;
    }
    const long r = idx / c;
    const int j = (int)(idx - r * c);
    const float xhat = (z[idx] - mean[j]) * rstd[j];
    const float k1 = sums[j] * inv_n, k2 = sums[c + j] * inv_n;
    const float dz = gamma[j] * rstd[j] * (dy[idx] - k1 - xhat * k2);
    if (dres) dres[(r + res_row0) * c + j] = dz;
    if (dh) {
      float v = dz;
      if (drop_p > 0.0f) {
        const float u = gwn_uniform(seed, salt, (unsigned long long)r * (unsigned)c + j);
        v = (u >= drop_p) ? v * (1.0f / (1.0f - drop_p)) : 0.0f;
      }
      dh[idx] = v;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// masked metrics (util.py:510-552, null_val = 0).  ws layout: [0] nonzero count,
// [1 .. 1+3*RED_BLOCKS) partial (mae, mape, mse) sums, [LOSS_CNT ..) partial nonzero-label counts
constexpr int LOSS_CNT_BLOCKS = 128;
// loss_terms blocks: few enough that the last-arriver count costs little (one same-address atomic
// per block is ~6-7 ns of serialised L2 work), enough to cover the [B][o][n][tf] output
constexpr int LOSS_TERM_BLOCKS = 256;
// adam_clipped blocks (grid-stride; same reasoning as LOSS_TERM_BLOCKS)
constexpr int ADAM_BLOCKS = 256;
constexpr int LOSS_CNT = 1 + 3 * RED_BLOCKS;

// arrival counter of loss_terms_kernel (reset by loss_count_kernel, which always runs first)
constexpr int LOSS_ARRIVE = LOSS_CNT + LOSS_CNT_BLOCKS;

__global__ void loss_count_kernel(const float* real, long rsb, long rsn, long rso, int B, int n,
                                  int o, float* ws) {
  __shared__ float sh[256];
  if (blockIdx.x == 0 && threadIdx.x == 0) *(int*)(ws + LOSS_ARRIVE) = 0;
  const long total = (long)B * n * o;
  float cnt = 0.0f;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < (int)total; i += 256 * gridDim.x) {  // (total < 2^31)
    const int oo = i % o;
    const int bv = i / o;
    const int v = bv % n;
    const int b = bv / n;
    cnt += (real[b * rsb + v * rsn + oo * rso] != 0.0f) ? 1.0f : 0.0f;
  }
  cnt = block_sum<256>(cnt, sh);
  if (threadIdx.x == 0) ws[LOSS_CNT + blockIdx.x] = cnt;
}

// one prediction's masked terms (util.py:510-552) and its loss gradient (d mae / d out)
__device__ __forceinline__ float loss_term(float out, float y, float mean, float std, float mask_scale,
                                          float inv_total, float& s_mae, float& s_mape, float& s_mse) {
  const float pred = out * std + mean;
  const float mask = (y != 0.0f) ? mask_scale : 0.0f;
  const float diff = pred - y;
  float mae = fabsf(diff) * mask;
  if (isnan(mae)) mae = 0.0f;
  float mape = fabsf(diff) / y * mask;
  if (isnan(mape)) mape = 0.0f;
  float mse = diff * diff * mask;
  if (isnan(mse)) mse = 0.0f;
  s_mae += mae;
  s_mape += mape;
  s_mse += mse;
  const float sg = (diff > 0.0f) ? 1.0f : ((diff < 0.0f) ? -1.0f : 0.0f);
  const float g = fabsf(diff) * mask;
  return isnan(g) ? 0.0f : sg * mask * inv_total * std;
}

// ROWS = false: out / dout are the reference's [B][o][n][tf]; ROWS = true: the head's slab rows,
// out[((t*B + b)*n + v)*ld_out + oo], dout alike with ld_dout (its columns o..ld_dout zeroed)
template <bool ROWS>
__global__ void loss_terms_kernel(const float* out, const float* real, long rsb, long rsn, long rso,
                                  int B, int o, int n, int tf, float mean, float std, float* dout,
                                  float* ws, float* metrics, int ld_out, int ld_dout) {
  __shared__ float sh[256];
  const long total = (long)B * o * n * tf;
  // every block re-derives the (exact, integer-valued) label count from the count partials
  const float cnt = block_sum<256>((threadIdx.x < LOSS_CNT_BLOCKS) ? ws[LOSS_CNT + threadIdx.x] : 0.0f, sh);
  const float label_total = (float)((long)B * n * o);
  const float mask_scale = (cnt > 0.0f) ? label_total / cnt : 0.0f;  // 1 / mean(mask)
  const float inv_total = 1.0f / (float)total;
  float s_mae = 0.0f, s_mape = 0.0f, s_mse = 0.0f;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    if (ROWS) {
      const long r = idx / o;
      const int oo = (int)(idx - r * o);
      const int v = (int)(r % n);
      const int b = (int)((r / n) % B);
      const float gr = loss_term(out[r * ld_out + oo], real[b * rsb + v * rsn + oo * rso], mean, std, mask_scale,
                                 inv_total, s_mae, s_mape, s_mse);
      if (dout) {
        float* row = dout + r * ld_dout;
        row[oo] = gr;
        if (oo == 0)
          for (int c = o; c < ld_dout; ++c) row[c] = 0.0f;
      }
    } else {
      const long r1 = idx / tf;
      const int v = (int)(r1 % n);
      const long r2 = r1 / n;
      const int oo = (int)(r2 % o);
      const int b = (int)(r2 / o);
      const float gr = loss_term(out[idx], real[b * rsb + v * rsn + oo * rso], mean, std, mask_scale, inv_total,
                                 s_mae, s_mape, s_mse);
      if (dout) dout[idx] = gr;
    }
  }
  s_mae = block_sum<256>(s_mae, sh);
  s_mape = block_sum<256>(s_mape, sh);
  s_mse = block_sum<256>(s_mse, sh);
  // hand-off to the last block to arrive (MI355X_MICROARCH.md, inter-workgroup visibility): sc1
  // (write-through) partial stores, an agent release before the one agent-scope add, and an agent
  // acquire in the last arriver before it reads every partial (sc1 loads); one lane per block, so
  // the fences cost ~2 x 1.7 us once per step
  __shared__ int last;
  if (threadIdx.x == 0) {
    __hip_atomic_store(ws + 1 + blockIdx.x * 3, s_mae, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(ws + 2 + blockIdx.x * 3, s_mape, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(ws + 3 + blockIdx.x * 3, s_mse, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int is_last = atomicAdd((int*)(ws + LOSS_ARRIVE), 1) == (int)gridDim.x - 1;
    if (is_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    last = is_last;
  }
  __syncthreads();
  if (!last) return;
  // the final sums, in block order per thread then the fixed block_sum tree (deterministic)
  float a = 0.0f, b = 0.0f, c = 0.0f;
  for (int i = threadIdx.x; i < (int)gridDim.x; i += 256) {
    a += __hip_atomic_load(ws + 1 + i * 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    b += __hip_atomic_load(ws + 2 + i * 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    c += __hip_atomic_load(ws + 3 + i * 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  a = block_sum<256>(a, sh);
  b = block_sum<256>(b, sh);
  c = block_sum<256>(c, sh);
  if (threadIdx.x == 0) {
    metrics[0] = (float)((double)a / (double)total);
    metrics[1] = (float)((double)b / (double)total);
    metrics[2] = sqrtf((float)((double)c / (double)total));
  }
}

// ---------------------------------------------------------------------------------------------
// clip_grad_norm_ + Adam over ranges of the flat buffers.  ws: [0 .. RED_BLOCKS) partial sq-sums,
// [RED_BLOCKS] clip coefficient.
__device__ __forceinline__ bool range_index(const long* lo, const long* hi, int nr, long i, long* out) {
  for (int r = 0; r < nr; ++r) {
    const long len = hi[r] - lo[r];
    if (i < len) { *out = lo[r] + i; return true; }
    i -= len;
  }
  return false;
}

__global__ void sqnorm_partial_kernel(const float* g, const long* lo, const long* hi, int nr,
                                      long active, float* ws) {
  __shared__ float sh[256];
  if (blockIdx.x == 0 && threadIdx.x == 0) *(int*)(ws + RED_BLOCKS + 1) = 0;  // adam_clipped's counter
  float s = 0.0f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < active;
       i += (long)gridDim.x * blockDim.x) {
    long k;
    if (range_index(lo, hi, nr, i, &k)) s += g[k] * g[k];
  }
  s = block_sum<256>(s, sh);
  if (threadIdx.x == 0) ws[blockIdx.x] = s;
}

// Adam with the clip coefficient computed in every block from the RED_BLOCKS sq-sum partials in
// ws (fixed order: every block derives the same coefficient), the step read before use (t = *step
// + 1) and advanced by the last block to finish (arrival counter at ws[RED_BLOCKS + 1], zeroed by
// the sq-sum kernel that precedes this launch), which also advances the dropout counter
// (seed_inc != 0) -- one launch for clip_coef + adam + the two counters.
__global__ void adam_clipped_kernel(float* p, float* g, float* m, float* v, const long* lo, const long* hi, int nr,
                                    long active, float* ws, long long* step, float max_norm, float lr, float beta1,
                                    float beta2, float eps, float wd, float* total_norm_out,
                                    unsigned long long* seed, unsigned long long seed_inc) {
  __shared__ float sh[256];
  __shared__ float s_coef;
  float part = 0.0f;
  for (int i = threadIdx.x; i < RED_BLOCKS; i += 256) part += ws[i];
  const float sq = block_sum<256>(part, sh);
  if (threadIdx.x == 0) {
    const float norm = sqrtf(sq);
    const float coef = max_norm / (norm + 1e-6f);
    s_coef = coef < 1.0f ? coef : 1.0f;
    if (blockIdx.x == 0 && total_norm_out) *total_norm_out = norm;
  }
  __syncthreads();
  const float coef = s_coef;
  const double t = (double)(*step + 1);
  const double bc1 = 1.0 - pow((double)beta1, t);
  const double bc2 = 1.0 - pow((double)beta2, t);
  const float step_size = (float)((double)lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  // four grid-stride elements per pass, every load issued before the first update (few blocks keep
  // the arrival count cheap; the passes were latency-bound one element at a time)
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i0 = blockIdx.x * (long)blockDim.x + threadIdx.x; i0 < active; i0 += 4 * stride) {
    long kk[4];
    bool ok[4];
    float gv[4], pv[4], mv[4], vv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long i = i0 + u * stride;
      ok[u] = i < active && range_index(lo, hi, nr, i, &kk[u]);
      if (ok[u]) {
        gv[u] = g[kk[u]]; pv[u] = p[kk[u]]; mv[u] = m[kk[u]]; vv[u] = v[kk[u]];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (!ok[u]) continue;
      const long k = kk[u];
      float gr = gv[u] * coef;
      g[k] = gr;
      if (wd != 0.0f) gr = gr + wd * pv[u];
      float mq = mv[u];
      mq = mq + (1.0f - beta1) * (gr - mq);
      const float vq = vv[u] * beta2 + (1.0f - beta2) * gr * gr;
      m[k] = mq;
      v[k] = vq;
      const float denom = sqrtf(vq) / bc2_sqrt + eps;
      p[k] = pv[u] - step_size * (mq / denom);
    }
  }
  // every block has read *step above: the last one to arrive advances it (and the dropout counter)
  __syncthreads();
  if (threadIdx.x == 0) {
    int* cnt = (int*)(ws + RED_BLOCKS + 1);
    if (atomicAdd(cnt, 1) == (int)gridDim.x - 1) {
      *step += 1;
      if (seed) *seed += seed_inc;
      atomicExch(cnt, 0);
    }
  }
}

// dst[i] = src[idx[i]] and the RED_BLOCKS partial sums of dst[i]^2 (the clip norm of a flat
// gradient whose inactive entries gather the zero slot) in one pass
__global__ void gather_sqnorm_kernel(const float* src, const int* idx, float* dst, long count, float* ws) {
  __shared__ float sh[256];
  if (blockIdx.x == 0 && threadIdx.x == 0) *(int*)(ws + RED_BLOCKS + 1) = 0;  // adam_clipped's counter
  float s = 0.0f;
  // four grid-stride elements per pass: their indices, then their values (the same sum order)
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i0 = blockIdx.x * (long)blockDim.x + threadIdx.x; i0 < count; i0 += 4 * stride) {
    int ix[4];
    float xv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) ix[u] = i0 + u * stride < count ? idx[i0 + u * stride] : 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) xv[u] = i0 + u * stride < count ? src[ix[u]] : 0.0f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (i0 + u * stride >= count) continue;
      dst[i0 + u * stride] = xv[u];
      s += xv[u] * xv[u];
    }
  }
  s = block_sum<256>(s, sh);
  if (threadIdx.x == 0) ws[blockIdx.x] = s;
}

// ---------------------------------------------------------------------------------------------
__global__ void gather_kernel(const float* src, const int* idx, float* dst, long count) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < count;
       i += (long)gridDim.x * blockDim.x)
    dst[i] = src[idx[i]];
}

// gather_kernel plus one computed segment: dst[sum_dst + j] = sum_v src[idx[sum_src + v*len + j]]
// (v in order, the same sums as sum_vectors_kernel over the gathered vectors)
__global__ void gather_sum_kernel(const float* src, const int* idx, float* dst, long count, long sum_src, int nvec,
                                  int len, long sum_dst) {
  const long total = count + len;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    if (i < count) {
      if (i < sum_dst || i >= sum_dst + len) dst[i] = src[idx[i]];
    } else {
      const long j = i - count;
      // the nvec source indices, then their values, eight at a time in flight (the same sum
      // order; a dependent index -> value chain per term made this 2 x nvec memory latencies)
      float s = 0.0f;
      for (int v0 = 0; v0 < nvec; v0 += 8) {
        int ix[8];
        float xv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) ix[u] = v0 + u < nvec ? idx[sum_src + (long)(v0 + u) * len + j] : 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) xv[u] = v0 + u < nvec ? src[ix[u]] : 0.0f;
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (v0 + u < nvec) s += xv[u];
      }
      dst[sum_dst + j] = s;
    }
  }
}

__global__ void to_nchw_kernel(const float* y, int B, int o, int n, int t, float* out) {
  const long total = (long)B * o * n * t;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int tt = (int)(idx % t);
    const long r1 = idx / t;
    const int v = (int)(r1 % n);
    const long r2 = r1 / n;
    const int oo = (int)(r2 % o);
    const int b = (int)(r2 / o);
    out[idx] = y[(((long)tt * B + b) * n + v) * o + oo];
  }
}

__global__ void from_nchw_kernel(const float* dout, int B, int o, int n, int t, float* dy, int ld) {
  const long total = (long)B * o * n * t;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int tt = (int)(idx % t);
    const long r1 = idx / t;
    const int v = (int)(r1 % n);
    const long r2 = r1 / n;
    const int oo = (int)(r2 % o);
    const int b = (int)(r2 / o);
    float* row = dy + (((long)tt * B + b) * n + v) * ld;
    row[oo] = dout[idx];
    if (oo == 0)
      for (int c = o; c < ld; ++c) row[c] = 0.0f;  // zero padding columns
  }
}

__global__ void sum_vectors_kernel(const float* x, int count, int len, long stride, float* out) {
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < len; j += gridDim.x * blockDim.x) {
    float s = 0.0f;
    for (int i = 0; i < count; ++i) s += x[(long)i * stride + j];
    out[j] = s;
  }
}

__global__ void increment_kernel(unsigned long long* c, unsigned long long inc) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *c += inc;
}

int grid_for(long total, int block = 256) {
  long g = (total + block - 1) / block;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

// =============================================================================================
int gwn_set_error(int code, const char* msg) {
  strncpy(g_err, msg ? msg : "", sizeof(g_err) - 1);
  g_err[sizeof(g_err) - 1] = 0;
  return code;
}

static int g_sync_check = -1;  // -1: read GWN_SYNC_CHECK on first use

int gwn_launch_status(const char* file, int line) {
  if (g_sync_check < 0) {
    const char* e = getenv("GWN_SYNC_CHECK");
    g_sync_check = (e && e[0] == '1') ? 1 : 0;
  }
  hipError_t e_ = hipGetLastError();
  if (e_ == hipSuccess && g_sync_check == 1) e_ = hipDeviceSynchronize();
  if (e_ == hipSuccess) return GWN_OK;
  char buf[256];
  snprintf(buf, sizeof(buf), "%s (%s:%d)", hipGetErrorString(e_), file, line);
  return gwn_set_error(GWN_ERR_HIP, buf);
}

// debugging (GWN_SYNC_CHECK): does [p, p + bytes) lie inside one device allocation?
int gwn_debug_range(const void* p, long bytes, const char* what) {
  if (g_sync_check != 1 || !p || bytes <= 0) return GWN_OK;
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p) != hipSuccess) {
    (void)hipGetLastError();
    char buf[256];
    snprintf(buf, sizeof(buf), "debug range: %s at %p is not in a device allocation", what, p);
    return gwn_set_error(GWN_ERR_ARG, buf);
  }
  const long off = (long)((const char*)p - (const char*)base);
  if (off + bytes > (long)size) {
    char buf[256];
    snprintf(buf, sizeof(buf), "debug range: %s [%p, +%ld) overruns its allocation [%p, +%zu) by %ld bytes", what,
             p, bytes, (void*)base, size, off + bytes - (long)size);
    return gwn_set_error(GWN_ERR_ARG, buf);
  }
  return GWN_OK;
}

extern "C" {

int gwn_version(void) { return 1; }
/* debugging: 1 = synchronise after every launch (GWN_SYNC_CHECK), 2 = suspended (e.g. while a
 * stream is being captured into a graph), 0 = off */
void gwn_set_sync_check(int mode) { g_sync_check = mode; }
const char* gwn_last_error(void) { return g_err; }

long gwn_abi_sizeof(const char* name) {
  if (!name) return -1;
  if (!strcmp(name, "gwn_gemm_desc")) return (long)sizeof(gwn_gemm_desc);
  if (!strcmp(name, "gwn_tcn_args")) return (long)sizeof(gwn_tcn_args);
  if (!strcmp(name, "gwn_tcn_bwd_args")) return (long)sizeof(gwn_tcn_bwd_args);
  if (!strcmp(name, "gwn_reduce_seg")) return (long)sizeof(gwn_reduce_seg);
  if (!strcmp(name, "gwn_gcn_args")) return (long)sizeof(gwn_gcn_args);
  if (!strcmp(name, "gwn_gcn_bwd_args")) return (long)sizeof(gwn_gcn_bwd_args);
  if (!strcmp(name, "gwn_wgrad_problem")) return (long)sizeof(gwn_wgrad_problem);
  if (!strcmp(name, "gwn_gram_layer")) return (long)sizeof(gwn_gram_layer);
  if (!strcmp(name, "gwn_bn_fold")) return (long)sizeof(gwn_bn_fold);
  return -1;
}

int gwn_gemm(const gwn_gemm_desc* d, hipStream_t s) {
  GWN_REQUIRE(d != nullptr, "gemm: null descriptor");
  return gwn_gemm_launch(*d, s);
}

long gwn_gemm_workspace_floats(int M, int N, int ksplit) {
  return ((long)M * N + M) * (ksplit > 1 ? ksplit : 0);  // + M: the optional ones column
}

// ---------------------------------------------------------------------------------------------
int gwn_nconv(const float* A, int lda, int transpose_a, const float* x, long ldx, float* y, long ldy,
              const float* y0, long ldy0, int n, int c, int slices, hipStream_t s) {
  GWN_REQUIRE(n > 0 && c > 0 && slices > 0, "nconv: bad shape");
  if (transpose_a && gwn_bigdiff_eligible(n, c, A, lda, x, ldx, y, ldy, y0, ldy0))
    return gwn_bigdiff(A, lda, x, ldx, y, ldy, y0, ldy0, n, slices, s);  // n > 512: large-graph kernel
  gwn_gemm_desc d = gemm_zero();
  d.A = A;
  if (transpose_a) { d.lda_m = 1; d.lda_k = lda; } else { d.lda_m = lda; d.lda_k = 1; }
  d.B = x; d.ldb_k = ldx; d.ldb_n = 1; d.b_nin = c; d.b_no_stride = (long)n * ldx;
  d.C = y; d.ldc_m = ldy; d.ldc_n = 1; d.c_nin = c; d.c_no_stride = (long)n * ldy;
  if (y0) { d.C0 = y0; d.ldc0_m = ldy0; d.ldc0_n = 1; d.c0_no_stride = (long)n * ldy0; d.beta = 1.0f; }
  d.M = n; d.N = c * slices; d.K = n;
  return gwn_gemm_launch(d, s);
}

int gwn_nconv2(const float* A, int lda, long a_bstride, int transpose_a, const float* x, long ldx, float* y,
               long ldy, int n, int c, int slices, int batch, hipStream_t s) {
  GWN_REQUIRE(n > 0 && c > 0 && slices > 0 && batch > 0 && A && x && y, "nconv2: bad shape");
  gwn_gemm_desc d = gemm_zero();
  d.A = A;
  if (transpose_a) { d.lda_m = 1; d.lda_k = lda; } else { d.lda_m = lda; d.lda_k = 1; }
  d.B = x; d.ldb_k = ldx; d.ldb_n = 1; d.b_nin = c; d.b_no_stride = (long)n * ldx;
  d.C = y; d.ldc_m = ldy; d.ldc_n = 1; d.c_nin = c; d.c_no_stride = (long)n * ldy;
  d.M = n; d.N = c * slices; d.K = n;
  d.batch = batch; d.a_bstride = a_bstride;
  d.b_bstride = (long)slices * n * ldx; d.c_bstride = (long)slices * n * ldy;
  return gwn_gemm_launch(d, s);
}

int gwn_nconv2_adj_grad(const float* x, long ldx, const float* dy, long lddy, int n, int c, int slices, int batch,
                        float* dA, int ld_dA, long dA_bstride, int accumulate, hipStream_t s) {
  GWN_REQUIRE(n > 0 && c > 0 && slices > 0 && batch > 0 && x && dy && dA, "nconv2_adj_grad: bad shape");
  gwn_gemm_desc d = gemm_zero();
  d.A = x; d.lda_m = ldx; d.lda_k = 1; d.a_kin = c; d.a_ko_stride = (long)n * ldx;
  d.B = dy; d.ldb_k = 1; d.ldb_n = lddy; d.b_kin = c; d.b_ko_stride = (long)n * lddy;
  d.C = dA; d.ldc_m = ld_dA; d.ldc_n = 1;
  if (accumulate) { d.C0 = dA; d.ldc0_m = ld_dA; d.ldc0_n = 1; d.beta = 1.0f; }
  d.M = n; d.N = n; d.K = c * slices;
  d.batch = batch; d.a_bstride = (long)slices * n * ldx; d.b_bstride = (long)slices * n * lddy;
  d.c_bstride = dA_bstride;
  return gwn_gemm_launch(d, s);
}

static int adj_grad_ksplit(int n, int c, int slices) {
  return pick_ksplit(n, n, c * slices);
}

long gwn_nconv_adj_grad_workspace_floats(int n, int c, int slices) {
  const int ks = adj_grad_ksplit(n, c, slices);
  const long g = gwn_gram_workspace_floats(n, slices);
  const long w = ks > 1 ? (long)ks * n * n : 0;
  return g > w ? g : w;
}

static bool gram_eligible(const float* x, long ldx, const float* dy, long lddy, int c) {
  return c == 32 && aligned16(x) && aligned16(dy) && (ldx & 3) == 0 && (lddy & 3) == 0;
}

int gwn_nconv_adj_grad(const float* x, long ldx, const float* dy, long lddy, int n, int c, int slices,
                       float* dA, int ld_dA, int accumulate, float* ws, hipStream_t s) {
  if (gram_eligible(x, ldx, dy, lddy, c))
    return gwn_gram(x, dy, nullptr, nullptr, ldx, lddy, n, slices, dA, ld_dA, accumulate, ws, s);
  gwn_gemm_desc d = gemm_zero();
  d.A = x; d.lda_m = ldx; d.lda_k = 1; d.a_kin = c; d.a_ko_stride = (long)n * ldx;
  d.B = dy; d.ldb_k = 1; d.ldb_n = lddy; d.b_kin = c; d.b_ko_stride = (long)n * lddy;
  d.C = dA; d.ldc_m = ld_dA; d.ldc_n = 1;
  if (accumulate) { d.C0 = dA; d.ldc0_m = ld_dA; d.ldc0_n = 1; d.beta = 1.0f; }
  d.M = n; d.N = n; d.K = c * slices;
  d.ksplit = adj_grad_ksplit(n, c, slices);
  d.part = ws;
  return gwn_gemm_launch(d, s);
}

// ---------------------------------------------------------------------------------------------
int gwn_adaptive_adj_fwd(const float* e1, const float* e2, int n, int dd, float* adp, int ld,
                         hipStream_t s) {
  GWN_REQUIRE(n > 0 && dd > 0 && ld >= n, "adaptive_adj_fwd: bad shape");
  adp_fwd_kernel<<<n, 256, 0, s>>>(e1, e2, n, dd, adp, ld);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

int gwn_adaptive_adj_fwd_batched(const float* e1, const float* e2, int batch, int n, int dd, float* adp, int ld,
                                 long adp_bstride, hipStream_t s) {
  GWN_REQUIRE(n > 0 && dd > 0 && ld >= n && batch > 0 && batch <= 65535 && adp_bstride >= (long)n * ld,
              "adaptive_adj_fwd_batched: bad shape");
  adp_fwd_kernel<<<dim3(n, batch), 256, 0, s>>>(e1, e2, n, dd, adp, ld, adp_bstride);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

int gwn_adaptive_adj_bwd(const float* e1, const float* e2, const float* adp, const float* dadp, int n,
                         int dd, int ld, float* de1, float* de2, float* ws, hipStream_t s) {
  GWN_REQUIRE(n > 0 && dd > 0 && dd <= ADP_MAXD && ld >= n, "adaptive_adj_bwd: bad shape (embedding rank <= 16)");
  // dL and dE1[v][k] = sum_w dL[v][w] e2[k][w] (one block per v), then dE2[k][w] = sum_v e1[v][k] dL[v][w]
  adp_bwd_kernel<<<n, 256, 0, s>>>(e1, e2, adp, dadp, n, dd, ld, ws, de1);
  GWN_CHECK_LAUNCH();
  adp_bwd_e2_kernel<<<(n + 15) / 16, 1024, 0, s>>>(e1, ws, n, dd, ld, de2);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

// ---------------------------------------------------------------------------------------------
int gwn_start_conv_fwd(const float* x, long sb, long sc, long sn, long st, int B, int cin, int n,
                       int t, int t0, const float* W, const float* bias, int c, float* out, float* xin,
                       hipStream_t s) {
  GWN_REQUIRE(t0 >= t && B > 0 && n > 0 && c > 0 && cin > 0, "start_conv: bad shape");
  const long total = (long)t0 * B * n * c;
  const long rows = (long)t0 * B * n;
  if (c == 32 && cin >= 1 && cin <= 4 && rows < (1L << 30)) {
    GWN_REQUIRE(((uintptr_t)out & 15) == 0, "start_conv: out 16-B aligned");
    const int grid = (int)((rows + 31) / 32 < 8192 ? (rows + 31) / 32 : 8192);
    switch (cin) {
      case 1: start_conv32_kernel<1><<<grid, 256, 0, s>>>(x, sb, sc, sn, st, B, n, t, t0, W, bias, out, xin); break;
      case 2: start_conv32_kernel<2><<<grid, 256, 0, s>>>(x, sb, sc, sn, st, B, n, t, t0, W, bias, out, xin); break;
      case 3: start_conv32_kernel<3><<<grid, 256, 0, s>>>(x, sb, sc, sn, st, B, n, t, t0, W, bias, out, xin); break;
      default: start_conv32_kernel<4><<<grid, 256, 0, s>>>(x, sb, sc, sn, st, B, n, t, t0, W, bias, out, xin); break;
    }
  } else {
    start_conv_kernel<<<grid_for(total), 256, 0, s>>>(x, sb, sc, sn, st, B, cin, n, t, t0, W, bias, c,
                                                      out, xin);
  }
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

// ---------------------------------------------------------------------------------------------
int gwn_gated_tcn_fwd(const gwn_tcn_args* a, hipStream_t s) {
  GWN_REQUIRE(a && a->c > 0 && a->P > 0 && a->ntaps >= 0 && a->c_out >= 0, "gated_tcn_fwd: bad shape");
  if (a->bn) {  // the layer below's BatchNorm finalized first (its own launch), then the folded TCN
    const gwn_bn_fold* f = a->bn;
    GWN_REQUIRE(a->c == 32 && a->bn_partials && a->bn_nparts > 0 && f->w_next && f->b_next && f->w_fold && f->b_fold &&
                    f->w_fold != f->w_next && f->gamma && f->beta && f->save_mean && f->save_rstd && f->scale,
                "gated_tcn_fwd: bn needs c == 32, bn_partials / bn_nparts, and bn's weights, outputs and w_fold / b_fold");
    int rc = gwn_batchnorm_fwd_fold(a->bn_partials, a->bn_nparts, a->c, f->gamma, f->beta, f->running_mean,
                                    f->running_var, f->momentum, f->eps, f->save_mean, f->save_rstd, f->scale,
                                    f->w_next, f->b_next, f->w_fold, f->b_fold, f->num_batches_tracked, s);
    if (rc) return rc;
    gwn_tcn_args t = *a;
    t.bn = nullptr;
    t.x_mean = f->save_mean;
    t.w_fg = f->w_fold;
    t.b_fg = f->b_fold;
    return gwn_gated_tcn_fwd(&t, s);
  }
  const int taps = a->ntaps > 0 ? a->ntaps : 2, co = a->c_out > 0 ? a->c_out : a->c;
  GWN_REQUIRE(a->t_in > a->dilation * (taps - 1), "gated_tcn_fwd: input shorter than the receptive field");
  GWN_REQUIRE(a->c % 16 == 0 && co % 16 == 0, "gated_tcn_fwd: channels must be multiples of 16");
  const int c = a->c, P = a->P, t_out = a->t_in - a->dilation * (taps - 1);
  if (c == 32 && taps == 2 && co == c && aligned16(a->x) && aligned16(a->fg)) return gwn_rowgemm_tcn_fwd(a, s);
  GWN_REQUIRE(a->fg != nullptr && !a->x_mean, "gated_tcn_fwd: fg may only be NULL (and x_mean set) on the c == 32 path");
  gwn_gemm_desc d = gemm_zero();
  d.A = a->x; d.lda_m = c; d.lda_k = 1; d.a_kin = c; d.a_row_shift = a->dilation * P;
  d.a_rows = a->t_in * P;
  d.B = a->w_fg; d.ldb_k = 1; d.ldb_n = taps * c;
  d.C = a->xg; d.ldc_m = a->ld_xg; d.ldc_n = 1;
  d.bias_n = a->b_fg;
  d.epi = EPI_GATE;
  d.aux = a->fg; d.ld_aux = 2 * co;
  d.aux2 = a->skipcat; d.ld_aux2 = a->ld_skip; d.aux2_row0 = a->skip_row0;
  d.M = t_out * P; d.N = 2 * co; d.K = taps * c;
  return gwn_gemm_launch(d, s);
}

static int tcn_w_ksplit(int rows, int c, int taps, int co) { return pick_ksplit(2 * co, taps * c, rows); }

// the weight gradient of the TCN runs on the row-reduction kernel when its tiles fit (gwn_wgrad)
static bool tcn_wgrad_rows(int c, int taps, int co) {
  return (2 * co) % 32 == 0 && c % 32 == 0 && (2 * co / 32) * (taps * c / 32) <= 16;
}

long gwn_gated_tcn_bwd_workspace_floats_ex(int t_in, int P, int c, int dilation, int ntaps, int c_out) {
  const int taps = ntaps > 0 ? ntaps : 2, co = c_out > 0 ? c_out : c;
  const int rows = (t_in - dilation * (taps - 1)) * P;
  if (rows <= 0 || c <= 0) return 0;
  const long g = gwn_gemm_workspace_floats(2 * co, taps * c, tcn_w_ksplit(rows, c, taps, co));
  const long w = tcn_wgrad_rows(c, taps, co) ? gwn_wgrad_workspace_floats(rows, 2 * co, taps * c) : 0;
  long m = g > w ? g : w;
  // BN statistics partials of the fused rowgemm epilogue, or of the generic fallback pass
  const long b = (long)(GWN_ROWGEMM_MAX_PARTS > RED_BLOCKS ? GWN_ROWGEMM_MAX_PARTS : RED_BLOCKS) * 2 * c;
  return m > b ? m : b;
}

long gwn_gated_tcn_bwd_workspace_floats(int t_in, int P, int c, int dilation) {
  return gwn_gated_tcn_bwd_workspace_floats_ex(t_in, P, c, dilation, 2, c);
}

int gwn_gated_tcn_bwd(const gwn_tcn_bwd_args* a, hipStream_t s) {
  GWN_REQUIRE(a && a->c % 16 == 0 && a->ntaps >= 0 && a->c_out >= 0, "gated_tcn_bwd: bad shape");
  const int taps = a->ntaps > 0 ? a->ntaps : 2, co = a->c_out > 0 ? a->c_out : a->c;
  GWN_REQUIRE(a->t_in > a->dilation * (taps - 1) && co % 16 == 0, "gated_tcn_bwd: bad shape");
  const bool square = taps == 2 && co == a->c;  // the row-GEMM fusions' shape
  GWN_REQUIRE(square || (!a->dfg_ready && !a->x_mean && !a->x_scale && !a->x_shift),
              "gated_tcn_bwd: dfg_ready / x_mean fusions need ntaps 2 and c_out == c");
  const int c = a->c, P = a->P, t_out = a->t_in - a->dilation * (taps - 1);
  const long rows = (long)t_out * P;
  GWN_REQUIRE(a->acc_row0 >= 0 && a->acc_row0 <= (long)a->t_in * P, "gated_tcn_bwd: bad acc_row0");
  if (a->bn_sums) GWN_REQUIRE(a->bn_z && a->bn_mean && a->bn_rstd && c <= 256 && 256 % c == 0,
                              "gated_tcn_bwd: BN statistics need bn_z, bn_mean, bn_rstd");
  if (!a->dfg_ready) {
    gate_bwd_kernel<<<grid_for(rows * co), 256, 0, s>>>(a->dxg, a->ld_dxg, a->dskip, a->ld_dskip,
                                                        a->skip_row0, a->fg, rows, co, a->dfg);
    GWN_CHECK_LAUNCH();
  }
  // dW_fg[j][tap*c + ci] = sum_r dfg[r][j] * x[r + tap*d*P][ci];  db_fg[j] = sum_r dfg[r][j]
  int rc = GWN_OK;
  gwn_gemm_desc d = gemm_zero();
  if (a->skip_weight_grads) {
    // caller computes dW_fg / db_fg itself (gwn_wgrad)
  } else if (tcn_wgrad_rows(c, taps, co)) {
    rc = gwn_wgrad_bn(a->dfg, 2 * co, 2 * co, a->x, c, (long)a->t_in * P, c, taps, (long)a->dilation * P, (int)rows,
                      a->x_mean, a->x_scale, a->x_shift, a->dw_fg, taps * c, a->db_fg, a->workspace, s);
  } else {
    GWN_REQUIRE(!a->x_mean && !a->x_scale && !a->x_shift, "gated_tcn_bwd: x_mean / x_scale / x_shift need c % 32 == 0");
    d.A = a->dfg; d.lda_m = 1; d.lda_k = 2 * co;
    d.B = a->x; d.ldb_k = c; d.ldb_n = 1; d.b_nin = c; d.b_no_stride = (long)a->dilation * P * c;
    d.C = a->dw_fg; d.ldc_m = taps * c; d.ldc_n = 1;
    d.ones_out = a->db_fg;
    d.M = 2 * co; d.N = taps * c; d.K = (int)rows;
    d.ksplit = tcn_w_ksplit((int)rows, c, taps, co);
    d.part = a->workspace;
    rc = gwn_gemm_launch(d, s);
  }
  if (rc) return rc;
  // dx[r'][ci] (+)= sum_tap sum_j dfg[r' - tap*d*P][j] * Wfg[j][tap*c + ci]
  if (c == 32 && square && aligned16(a->dfg) && aligned16(a->dx)) {
    rc = gwn_rowgemm_tcn_bwd_data(a, s);
    if (rc || !a->bn_sums) return rc;
    colsum_final_wide_kernel<<<2 * c, 256, 0, s>>>(a->workspace, gwn_rowgemm_tcn_bwd_nparts(a), 2 * c,
                                                   a->bn_sums, 0);
    GWN_CHECK_LAUNCH();
    return GWN_OK;
  }
  if (a->accumulate_dx && a->acc_row0 > 0) {
    if (hipMemsetAsync(a->dx, 0, (size_t)a->acc_row0 * c * sizeof(float), s) != hipSuccess)
      return gwn_set_error(GWN_ERR_HIP, "gated_tcn_bwd: memset failed");
  }
  d = gemm_zero();
  d.A = a->dfg; d.lda_m = 2 * co; d.lda_k = 1; d.a_kin = 2 * co; d.a_row_shift = -a->dilation * P;
  d.a_rows = (int)rows;
  d.B = a->w_fg; d.ldb_k = taps * c; d.ldb_n = 1; d.b_kin = 2 * co; d.b_ko_stride = c;
  d.C = a->dx; d.ldc_m = c; d.ldc_n = 1;
  if (a->accumulate_dx) { d.C0 = a->dx; d.ldc0_m = c; d.ldc0_n = 1; d.beta = 1.0f; }
  d.M = a->t_in * P; d.N = c; d.K = taps * 2 * co;
  rc = gwn_gemm_launch(d, s);
  if (rc || !a->bn_sums) return rc;
  const long rows_in = (long)a->t_in * P;
  bn_bwd_partial_kernel<<<RED_BLOCKS, 256, 0, s>>>(a->dx, a->bn_z, a->bn_mean, a->bn_rstd, rows_in, c,
                                                   a->workspace);
  GWN_CHECK_LAUNCH();
  colsum_final_wide_kernel<<<2 * c, 256, 0, s>>>(a->workspace, RED_BLOCKS, 2 * c, a->bn_sums, 0);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

// ---------------------------------------------------------------------------------------------
static int gcn_fwd_unfolded(const gwn_gcn_args* a, hipStream_t s);

int gwn_gcn_fwd(const gwn_gcn_args* a, hipStream_t s) {
  GWN_REQUIRE(a && a->rows > 0 && a->n > 0 && a->rows % a->n == 0, "gcn_fwd: rows must be slices*n");
  GWN_REQUIRE(a->drop_p <= 0.0f || (long long)a->rows * (a->c_out > 0 ? a->c_out : a->c) < (1LL << 32),
              "gcn_fwd: dropout masks index rows*c_out elements in 32 bits (gwn_uniform)");
  const gwn_bn_fold* f = a->bn_fold;
  if (f) {
    const int co = a->c_out > 0 ? a->c_out : a->c;
    GWN_REQUIRE(co == 32 && a->bn_partials && !a->bn_out && f->gamma && f->beta && f->save_mean && f->save_rstd &&
                    f->scale,
                "gcn_fwd: bn_fold needs c_out == 32, bn_partials, no bn_out, gamma / beta and the outputs");
    GWN_REQUIRE(!f->w_next || (f->b_next && f->w_fold && f->b_fold && f->w_fold != f->w_next),
                "gcn_fwd: bn_fold.w_next needs b_next, w_fold, b_fold (w_fold not aliasing w_next)");
  }
  const int c = a->c, n = a->n;
  const int co = a->c_out > 0 ? a->c_out : c;
  gwn_gcn_args local;
  if (a->tcn) {
    GWN_REQUIRE(a->tcn->xg == a->h && a->tcn->ld_xg == a->ld_h, "gcn_fwd: tcn must write xg into h (ld_xg = ld_h)");
    if (!gwn_gcn_tcn_fusable(a)) {  // the TCN as its own launch, then the diffusion without it
      const int rc = gwn_gated_tcn_fwd(a->tcn, s);
      if (rc) return rc;
      local = *a;
      local.tcn = nullptr;
      a = &local;
    }
  }
  int used = (int)gwn_bn_part_slots(a->rows / n);  // the slots that can hold rows (the t16 kernels: their grid)
  int rc = (co == c && gwn_gcn_fused_eligible(c, n, a->nsup, a->ld_sup))
               ? gwn_gcn_fused_fwd_launch(a, a->bn_partials, s, &used)
               : gcn_fwd_unfolded(a, s);
  if (rc) return rc;
  if (a->bn_slots_used) *a->bn_slots_used = used;
  if (!f) return rc;
  return gwn_batchnorm_fwd_fold(a->bn_partials, used, co, f->gamma, f->beta,
                                f->running_mean, f->running_var, f->momentum, f->eps, f->save_mean, f->save_rstd,
                                f->scale, f->w_next, f->b_next, f->w_fold, f->b_fold, f->num_batches_tracked, s);
}

static int gcn_fwd_unfolded(const gwn_gcn_args* a, hipStream_t s) {
  const int c = a->c, n = a->n, slices = a->rows / n;
  GWN_REQUIRE(a->c_out >= 0, "gcn_fwd: bad c_out");
  const int co = a->c_out > 0 ? a->c_out : c;
  GWN_REQUIRE(a->sup_batch <= 1, "gcn_fwd: per-sample supports need the fused path (c == 32, n <= 512)");
  GWN_REQUIRE(!a->no_pieces && !a->bn_out && !a->residual_scale && !a->residual_mean,
              "gcn_fwd: no_pieces / bn_out / residual_scale need the fused path (c == 32, n <= 512)");
  const int width = (2 * a->nsup + 1) * c;
  for (int k = 0; k < a->nsup; ++k) {
    float* x1 = a->h + (1 + 2 * k) * c;
    float* x2 = a->h + (2 + 2 * k) * c;
    int rc = gwn_nconv(a->sup[k], a->ld_sup, 1, a->h, a->ld_h, x1, a->ld_h, nullptr, 0, n, c, slices, s);
    if (rc) return rc;
    rc = gwn_nconv(a->sup[k], a->ld_sup, 1, x1, a->ld_h, x2, a->ld_h, nullptr, 0, n, c, slices, s);
    if (rc) return rc;
  }
  gwn_gemm_desc d = gemm_zero();
  d.A = a->h; d.lda_m = a->ld_h; d.lda_k = 1;
  d.B = a->w_mlp; d.ldb_k = 1; d.ldb_n = width;
  d.C = a->z; d.ldc_m = co; d.ldc_n = 1;
  d.bias_n = a->b_mlp;
  d.C0 = a->residual; d.ldc0_m = co; d.ldc0_n = 1; d.beta = 1.0f;
  d.seed_ptr = a->seed_ptr; d.seed_salt = a->salt; d.drop_p = a->drop_p;
  d.M = a->rows; d.N = co; d.K = width;
  int rc = gwn_gemm_launch(d, s);
  if (rc || !a->bn_partials) return rc;
  GWN_REQUIRE(co <= 256 && 256 % co == 0, "gcn_fwd: BN partials need c_out | 256");
  bn_partial_kernel<<<slices, 256, 0, s>>>(a->z, a->rows, co, a->bn_partials);  // one chunk per slice
  GWN_CHECK_LAUNCH();
  const long slots = gwn_bn_part_slots(slices);  // the slots past the slices hold no rows
  if (slots > slices && hipMemsetAsync(a->bn_partials + (long)slices * 3 * co, 0,
                                       (size_t)(slots - slices) * 3 * co * sizeof(float), s) != hipSuccess)
    return gwn_set_error(GWN_ERR_HIP, "gcn_fwd: BN partial tail memset failed");
  return GWN_OK;
}

static int gcn_w_ksplit(int rows, int c, int width) { return pick_ksplit(c, width, rows); }

long gwn_gcn_bwd_workspace_floats(int rows, int n, int c, int nsup) {
  return gwn_gcn_bwd_workspace_floats_ex(rows, n, c, nsup, c);
}

long gwn_gcn_bwd_workspace_floats_ex(int rows, int n, int c, int nsup, int c_out) {
  const int co = c_out > 0 ? c_out : c;
  const int width = (2 * nsup + 1) * c;
  long w = gwn_gemm_workspace_floats(co, width, gcn_w_ksplit(rows, co, width));
  const long g = gwn_nconv_adj_grad_workspace_floats(n, c, rows / n);
  const long v = gwn_wgrad_workspace_floats(rows, co, width);
  const long gr = gwn_gram_workspace_floats(n, rows / n);  // any slice count up to rows / n
  if (v > w) w = v;
  if (gr > w) w = gr;
  return g > w ? g : w;
}

long gwn_gcn_ksplit_ws_floats(int rows, int n, int nsup) {
  if (rows <= 0 || n <= 0 || nsup <= 0) return 0;
  return (long)(rows / n) * nsup * ((n + 31) / 32 * 32) * 32;
}

int gwn_gcn_bwd(const gwn_gcn_bwd_args* a, hipStream_t s) {
  GWN_REQUIRE(a && a->rows > 0 && a->n > 0 && a->rows % a->n == 0, "gcn_bwd: rows must be slices*n");
  GWN_REQUIRE(a->drop_p <= 0.0f || (long long)a->rows * (a->c_out > 0 ? a->c_out : a->c) < (1LL << 32),
              "gcn_bwd: dropout masks index rows*c_out elements in 32 bits (gwn_uniform)");
  const int c = a->c, n = a->n, slices = a->rows / n;
  GWN_REQUIRE(a->c_out >= 0, "gcn_bwd: bad c_out");
  const int co = a->c_out > 0 ? a->c_out : c;
  const int width = (2 * a->nsup + 1) * c;
  const bool fused = co == c && a->sup_t && gwn_gcn_fused_eligible(c, n, a->nsup, a->ld_sup);
  GWN_REQUIRE(fused || (!a->bn_dy && !a->dfg && a->sup_batch <= 1),
              "gcn_bwd: the BN / gate fusions and per-sample supports need the fused path "
              "(sup_t given, c == 32, n <= 512)");
  const float* dh = a->bn_dy ? a->dh_out : a->dh;
  const bool wgrads = !a->skip_weight_grads;  // else the caller runs gwn_wgrad / gwn_gram itself
  // with tg4 the bf16 tile backward writes t1 / t2 there instead of dhcat's columns c..3c, so the
  // in-library adjacency gram (which reads those columns) would see stale memory
  GWN_REQUIRE(!a->tg4 || !wgrads || a->adp_index < 0 || !a->dadp,
              "gcn_bwd: tg4 needs skip_weight_grads (the caller runs gwn_gram_g4_bf16 on tg4)");
  int rc = GWN_OK;
  if (fused) {
    // fused: dxg -> dhcat piece 0 (or dfg through the gate epilogue); for the adaptive support
    // dx1 -> piece 1, dx2 -> piece 2
    float* t1 = a->dhcat + c;
    float* t2 = a->dhcat + 2 * c;
    rc = gwn_gcn_fused_bwd_launch(a, a->sup_t, a->dhcat, a->ld_dhcat, t1, t2, a->ld_dhcat, s);
    if (rc) return rc;
  }
  // dW_mlp[j][k] = sum_r dh[r][j] h[r][k];  db_mlp[j] = sum_r dh[r][j]
  gwn_gemm_desc d = gemm_zero();
  if (!wgrads) {
  } else if (co % 32 == 0 && width % 32 == 0 && (co / 32) * (width / 32) <= 16) {
    rc = gwn_wgrad(dh, co, co, a->h, a->ld_h, a->rows, width, 1, 0, a->rows, a->dw_mlp, width, a->db_mlp,
                   a->workspace, s);
  } else {
    d.A = dh; d.lda_m = 1; d.lda_k = co;
    d.B = a->h; d.ldb_k = a->ld_h; d.ldb_n = 1;
    d.C = a->dw_mlp; d.ldc_m = width; d.ldc_n = 1;
    d.ones_out = a->db_mlp;
    d.M = co; d.N = width; d.K = a->rows;
    d.ksplit = gcn_w_ksplit(a->rows, co, width);
    d.part = a->workspace;
    rc = gwn_gemm_launch(d, s);
  }
  if (rc) return rc;
  if (fused) {
    float* t1 = a->dhcat + c;
    float* t2 = a->dhcat + 2 * c;
    if (wgrads && a->adp_index >= 0 && a->adp_index < a->nsup && a->dadp) {
      // dA = sum xg (x) dx1 + sum x1 (x) dx2: one launch over both pairs
      const int k = a->adp_index;
      const float* x1 = a->h + (1 + 2 * k) * c;
      if (gram_eligible(a->h, a->ld_h, t1, a->ld_dhcat, c) && gram_eligible(x1, a->ld_h, t2, a->ld_dhcat, c))
        return gwn_gram_dtype(a->h, t1, x1, t2, a->ld_h, a->ld_dhcat, n, slices, a->dadp, a->ld_sup,
                              a->accumulate_dadp, a->workspace, a->split_planes >= 1 ? 1 : 0, s);
      rc = gwn_nconv_adj_grad(a->h, a->ld_h, t1, a->ld_dhcat, n, c, slices, a->dadp, a->ld_sup,
                              a->accumulate_dadp, a->workspace, s);
      if (rc) return rc;
      rc = gwn_nconv_adj_grad(x1, a->ld_h, t2, a->ld_dhcat, n, c, slices, a->dadp, a->ld_sup, 1,
                              a->workspace, s);
    }
    return rc;
  }
  // dhcat[r][k] = sum_j dh[r][j] W[j][k]
  d = gemm_zero();
  d.A = a->dh; d.lda_m = co; d.lda_k = 1;
  d.B = a->w_mlp; d.ldb_k = width; d.ldb_n = 1;
  d.C = a->dhcat; d.ldc_m = a->ld_dhcat; d.ldc_n = 1;
  d.M = a->rows; d.N = width; d.K = co;
  rc = gwn_gemm_launch(d, s);
  if (rc) return rc;
  // A x = (A^T)^T x: with the transposed supports the products run on the transpose_a = 1 kernels
  // (the large-graph diffusion for n > 512)
  const float* const* sa = a->sup_t ? a->sup_t : a->sup;
  const int ta = a->sup_t ? 1 : 0;
  for (int k = 0; k < a->nsup; ++k) {
    float* t1 = a->dhcat + (1 + 2 * k) * c;        // dL/dx1 (gets the x2 path added)
    const float* t2 = a->dhcat + (2 + 2 * k) * c;  // dL/dx2
    // x2 = A^T x1  =>  dx1 += A dx2
    rc = gwn_nconv(sa[k], a->ld_sup, ta, t2, a->ld_dhcat, t1, a->ld_dhcat, t1, a->ld_dhcat, n, c, slices, s);
    if (rc) return rc;
    if (wgrads && k == a->adp_index && a->dadp) {
      // dA = sum xg (x) dx1  +  sum x1 (x) dx2
      rc = gwn_nconv_adj_grad(a->h, a->ld_h, t1, a->ld_dhcat, n, c, slices, a->dadp, a->ld_sup,
                              a->accumulate_dadp, a->workspace, s);
      if (rc) return rc;
      rc = gwn_nconv_adj_grad(a->h + (1 + 2 * k) * c, a->ld_h, t2, a->ld_dhcat, n, c, slices, a->dadp,
                              a->ld_sup, 1, a->workspace, s);
      if (rc) return rc;
    }
    // x1 = A^T xg  =>  dxg += A dx1   (dxg is piece 0 of dhcat)
    rc = gwn_nconv(sa[k], a->ld_sup, ta, t1, a->ld_dhcat, a->dhcat, a->ld_dhcat, a->dhcat, a->ld_dhcat, n, c,
                   slices, s);
    if (rc) return rc;
  }
  return GWN_OK;
}

// ---------------------------------------------------------------------------------------------
long gwn_batchnorm_workspace_floats(int rows, int c) {
  (void)rows;
  return (long)RED_BLOCKS * 3 * (c > 0 ? c : 1) + 2L * c;
}

int gwn_batchnorm_fwd(const float* z, int rows, int c, const float* gamma, const float* beta,
                      float* running_mean, float* running_var, float momentum, float eps, int training,
                      float* out, float* save_mean, float* save_rstd, float* ws, hipStream_t s) {
  GWN_REQUIRE(rows > 0 && c > 0 && c <= 256 && 256 % c == 0, "batchnorm_fwd: c must divide 256");
  const long total = (long)rows * c;
  if (training) {
    bn_partial_kernel<<<RED_BLOCKS, 256, 0, s>>>(z, rows, c, ws);
    GWN_CHECK_LAUNCH();
    bn_finalize_kernel<<<c, 256, 0, s>>>(ws, RED_BLOCKS, c, momentum, eps, running_mean, running_var,
                                         save_mean, save_rstd, nullptr);
    GWN_CHECK_LAUNCH();
    bn_apply_kernel<<<grid_for(total), 256, 0, s>>>(z, rows, c, save_mean, save_rstd, nullptr, eps,
                                                    gamma, beta, out);
  } else {
    bn_apply_kernel<<<grid_for(total), 256, 0, s>>>(z, rows, c, running_mean, nullptr, running_var,
                                                    eps, gamma, beta, out);
    if (save_mean && save_rstd) {
      // the statistics an eval-mode backward differentiates through (gwn_batchnorm_bwd, batch_stats 0)
      GWN_CHECK_LAUNCH();
      bn_running_stats_kernel<<<(c + 255) / 256, 256, 0, s>>>(running_mean, running_var, c, eps, save_mean,
                                                             save_rstd);
    }
  }
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

int gwn_batchnorm_fwd_partials(const float* z, int rows, int c, const float* partials, int nparts,
                               const float* gamma, const float* beta, float* running_mean, float* running_var,
                               float momentum, float eps, float* out, float* save_mean, float* save_rstd,
                               long long* num_batches_tracked, hipStream_t s) {
  GWN_REQUIRE(rows > 0 && c > 0 && nparts > 0, "batchnorm_fwd_partials: bad shape");
  bn_finalize_kernel<<<c, 256, 0, s>>>(partials, nparts, c, momentum, eps, running_mean, running_var,
                                       save_mean, save_rstd, num_batches_tracked);
  GWN_CHECK_LAUNCH();
  const long total = (long)rows * c;
  bn_apply_kernel<<<grid_for(total), 256, 0, s>>>(z, rows, c, save_mean, save_rstd, nullptr, eps, gamma,
                                                  beta, out);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

int gwn_batchnorm_fwd_fold(const float* partials, int nparts, int c, const float* gamma, const float* beta,
                           float* running_mean, float* running_var, float momentum, float eps, float* save_mean,
                           float* save_rstd, float* scale, const float* w_next, const float* b_next, float* w_fold,
                           float* b_fold, long long* num_batches_tracked, hipStream_t s) {
  GWN_REQUIRE(c == 32 && nparts > 0 && partials && gamma && beta && save_mean && save_rstd && scale,
              "batchnorm_fwd_fold: needs c == 32, the partials, gamma / beta and the outputs");
  GWN_REQUIRE(!w_next || (b_next && w_fold && b_fold && w_fold != w_next),
              "batchnorm_fwd_fold: w_next needs b_next, w_fold, b_fold (w_fold not aliasing w_next)");
  bn_finalize_fold_kernel<<<c, 256, 0, s>>>(partials, nparts, c, momentum, eps, gamma, beta, running_mean,
                                            running_var, save_mean, save_rstd, scale, w_next, b_next, w_fold, b_fold,
                                            num_batches_tracked);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

int gwn_batchnorm_bwd(const float* dy, const float* z, int rows, int c, const float* gamma,
                      const float* save_mean, const float* save_rstd, float* dgamma, float* dbeta,
                      float* dres, int res_row0, float* dh, const unsigned long long* seed_ptr,
                      unsigned long long salt, float drop_p, int batch_stats, float* ws, hipStream_t s) {
  GWN_REQUIRE(rows > 0 && c > 0 && c <= 256 && 256 % c == 0, "batchnorm_bwd: c must divide 256");
  GWN_REQUIRE(drop_p <= 0.0f || (long long)rows * c < (1LL << 32),
              "batchnorm_bwd: dropout masks index rows*c elements in 32 bits (gwn_uniform)");
  float* part = ws;
  float* sums = ws + (long)RED_BLOCKS * 3 * c;  // [2][c]: sum dy, sum dy*xhat
  bn_bwd_partial_kernel<<<RED_BLOCKS, 256, 0, s>>>(dy, z, save_mean, save_rstd, rows, c, part);
  GWN_CHECK_LAUNCH();
  colsum_final_wide_kernel<<<2 * c, 256, 0, s>>>(part, RED_BLOCKS, 2 * c, sums, 0);
  GWN_CHECK_LAUNCH();
  const long total = (long)rows * c + (long)res_row0 * c;
  // batch statistics: the mean / xhat terms of d(mean), d(var); running statistics: affine only
  const float inv_n = batch_stats ? 1.0f / (float)rows : 0.0f;
  bn_bwd_apply_kernel<<<grid_for(total), 256, 0, s>>>(dy, z, rows, c, gamma, save_mean, save_rstd, sums,
                                                      inv_n, dres, res_row0, dh, seed_ptr, salt, drop_p,
                                                      dgamma, dbeta);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

long gwn_colsum_workspace_floats(int rows, int ncol) {
  (void)rows;
  return (long)RED_BLOCKS * ncol;
}

int gwn_colsum(const float* dy, int rows, int ncol, long ld, float* out, int accumulate, float* ws,
               hipStream_t s) {
  GWN_REQUIRE(rows > 0 && ncol > 0, "colsum: bad shape");
  colsum_partial_kernel<0><<<RED_BLOCKS, 256, 0, s>>>(dy, ld, nullptr, 0, nullptr, nullptr, rows, ncol, ws);
  GWN_CHECK_LAUNCH();
  colsum_final_wide_kernel<<<ncol, 256, 0, s>>>(ws, RED_BLOCKS, ncol, out, accumulate);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

// ---------------------------------------------------------------------------------------------
long gwn_masked_loss_workspace_floats(int B, int o, int n, int tf) {
  (void)B; (void)o; (void)n; (void)tf;
  return LOSS_ARRIVE + 1;
}

int gwn_masked_loss(const float* out, const float* real, long rsb, long rsn, long rso, int B, int o,
                    int n, int tf, float mean, float std, float* metrics, float* dout, float* ws,
                    hipStream_t s) {
  GWN_REQUIRE(B > 0 && o > 0 && n > 0 && tf > 0 && (long)B * o * n * tf < (1L << 31), "masked_loss: bad shape");
  loss_count_kernel<<<LOSS_CNT_BLOCKS, 256, 0, s>>>(real, rsb, rsn, rso, B, n, o, ws);
  GWN_CHECK_LAUNCH();
  loss_terms_kernel<false><<<LOSS_TERM_BLOCKS, 256, 0, s>>>(out, real, rsb, rsn, rso, B, o, n, tf, mean, std, dout,
                                                             ws, metrics, 0, 0);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

int gwn_masked_loss_rows(const float* y, int ld_y, const float* real, long rsb, long rsn, long rso, int B, int o,
                         int n, int tf, float mean, float std, float* metrics, float* dy, int ld_dy, float* ws,
                         hipStream_t s) {
  GWN_REQUIRE(B > 0 && o > 0 && n > 0 && tf > 0 && ld_y >= o && (!dy || ld_dy >= o) && (long)B * o * n * tf < (1L << 31),
              "masked_loss_rows: bad shape");
  loss_count_kernel<<<LOSS_CNT_BLOCKS, 256, 0, s>>>(real, rsb, rsn, rso, B, n, o, ws);
  GWN_CHECK_LAUNCH();
  loss_terms_kernel<true><<<LOSS_TERM_BLOCKS, 256, 0, s>>>(y, real, rsb, rsn, rso, B, o, n, tf, mean, std, dy, ws,
                                                           metrics, ld_y, ld_dy);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

// ---------------------------------------------------------------------------------------------
long gwn_clip_adam_workspace_floats(long total) {
  (void)total;
  return RED_BLOCKS + 2;  // sq-sum partials, (unused), arrival counter
}

int gwn_adam_clipped(float* params, float* grads, float* exp_avg, float* exp_avg_sq, const long* lo,
                     const long* hi, int nranges, long active, float max_norm, float lr, float beta1,
                     float beta2, float eps, float wd, long long* step_ptr, float* ws, float* total_norm_out,
                     unsigned long long* seed, unsigned long long seed_inc, hipStream_t s) {
  GWN_REQUIRE(nranges > 0 && active > 0, "adam_clipped: empty");
  const long want = (active + 255) / 256;
  const int blocks = (int)(want < ADAM_BLOCKS ? want : ADAM_BLOCKS);
  adam_clipped_kernel<<<blocks, 256, 0, s>>>(params, grads, exp_avg, exp_avg_sq, lo, hi, nranges, active,
                                                       ws, step_ptr, max_norm, lr, beta1, beta2, eps, wd,
                                                       total_norm_out, seed, seed_inc);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

int gwn_clip_adam(float* params, float* grads, float* exp_avg, float* exp_avg_sq, const long* lo,
                  const long* hi, int nranges, long active, float max_norm, float lr, float beta1,
                  float beta2, float eps, float wd, long long* step_ptr, float* ws,
                  float* total_norm_out, hipStream_t s) {
  GWN_REQUIRE(nranges > 0 && active > 0, "clip_adam: empty");
  sqnorm_partial_kernel<<<RED_BLOCKS, 256, 0, s>>>(grads, lo, hi, nranges, active, ws);
  GWN_CHECK_LAUNCH();
  return gwn_adam_clipped(params, grads, exp_avg, exp_avg_sq, lo, hi, nranges, active, max_norm, lr, beta1, beta2,
                          eps, wd, step_ptr, ws, total_norm_out, nullptr, 0, s);
}

int gwn_sqnorm_partials(const float* grads, const long* lo, const long* hi, int nranges, long active, float* ws,
                        hipStream_t s) {
  GWN_REQUIRE(nranges > 0 && active > 0, "sqnorm_partials: empty");
  sqnorm_partial_kernel<<<RED_BLOCKS, 256, 0, s>>>(grads, lo, hi, nranges, active, ws);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

int gwn_gather_sqnorm(const float* src, const int* idx, float* dst, long count, float* ws, hipStream_t s) {
  GWN_REQUIRE(count > 0, "gather_sqnorm: empty");
  gather_sqnorm_kernel<<<RED_BLOCKS, 256, 0, s>>>(src, idx, dst, count, ws);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

int gwn_gather(const float* src, const int* idx, float* dst, long count, hipStream_t s) {
  if (count <= 0) return GWN_OK;
  gather_kernel<<<grid_for(count), 256, 0, s>>>(src, idx, dst, count);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

int gwn_gather_sum(const float* src, const int* idx, float* dst, long count, long sum_src, int nvec, int len,
                   long sum_dst, hipStream_t s) {
  GWN_REQUIRE(count > 0 && nvec >= 0 && len >= 0 && sum_src >= 0 && sum_src + (long)nvec * len <= count &&
                  sum_dst >= 0 && sum_dst + len <= count,
              "gather_sum: segments outside [0, count)");
  gather_sum_kernel<<<grid_for(count + len), 256, 0, s>>>(src, idx, dst, count, sum_src, nvec, len, sum_dst);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

int gwn_to_nchw(const float* y, int B, int o, int n, int t, float* out, hipStream_t s) {
  const long total = (long)B * o * n * t;
  to_nchw_kernel<<<grid_for(total), 256, 0, s>>>(y, B, o, n, t, out);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

int gwn_from_nchw(const float* dout, int B, int o, int n, int t, float* dy, hipStream_t s) {
  return gwn_from_nchw_ld(dout, B, o, n, t, dy, o, s);
}

int gwn_from_nchw_ld(const float* dout, int B, int o, int n, int t, float* dy, int ld_dy, hipStream_t s) {
  GWN_REQUIRE(ld_dy >= o, "from_nchw: ld_dy < o");
  const long total = (long)B * o * n * t;
  from_nchw_kernel<<<grid_for(total), 256, 0, s>>>(dout, B, o, n, t, dy, ld_dy);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

int gwn_sum_vectors(const float* x, int count, int len, long stride, float* out, hipStream_t s) {
  sum_vectors_kernel<<<(len + 255) / 256, 256, 0, s>>>(x, count, len, stride, out);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

int gwn_increment_u64(unsigned long long* counter, unsigned long long inc, hipStream_t s) {
  increment_kernel<<<1, 64, 0, s>>>(counter, inc);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

}  // extern "C"
