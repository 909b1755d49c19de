// Weight (+ bias) gradients of the channels-last 1x1 / dilated convolutions:
//     dW[j][k] = sum_r dY[r][j] * X[r + tap(k)*shift][col(k)],    db[j] = sum_r dY[r][j]
// with j < J (32 or 64), k < Kc = ntaps * Kt, tap(k) = k / Kt, col(k) = k % Kt, r < R (all
// positions: ~10^5 rows).  Used for the gcn mlp (J = 32, Kc = 224, X = the concat buffer h) and the
// gated TCN (J = 64, Kc = 2 taps x 32).  Memory-bound: every input byte is read once from HBM.
//
// A wave owns one 32x32 output tile for its whole life; a workgroup holds all (J/32)*(Kc/32) tiles
// and walks one contiguous row range, so the partial of a workgroup is the full dW.  An MFMA
// k-step covers two rows: lane (i, h) loads dY[r + h][32*jt + i] (A operand) and
// X[r + h (+shift)][32*kt + i] (B operand) — each wave-load instruction is two 128-B row
// segments.  No LDS, no barriers; 16 k-steps of loads are in flight ahead of the MFMAs.  The
// bias gradient rides along on the kt == 0 waves (VALU sums of the A fragments).  Workgroup
// partials [nblk][J*Kc + J] are summed in a fixed order by the reduce kernel (deterministic).
#include "gwn_internal.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int D = 16;  // k-steps (row pairs) per batch
#ifndef WGRAD_WAVES_PER_CU
#define WGRAD_WAVES_PER_CU 8  // target resident waves per CU (whole workgroups); 8 beat 16 and 32 (fewer
                              // partials to write and reduce: mlp dW 37 vs 41 us at T=12, +1 % per step)
#endif

struct Wgrad {
  const float* dY; long ldy; int J;
  const float* X; long ldx; long x_rows; int Kt, ntaps; long shift;
  int R, nblk;
  float* part;  // [nblk][J*Kc + J]
  const float* x_mean; const float* x_scale; const float* x_shift;  // AFF: X = (X - mean) * scale + shift
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float bld(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ int crow(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }

template <bool AFF>
__global__ __launch_bounds__(1024) void wgrad_kernel(const Wgrad g) {
  const int lane = threadIdx.x & 63, half = lane >> 5, col = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (scalar) tile
  const int Kc = g.ntaps * g.Kt, nkt = Kc / 32;
  const int jt = wave / nkt, kt = wave % nkt;
  const int tap = (32 * kt) / g.Kt, xc = 32 * kt - tap * g.Kt;
  const int r0 = (int)((long)g.R * blockIdx.x / g.nblk), r1 = (int)((long)g.R * (blockIdx.x + 1) / g.nblk);

  // buffer windows end at this workgroup's last row: rows >= r1 read zeros with no per-lane
  // predicate (a predicated offset would be compiled into branches around the loads)
  const long xshift = (long)tap * g.shift;
  const __amdgpu_buffer_rsrc_t ry = rsrc(g.dY, (long)r1 * g.ldy * 4);
  const __amdgpu_buffer_rsrc_t rx = rsrc(g.X, (r1 + xshift) * g.ldx * 4);
  // AFF (BatchNorm on load): zero rows past r1 become finite junk, but their dY rows are zero too
  const float xmu = AFF ? g.x_mean[xc + col] : 0.0f;
  const float xsc = AFF ? g.x_scale[xc + col] : 1.0f, xsh = AFF ? g.x_shift[xc + col] : 0.0f;
  auto load = [&](int r, float* a, float* b) {
    const int oy = (int)(((long)(r + half) * g.ldy + 32 * jt + col) * 4);
    const int ox = (int)((((long)(r + half) + xshift) * g.ldx + xc + col) * 4);
#pragma unroll
    for (int s = 0; s < D; ++s) {
      a[s] = bld(ry, oy + (int)(2 * s * g.ldy * 4));
      b[s] = bld(rx, ox + (int)(2 * s * g.ldx * 4));
    }
    if (AFF) {
#pragma unroll
      for (int s = 0; s < D; ++s) b[s] = fmaf(b[s] - xmu, xsc, xsh);
    }
  };

  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
  float bsum = 0.0f;
  float a[D], b[D];
  load(r0, a, b);
  for (int r = r0; r < r1; r += 2 * D) {
    float an[D], bn[D];
    load(r + 2 * D, an, bn);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < D; ++s) {
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b[s], acc, 0, 0, 0);
      bsum += a[s];
    }
#pragma unroll
    for (int s = 0; s < D; ++s) { a[s] = an[s]; b[s] = bn[s]; }
  }
  // D[j][k]: col = lane&31 -> k, rows -> j
  const int stride = g.J * Kc + g.J;
  float* out = g.part + (long)blockIdx.x * stride;
#pragma unroll
  for (int i = 0; i < 16; ++i) out[(32 * jt + crow(i, half)) * Kc + 32 * kt + col] = acc[i];
  if (kt == 0) {
    // lane (i, h) summed rows of parity h for j = 32 jt + i: add the two halves
    const float other = __shfl_xor(bsum, 32);
    if (half == 0) out[g.J * Kc + 32 * jt + col] = bsum + other;
  }
}

// dW[j][k] (ld_w) and db[j] from the workgroup partials: 32 consecutive outputs per workgroup x 8
// partial lanes (lane l sums partials l, l+8, ...; every wave-load is two 128-B segments), then a
// fixed-order tree over the 8 lanes
__global__ void wgrad_reduce_kernel(const float* part, int nblk, int J, int Kc, float* dW, long ld_w, float* db) {
  __shared__ float sh[256];
  const int stride = J * Kc + J;
  const int ej = threadIdx.x & 31, l = threadIdx.x >> 5;
  const int idx = blockIdx.x * 32 + ej;
  // four independent chains per lane keep four loads in flight; merged in a fixed order
  float v0 = 0.0f, v1 = 0.0f, v2 = 0.0f, v3 = 0.0f;
  if (idx < stride) {
    const float* p = part + idx;
    int b = l;
    for (; b + 24 < nblk; b += 32) {
      v0 += p[(long)b * stride];
      v1 += p[(long)(b + 8) * stride];
      v2 += p[(long)(b + 16) * stride];
      v3 += p[(long)(b + 24) * stride];
    }
    for (; b < nblk; b += 8) v0 += p[(long)b * stride];
  }
  sh[threadIdx.x] = (v0 + v1) + (v2 + v3);
  __syncthreads();
#pragma unroll
  for (int w = 4; w > 0; w >>= 1) {
    if (l < w) sh[threadIdx.x] += sh[threadIdx.x + 32 * w];
    __syncthreads();
  }
  if (l != 0 || idx >= stride) return;
  if (idx < J * Kc) dW[(long)(idx / Kc) * ld_w + idx % Kc] = sh[ej];
  else if (db) db[idx - J * Kc] = sh[ej];
}

// One launch reduces many partial sets (the deferred weight gradients of a whole backward,
// gwn_reduce_partials): block b belongs to the segment whose block range holds it; each block sums
// 32 consecutive outputs of its segment over the segment's partials with the wgrad_reduce_kernel
// scheme (8 partial lanes x 4 chains, fixed-order tree); output i < J*Kc -> out[(i / Kc) * ld + i % Kc],
// else out2[i - J*Kc].
constexpr int MAXSEG = 32;  // the table travels as a kernel argument (<= 4 KB)
struct SegTable {
  gwn_reduce_seg seg[MAXSEG];
  int first_block[MAXSEG + 1];
  int nseg;
};

__global__ void reduce_segments_kernel(const SegTable t) {
  __shared__ float sh[256];
  int si = 0;
  while (si + 1 < t.nseg && (int)blockIdx.x >= t.first_block[si + 1]) ++si;
  const gwn_reduce_seg& g = t.seg[si];
  const int ej = threadIdx.x & 31, l = threadIdx.x >> 5;
  const long i = (long)(blockIdx.x - t.first_block[si]) * 32 + ej;
  const long jk = (long)g.J * g.Kc, outs = jk + g.J;
  const long dbo = g.db_off ? g.db_off : jk;
  float v0 = 0.0f, v1 = 0.0f, v2 = 0.0f, v3 = 0.0f;
  if (i < outs) {
    const float* p = g.part + (i < jk ? i : dbo + (i - jk));
    const long st = g.part_stride;
    int b = l;
    for (; b + 24 < g.nparts; b += 32) {
      v0 += p[(long)b * st];
      v1 += p[(long)(b + 8) * st];
      v2 += p[(long)(b + 16) * st];
      v3 += p[(long)(b + 24) * st];
    }
    for (; b < g.nparts; b += 8) v0 += p[(long)b * st];
  }
  sh[threadIdx.x] = (v0 + v1) + (v2 + v3);
  __syncthreads();
#pragma unroll
  for (int w = 4; w > 0; w >>= 1) {
    if (l < w) sh[threadIdx.x] += sh[threadIdx.x + 32 * w];
    __syncthreads();
  }
  if (l != 0 || i >= outs) return;
  if (i < jk) g.out[(i / g.Kc) * g.ld_out + i % g.Kc] = sh[ej];
  else if (g.out2) g.out2[i - jk] = sh[ej];
}

// Narrow inputs (the start conv: Kc = in_dim = 2 channels, J = 32): 256-thread workgroups over
// contiguous row ranges, thread (row lane l, channel j) accumulating dY[r][j] * X[r][k] (k < Kc)
// and dY[r][j] over rows r = l mod 8; the 8 row lanes are folded in a fixed order and the
// workgroup partial [J*Kc + J] written for gwn_reduce_partials.
// 1024-thread workgroups (round 2; 256 took 25 us for the start conv's 22 MB dY: too few loads in
// flight for a latency-bound stream with the partial count capped for the reduction)
constexpr int SMALL_KC = 4, SMALL_BLK = 512, SMALL_ROWS = 64, SMALL_T = 1024;  // <= 512 workgroups (partials to reduce)
__global__ __launch_bounds__(SMALL_T) void wgrad_small_kernel(const float* dY, long ldy, int J, const float* X, long ldx,
                                                              int Kc, int R, float* part) {
  __shared__ float sh[SMALL_KC + 1][SMALL_T];
  const int j = threadIdx.x % J, l = threadIdx.x / J, lanes = SMALL_T / J;
  const int r0 = (int)((long)R * blockIdx.x / gridDim.x), r1 = (int)((long)R * (blockIdx.x + 1) / gridDim.x);
  float acc[SMALL_KC + 1];
#pragma unroll
  for (int k = 0; k <= SMALL_KC; ++k) acc[k] = 0.0f;
  if (l < lanes) {
#pragma unroll 8
    for (int r = r0 + l; r < r1; r += lanes) {
      const float dy = dY[(long)r * ldy + j];
#pragma unroll
      for (int k = 0; k < SMALL_KC; ++k)
        if (k < Kc) acc[k] = fmaf(dy, X[(long)r * ldx + k], acc[k]);
      acc[SMALL_KC] += dy;
    }
  }
#pragma unroll
  for (int k = 0; k <= SMALL_KC; ++k) sh[k][threadIdx.x] = acc[k];
  __syncthreads();
  if (l != 0) return;
  float* out = part + (long)blockIdx.x * (J * Kc + J);
#pragma unroll
  for (int k = 0; k <= SMALL_KC; ++k) {
    if (k < Kc || k == SMALL_KC) {
      float v = 0.0f;
      for (int q = 0; q < lanes; ++q) v += sh[k][q * J + j];
      if (k < Kc) out[j * Kc + k] = v;
      else out[J * Kc + j] = v;
    }
  }
}

// J = 32 with 16-B aligned dY rows (the start conv's weight gradient): lane (row slot, quad) owns
// channels 4 quad .. +3 of every eighth row of its share (one 16-B dY load and one Kc-float X load
// per row), the eight row slots of a wave summed by lane exchange, the sixteen waves through LDS in
// a fixed order.  (The generic form: one channel per lane, 14.4 us per METR step.)
__global__ __launch_bounds__(SMALL_T) void wgrad_small32_kernel(const float* dY, long ldy, const float* X, long ldx,
                                                               int Kc, int R, float* part) {
  __shared__ float sh[SMALL_T / 64][8][4 * (SMALL_KC + 1)];
  const int qd = threadIdx.x & 7, slot = threadIdx.x >> 3, nslot = SMALL_T / 8;
  const int r0 = (int)((long)R * blockIdx.x / gridDim.x), r1 = (int)((long)R * (blockIdx.x + 1) / gridDim.x);
  float acc[4][SMALL_KC + 1];
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int k = 0; k <= SMALL_KC; ++k) acc[e][k] = 0.0f;
#pragma unroll 4
  for (int r = r0 + slot; r < r1; r += nslot) {
    const float4 dy = *(const float4*)(dY + (long)r * ldy + 4 * qd);
    const float d4[4] = {dy.x, dy.y, dy.z, dy.w};
    float xk[SMALL_KC];
#pragma unroll
    for (int k = 0; k < SMALL_KC; ++k) xk[k] = k < Kc ? X[(long)r * ldx + k] : 0.0f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
#pragma unroll
      for (int k = 0; k < SMALL_KC; ++k) acc[e][k] = fmaf(d4[e], xk[k], acc[e][k]);
      acc[e][SMALL_KC] += d4[e];
    }
  }
  // the wave's eight row slots (lane bits 3..5) summed by exchange
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int k = 0; k <= SMALL_KC; ++k) {
      float v = acc[e][k];
      v += __shfl_xor(v, 8);
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      acc[e][k] = v;
    }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane < 8) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int k = 0; k <= SMALL_KC; ++k) sh[wave][lane][e * (SMALL_KC + 1) + k] = acc[e][k];
  }
  __syncthreads();
  if (threadIdx.x >= 32) return;
  const int j = threadIdx.x, q = j >> 2, e = j & 3;
  float* out = part + (long)blockIdx.x * (32 * Kc + 32);
#pragma unroll
  for (int k = 0; k <= SMALL_KC; ++k) {
    if (k < Kc || k == SMALL_KC) {
      float v = 0.0f;
      for (int w = 0; w < SMALL_T / 64; ++w) v += sh[w][q][e * (SMALL_KC + 1) + k];
      if (k < Kc) out[j * Kc + k] = v;
      else out[32 * Kc + j] = v;
    }
  }
}

int wgrad_nblk(int R, int waves_per_blk) {
  // a whole number of workgroups per CU (256 CUs), ~WGRAD_WAVES_PER_CU waves per CU; >= 256 rows per workgroup
  int per_cu = WGRAD_WAVES_PER_CU / waves_per_blk;
  if (per_cu < 1) per_cu = 1;
  int nb = 256 * per_cu;
  const int byrows = R / 256;
  if (nb > byrows) nb = byrows;
  return nb < 1 ? 1 : nb;
}

}  // namespace

int gwn_wgrad_partial_count(int R, int J, int Kc) {
  if (R <= 0) return 0;
  if (Kc <= SMALL_KC && J > 0 && J <= 256 && 256 % J == 0) {
    const int nb = (R + SMALL_ROWS - 1) / SMALL_ROWS;
    return nb < SMALL_BLK ? nb : SMALL_BLK;
  }
  if (J < 32 || Kc < 32 || J % 32 || Kc % 32) return 0;
  return wgrad_nblk(R, (J / 32) * (Kc / 32));
}

long gwn_wgrad_workspace_floats(int R, int J, int Kc) {
  if (J < 32 || Kc < 32 || J % 32 || Kc % 32 || R <= 0) return 0;  // not eligible: no workspace
  return (long)wgrad_nblk(R, (J / 32) * (Kc / 32)) * (J * Kc + J);
}

// dW[j][k] = sum_r dY[r][j] X[r + (k / Kt) * shift][k % Kt]; db[j] = sum_r dY[r][j] (db may be NULL)
int gwn_wgrad(const float* dY, long ldy, int J, const float* X, long ldx, long x_rows, int Kt, int ntaps,
              long shift, int R, float* dW, long ld_w, float* db, float* ws, hipStream_t s) {
  return gwn_wgrad_bn(dY, ldy, J, X, ldx, x_rows, Kt, ntaps, shift, R, nullptr, nullptr, nullptr, dW, ld_w, db, ws,
                      s);
}

// the same with X = (X - x_mean[k % Kt]) * x_scale[k % Kt] + x_shift[k % Kt] on load (all NULL: plain)
int gwn_wgrad_bn(const float* dY, long ldy, int J, const float* X, long ldx, long x_rows, int Kt, int ntaps,
                 long shift, int R, const float* x_mean, const float* x_scale, const float* x_shift, float* dW,
                 long ld_w, float* db, float* ws, hipStream_t s) {
  GWN_REQUIRE(!x_scale == !x_shift && !x_scale == !x_mean, "wgrad: x_mean, x_scale and x_shift go together");
  const int Kc = Kt * ntaps;
  GWN_REQUIRE(J % 32 == 0 && Kt % 32 == 0 && R > 0 && ws, "wgrad: J and Kt must be multiples of 32");
  const int wpb = (J / 32) * (Kc / 32);
  GWN_REQUIRE(wpb <= 16, "wgrad: at most 16 output tiles");
  GWN_REQUIRE((long)R * ldy * 4 < 0x7fff0000L && x_rows * ldx * 4 < 0x7fff0000L,
              "wgrad: operand beyond a 2 GB buffer window");
  GWN_REQUIRE(x_rows >= (long)R + (ntaps - 1) * shift, "wgrad: X rows do not cover the taps");
  Wgrad g = {};
  g.dY = dY; g.ldy = ldy; g.J = J;
  g.X = X; g.ldx = ldx; g.x_rows = x_rows; g.Kt = Kt; g.ntaps = ntaps; g.shift = shift;
  g.R = R; g.nblk = wgrad_nblk(R, wpb);
  g.part = ws;
  g.x_mean = x_mean; g.x_scale = x_scale; g.x_shift = x_shift;
  if (x_scale) wgrad_kernel<true><<<g.nblk, 64 * wpb, 0, s>>>(g);
  else wgrad_kernel<false><<<g.nblk, 64 * wpb, 0, s>>>(g);
  GWN_CHECK_LAUNCH();
  if (!dW) return GWN_OK;  // partials only (gwn_wgrad_partials)
  const int outs = J * Kc + J;
  wgrad_reduce_kernel<<<(outs + 31) / 32, 256, 0, s>>>(ws, g.nblk, J, Kc, dW, ld_w, db);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

// partials only: part [gwn_wgrad_partial_count(R, J, Kc)][J*Kc + J], reduced later by
// gwn_reduce_partials (kind 0)
int gwn_wgrad_partials(const float* dY, long ldy, int J, const float* X, long ldx, long x_rows, int Kt, int ntaps,
                       long shift, int R, const float* x_mean, const float* x_scale, const float* x_shift, float* part,
                       hipStream_t s) {
  GWN_REQUIRE(part != nullptr, "wgrad_partials: part is required");
  if (Kt * ntaps <= SMALL_KC && J > 0 && J <= 256 && 256 % J == 0) {  // narrow inputs (1x1, no affine)
    GWN_REQUIRE(ntaps == 1 && !x_mean && !x_scale && !x_shift && x_rows >= R, "wgrad_partials: narrow form is 1x1, plain");
    if (J == 32 && ldy % 4 == 0 && ((uintptr_t)dY & 15) == 0)
      wgrad_small32_kernel<<<gwn_wgrad_partial_count(R, J, Kt), SMALL_T, 0, s>>>(dY, ldy, X, ldx, Kt, R, part);
    else
      wgrad_small_kernel<<<gwn_wgrad_partial_count(R, J, Kt), SMALL_T, 0, s>>>(dY, ldy, J, X, ldx, Kt, R, part);
    GWN_CHECK_LAUNCH();
    return GWN_OK;
  }
  return gwn_wgrad_bn(dY, ldy, J, X, ldx, x_rows, Kt, ntaps, shift, R, x_mean, x_scale, x_shift, nullptr, 0, nullptr,
                      part, s);
}

int gwn_reduce_partials(const gwn_reduce_seg* segs, int nseg, hipStream_t s) {
  GWN_REQUIRE(nseg >= 0 && nseg <= MAXSEG && (nseg == 0 || segs), "reduce_partials: 0..32 segments");
  SegTable t = {};
  int blocks = 0;
  for (int i = 0; i < nseg; ++i) {
    const gwn_reduce_seg& g = segs[i];
    const long dbo = g.db_off ? g.db_off : (long)g.J * g.Kc;
    GWN_REQUIRE(g.part && g.out && g.nparts > 0 && g.J > 0 && g.Kc > 0 && g.ld_out >= g.Kc &&
                    dbo >= (long)g.J * g.Kc && g.part_stride >= dbo + g.J,
                "reduce_partials: segment needs part, out, nparts > 0, J, Kc, ld_out >= Kc, db_off >= J*Kc, "
                "stride >= db_off + J");
    const long outs = (long)g.J * g.Kc + g.J;
    t.seg[i] = g;
    t.first_block[i] = blocks;
    blocks += (int)((outs + 31) / 32);
  }
  t.first_block[nseg] = blocks;
  t.nseg = nseg;
  if (!blocks) return GWN_OK;
  reduce_segments_kernel<<<blocks, 256, 0, s>>>(t);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}
