// Grouped weight (+ bias) gradients: ONE launch for the same 1x1 / dilated conv weight of several
// layers (the deferred weight gradients of a whole backward: the gcn mlp of every layer, the gated
// TCN of every layer), each problem p
//     dW_p[j][k] = sum_r dY_p[r][j] * X_p[r + tap(k)*shift_p][col(k)],   db_p[j] = sum_r dY_p[r][j]
// with tap(k) = k / Kt, col(k) = k % Kt (k < Kc = ntaps*Kt), and X optionally normalised on load
// (BatchNorm folded: X = (X - mean) * scale + shift).  Replaces the per-layer wgrad_kernel launches
// (model.py:135-151 and the gcn mlp of model.py:41-55: their weight.grad / bias.grad).
//
// Why (round-3 kernel trace, METR B=64): one launch per layer paid ~9 us of fixed cost (ramp,
// tail, one latency-bound batch per workgroup at the small T) on 18-43 us kernels, and every one
// of the 7 waves of a workgroup re-read the same dY rows with 4-B loads.  Here:
//  * the layers' rows are dealt to one grid (one 4-wave workgroup per CU, workgroups per problem
//    in proportion to its rows), so the fixed cost is paid once;
//  * v_mfma_f32_16x16x4_f32 with K = 4 rows: lane (q, i) = (l / 16, l % 16) loads row r0 + q, and
//    ONE wide load per lane per operand chunk feeds several MFMAs -- dY: 8 B (J = 32: channels
//    2i, 2i+1 -> two 16-row output tiles) or 16 B (J = 64: 4i .. 4i+3 -> four); X: 16 B (64
//    columns, four 16-column tiles) or 8 B (32 columns, two).  A wave owns every output tile of
//    its column group, so dY is read once per row;
//  * PD quads (4 rows each) of loads in flight per wave (the buffer ring is unrolled, waits are
//    counted in issue order);
//  * the WR row-group waves of a workgroup are summed through LDS in a fixed order and the
//    workgroup writes one partial [J*Kc + J] (bias last), reduced later by gwn_reduce_partials
//    (deterministic; no float atomics).
#include "gwn_internal.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

namespace {

constexpr int GMAX = 8;  // problems per launch

struct WProb {
  const float* dY; long ldy;
  const float* X; long ldx; long x_rows; long shift;
  const __bf16* Xb; long ldxb;  // XB: columns 32 .. 224 (the bf16 mode's hop pieces)
  const float* mean; const float* scale; const float* shiftb;
  float* part;
  int R, nb, b0;  // rows, workgroups, first workgroup of this problem
};
struct WGroup {
  WProb p[GMAX];
  int nprob, Kt;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}

// JW: dY floats per lane (2: J = 32, 4: J = 64); NX16 / NX8: 64- / 32-column X chunks of a column
// group; WK column groups x WR = 4 / WK row groups per 4-wave workgroup; PD quads in flight.
// XB (the gcn mlp in bf16 mode, Kc = 224): column chunk 0 (32 fp32 columns, 8-B loads) from X, the
// hop pieces from Xb as bf16 -- a 16-B load (8 columns per lane: 128) and an 8-B load (4: 64);
// converted to fp32 in registers (exact), the same 14 output tiles as the fp32 form
// (two workgroups per CU for the gcn-mlp shape -- row groups summed through two LDS slots, 4 quads in
// flight -- measured within noise)
template <int JW, int NX16, int NX8, int WK, int PD, bool AFF, bool XB = false>
__global__ __launch_bounds__(256) void wgrad_group_kernel(const WGroup G) {
  constexpr int J = 16 * JW;
  constexpr int KCG = 64 * NX16 + 32 * NX8;  // columns of a column group
  constexpr int KC = WK * KCG;
  constexpr int WR = 4 / WK;
  constexpr int NT = 4 * NX16 + 2 * NX8;     // 16-column output tiles per J-tile row
  constexpr int XR = 4 * NX16 + 2 * NX8;     // X floats per lane per quad
  static_assert(!XB || (NX16 == 3 && NX8 == 1 && WK == 1 && !AFF), "XB: the gcn mlp shape only");
  extern __shared__ float red[];             // [WR][J*KC + J]

  // the problem of this workgroup (a short scalar search)
  int pi = 0;
  while (pi + 1 < G.nprob && (int)blockIdx.x >= G.p[pi + 1].b0) ++pi;
  const WProb& P = G.p[pi];
  const int b = blockIdx.x - P.b0;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int kg = wave % WK, rg = wave / WK;
  const int lane = threadIdx.x & 63, q = lane >> 4, i = lane & 15;
  const int r0 = (int)((long)P.R * b / P.nb), r1 = (int)((long)P.R * (b + 1) / P.nb);
  const __amdgpu_buffer_rsrc_t ry = rsrc(P.dY, (long)r1 * P.ldy * 4);
  const __amdgpu_buffer_rsrc_t rx = rsrc(P.X, P.x_rows * P.ldx * 4);
  const __amdgpu_buffer_rsrc_t rxb = rsrc(XB ? (const void*)P.Xb : (const void*)P.X, XB ? P.x_rows * P.ldxb * 2 : 0);

  // per-chunk X column / tap offsets (floats) and the lane's affine constants
  int xoff[NX16 + NX8];
  float mu[XR], sc[XR], sh[XR];
#pragma unroll
  for (int c = 0; c < NX16 + NX8; ++c) {
    const int col0 = kg * KCG + (c < NX16 ? 64 * c : 64 * NX16 + 32 * (c - NX16));
    const int tap = col0 / G.Kt, xc = col0 - tap * G.Kt;
    const int lc = xc + (c < NX16 ? 4 * i : 2 * i);
    xoff[c] = (int)(tap * P.shift * P.ldx) + lc;
    const int base = c < NX16 ? 4 * c : 4 * NX16 + 2 * (c - NX16);
    const int w = c < NX16 ? 4 : 2;
#pragma unroll
    for (int e = 0; e < w; ++e) {
      mu[base + e] = AFF ? P.mean[lc + e] : 0.0f;
      sc[base + e] = AFF ? P.scale[lc + e] : 1.0f;
      sh[base + e] = AFF ? P.shiftb[lc + e] : 0.0f;
    }
  }

  f32x4 acc[JW][NT];
#pragma unroll
  for (int e = 0; e < JW; ++e)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[e][t] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  float bsum[JW];
#pragma unroll
  for (int e = 0; e < JW; ++e) bsum[e] = 0.0f;

  // quads (4 rows) of this workgroup: quad u covers rows r0 + 4u .. +3; row group rg takes u = rg mod WR
  const int nq = (r1 - r0 + 3) >> 2;
  float ybuf[PD][JW];
  float xbuf[PD][XR];
  auto load = [&](int u, float* yv, float* xv) {
    const int row = r0 + 4 * u + q;  // past r1 (or past the quads): zeros from the dY window
    const int oy = (u < nq) ? (int)(((long)row * P.ldy + JW * i) * 4) : 0x7ffffff0;
    if constexpr (JW == 2) {
      const f32x2 v = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(ry, oy, 0, 0));
      yv[0] = v[0]; yv[1] = v[1];
    } else {
      const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ry, oy, 0, 0));
#pragma unroll
      for (int e = 0; e < JW; ++e) yv[e] = v[e];
    }
    if constexpr (XB) {
      const int ox = (u < nq) ? (int)(((long)row * P.ldx + 2 * i) * 4) : 0x7ffffff0;
      const f32x2 v0 = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rx, ox, 0, 0));
      xv[0] = v0[0]; xv[1] = v0[1];
      const int ob = (u < nq) ? (int)(((long)row * P.ldxb + 8 * i) * 2) : 0x7ffffff0;
      const int ob2 = (u < nq) ? (int)(((long)row * P.ldxb + 128 + 4 * i) * 2) : 0x7ffffff0;
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      const u32x4 b1 = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rxb, ob, 0, 0));
      const u32x2 b2 = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rxb, ob2, 0, 0));
      // bf16 -> fp32: the high half of a float (exact)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        xv[2 + 2 * e] = __builtin_bit_cast(float, b1[e] << 16);
        xv[3 + 2 * e] = __builtin_bit_cast(float, b1[e] & 0xffff0000u);
      }
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        xv[10 + 2 * e] = __builtin_bit_cast(float, b2[e] << 16);
        xv[11 + 2 * e] = __builtin_bit_cast(float, b2[e] & 0xffff0000u);
      }
      return;
    }
    const long xrow = (long)row * P.ldx;
#pragma unroll
    for (int c = 0; c < NX16 + NX8; ++c) {
      const int ox = (u < nq) ? (int)((xrow + xoff[c]) * 4) : 0x7ffffff0;
      if (c < NX16) {
        const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, ox, 0, 0));
#pragma unroll
        for (int e = 0; e < 4; ++e) xv[4 * c + e] = v[e];
      } else {
        const f32x2 v = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rx, ox, 0, 0));
        xv[4 * NX16 + 2 * (c - NX16)] = v[0];
        xv[4 * NX16 + 2 * (c - NX16) + 1] = v[1];
      }
    }
  };
  auto compute = [&](const float* yv, const float* xv) {
    float xa[XR];
#pragma unroll
    for (int e = 0; e < XR; ++e) xa[e] = AFF ? fmaf(xv[e] - mu[e], sc[e], sh[e]) : xv[e];
#pragma unroll
    for (int e = 0; e < JW; ++e) {
      bsum[e] += yv[e];
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[e][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(yv[e], xa[t], acc[e][t], 0, 0, 0);
    }
  };
  // the ring: slot s holds quad u0 + s*WR; loads run PD quads ahead of the products
#pragma unroll
  for (int s = 0; s < PD; ++s) load(rg + s * WR, ybuf[s], xbuf[s]);
  for (int u0 = rg; u0 < nq; u0 += PD * WR) {
#pragma unroll
    for (int s = 0; s < PD; ++s) {
      compute(ybuf[s], xbuf[s]);
      load(u0 + (s + PD) * WR, ybuf[s], xbuf[s]);
    }
  }
  // AFF: quads past nq loaded zeros for dY (out of window) and junk-free zeros for X (offset out
  // of range), and rows in [r1, 4 nq) read zero dY -- they add nothing

  // bias: lane (q, i) summed channel JW i + e over rows of parity q: fold the four q groups
#pragma unroll
  for (int e = 0; e < JW; ++e) {
    bsum[e] += __shfl_xor(bsum[e], 16);
    bsum[e] += __shfl_xor(bsum[e], 32);
  }
  // row-group partials through LDS: red[rg][j * KC + k], bias at red[rg][J*KC + j]
  constexpr int SLOT = J * KC + J;
  float* my = red + rg * SLOT;
#pragma unroll
  for (int e = 0; e < JW; ++e)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      // tile t: columns of chunk c (16-B chunks: 4 tiles, column 4 i + e'; 8-B: 2 tiles, 2 i + e')
      const int c = t < 4 * NX16 ? t / 4 : NX16 + (t - 4 * NX16) / 2;
      const int ep = t < 4 * NX16 ? t % 4 : (t - 4 * NX16) % 2;
      const int col0 = kg * KCG + (c < NX16 ? 64 * c : 64 * NX16 + 32 * (c - NX16));
      // XB: X floats 0-1 = fp32 columns 2i + e, 2-9 = bf16 columns 32 + 8i + e, 10-13 = 160 + 4i + e
      const int k = XB ? (t < 2 ? 2 * i + t : (t < 10 ? 32 + 8 * i + (t - 2) : 160 + 4 * i + (t - 10)))
                       : col0 + (c < NX16 ? 4 * i : 2 * i) + ep;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = JW * (4 * q + r) + e;
        my[j * KC + k] = acc[e][t][r];
      }
    }
  if (kg == 0 && q == 0) {
#pragma unroll
    for (int e = 0; e < JW; ++e)
      my[J * KC + JW * i + e] = bsum[e];
  }
  __syncthreads();
  float* out = P.part + (long)b * SLOT;
  for (int o = threadIdx.x; o < SLOT; o += 256) {
    float v = red[o];
#pragma unroll
    for (int g = 1; g < WR; ++g) v += red[g * SLOT + o];
    out[o] = v;
  }
}

struct Shape {
  int J, Kt, ntaps;
};

template <int JW, int NX16, int NX8, int WK, int PD, bool XB = false>
int launch(const WGroup& g, bool aff, int blocks, size_t lds, hipStream_t s) {
  auto k = aff ? wgrad_group_kernel<JW, NX16, NX8, WK, PD, true, false>
               : wgrad_group_kernel<JW, NX16, NX8, WK, PD, false, XB>;
  static bool attr[2] = {false, false};
  if (!attr[aff]) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr[aff] = true;
  }
  k<<<blocks, 256, lds, s>>>(g);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

// the built shapes: (J, Kt, ntaps) -> kernel, LDS bytes
int shape_kind(int J, int Kt, int ntaps) {
  if (J == 32 && Kt == 224 && ntaps == 1) return 1;  // gcn mlp, 3 supports (W = 7 x 32)
  if (J == 64 && Kt == 32 && ntaps == 2) return 2;   // gated TCN, kernel_size 2
  if (J == 32 && Kt == 512 && ntaps == 1) return 3;  // end_conv_2 (12 -> 32 padded rows), E = 512
  return 0;
}
size_t shape_lds(int kind) {
  switch (kind) {
    case 1: return (size_t)4 * (32 * 224 + 32) * 4;  // WR = 4
    case 2: return (size_t)4 * (64 * 64 + 64) * 4;   // WR = 4
    case 3: return (size_t)1 * (32 * 512 + 32) * 4;  // WK = 4, WR = 1
    default: return 0;
  }
}
int shape_wgs_per_cu(int kind) { return kind ? (int)((160 * 1024) / shape_lds(kind)) : 0; }

}  // namespace

extern "C" int gwn_wgrad_group_supported(int J, int Kt, int ntaps) { return shape_kind(J, Kt, ntaps) ? 1 : 0; }

// workgroups of each problem (nparts[p], the partial slots it writes): the device's CUs x the
// workgroups a CU holds, dealt in proportion to the rows (largest remainder, >= 1 each, and never
// more than one per 64 rows).  Returns the total, 0 for an unsupported shape.
extern "C" int gwn_wgrad_group_plan(const int* R, int nprob, int J, int Kt, int ntaps, int* nparts) {
  const int kind = shape_kind(J, Kt, ntaps);
  if (!kind || nprob < 1 || nprob > GMAX) return 0;
  long tot = 0;
  for (int p = 0; p < nprob; ++p) {
    if (R[p] <= 0) return 0;
    tot += R[p];
  }
  const int target = gwn_device_cus() * shape_wgs_per_cu(kind);
  int used = 0;
  double rem[GMAX];
  for (int p = 0; p < nprob; ++p) {
    const double share = (double)target * R[p] / (double)tot;
    int nb = (int)share;
    rem[p] = share - nb;
    const int cap = (R[p] + 63) / 64;
    if (nb < 1) nb = 1;
    if (nb > cap) nb = cap;
    nparts[p] = nb;
    used += nb;
  }
  while (used < target) {  // largest remainder first (ties: lower index), within each cap
    int best = -1;
    for (int p = 0; p < nprob; ++p)
      if (nparts[p] < (R[p] + 63) / 64 && (best < 0 || rem[p] > rem[best])) best = p;
    if (best < 0) break;
    nparts[best] += 1;
    rem[best] = -1.0;
    used += 1;
  }
  return used;
}

extern "C" int gwn_wgrad_group(const gwn_wgrad_problem* probs, int nprob, int J, int Kt, int ntaps, hipStream_t s) {
  const int kind = shape_kind(J, Kt, ntaps);
  GWN_REQUIRE(kind, "wgrad_group: shape not built (J, Kt, ntaps) in {(32, 224, 1), (64, 32, 2), (32, 512, 1)}");
  GWN_REQUIRE(probs && nprob >= 1 && nprob <= GMAX, "wgrad_group: 1..8 problems");
  int R[GMAX], nb[GMAX];
  for (int p = 0; p < nprob; ++p) R[p] = probs[p].R;
  const int blocks = gwn_wgrad_group_plan(R, nprob, J, Kt, ntaps, nb);
  GWN_REQUIRE(blocks > 0, "wgrad_group: every problem needs R > 0");
  WGroup g = {};
  g.nprob = nprob;
  g.Kt = Kt;
  const bool aff = probs[0].x_mean != nullptr;
  const bool xb = probs[0].Xb != nullptr;
  GWN_REQUIRE(!xb || (kind == 1 && !aff), "wgrad_group: Xb (bf16 hop pieces) is for the gcn-mlp shape, no affine");
  int b0 = 0;
  for (int p = 0; p < nprob; ++p) {
    const gwn_wgrad_problem& q = probs[p];
    GWN_REQUIRE(q.dY && q.X && q.part && q.ldy >= J && q.ldx >= Kt && q.ldy % 4 == 0 && q.ldx % 4 == 0 &&
                    ((uintptr_t)q.dY & 15) == 0 && ((uintptr_t)q.X & 15) == 0,
                "wgrad_group: dY, X, part required; ldy >= J, ldx >= Kt, multiples of 4; 16-B aligned operands");
    GWN_REQUIRE((q.x_mean != nullptr) == aff && !q.x_mean == !q.x_scale && !q.x_mean == !q.x_shift,
                "wgrad_group: x_mean / x_scale / x_shift go together, for every problem or none");
    GWN_REQUIRE((q.Xb != nullptr) == xb && (!xb || (q.ldxb >= 192 && q.ldxb % 8 == 0 && ((uintptr_t)q.Xb & 15) == 0 &&
                                                    (long)q.R * q.ldxb * 2 < 0x7fff0000L)),
                "wgrad_group: Xb for every problem or none; ldxb >= 192, a multiple of 8, 16-B aligned");
    GWN_REQUIRE(q.x_rows >= (long)q.R + (ntaps - 1) * q.shift && q.shift >= 0, "wgrad_group: X rows do not cover the taps");
    GWN_REQUIRE((long)q.R * q.ldy * 4 < 0x7fff0000L && q.x_rows * q.ldx * 4 < 0x7fff0000L,
                "wgrad_group: operand beyond a 2 GB buffer window");
    WProb& w = g.p[p];
    w.dY = q.dY; w.ldy = q.ldy; w.X = q.X; w.ldx = q.ldx; w.x_rows = q.x_rows; w.shift = q.shift;
    w.mean = q.x_mean; w.scale = q.x_scale; w.shiftb = q.x_shift;
    w.part = q.part; w.R = q.R; w.nb = nb[p]; w.b0 = b0;
    w.Xb = (const __bf16*)q.Xb; w.ldxb = q.ldxb;
    b0 += nb[p];
  }
  const size_t lds = shape_lds(kind);
  // quads in flight per wave (8 / 10 / 10; 4 / 6 / 6 measured slower on the TCN shape: 87 vs 74 us
  // per METR step): the mlp launch holds one workgroup (one wave per SIMD) per CU, so its loads in
  // flight are all the latency hiding it has
  switch (kind) {
    case 1: return xb ? launch<2, 3, 1, 1, 8, true>(g, false, blocks, lds, s) : launch<2, 3, 1, 1, 8>(g, aff, blocks, lds, s);
    case 2: return launch<4, 0, 2, 1, 10>(g, aff, blocks, lds, s);
    default: return launch<2, 2, 0, 4, 10>(g, aff, blocks, lds, s);
  }
}
