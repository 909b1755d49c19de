// Adaptive-support gradient ("gram"): the backward of nconv w.r.t. the support,
//     dA[v][w] (+)= sum_p sum_s sum_c X_p[s*n + v][c] * T_p[s*n + w][c]      (p < npairs <= 2)
// over all slices s of a layer (model.py:12-14 differentiated w.r.t. A; two pairs per layer for
// order 2: (xg, dx1) and (x1, dx2)).  M = N = n (<= 224 here), K = slices * 32 per pair.
//
// One wave per (32x64 output block = one row tile x two column tiles, slice range).  The
// contraction is laid onto v_mfma_f32_32x32x2_f32 PERMUTED: step j takes channel c = 16h + j in
// lane half h, so lane (i, h) needs the 16 contiguous floats X[s*n + 32*vt + i][16h ..] (A) and
// T[s*n + 32*wt + i][16h ..] (B) — four 16-B buffer loads each, nodes >= n reading zeros
// (out-of-range offset).  Each A fragment feeds two accumulator chains (0.375 loads per MFMA
// instead of 1).  The K loop walks (slice, pair) steps with the next step's 12 fragments in flight
// while the current step's 32 MFMAs run (pairs unrolled: scalar buffer resources).  No LDS, no
// barriers.  Measured (tools/bench_gcn.py under rocprofv3, T=12, 768 slices): 72 us against 78 us
// for one 32x32 tile per wave; a whole slice in flight (200 VGPRs) or 4096 waves were slower.
// Still ~55 TFLOP/s: each 16-B fragment load touches 32 rows (32 cache lines per instruction).
// Waves of one slice range are placed on one XCD (blocks round-robin over the 8 XCDs), so the
// 7x re-reads of each row block hit that XCD's L2.  Partials [nsplit][npad][npad] are summed in
// a fixed order by a second kernel (deterministic).
#include "gwn_internal.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int OOR = 0x7ffffff0;
constexpr int NXCD = 8;
#ifndef GRAM_WAVES
#define GRAM_WAVES 2048  // target wave count of a gram launch (1792: 263.8 us per METR step, 2048: 242.4, 3072: 273.2, 4096: 245.2)
#endif

constexpr int GL = 8;  // layers of a grouped launch (gwn_gram_group)
struct Gram {
  const float* X[GL][2]; const float* T[GL][2]; int npairs;  // pair 1 used iff npairs == 2
  int lslices[GL], lsplit0[GL + 1], nlayers;  // layer l: its slices, splits [lsplit0[l], lsplit0[l+1])
  long ldx, ldt;
  int n, nt, nsplit;  // nt = ceil(n / 32); nsplit = all layers' splits
  float* part;        // [nsplit][32 nt][32 nt]
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ int crow(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ bf16x8 to_bf16x8(const float4& a, const float4& b) {
  bf16x8 r;
  r[0] = (__bf16)a.x; r[1] = (__bf16)a.y; r[2] = (__bf16)a.z; r[3] = (__bf16)a.w;
  r[4] = (__bf16)b.x; r[5] = (__bf16)b.y; r[6] = (__bf16)b.z; r[7] = (__bf16)b.w;
  return r;
}

// BF16: the same loads, each lane's 16 channels (16h .. 16h+15) as two bf16x8 K-groups of
// v_mfma_f32_32x32x16_bf16 (K permuted alike on both operands: group s of half h = channels
// 16h + 8s .. +7), 2 MFMAs per tile and slice instead of 16 (the bf16 mode's adaptive-support
// gradient; fp32 accumulation)
// LINES: each (slice, pair) step's 96 rows x 128 B (32 rows of X, 64 of T) arrive by full-line
// loads (64 lanes x 16 B = 8 whole rows per instruction) into the wave's LDS image [96][36]
// (padded rows: conflict-free ds_read_b128), from which the lanes read their fragments -- instead
// of fragment-shaped loads that touch 32 rows (16 B of each) per instruction
template <int NP, bool BF16 = false, bool LINES = false>
__global__ __launch_bounds__(64) void gram_kernel(const Gram g) {
  const int lane = threadIdx.x, half = lane >> 5, col = lane & 31;
  const int ntp = (g.nt + 1) / 2;  // column tile pairs
  const int per_split = g.nt * ntp;
  // XCD-aware placement: block b runs on XCD b % 8; keep every block of one split on one XCD
  const int b = blockIdx.x, xcd = b % NXCD, j = b / NXCD;
  const int blk = j % per_split, split = (j / per_split) * NXCD + xcd;
  if (split >= g.nsplit) return;
  const int vt = blk / ntp, wt0 = 2 * (blk % ntp);
  const bool two = wt0 + 1 < g.nt;  // wave-uniform: the last pair of an odd tile count has one tile
  // the layer of this split (grouped launch) and its slice range within that layer
  int L = 0;
  while (L + 1 < g.nlayers && split >= g.lsplit0[L + 1]) ++L;
  const int lsl = g.lslices[L], ls = split - g.lsplit0[L], lns = g.lsplit0[L + 1] - g.lsplit0[L];
  const int s0 = (int)((long)lsl * ls / lns), s1 = (int)((long)lsl * (ls + 1) / lns);

  __amdgpu_buffer_rsrc_t rx[NP], rt[NP];
  const long rows = (long)lsl * g.n;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    rx[p] = rsrc(g.X[L][p], rows * g.ldx * 4);
    rt[p] = rsrc(g.T[L][p], rows * g.ldt * 4);
  }
  const int v = 32 * vt + col, w0 = 32 * wt0 + col, w1 = w0 + 32;
  // fragments of (slice s, pair p); p must be a compile-time constant after unrolling so the buffer
  // resource stays scalar (a run-time select makes it a per-lane value: waterfall loops per load).
  // Past the last slice every offset is out of range (zeros).
  auto load = [&](int s, int p, float4* fa, float4* fb) {
    const bool ok = s < s1;
    const long base = (long)s * g.n;
    if (LINES) {  // float4 f = q*64 + lane of the step's [96 rows][8 float4] image
#pragma unroll
      for (int q = 0; q < 12; ++q) {
        const int f = q * 64 + lane, rr = f >> 3, c4 = f & 7;
        float4 v;
        if (rr < 32) {
          const int vv = 32 * vt + rr;
          const int o = (ok && vv < g.n) ? (int)(((base + vv) * g.ldx + 4 * c4) * 4) : OOR;
          v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx[p], o, 0, 0));
        } else {
          const int ww = 32 * wt0 + (rr - 32);
          const int o = (ok && ww < g.n && (rr < 64 || two)) ? (int)(((base + ww) * g.ldt + 4 * c4) * 4) : OOR;
          v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt[p], o, 0, 0));
        }
        if (q < 4) fa[q] = v;
        else fb[q - 4] = v;
      }
      return;
    }
    const int ox = (ok && v < g.n) ? (int)(((base + v) * g.ldx + 16 * half) * 4) : OOR;
    const int o0 = (ok && w0 < g.n) ? (int)(((base + w0) * g.ldt + 16 * half) * 4) : OOR;
    const int o1 = (ok && two && w1 < g.n) ? (int)(((base + w1) * g.ldt + 16 * half) * 4) : OOR;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      fa[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx[p], ox, 16 * q, 0));
      fb[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt[p], o0, 16 * q, 0));
      fb[4 + q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt[p], o1, 16 * q, 0));
    }
  };

  f32x16 acc0, acc1;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    acc0[r] = 0.0f;
    acc1[r] = 0.0f;
  }
  float4 fa[4], fb[8];
  extern __shared__ float4 gimg4[];
  float* gimg = (float*)gimg4;
  // LINES: the staged lines -> the wave's image -> this lane's fragments (rows col, 32 + col, 64 + col)
  auto restage = [&](float4* fa_, float4* fb_) {
    if (!LINES) return;
#pragma unroll
    for (int q = 0; q < 12; ++q) {
      const int f = q * 64 + lane, rr = f >> 3, c4 = f & 7;
      *(float4*)(gimg + rr * 36 + 4 * c4) = q < 4 ? fa_[q] : fb_[q - 4];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      fa_[q] = *(const float4*)(gimg + col * 36 + 16 * half + 4 * q);
      fb_[q] = *(const float4*)(gimg + (32 + col) * 36 + 16 * half + 4 * q);
      fb_[4 + q] = *(const float4*)(gimg + (64 + col) * 36 + 16 * half + 4 * q);
    }
  };
  load(s0, 0, fa, fb);
  restage(fa, fb);
  for (int s = s0; s < s1; ++s) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      float4 na[4], nb[8];
      if (p + 1 < NP) load(s, p + 1, na, nb);
      else load(s + 1, 0, na, nb);
      __builtin_amdgcn_sched_barrier(0);
      if (BF16) {
#pragma unroll
        for (int sg = 0; sg < 2; ++sg) {
          const bf16x8 av = to_bf16x8(fa[2 * sg], fa[2 * sg + 1]);
          acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, to_bf16x8(fb[2 * sg], fb[2 * sg + 1]), acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, to_bf16x8(fb[4 + 2 * sg], fb[5 + 2 * sg]), acc1, 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].x, fb[q].x, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].x, fb[4 + q].x, acc1, 0, 0, 0);
          acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].y, fb[q].y, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].y, fb[4 + q].y, acc1, 0, 0, 0);
          acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].z, fb[q].z, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].z, fb[4 + q].z, acc1, 0, 0, 0);
          acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].w, fb[q].w, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].w, fb[4 + q].w, acc1, 0, 0, 0);
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        fa[q] = na[q];
        fb[q] = nb[q];
        fb[4 + q] = nb[4 + q];
      }
      restage(fa, fb);
    }
  }
  // D[v][w]: col = lane&31 -> w, rows -> v
  const int np = 32 * g.nt;
  float* out = g.part + (long)split * np * np + (long)(32 * vt) * np + 32 * wt0 + col;
#pragma unroll
  for (int r = 0; r < 16; ++r) out[(long)crow(r, half) * np] = acc0[r];
  if (two) {
#pragma unroll
    for (int r = 0; r < 16; ++r) out[(long)crow(r, half) * np + 32] = acc1[r];
  }
}

// dA[v][w] (+)= sum_split part[split][v][w], fixed order.  A 256-thread block takes 64 outputs x 4
// contiguous quarters of the splits (8 independent chains per thread: loads in flight together),
// the quarters merged in LDS as (q0 + q1) + (q2 + q3): four times the blocks of a thread per
// output (a 224 x 224 output is 49k threads -- under a fifth of the chip's wave slots)
__global__ __launch_bounds__(256) void gram_reduce_kernel(const float* part, int nsplit, int n, int np, float* dA,
                                                          int ld, int accumulate) {
  __shared__ float sh[4][64];
  const int o = threadIdx.x & 63, qq = threadIdx.x >> 6;
  const long idx = blockIdx.x * 64L + o;
  const bool ok = idx < (long)n * n;
  const int v = ok ? (int)(idx / n) : 0, w = ok ? (int)(idx - (long)v * n) : 0;
  const float* p = part + (long)v * np + w;
  const long st = (long)np * np;
  const int k0 = nsplit * qq / 4, k1 = nsplit * (qq + 1) / 4;
  float a[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
  int k = k0;
  if (ok) {
    for (; k + 8 <= k1; k += 8)
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] += p[(k + u) * st];
    for (; k < k1; ++k) a[(k - k0) & 7] += p[k * st];
  }
  sh[qq][o] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  if (qq != 0 || !ok) return;
  const float s = (sh[0][o] + sh[1][o]) + (sh[2][o] + sh[3][o]);
  float* d = dA + (long)v * ld + w;
  *d = accumulate ? *d + s : s;
}

inline unsigned gram_reduce_blocks(int n) { return (unsigned)(((long)n * n + 63) / 64); }

constexpr size_t GRAM_IMG = 96 * 36 * sizeof(float);  // LINES: a wave's [96][36] image

int gram_nsplit(int n, int slices) {
  const int nt = (n + 31) / 32;
  // ~1.8k waves over 256 CUs (each with two accumulator chains), a multiple of the XCD count, and
  // preferably a divisor of the slice count so every split walks the same number of slices
  // (T=12 at B=64: 64 splits of 12 slices, 65 us, against 88 uneven splits 73 us).  More splits
  // cost partial-sum traffic (splits x np^2 floats) and fewer leave SIMDs idle.
  int target = GRAM_WAVES / (nt * ((nt + 1) / 2));
  target = (target / NXCD) * NXCD;
  if (target < NXCD) target = NXCD;
  if (target > slices) target = slices;
  for (int ns = target; ns >= 2 * NXCD && ns >= target / 2; ns -= NXCD)
    if (slices % ns == 0) return ns;
  return target < 1 ? 1 : target;
}

// ---------------------------------------------------------------------------------------------
// The bf16 mode's gram on bf16 operands in the 16-node tiled activation layout (gwn_gcn_args.xg4
// / gwn_gcn_bwd_args.tg4, include/gwn.h): a (slice, node tile) block is one KiB, lane (g, j)
// holding the 16 B of node 16 vt + j, channels 4g .. 4g+3 then 16+4g .. 16+4g+3 -- exactly its
// k-group of v_mfma_f32_16x16x32_bf16 (the same channel permutation on both operands).  One wave
// owns a TB x TB block of 16-node output tiles over a slice range; per (slice, pair) it issues 2 TB
// 16-B loads (each a contiguous KiB) for TB^2 MFMAs, the next step's loads in flight.  The operand
// re-reads (ceil(nt / TB) per side) are the cost: L2-to-CU bandwidth bound, hence bf16 operands
// written by the producers (half the bytes of fp32).  PEMS bf16 (N = 325, 7 layers): 658 us per
// step on the row-fragment gram_kernel<., true> (a load per 32 rows), 344 on fp32 tiled operands
// (TB = 2), 167 on bf16 ones, TB = 2 / 3 / 4 alike (21.51k / 21.54k / 21.53k samples/s).
typedef float f32x4g __attribute__((ext_vector_type(4)));
constexpr int G4_WAVES = 2048;  // target waves of a launch
constexpr int G4_TB = 3;        // 16-node tiles per side of a wave's output block

struct GramG4 {
  const void* X[2]; const void* T[2];    // [slices][nt] KiB each
  int nt, slices, nsplit, npair, nb;     // nb = ceil(nt / TB) output blocks per side
  long np;                               // partial row stride (32 * ceil(n / 32))
  float* part;                           // [nsplit][np][np]
};

template <int TB>
__global__ __launch_bounds__(64) void gram_g4_kernel(const GramG4 g) {
  const int lane = threadIdx.x, gq = lane >> 4, j = lane & 15;
  const int b = blockIdx.x, xcd = b % NXCD, q = b / NXCD;
  const int per_split = g.nb * g.nb;
  const int blk = q % per_split, split = (q / per_split) * NXCD + xcd;  // a split's blocks share an XCD
  if (split >= g.nsplit) return;
  const int vt0 = TB * (blk / g.nb), wt0 = TB * (blk % g.nb);
  const int s0 = (int)((long)g.slices * split / g.nsplit), s1 = (int)((long)g.slices * (split + 1) / g.nsplit);
  const long bytes = (long)g.slices * g.nt * 1024;
  __amdgpu_buffer_rsrc_t rx[2], rt[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    rx[p] = rsrc(g.X[p], bytes);
    rt[p] = rsrc(g.T[p], bytes);
  }
  // block (s, tile) at (s * nt + tile) KiB; lane's 16 B at lane * 16; tiles past nt (wave-uniform)
  // read zeros
  auto off = [&](int s_, int tile) {
    return tile < g.nt && s_ < s1 ? (int)(((long)s_ * g.nt + tile) * 1024 + lane * 16) : OOR;
  };
  f32x4g acc[TB][TB];
#pragma unroll
  for (int x = 0; x < TB; ++x)
#pragma unroll
    for (int y = 0; y < TB; ++y) acc[x][y] = f32x4g{0.0f, 0.0f, 0.0f, 0.0f};
  // fragments of (slice, pair); p unrolled so the buffer resources stay scalar
  auto load = [&](int s_, int p, bf16x8* av, bf16x8* bv) {
#pragma unroll
    for (int t = 0; t < TB; ++t) {
      av[t] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rx[p], off(s_, vt0 + t), 0, 0));
      bv[t] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rt[p], off(s_, wt0 + t), 0, 0));
    }
  };
  bf16x8 a[TB], bb[TB];
  load(s0, 0, a, bb);
  for (int s_ = s0; s_ < s1; ++s_) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      if (p >= g.npair) break;
      bf16x8 na[TB], nb[TB];
      if (p + 1 < g.npair) load(s_, 1, na, nb);
      else load(s_ + 1, 0, na, nb);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int x = 0; x < TB; ++x)
#pragma unroll
        for (int y = 0; y < TB; ++y) acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[x], bb[y], acc[x][y], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < TB; ++t) {
        a[t] = na[t];
        bb[t] = nb[t];
      }
    }
  }
  // D[v][w]: lane (g, j) holds rows 4 g + r of the tile, column j
  float* out = g.part + (long)split * g.np * g.np;
#pragma unroll
  for (int x = 0; x < TB; ++x)
#pragma unroll
    for (int y = 0; y < TB; ++y) {
      if (vt0 + x >= g.nt || wt0 + y >= g.nt) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        out[(long)(16 * (vt0 + x) + 4 * gq + r) * g.np + 16 * (wt0 + y) + j] = acc[x][y][r];
    }
}

int gram_g4_nsplit(int nb, int slices) {
  int target = G4_WAVES / (nb * nb);
  target = (target / NXCD) * NXCD;
  if (target < NXCD) target = NXCD;
  if (target > slices) target = slices;
  return target < 1 ? 1 : target;
}

}  // namespace

// dA (+)= sum_s X1_s T1_s^T (+ X2_s T2_s^T) on bf16 operands in the 16-node tiled activation layout
int gwn_gram_g4_bf16(const void* x1, const void* t1, const void* x2, const void* t2, int n, int slices, float* dA,
                int ld_dA, int accumulate, float* ws, hipStream_t s) {
  GWN_REQUIRE(n > 0 && slices > 0 && x1 && t1 && ws && !x2 == !t2, "gram_g4_bf16: bad arguments");
  GramG4 g = {};
  g.X[0] = x1; g.T[0] = t1; g.X[1] = x2 ? x2 : x1; g.T[1] = t2 ? t2 : t1;
  g.npair = x2 ? 2 : 1;
  g.nt = (n + 15) / 16;
  g.nb = (g.nt + G4_TB - 1) / G4_TB;
  g.slices = slices;
  g.nsplit = gram_g4_nsplit(g.nb, slices);
  g.np = 32L * ((n + 31) / 32);
  g.part = ws;
  GWN_REQUIRE((long)slices * g.nt * 1024 < 0x7fff0000L, "gram_g4_bf16: operand beyond a 2 GB buffer window");
  GWN_REQUIRE((long)g.nsplit * g.np * g.np <= gwn_gram_workspace_floats(n, slices) ||
                  (long)g.nsplit * g.np * g.np <= gwn_gram_g4_workspace_floats(n, slices),
              "gram_g4_bf16: workspace");
  const int blocks = ((g.nsplit + NXCD - 1) / NXCD) * NXCD * g.nb * g.nb;
  gram_g4_kernel<G4_TB><<<blocks, 64, 0, s>>>(g);
  GWN_CHECK_LAUNCH();
  gram_reduce_kernel<<<gram_reduce_blocks(n), 256, 0, s>>>(ws, g.nsplit, n, (int)g.np, dA, ld_dA, accumulate);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

long gwn_gram_g4_workspace_floats(int n, int slices) {
  const int nt = (n + 15) / 16;
  const long np = 32L * ((n + 31) / 32);
  return (long)gram_g4_nsplit((nt + G4_TB - 1) / G4_TB, slices) * np * np;
}

// Partial-sum floats of a gram launch over AT MOST `slices` slices.  gram_nsplit is not monotone
// in the slice count (it prefers divisors: 56 slices take 56 splits, 96 take 48), so a workspace
// sized for the largest layer is bounded by the split target, not by that layer's own split count.
long gwn_gram_workspace_floats(int n, int slices) {
  const int nt = (n + 31) / 32, np = 32 * nt;
  int bound = GRAM_WAVES / (nt * ((nt + 1) / 2));
  bound = (bound / NXCD) * NXCD;
  if (bound < NXCD) bound = NXCD;
  if (bound > slices) bound = slices;
  return (long)bound * np * np;
}

// dA (+)= sum over slices of X1^T T1 (+ X2^T T2); c = 32 channels per slice row
int gwn_gram(const float* x1, const float* t1, const float* x2, const float* t2, long ldx, long ldt, int n,
             int slices, float* dA, int ld_dA, int accumulate, float* ws, hipStream_t s) {
  return gwn_gram_dtype(x1, t1, x2, t2, ldx, ldt, n, slices, dA, ld_dA, accumulate, ws, 0, s);
}

// the same contraction on bf16 MFMA operands with fp32 accumulation (the bf16 mode's gram)
int gwn_gram_bf16(const float* x1, const float* t1, const float* x2, const float* t2, long ldx, long ldt, int n,
                  int slices, float* dA, int ld_dA, int accumulate, float* ws, hipStream_t s) {
  return gwn_gram_dtype(x1, t1, x2, t2, ldx, ldt, n, slices, dA, ld_dA, accumulate, ws, 1, s);
}

int gwn_gram_dtype(const float* x1, const float* t1, const float* x2, const float* t2, long ldx, long ldt, int n,
                   int slices, float* dA, int ld_dA, int accumulate, float* ws, int bf16, hipStream_t s) {
  GWN_REQUIRE(n > 0 && slices > 0 && x1 && t1 && ws, "gram: bad arguments");
  GWN_REQUIRE(((uintptr_t)x1 & 15) == 0 && ((uintptr_t)t1 & 15) == 0 && (ldx & 3) == 0 && (ldt & 3) == 0 &&
                  (!x2 || (((uintptr_t)x2 & 15) == 0 && ((uintptr_t)t2 & 15) == 0)),
              "gram: operands must be 16-B aligned with ld % 4 == 0");
  GWN_REQUIRE((long)slices * n * (ldx > ldt ? ldx : ldt) * 4 < 0x7fff0000L, "gram: operand beyond a 2 GB buffer window");
  Gram g = {};
  g.X[0][0] = x1; g.T[0][0] = t1; g.X[0][1] = x2; g.T[0][1] = t2;
  g.npairs = x2 ? 2 : 1;
  g.ldx = ldx; g.ldt = ldt;
  g.n = n; g.nt = (n + 31) / 32;
  g.nsplit = gram_nsplit(n, slices);
  g.nlayers = 1; g.lslices[0] = slices; g.lsplit0[0] = 0; g.lsplit0[1] = g.nsplit;
  g.part = ws;
  {
    const long rows = (long)slices * n;  // the loads stay inside rows * ld of each operand
    GWN_DEBUG_RANGE(x1, ((rows - 1) * ldx + 32) * 4, "gram x1");
    GWN_DEBUG_RANGE(t1, ((rows - 1) * ldt + 32) * 4, "gram t1");
    if (x2) GWN_DEBUG_RANGE(x2, ((rows - 1) * ldx + 32) * 4, "gram x2");
    if (x2) GWN_DEBUG_RANGE(t2, ((rows - 1) * ldt + 32) * 4, "gram t2");
    const long np = 32L * g.nt;
    GWN_DEBUG_RANGE(ws, g.nsplit * np * np * 4, "gram partials");
    GWN_DEBUG_RANGE(dA, ((long)(n - 1) * ld_dA + n) * 4, "gram dA");
  }
  const int per_split = g.nt * ((g.nt + 1) / 2);
  const int blocks = ((g.nsplit + NXCD - 1) / NXCD) * NXCD * per_split;
  if (bf16) {
    if (g.npairs == 2) gram_kernel<2, true><<<blocks, 64, 0, s>>>(g);
    else gram_kernel<1, true><<<blocks, 64, 0, s>>>(g);
  } else {  // fp32: full-line operand loads restaged per wave (the fragment-shaped loads: 317 vs 264 us)
    if (g.npairs == 2) gram_kernel<2, false, true><<<blocks, 64, GRAM_IMG, s>>>(g);
    else gram_kernel<1, false, true><<<blocks, 64, GRAM_IMG, s>>>(g);
  }
  GWN_CHECK_LAUNCH();
  gram_reduce_kernel<<<gram_reduce_blocks(n), 256, 0, s>>>(ws, g.nsplit, n, 32 * g.nt, dA, ld_dA,
                                                                     accumulate);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

// ---------------------------------------------------------------------------------------------
// Grouped gram: the adaptive-support gradient of every layer of a backward in ONE launch (and one
// reduction), all layers accumulating into the same dA.  The gram_kernel waves of a layer-size
// launch are latency-bound at the small T (METR B=64, round-4 trace: ~7.7 us fixed per launch + a
// 5.5 us reduce each, on 22-63 us kernels); here the wave target is dealt to the layers in
// proportion to their slices, every split inside one layer.
namespace {
int gram_group_plan(int n, const int* slices, int nlayers, int* nsp) {
  const int nt = (n + 31) / 32;
  int target = GRAM_WAVES / (nt * ((nt + 1) / 2));
  target = (target / NXCD) * NXCD;
  if (target < NXCD) target = NXCD;
  long tot = 0;
  for (int l = 0; l < nlayers; ++l) tot += slices[l];
  int used = 0;
  for (int l = 0; l < nlayers; ++l) {
    int k = (int)((double)target * slices[l] / (double)tot + 0.5);
    if (k < 1) k = 1;
    if (k > slices[l]) k = slices[l];
    nsp[l] = k;
    used += k;
  }
  return used;
}

// ---------------------------------------------------------------------------------------------
// CU-resident gram (fp32, n <= 256): the whole contraction as one split-K GEMM per CU.  A 16-wave
// workgroup per CU keeps the entire [np16][np16] output (np16 = 16 ceil(n / 16); 16-node tiles of
// v_mfma_f32_16x16x4_f32, a contiguous row-major run of <= MAXT tiles per wave, 4 accumulator
// registers each) over an equal range of the launch's (layer, slice, pair) steps.  Each step's X
// and T rows (np16 x 32 floats each) are staged ONCE per CU into LDS -- double-buffered, the next
// step's loads in flight during the current step's products, one barrier per step -- and read by
// all 16 waves, so an operand row crosses L2 -> CU once per CU instead of once per 32 x 64 output
// block (gram_kernel: ~2.2 GB of fragment traffic per METR step).  The K permutation of
// gram_kernel: lane group q takes channels 8q .. 8q+7 (two ds_read_b128 per operand and tile), the
// same on both operands.  Partials [CU][np16][np16], summed in a fixed order by gram_reduce_kernel.
constexpr int GCU_LDR = 36;  // LDS row stride (floats): the 16 rows of a ds_read_b128 pass on distinct banks
typedef __attribute__((address_space(3))) void* lds_ptr_t;
constexpr int GCG_NB = 4;  // LDS step buffers: three steps' operands in flight
// s_waitcnt vmcnt(n) (n <= 15), expcnt / lgkmcnt not waited on
#define GCG_WAIT_VM(n) __builtin_amdgcn_s_waitcnt(0x0F70 | (n))

struct GramCu {
  const float* X[GL][2]; const float* T[GL][2];
  int lsteps0[GL + 1];  // layer l's steps [lsteps0[l], lsteps0[l+1]) = (slice, pair), pair fastest
  int nlayers;
  long ldx, ldt;
  int n, nt16;
  float* part;  // [gridDim.x][16 nt16][16 nt16]
};

template <int MAXT>
__global__ __launch_bounds__(1024) void gram_cu_kernel(const GramCu g) {
  extern __shared__ float4 gcu_lds4[];
  float* lds = (float*)gcu_lds4;
  const int rows = 16 * g.nt16, opf = rows * GCU_LDR;  // staged rows per operand (>= n: zeros)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, q = lane >> 4, i = lane & 15;
  const int total = g.lsteps0[g.nlayers];
  const int st0 = (int)((long)total * blockIdx.x / gridDim.x), st1 = (int)((long)total * (blockIdx.x + 1) / gridDim.x);
  const int ntiles = g.nt16 * g.nt16;
  const int tb = ntiles * wave / 16, cnt = ntiles * (wave + 1) / 16 - tb;
  f32x4g acc[MAXT];
#pragma unroll
  for (int u = 0; u < MAXT; ++u) acc[u] = f32x4g{0.0f, 0.0f, 0.0f, 0.0f};
  // staging: operand rows as float4 e = row * 8 + quad, e < rows * 8 <= 2048: two per thread
  const int per = rows * 8;
  float4 sx[2], stt[2];
  auto stage_load = [&](int st) {
    int L = 0;
    while (L + 1 < g.nlayers && st >= g.lsteps0[L + 1]) ++L;
    const int ls = st - g.lsteps0[L], sl = ls >> 1, p = ls & 1;
    const long base = (long)sl * g.n;
    const __amdgpu_buffer_rsrc_t rx = rsrc(g.X[L][p] + base * g.ldx, (long)g.n * g.ldx * 4);
    const __amdgpu_buffer_rsrc_t rt = rsrc(g.T[L][p] + base * g.ldt, (long)g.n * g.ldt * 4);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = (int)threadIdx.x + 1024 * u, r = e >> 3, c4 = e & 7;
      const bool ok = e < per && r < g.n;
      sx[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx, ok ? (int)((r * g.ldx + 4 * c4) * 4) : OOR, 0, 0));
      stt[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, ok ? (int)((r * g.ldt + 4 * c4) * 4) : OOR, 0, 0));
    }
  };
  auto stage_store = [&](int buf) {
    float* xi = lds + buf * 2 * opf;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = (int)threadIdx.x + 1024 * u, r = e >> 3, c4 = e & 7;
      if (e < per) {
        *(float4*)(xi + r * GCU_LDR + 4 * c4) = sx[u];
        *(float4*)(xi + opf + r * GCU_LDR + 4 * c4) = stt[u];
      }
    }
  };
  // (LDS-DMA staging of the step rows, no staging registers, measured slower here: 195 vs 170 us --
  // the fp32 step computes longer than the load latency, one register-staged step in flight suffices)
  auto frag = [&](const float* img, int t16, float4* f) {
    const float* r = img + (16 * t16 + i) * GCU_LDR + 8 * q;
    f[0] = *(const float4*)r;
    f[1] = *(const float4*)(r + 4);
  };
  if (st0 < st1) {
    stage_load(st0);
    stage_store(0);
  }
  __syncthreads();
  int buf = 0;
  for (int st = st0; st < st1; ++st) {
    const bool more = st + 1 < st1;
    if (more) stage_load(st + 1);
    const float* xi = lds + buf * 2 * opf;
    const float* ti_ = xi + opf;
    // (the 16 waves of the CU hide the LDS latency: no in-wave prefetch, which would cost 8 of the
    // registers the accumulators need)
#pragma unroll
    for (int u = 0; u < MAXT; ++u) {
      if (u < cnt) {
        const int t = tb + u, ti = t / g.nt16;
        float4 a[2], b[2];
        frag(xi, ti, a);
        frag(ti_, t - ti * g.nt16, b);
        const float av[8] = {a[0].x, a[0].y, a[0].z, a[0].w, a[1].x, a[1].y, a[1].z, a[1].w};
        const float bv[8] = {b[0].x, b[0].y, b[0].z, b[0].w, b[1].x, b[1].y, b[1].z, b[1].w};
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kk], bv[kk], acc[u], 0, 0, 0);
      }
    }
    if (more) stage_store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // D[v][w]: lane (q, i) holds rows 16 ti + 4 q + r, column 16 tj + i
  const long np = rows;
  float* out = g.part + (long)blockIdx.x * np * np;
#pragma unroll
  for (int u = 0; u < MAXT; ++u) {
    if (u < cnt) {
      const int t = tb + u, ti = t / g.nt16, tj = t - ti * g.nt16;
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(long)(16 * ti + 4 * q + r) * np + 16 * tj + i] = acc[u][r];
    }
  }
}

// The bf16 mode's CU-resident gram on the tiled bf16 operands (gwn_gram_g4_bf16's layout: a KiB per
// (slice, 16-node tile), lane (g, j)'s 16 B its k-group of v_mfma_f32_16x16x32_bf16).  Like
// gram_cu_kernel, but the 16x16 output tiles of one CU would need ~28 per wave at n = 325, so the
// workgroups come in two halves (blockIdx bit 3): half h keeps output tile rows [vt0, vt0 + R) of
// every column (<= MAXT tiles per wave) and walks its own equal share of ALL the (layer, slice,
// pair) steps; per step it stages R KiB of X and nt KiB of T (double-buffered, the next step's
// 16-B loads in flight) and each wave runs one MFMA per tile, the X fragment reloaded only when
// its row changes.  Partial slot kb (kernel) holds half 0's rows of share kb and half 1's
// rows of share kb: [grid / 2][np][np], reduced in a fixed order.
struct GramCuG4 {
  const char* X[GL]; const char* T[GL];  // layer l: pair p's operand at + p * slices * nt KiB
  int lslices[GL], lsteps0[GL + 1], nlayers;
  int nt, vmid;                          // tile rows [0, vmid) in half 0, [vmid, nt) in half 1
  long np;
  float* part;
};


template <int MAXT>
__global__ __launch_bounds__(1024) void gram_cu_g4_kernel(const GramCuG4 g) {
  extern __shared__ float4 gcg_lds4[];
  // the two halves of share kb are workgroups 16 q + x and 16 q + 8 + x (kb = 8 q + x): the same XCD
  // (dispatch deals workgroups to the 8 XCDs round-robin), so the T stream both read per step comes
  // from that XCD's L2 for the second of them (pairs 2 kb, 2 kb + 1 sat on two XCDs: 1.71x the
  // algorithmic bytes, profiles/r04/pmc_pems_summary.txt)
  const int h = (blockIdx.x >> 3) & 1, kb = ((blockIdx.x >> 4) << 3) | (blockIdx.x & 7), nh = gridDim.x >> 1;
  const int vt0 = h ? g.vmid : 0, R = h ? g.nt - g.vmid : g.vmid;
  const int nblk = R + g.nt;  // KiB staged per step
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int gq = lane >> 4, j = lane & 15;
  const int total = g.lsteps0[g.nlayers];
  const int st0 = (int)((long)total * kb / nh), st1 = (int)((long)total * (kb + 1) / nh);
  const int nst = st1 - st0;
  const int ntiles = R * g.nt;
  const int tb = ntiles * wave / 16, cnt = ntiles * (wave + 1) / 16 - tb;
  f32x4g acc[MAXT];
#pragma unroll
  for (int u = 0; u < MAXT; ++u) acc[u] = f32x4g{0.0f, 0.0f, 0.0f, 0.0f};
  const int bufk = nblk * 64;                    // float4 per step buffer
  float4* sink = gcg_lds4 + GCG_NB * bufk;       // the target of the padding waves' loads
  // step st's operands into buffer b by 16-B LDS-DMA loads (buffer_load ... lds): wave w moves
  // KiB blocks w, w + 16 (a block = one wave instruction, lane-linear); every wave issues
  // exactly two per step (past nblk: a zero load into the sink) so the vmcnt waits are uniform
  auto issue = [&](int st, int b) {
    int L = 0;
    while (L + 1 < g.nlayers && st >= g.lsteps0[L + 1]) ++L;
    const int ls = st - g.lsteps0[L], sl = ls >> 1, p = ls & 1;
    const long blk0 = ((long)p * g.lslices[L] + sl) * g.nt;  // KiB index of the step's slice
    const __amdgpu_buffer_rsrc_t rx =
        rsrc(g.X[L] + (blk0 + vt0) * 1024, (long)R * 1024);
    const __amdgpu_buffer_rsrc_t rt = rsrc(g.T[L] + blk0 * 1024, (long)g.nt * 1024);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int blk = wave + 16 * i;
      float4* dst = blk < nblk ? gcg_lds4 + b * bufk + blk * 64 : sink;
      if (blk < R)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr_t)dst, 16, blk * 1024 + lane * 16, 0, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rt, (lds_ptr_t)dst, 16,
                                                 blk < nblk ? (blk - R) * 1024 + lane * 16 : 0x7ffffff0, 0, 0, 0);
    }
  };
#pragma unroll
  for (int c = 0; c < GCG_NB - 1; ++c)
    if (c < nst) issue(st0 + c, c);
  for (int c = 0; c < nst; ++c) {
    // this wave's loads of step c have landed (steps c+1, c+2 may still be in flight), then the
    // barrier: every wave's part of step c landed and every wave is done with step c-1, whose
    // buffer the next issue reuses
    if (c + 2 < nst) GCG_WAIT_VM(4);
    else if (c + 1 < nst) GCG_WAIT_VM(2);
    else GCG_WAIT_VM(0);
    __builtin_amdgcn_s_barrier();
    if (c + GCG_NB - 1 < nst) issue(st0 + c + GCG_NB - 1, (c + GCG_NB - 1) % GCG_NB);
    const float4* img = gcg_lds4 + (c % GCG_NB) * bufk;
    bf16x8 a = {};
    int rprev = -1;
#pragma unroll
    for (int u = 0; u < MAXT; ++u) {
      if (u < cnt) {
        const int t = tb + u, r = t / g.nt, cc = t - r * g.nt;
        if (r != rprev) {
          a = __builtin_bit_cast(bf16x8, img[r * 64 + lane]);
          rprev = r;
        }
        const bf16x8 b = __builtin_bit_cast(bf16x8, img[(R + cc) * 64 + lane]);
        acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[u], 0, 0, 0);
      }
    }
  }
  // D[v][w]: lane (gq, j) holds rows 4 gq + r of the tile, column j
  float* out = g.part + (long)kb * g.np * g.np;
#pragma unroll
  for (int u = 0; u < MAXT; ++u) {
    if (u < cnt) {
      const int t = tb + u, r = t / g.nt, cc = t - r * g.nt;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) out[(long)(16 * (vt0 + r) + 4 * gq + rr) * g.np + 16 * cc + j] = acc[u][rr];
    }
  }
}

// the CU-resident gram applies (GWN_GRAM_CU=0: gram_kernel)
bool gram_cu_ok(int n) {
  const char* e = getenv("GWN_GRAM_CU");
  if (e && e[0] == '0') return false;
  return n <= 256;
}
size_t gram_cu_lds(int n) {
  return (size_t)2 * 2 * 16 * ((n + 15) / 16) * GCU_LDR * sizeof(float);
}
}  // namespace

long gwn_gram_group_workspace_floats(int n, const int* slices, int nlayers) {
  if (n <= 0 || nlayers < 1 || nlayers > GL || !slices) return 0;
  int nsp[GL];
  for (int l = 0; l < nlayers; ++l)
    if (slices[l] <= 0) return 0;
  const long np = 32L * ((n + 31) / 32);
  const long classic = (long)gram_group_plan(n, slices, nlayers, nsp) * np * np;
  const long np16 = 16L * ((n + 15) / 16);
  const long cu = n <= 256 ? (long)gwn_device_cus() * np16 * np16 : 0;  // gram_cu_kernel's partials
  return classic > cu ? classic : cu;
}

int gwn_gram_group(const gwn_gram_layer* layers, int nlayers, long ldx, long ldt, int n, float* dA, int ld_dA,
                   int accumulate, float* ws, hipStream_t s) {
  GWN_REQUIRE(layers && nlayers >= 1 && nlayers <= GL && n > 0 && dA && ws, "gram_group: 1..8 layers, n, dA, ws");
  GWN_REQUIRE((ldx & 3) == 0 && (ldt & 3) == 0, "gram_group: ld % 4 == 0");
  Gram g = {};
  int sl[GL], nsp[GL];
  for (int l = 0; l < nlayers; ++l) {
    const gwn_gram_layer& q = layers[l];
    GWN_REQUIRE(q.slices > 0 && q.x1 && q.t1 && q.x2 && q.t2 && ((uintptr_t)q.x1 & 15) == 0 &&
                    ((uintptr_t)q.t1 & 15) == 0 && ((uintptr_t)q.x2 & 15) == 0 && ((uintptr_t)q.t2 & 15) == 0,
                "gram_group: every layer needs slices > 0 and both 16-B aligned pairs");
    GWN_REQUIRE((long)q.slices * n * (ldx > ldt ? ldx : ldt) * 4 < 0x7fff0000L,
                "gram_group: operand beyond a 2 GB buffer window");
    g.X[l][0] = q.x1; g.T[l][0] = q.t1; g.X[l][1] = q.x2; g.T[l][1] = q.t2;
    sl[l] = q.slices;
  }
  g.nsplit = gram_group_plan(n, sl, nlayers, nsp);
  g.nlayers = nlayers;
  g.lsplit0[0] = 0;
  for (int l = 0; l < nlayers; ++l) {
    g.lslices[l] = sl[l];
    g.lsplit0[l + 1] = g.lsplit0[l] + nsp[l];
  }
  if (gram_cu_ok(n)) {
    GramCu c = {};
    c.nlayers = nlayers;
    c.lsteps0[0] = 0;
    for (int l = 0; l < nlayers; ++l) {
      for (int p = 0; p < 2; ++p) {
        c.X[l][p] = g.X[l][p];
        c.T[l][p] = g.T[l][p];
      }
      c.lsteps0[l + 1] = c.lsteps0[l] + 2 * sl[l];
    }
    c.ldx = ldx; c.ldt = ldt;
    c.n = n; c.nt16 = (n + 15) / 16;
    c.part = ws;
    const int grid = gwn_device_cus();
    const long np16 = 16L * c.nt16;
    GWN_DEBUG_RANGE(ws, grid * np16 * np16 * 4, "gram_group (CU) partials");
    GWN_DEBUG_RANGE(dA, ((long)(n - 1) * ld_dA + n) * 4, "gram_group dA");
    const size_t lds = gram_cu_lds(n);
    const int need = (c.nt16 * c.nt16 + 15) / 16;  // tiles per wave
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)gram_cu_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)gram_cu_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)gram_cu_kernel<11>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)gram_cu_kernel<12>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)gram_cu_kernel<16>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr = true;
    }
    if (need <= 4) gram_cu_kernel<4><<<grid, 1024, lds, s>>>(c);
    else if (need <= 8) gram_cu_kernel<8><<<grid, 1024, lds, s>>>(c);
    else if (need <= 11) gram_cu_kernel<11><<<grid, 1024, lds, s>>>(c);  // n = 161 .. 208
    else if (need <= 12) gram_cu_kernel<12><<<grid, 1024, lds, s>>>(c);
    else gram_cu_kernel<16><<<grid, 1024, lds, s>>>(c);
    GWN_CHECK_LAUNCH();
    gram_reduce_kernel<<<gram_reduce_blocks(n), 256, 0, s>>>(ws, grid, n, (int)np16, dA, ld_dA, accumulate);
    GWN_CHECK_LAUNCH();
    return GWN_OK;
  }
  g.npairs = 2;
  g.ldx = ldx; g.ldt = ldt;
  g.n = n; g.nt = (n + 31) / 32;
  g.part = ws;
  const long np = 32L * g.nt;
  GWN_DEBUG_RANGE(ws, g.nsplit * np * np * 4, "gram_group partials");
  GWN_DEBUG_RANGE(dA, ((long)(n - 1) * ld_dA + n) * 4, "gram_group dA");
  const int per_split = g.nt * ((g.nt + 1) / 2);
  const int blocks = ((g.nsplit + NXCD - 1) / NXCD) * NXCD * per_split;
  gram_kernel<2, false, true><<<blocks, 64, GRAM_IMG, s>>>(g);
  GWN_CHECK_LAUNCH();
  gram_reduce_kernel<<<gram_reduce_blocks(n), 256, 0, s>>>(ws, g.nsplit, n, (int)np, dA, ld_dA, accumulate);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

// ---------------------------------------------------------------------------------------------
namespace {
// tiles per wave of gram_cu_g4_kernel's larger half
inline int gcg_need(int nt) { return (((nt + 1) / 2) * nt + 15) / 16; }
}  // namespace

// 0 where gwn_gram_g4_group does not apply (n > 368: more than 16 output tiles per wave)
long gwn_gram_g4_group_workspace_floats(int n, const int* slices, int nlayers) {
  if (n <= 0 || nlayers < 1 || nlayers > GL || !slices || gcg_need((n + 15) / 16) > 16) return 0;
  const long np = 32L * ((n + 31) / 32);
  return (long)(gwn_device_cus() / 16 * 8) * np * np;
}

int gwn_gram_g4_group(const gwn_gram_layer* layers, int nlayers, int n, float* dA, int ld_dA, int accumulate,
                      float* ws, hipStream_t s) {
  GWN_REQUIRE(layers && nlayers >= 1 && nlayers <= GL && n > 0 && dA && ws, "gram_g4_group: 1..8 layers, n, dA, ws");
  const int nt = (n + 15) / 16;
  GWN_REQUIRE(gcg_need(nt) <= 16, "gram_g4_group: n up to 368 (16 output tiles per wave)");
  GramCuG4 g = {};
  g.nlayers = nlayers;
  g.lsteps0[0] = 0;
  for (int l = 0; l < nlayers; ++l) {
    const gwn_gram_layer& q = layers[l];
    GWN_REQUIRE(q.slices > 0 && q.x1 && q.t1 && ((uintptr_t)q.x1 & 15) == 0 && ((uintptr_t)q.t1 & 15) == 0 &&
                    q.x2 == (const float*)((const char*)q.x1 + (long)q.slices * nt * 1024) &&
                    q.t2 == (const float*)((const char*)q.t1 + (long)q.slices * nt * 1024),
                "gram_g4_group: every layer's x2 / t2 must follow x1 / t1 (the xg4 / tg4 layout), 16-B aligned");
    g.X[l] = (const char*)q.x1;
    g.T[l] = (const char*)q.t1;
    g.lslices[l] = q.slices;
    g.lsteps0[l + 1] = g.lsteps0[l] + 2 * q.slices;
  }
  g.nt = nt;
  g.vmid = (nt + 1) / 2;
  g.np = 32L * ((n + 31) / 32);
  g.part = ws;
  const int grid = (gwn_device_cus() / 16) * 16;  // (XCD-paired halves: a multiple of 16 workgroups)
  GWN_DEBUG_RANGE(ws, (long)(grid / 2) * g.np * g.np * 4, "gram_g4_group partials");
  GWN_DEBUG_RANGE(dA, ((long)(n - 1) * ld_dA + n) * 4, "gram_g4_group dA");
  const size_t lds = (size_t)(GCG_NB * (g.vmid + nt) + 1) * 1024;  // + the sink
  GWN_REQUIRE(lds <= 160 * 1024 && g.vmid + nt <= 32, "gram_g4_group: a step's operands exceed LDS");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gram_cu_g4_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)gram_cu_g4_kernel<16>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const int need = gcg_need(nt);
  if (need <= 8) gram_cu_g4_kernel<8><<<grid, 1024, lds, s>>>(g);
  else gram_cu_g4_kernel<16><<<grid, 1024, lds, s>>>(g);
  GWN_CHECK_LAUNCH();
  gram_reduce_kernel<<<gram_reduce_blocks(n), 256, 0, s>>>(ws, grid / 2, n, (int)g.np, dA, ld_dA, accumulate);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}
