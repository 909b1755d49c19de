// Fused diffusion graph convolution (gcn.forward, reference model.py:41-55, + residual model.py:234)
// and its backward, for C = 32 channels and N <= 512 nodes: the persistent 16-node tile kernels
// (one 16-wave workgroup per CU over an equal range of the launch's 16-node tiles; f32 operands on
// v_mfma_f32_16x16x4_f32, bf16 operands on v_mfma_f32_16x16x32_bf16), the gated TCN and the layer
// below's BatchNorm finalize fused into the f32 forward's staging, and the gwn_gcn_fwd /
// gwn_gcn_bwd dispatch between them and the whole-slice schedules of gcn_slice.hip.
//
// Contract on the supports: [np][ld] with np = 32*ceil(n/32) <= ld, ZERO outside [n][n]
// (the executor keeps padded copies), so the K loops run whole node batches unguarded.
#include "gcn_common.h"

using namespace gcnk;

namespace {

// ---------------------------------------------------------------------------------------------
// 16-node tiles (v_mfma_f32_16x16x4_f32): the power-schedule forward with one wave per 16-node
// tile.  Against the 32-node tile waves it pads 207 nodes to 208 rows instead of 224 (7 % fewer
// MFMAs), gives a slice 13 equal waves instead of 7 (the SIMD imbalance of 7 waves on 4 SIMDs:
// 2,2,2,1), and needs fewer registers per wave (4-register accumulators), so two workgroups share
// a CU at 6-7 waves per SIMD.
//   diffusion (piece p of support k, channel half hf): D[c][w] = sum_v x[v][c] * G[v][w] with
//     A operand x[v0 + lane/16][16 hf + lane%16] (LDS image, row stride LDR16: conflict-free),
//     B operand G[v0 + lane/16][w0 + lane%16] (support row segments, L2-resident), and
//     lane l holding D[16 hf + 4 (l/16) + r][w0 + l%16] in register r;
//   mlp: z[w][o] += sum_c W[o][c] piece[c][w] with the contraction PERMUTED so that the pieces
//     feed the B operand straight from the accumulators: step s of half hf takes, in lane group
//     g = l/16, channel 16 hf + 4 g + s (register s), and the A operand W^T[that channel][o] from
//     the transposed weights (16 consecutive floats per lane group);
//   z tile: lane l holds z[w0 + l%16][16 oh + 4 (l/16) + r]: 16-B epilogue rows per lane.
// ---------------------------------------------------------------------------------------------
typedef float f32x4v __attribute__((ext_vector_type(4)));
constexpr int T16_RING = 4;   // k-steps (4 support rows each) of support fragments in flight
constexpr int T16_WAVES = 16; // waves of a t16 workgroup (one workgroup per CU, persistent over a tile range)
constexpr int T16_MAXIMG = 4; // slice images a workgroup holds at once (LDS permitting)
// Tile order within a phase: slice-major (wave w takes every 16th tile; a column-major order
// sharing support fragments in L1 measured slower).

// rows of a slice image: the tiles' rows, and the diffusion loop's reads (4 rows per k-step, one
// k-step ahead, whole rings of T16_RING k-steps); rows >= n are zero
__host__ __device__ inline int t16_img_rows(int n) {
  const int nt16 = (n + 15) / 16;
  const int nk = (n + 3) / 4, nkp = (nk + T16_RING - 1) / T16_RING * T16_RING;
  return 16 * nt16 > 4 * nkp + 4 ? 16 * nt16 : 4 * nkp + 4;
}

// Slice image in LDS: two channel halves, each [rows][16] (no padding): lane (g, j) of the
// diffusion's A-operand read (row 4 ks + g, channel 16 hf + j) hits bank 16 g + j of 64.  The
// half stride hs = rows * 16 floats is a multiple of 64 (ds_read2st64 pairs the two halves).
// the t16 kernels' 16-B output stores (z, dres / dh_out, dxg / t1 / t2, dfg): plain (non-temporal
// measured slower: 24.64k / 23.54k vs 24.79k / 23.67k samples/s METR / PEMS)
__device__ __forceinline__ void t16_st4(float* p, float4 v) { *(float4*)p = v; }
constexpr int LDW16 = 36;  // LDS row stride of the staged channel maps: lane groups g hit banks 16 g + j

// LDS of a t16 workgroup: the channel maps of all 2K+1 pieces (32 x LDW16 floats each), the waves'
// BN partials [16][3][32], and maximg slice images
// fused TCN (FusedFwd.tcn): the region of the waves' BN partials (used only by the final flush)
// first holds the TCN weights [64 outputs in MFMA-tile order][LDT_TCN], the input means and the biases
constexpr int LDT_TCN = 68;  // 2c + 4: a ds_read_b128 pass of 16 rows hits distinct banks
// region layout: weights [64][LDT_TCN], input means [32], biases [64], the TCN's pointers / sizes
// (TcnLds, 16 floats), BatchNorm scales [32]
constexpr int TW_MEAN = 64 * LDT_TCN, TW_BIAS = TW_MEAN + 32, TW_PAR = TW_BIAS + 64, TW_SCALE = TW_PAR + 16;
constexpr int T16_TCN_REGION = TW_SCALE + 32;
__host__ __device__ constexpr int t16_region(bool tcn) { return tcn ? T16_TCN_REGION : T16_WAVES * 3 * CH; }
static_assert(T16_TCN_REGION >= T16_WAVES * 3 * CH, "the TCN region holds the BN partials' space");
size_t t16_lds_bytes(int n, int nsup, int maximg, bool tcn = false) {
  return (size_t)((2 * nsup + 1) * CH * LDW16 + t16_region(tcn) + maximg * t16_img_rows(n) * CH) * sizeof(float);
}

// the channel maps M_p[out][in] of pieces p < npieces into LDS transposed, m[(p*32 + in)*LDW16 +
// out] (t16_mlp's 16 ds_read_b32 per piece; the untransposed layout read as ds_read_b128 measured no
// faster), from the mlp weights W [32][ld_w] (row = mlp output channel): forward M_p = W[:,
// p-block] (strided 4-B loads), backward M_p = W[:, p-block]^T (rows of W, 16-B loads)
// (Both of round 6's batched forms of this copy -- a thread's 7 strided loads in flight at once, or
// W read row by row with 8 loads in flight -- measured 0.5-0.7 % slower per METR step than this
// element loop, same box; profiles/r06/load_batching.)
__device__ __forceinline__ void t16_stage_maps(const float* w, int ld_w, bool backward, int npieces, float* dst) {
  if (backward) {
    const int total = npieces * CH * 8;  // float4s
    for (int e = threadIdx.x; e < total; e += blockDim.x) {
      const int r = e >> 3, q = e & 7;  // r = p*32 + out
      *(float4*)(dst + r * LDW16 + 4 * q) = *(const float4*)(w + (long)(r & 31) * ld_w + (r >> 5) * CH + 4 * q);
    }
  } else {
    const int total = npieces * CH * CH;
    for (int e = threadIdx.x; e < total; e += blockDim.x) {
      const int r = e >> 5, o = e & 31;  // r = p*32 + c
      dst[r * LDW16 + o] = w[(long)o * ld_w + (r >> 5) * CH + (r & 31)];
    }
  }
}

// rows [0, rows) of a slice's node features (rows >= n zero) into the two-half LDS image
__device__ __forceinline__ void global_to_lds16(const float* src, long ld, int n, int rows, float* buf) {
  const int hs = rows * 16;
  if ((((uintptr_t)src) & 15) == 0 && (ld & 3) == 0) {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)((long)n * ld * 4), 0x00020000);
    const int total = rows * 8;
    for (int e0 = 0; e0 < total; e0 += 4 * (int)blockDim.x) {
      float4 v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = e0 + threadIdx.x + i * blockDim.x;
        const int off = e < total ? (int)(((long)(e >> 3) * ld + 4 * (e & 7)) * 4) : 0x7ffffff0;
        v[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = e0 + threadIdx.x + i * blockDim.x;
        if (e < total) *(float4*)(buf + ((e >> 2) & 1) * hs + (e >> 3) * 16 + 4 * (e & 3)) = v[i];
      }
    }
  } else {
    for (int e = threadIdx.x; e < rows * CH; e += blockDim.x) {
      const int w = e / CH, c = e % CH;
      buf[(c >> 4) * hs + w * 16 + (c & 15)] = w < n ? src[(long)w * ld + c] : 0.0f;
    }
  }
}

// A phase's staging: rows [0, rows) of nsl consecutive slices (src: slice 0's row 0, slice stride
// n * ld floats, 16-B aligned, ld % 4 == 0; rows >= n load as zeros) as float4 elements e ->
// put(slice, row, quad, value).  Each thread's U elements of a round are all loaded before the
// first put, and the rounds run over the whole phase (not slice by slice): one memory round trip
// per U * blockDim elements.  mid() runs once with round 0's loads in flight (the channel-map
// staging shares their round trip).
template <int U, typename Put, typename Mid>
__device__ __forceinline__ void stage_rows4(const float* src, long ld, int n, int rows, int nsl, Put put, Mid mid) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)((long)nsl * n * ld * 4), 0x00020000);
  const int per = rows * 8, total = nsl * per;
  bool first = true;
  for (int e0 = threadIdx.x; e0 < total || first; e0 += U * (int)blockDim.x) {
    float4 v[U];
    int key[U];  // (slice * rows + row) * 8 + quad, -1 past the phase
#pragma unroll
    for (int i = 0; i < U; ++i) {
      const int e = e0 + i * (int)blockDim.x;
      const int sl = e / per, rem = e - sl * per, w = rem >> 3, q = rem & 7;
      const bool ok = e < total && w < n;
      v[i] = __builtin_bit_cast(
          float4, __builtin_amdgcn_raw_buffer_load_b128(r, ok ? (int)(((long)(sl * n + w) * ld + 4 * q) * 4) : 0x7ffffff0, 0, 0));
      key[i] = e < total ? e : -1;
    }
    if (first) {
      mid();
      first = false;
    }
#pragma unroll
    for (int i = 0; i < U; ++i)
      if (key[i] >= 0) {
        const int sl = key[i] / per, rem = key[i] - sl * per;
        put(sl, rem >> 3, rem & 7, v[i]);
      }
  }
}

// A lane's running BatchNorm partial over the nodes it held in the wave's tiles (Welford, tile
// order): lane (g, j) keeps the 8 channels 16 (q >> 2) + 4 g + (q & 3) of node j of each tile.  The
// 16 lanes of a row group are merged once, at the flush (t16_bn_lanes) -- not per tile, which cost
// two 4-step DPP reductions per channel and tile.
struct BnRun {
  float n, mean[8], m2[8];
};
__device__ __forceinline__ void bn_init(BnRun& bn, float*) {
  bn.n = 0.0f;
#pragma unroll
  for (int q = 0; q < 8; ++q) bn.mean[q] = bn.m2[q] = 0.0f;
}

// z tile epilogue (fwd_tile_epilogue's arithmetic on the 16-node tile layout): bias, dropout,
// residual (BN of the layer below applied on load), z or eval-BN output store; the tile's BN
// partial merged into the wave's running one
// seed: *a.seed_ptr, read once per workgroup by the caller (t16_seed) -- per tile it was a dependent
// global load in every epilogue
__device__ __forceinline__ unsigned long long t16_seed(const FusedFwd& a) {
  return (a.seed_ptr && a.drop_p > 0.0f) ? *a.seed_ptr : 0ull;
}
__device__ __forceinline__ void t16_epilogue(const FusedFwd& a, const f32x4v* hacc, long row0, int w0, int lane,
                                             int n, BnRun& bn, unsigned long long seed,
                                             const float* res_mean = nullptr, const float* res_scale = nullptr) {
  if (!res_mean) res_mean = a.res_mean;
  if (!res_scale) res_scale = a.res_scale;
  const int g = lane >> 4, j = lane & 15;
  const int w = w0 + j;
  const bool valid = w < n;
  const long m = row0 + min(w, n - 1);
  const float keep_scale = (a.drop_p > 0.0f) ? 1.0f / (1.0f - a.drop_p) : 1.0f;
  float* dst = a.x_out ? a.x_out : a.z;
  float v[8];
#pragma unroll
  for (int oh = 0; oh < 2; ++oh) {
    const int c0 = 16 * oh + 4 * g;
    const float4 bq = *(const float4*)(a.b_mlp + c0);
    const float4 rq = *(const float4*)(a.residual + m * CH + c0);
    const float* bias = (const float*)&bq;
    const float* rv = (const float*)&rq;
    float4 mq, sq, hq;
    if (a.res_scale) {
      mq = *(const float4*)(res_mean + c0);
      sq = *(const float4*)(res_scale + c0);
      hq = *(const float4*)(a.res_shift + c0);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float x = hacc[oh][e] + bias[e];
      if (a.drop_p > 0.0f) {
        const float u = gwn_uniform(seed, a.salt, (unsigned long long)m * CH + c0 + e);
        x = (u >= a.drop_p) ? x * keep_scale : 0.0f;
      }
      x += a.res_scale ? fmaf(rv[e] - ((const float*)&mq)[e], ((const float*)&sq)[e], ((const float*)&hq)[e]) : rv[e];
      v[4 * oh + e] = x;
    }
    if (a.x_out) {  // eval BatchNorm, the arithmetic of bn_apply_kernel (ops.hip)
      const float4 rm = *(const float4*)(a.bn_rm + c0), rvv = *(const float4*)(a.bn_rv + c0);
      const float4 gq = *(const float4*)(a.bn_g + c0), bb = *(const float4*)(a.bn_b + c0);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        v[4 * oh + e] = (v[4 * oh + e] - ((const float*)&rm)[e]) *
                            (1.0f / sqrtf(((const float*)&rvv)[e] + a.bn_eps)) * ((const float*)&gq)[e] +
                        ((const float*)&bb)[e];
    }
    if (valid) t16_st4(dst + m * CH + c0, make_float4(v[4 * oh], v[4 * oh + 1], v[4 * oh + 2], v[4 * oh + 3]));
  }
  if (a.bn_part == nullptr || a.x_out || !valid) return;
  bn.n += 1.0f;
  const float inv = 1.0f / bn.n;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float d = v[q] - bn.mean[q];
    bn.mean[q] = fmaf(d, inv, bn.mean[q]);
    bn.m2[q] = fmaf(d, v[q] - bn.mean[q], bn.m2[q]);
  }
}

// the 16 lanes of each row group merged (Chan, rotations by 8, 4, 2, 1 within the row): lane j = 0
// of a group then holds the group's partial (each lane merges in its own order; lane 0's is fixed)
template <int CTRL>
__device__ __forceinline__ float row_ror(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ void bn_lane_step(BnRun& bn) {
  const float nb = row_ror<CTRL>(bn.n);
  const float tot = bn.n + nb;
  const float wb = tot > 0.0f ? nb / tot : 0.0f, wab = tot > 0.0f ? bn.n * nb / tot : 0.0f;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float mb = row_ror<CTRL>(bn.mean[q]), qb = row_ror<CTRL>(bn.m2[q]);
    const float d = mb - bn.mean[q];
    bn.mean[q] = fmaf(d, wb, bn.mean[q]);
    bn.m2[q] = bn.m2[q] + qb + d * d * wab;
  }
  bn.n = tot;
}
__device__ __forceinline__ void t16_bn_lanes(BnRun& bn) {
  bn_lane_step<0x128>(bn);  // row_ror 8, 4, 2, 1
  bn_lane_step<0x124>(bn);
  bn_lane_step<0x122>(bn);
  bn_lane_step<0x121>(bn);
}

// the waves' running partials (wave order) -> the workgroup's BN partial, slot blockIdx.x
__device__ __forceinline__ void t16_bn_flush(const FusedFwd& a, const BnRun& bn, float* wpart) {
  if (a.bn_part == nullptr || a.x_out) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  BnRun bl = bn;
  t16_bn_lanes(bl);
  if (j == 0) {
    float* wp = wpart + wave * 3 * CH;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = 16 * (q >> 2) + 4 * g + (q & 3);
      wp[c] = bl.n;
      wp[CH + c] = bl.mean[q];
      wp[2 * CH + c] = bl.m2[q];
    }
  }
  __syncthreads();
  if (threadIdx.x < CH) {
    const int c = threadIdx.x;
    float nn = 0.0f, mean = 0.0f, m2 = 0.0f;
    for (int wv = 0; wv < (int)(blockDim.x >> 6); ++wv) {
      const float nb = wpart[wv * 3 * CH + c];
      if (nb <= 0.0f) continue;
      const float mb = wpart[wv * 3 * CH + CH + c], qb = wpart[wv * 3 * CH + 2 * CH + c];
      const float tot = nn + nb;
      const float d = mb - mean;
      mean += d * (nb / tot);
      m2 += qb + d * d * (nn * nb / tot);
      nn = tot;
    }
    float* sp = a.bn_part + (long)blockIdx.x * 3 * CH;
    sp[c] = nn;
    sp[CH + c] = mean;
    sp[2 * CH + c] = m2;
  }
  // the slots past the grid (gwn_bn_part_slots: at least one per slice) hold no rows
  for (long slot = blockIdx.x + gridDim.x; slot < a.bn_slots; slot += gridDim.x)
    if (threadIdx.x < 3 * CH) a.bn_part[slot * 3 * CH + threadIdx.x] = 0.0f;
}

// gwn_gcn_args.clock: the workgroup's (start, end) device wall clock into slot blockIdx.x, each a
// plain store (no atomic, no load: nothing waits on memory and nothing is held in registers across
// the kernel); every launch overwrites the call site's slots
__device__ __forceinline__ void t16_clock_start(const FusedFwd& a) {
  if (a.clk != nullptr && threadIdx.x == 0) a.clk[2 * blockIdx.x] = wall_clock64();
}
__device__ __forceinline__ void t16_clock_end(const FusedFwd& a) {
  if (a.clk == nullptr) return;
  __syncthreads();
  if (threadIdx.x == 0) a.clk[2 * blockIdx.x + 1] = wall_clock64();
}

// the channel map of one piece held in accumulators acc[hf] (register s = input channel
// 16 hf + 4 g + s): hacc[oh] (output channel 16 oh + 4 g + r) += M x piece with the A operand
// M[out][in] read as m[in * ld_m + out] (t16_stage_maps: forward the piece's block of W, backward
// its transpose, i.e. W^T applied to dh)
__device__ __forceinline__ void t16_mlp(const float* m, int ld_m, const f32x4v* acc, int lane, f32x4v* hacc) {
  const int g = lane >> 4, j = lane & 15;
  float wf[2][2][4];
#pragma unroll
  for (int hf = 0; hf < 2; ++hf)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int oh = 0; oh < 2; ++oh) wf[hf][oh][s] = m[(16 * hf + 4 * g + s) * ld_m + 16 * oh + j];
  // all fragment reads in flight before the first product (one LDS latency)
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int hf = 0; hf < 2; ++hf)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int oh = 0; oh < 2; ++oh)
        hacc[oh] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[hf][oh][s], acc[hf][s], hacc[oh], 0, 0, 0);
}

// bf16 mlp (gwn_dtype GWN_DTYPE_BF16_MLP, the bf16 tile kernels): a piece's channel map as
// v_mfma_f32_16x16x32_bf16 A operands in LDS, [piece][out half oh][lane][8 bf16] with lane (g, j)
// holding M[16 oh + j][k] for the permuted K group k = 4g .. 4g+3, 16+4g .. 16+4g+3 -- the
// channels a lane's accumulators hold (acc[hf][e]: channel 16 hf + 4 g + e), so the piece itself
// is the B operand as it stands: 2 MFMAs per piece instead of 16 f32 ones.  Forward M_p = W[:,
// p-block]; backward M_p = its transpose (W^T applied to dh).
typedef __bf16 bf16x8m __attribute__((ext_vector_type(8)));
__device__ __forceinline__ int mlp_perm(int g, int e) { return e < 4 ? 4 * g + e : 16 + 4 * g + (e - 4); }
__device__ __forceinline__ void t16_stage_maps_bf16(const float* w, int ld_w, bool backward, int npieces, __bf16* dst) {
  for (int t = threadIdx.x; t < npieces * 2 * 64; t += blockDim.x) {
    const int p = t >> 7, oh = (t >> 6) & 1, lane = t & 63, g = lane >> 4, j = lane & 15;
    const int row = 16 * oh + j;
    bf16x8m v;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = mlp_perm(g, e);
      v[e] = (__bf16)(backward ? w[(long)k * ld_w + p * CH + row] : w[(long)row * ld_w + p * CH + k]);
    }
    *(bf16x8m*)(dst + (long)t * 8) = v;
  }
}
// the piece in the t16 accumulator layout (acc[hf][e]: channel 16 hf + 4 g + e) as the B operand
// of t16_mlp_b; its halves are also the bf16 piece store's 4-channel groups
__device__ __forceinline__ bf16x8m t16_pack_b(const f32x4v* acc) {
  bf16x8m b;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    b[e] = (__bf16)acc[0][e];
    b[4 + e] = (__bf16)acc[1][e];
  }
  return b;
}
// hacc[oh] += M_p x piece, bf16 operands: both A fragments are read before the first product
// (one LDS latency per piece, not two)
__device__ __forceinline__ void t16_mlp_bp(const __bf16* maps, int p, const bf16x8m b, int lane, f32x4v* hacc) {
  const bf16x8m a0 = *(const bf16x8m*)(maps + ((p * 2 + 0) * 64 + lane) * 8);
  const bf16x8m a1 = *(const bf16x8m*)(maps + ((p * 2 + 1) * 64 + lane) * 8);
  __builtin_amdgcn_sched_barrier(0);
  hacc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b, hacc[0], 0, 0, 0);
  hacc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b, hacc[1], 0, 0, 0);
}
__device__ __forceinline__ void t16_mlp_b(const __bf16* maps, int p, const f32x4v* acc, int lane, f32x4v* hacc) {
  t16_mlp_bp(maps, p, t16_pack_b(acc), lane, hacc);
}
// node w0 + j's column of a channel-major bf16 image [32][s16] as t16_mlp_bp's B operand (channels
// 4 g .. +3, 16 + 4 g .. +3): the bf16 mode's piece 0 / dh operand without re-reading fp32 rows
__device__ __forceinline__ bf16x8m t16_img_col_b(const __bf16* img, int s16, int w0, int lane) {
  const int g = lane >> 4, j = lane & 15;
  const __bf16* xi = img + w0 + j;
  bf16x8m b;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    b[e] = xi[(4 * g + e) * s16];
    b[4 + e] = xi[(16 + 4 * g + e) * s16];
  }
  return b;
}

// both powers of one support for the wave's 16-node tile: acc[q][hf] (q = 0: G1, 1: G2) holds
// D[16 hf + 4 g + r][w0 + j] = sum_v img[v][16 hf + 4 g + r] G_q[v][w0 + j]
// The supports come in gwn_support_g4's k-interleaved layout: one 16-B load per lane fetches the
// fragments of four k-steps (a wave's load is one contiguous KiB).  Per-k-step 4-B fragment loads
// of the padded [np][ld] supports held the MFMA pipes at ~0.70 busy in the isolated loop
// (tools/t16_loop_probe.hip, 16 waves per CU: L1 / address processing per load instruction),
// these at 0.93.  Fragments run one group (4 k-steps) ahead: the group's load pair is issued
// before the previous group's products, so every wait is vmcnt(2).
__device__ __forceinline__ void t16_diffuse(const float* img, int hs, const float* G1, const float* G2, int n, int tile,
                                            int lane, f32x4v (*acc)[2]) {
  const int g = lane >> 4, j = lane & 15;
  const int nt = (n + 15) >> 4, nkg = nt;  // k-groups of 16 rows: ceil(n / 16), as the column tiles
  const int bytes = nkg * nt * 1024;
  const __amdgpu_buffer_rsrc_t r1 = __builtin_amdgcn_make_buffer_rsrc((void*)G1, (short)0, bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t r2 = __builtin_amdgcn_make_buffer_rsrc((void*)G2, (short)0, bytes, 0x00020000);
  // group kg of this tile: 1 KiB block kg * nt + tile, lane l's 16 B (k-steps 4 kg .. 4 kg + 3)
  auto off = [&](int kg) { return ((kg * nt + tile) * 64 + lane) * 16; };
  f32x4v a1[2], a2[2];
  a1[0] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(r1, off(0), 0, 0));
  a2[0] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(r2, off(0), 0, 0));
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int q = 0; q < 2; ++q) acc[q][0] = acc[q][1] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
  const float* xp = img + g * 16 + j;
  // image operands one k-step ahead: the LDS latency hides behind the current step's products
  float xa = xp[0], xb = xp[hs];
  // group kg (fragments in buffer kg & 1); the next group's pair is requested first (past the
  // last group the offsets leave the buffer range: zeros, no traffic)
  auto group = [&](int kg, int bsel) {
    a1[bsel ^ 1] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(r1, off(kg + 1), 0, 0));
    a2[bsel ^ 1] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(r2, off(kg + 1), 0, 0));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ks = 4 * kg + i;
      // the image has 4 * nkp + 4 rows (t16_img_rows): step nkp's read stays inside
      const float na = xp[4 * (ks + 1) * 16], nb = xp[hs + 4 * (ks + 1) * 16];
      __builtin_amdgcn_sched_barrier(0);
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa, a1[bsel][i], acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(xb, a1[bsel][i], acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa, a2[bsel][i], acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(xb, a2[bsel][i], acc[1][1], 0, 0, 0);
      xa = na;
      xb = nb;
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  int kg = 0;
  for (; kg + 2 <= nkg; kg += 2) {
    group(kg, 0);
    group(kg + 1, 1);
  }
  if (kg < nkg) group(kg, 0);
}

// the image rows of the wave's tile as B operands in the permuted channel order of t16_mlp
__device__ __forceinline__ void t16_rows(const float* img, int hs, int w0, int lane, f32x4v* x) {
  const int g = lane >> 4, j = lane & 15;
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    const float4 q = *(const float4*)(img + hf * hs + (w0 + j) * 16 + 4 * g);
    x[hf] = f32x4v{q.x, q.y, q.z, q.w};
  }
}

// Tile range of a t16 workgroup: the launch's slices x nt tiles in slice-major order, cut into
// gridDim.x equal contiguous ranges (one workgroup per CU: every CU gets the same number of tiles,
// whatever the slice count -- no partial last round of whole slices).  The range is worked in
// phases of at most maximg slices: their images staged, one barrier, then wave w takes the
// phase's tiles t with t % nwaves == w (the 16 waves of a CU spread over its 4 SIMDs evenly).
struct T16Range {
  long tb, te;
};
__device__ __forceinline__ T16Range t16_range(int slices, int nt) {
  const long total = (long)slices * nt;
  return {total * blockIdx.x / gridDim.x, total * (blockIdx.x + 1) / gridDim.x};
}

// a tile's 32 channels (lane (g, j): node w0 + j, channels 16 hf + 4 g .. + 3, as the t16
// accumulators) as bf16 into the tiled activation layout of gwn_gram_g4_bf16: one KiB per (slice,
// tile) of operand `which` (regions of slices * nt KiB), lane (g, j)'s 16 B = channels 4g .. 4g+3
// then 16+4g .. 16+4g+3 (its MFMA k-group)
typedef __bf16 bf16x8g __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void t16_store_g4(void* base, int which, int slices, int slice, int nt, int tile, int lane,
                                             const f32x4v* v) {
  bf16x8g r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    r[i] = (__bf16)v[0][i];
    r[4 + i] = (__bf16)v[1][i];
  }
  *(bf16x8g*)((char*)base + (((long)which * slices + slice) * nt + tile) * 1024 + lane * 16) = r;
}

// ---- the gated TCN fused into the f32 tile forward's staging (FusedFwd.tcn) ----
// xg[r][c] = tanh(f) sigmoid(g) with (f, g)[r] = w_fg [x[r] | x[r + tap_rows]] + b_fg (model.py:
// 206-212; rowgemm.hip's gwn_rowgemm_tcn_fwd computes the same as a separate launch).  One unit = a
// 16-node group of one output slice on v_mfma_f32_16x16x4_f32, in the transposed orientation
//   D[o][w] = sum_k W[o][k] X[w][k]        (M = 64 gate outputs in four 16-row tiles, N = nodes)
// with the contraction permuted so that lane group g takes k = 16 g + kk at step kk: its B operand
// is 16 contiguous floats of its node's row (tap g >> 1, channels 16 (g & 1) ..), its A operand 16
// contiguous floats of a weight row (ds_read_b128 x 4).  Tile t of the outputs holds channel
// 16 (t >> 1) + i's filter (t even) or gate (t odd) row, so lane (g, j) ends with f and g of the
// same four channels 16 hf + 4 g + r of node w0 + j: the gate is elementwise in registers, and
// the result is a float4 of the two-half slice image as it stands.

// the TCN's pointers and sizes as the staging reads them: parked in LDS with the weights, so that
// they do not hold scalar registers through the tile loop (which then spilled)
struct TcnLds {
  const float* x; float* fg; float* skip; float* h;
  long tap_rows, ld_skip, skip_row0;
  int x_bytes, ld_h;
};
static_assert(sizeof(TcnLds) <= 16 * sizeof(float), "TcnLds in its LDS slot");
__device__ __forceinline__ const TcnLds* tcn_lds(const float* tw) { return (const TcnLds*)(tw + TW_PAR); }
template <typename T>
__device__ __forceinline__ T tcn_uniform(const T& v) {  // an LDS-held value as a wave-uniform scalar
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "4- or 8-byte values");
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
  } else {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffff)), hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __builtin_bit_cast(T, (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
  }
}

// the layer below's BatchNorm from its partials (gwn_tcn_args.bn), in every workgroup: thread (sub,
// c) merges slots sub, sub + 32, ... of channel c in double (coalesced rows), the 32 subs meet in
// scratch (LDS, 3 KiB floats x 4) and channel c's thread merges them in order -> mean and scale =
// gamma * rstd at tw[TW_MEAN] / tw[TW_SCALE]; workgroup 0 writes gwn_batchnorm_fwd_fold's outputs
// but w_fold / b_fold (t16_tcn_stage_weights).  Every workgroup computes bit-identical values.
__device__ __forceinline__ void t16_tcn_bn_finalize(const FusedFwd& a, float* tw, float* scratch) {
  const auto& f = a.tcn.bn;
  const int c = threadIdx.x & 31, sub = threadIdx.x >> 5, nsub = blockDim.x >> 5;
  // the partials (count, mean, M2) as fp64 sums n, S = sum n_b mean_b, Q = sum (M2_b + n_b mean_b^2):
  // no division per merge (a Chan merge divides per partial, a serial chain per thread); mean = S/n,
  // M2 = Q - S mean in fp64 (fp32 inputs: the cancellation costs ~1e-16 (1 + mean^2/var) of var)
  double n = 0.0, s1 = 0.0, s2 = 0.0;
  constexpr int U = 12;  // (768 partials: two rounds of loads per thread)
  for (int i0 = sub; i0 < f.nparts; i0 += U * nsub) {
    float nb[U], mb[U], qb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // unconditional loads (a slot past nparts reads slot 0, then counts 0)
      const int i = i0 + u * nsub;
      const float* pp = f.part + (long)(i < f.nparts ? i : 0) * 3 * CH;
      nb[u] = pp[c];
      mb[u] = pp[CH + c];
      qb[u] = pp[2 * CH + c];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + u * nsub >= f.nparts) nb[u] = 0.0f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (nb[u] <= 0.0f) continue;
      const double nm = (double)nb[u] * (double)mb[u];
      n += nb[u];
      s1 += nm;
      s2 += (double)qb[u] + nm * (double)mb[u];
    }
  }
  // the nsub sums of a channel: a fixed-order tree in LDS (fp64)
  double* sd = (double*)scratch;
  sd[(sub * 3) * CH + c] = n;
  sd[(sub * 3 + 1) * CH + c] = s1;
  sd[(sub * 3 + 2) * CH + c] = s2;
  __syncthreads();
  for (int w = nsub >> 1; w > 0; w >>= 1) {
    if (sub < w)
#pragma unroll
      for (int e = 0; e < 3; ++e) sd[(sub * 3 + e) * CH + c] += sd[((sub + w) * 3 + e) * CH + c];
    __syncthreads();
  }
  if (threadIdx.x < CH) {
    n = sd[c];
    const double mean = n > 0.0 ? sd[CH + c] / n : 0.0;
    const double m2d = sd[2 * CH + c] - sd[CH + c] * mean;
    const double m2 = m2d > 0.0 ? m2d : 0.0;
    const double var = n > 0.0 ? m2 / n : 0.0;
    const float rs = (float)(1.0 / sqrt(var + (double)f.eps));
    const float sc = rs * f.gamma[c];  // bn(z) = (z - mean) * sc + beta
    tw[TW_MEAN + c] = (float)mean;
    tw[TW_SCALE + c] = sc;
    if (blockIdx.x == 0) {
      f.save_mean[c] = (float)mean;
      f.save_rstd[c] = rs;
      f.scale[c] = sc;
      if (f.rm) {
        const double unbiased = n > 1.0 ? m2 / (n - 1.0) : var;
        f.rm[c] = (float)((1.0 - f.mom) * f.rm[c] + f.mom * mean);
        f.rv[c] = (float)((1.0 - f.mom) * f.rv[c] + f.mom * unbiased);
      }
      if (c == 0 && f.nbt) *f.nbt += 1;
    }
  }
  __syncthreads();
}

// the TCN weights (rows in MFMA-tile order), input means and biases into the staging region; with
// bn, first the finalize (scratch: the channel maps' LDS, staged afterwards), then the weights
// folded (w * scale, b + w beta; workgroup 0 also writes w_fold / b_fold)
__device__ __forceinline__ void t16_tcn_stage_weights(const FusedFwd& a, float* tw, float* scratch) {
  static_assert(T16_WAVES * 64 == 1024, "the staging maps 64 x 64 weights four per thread");
  const bool bn = a.tcn.bn.part != nullptr;
  // the raw weights and the bias-fold operands do not depend on the statistics: loaded first, so
  // their latency overlaps the finalize's
  float wr[4], wb[4], bb[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e = threadIdx.x + 1024 * q, ti = e >> 6, k = e & 63, t = ti >> 4, i = ti & 15;
    wr[q] = a.tcn.w[(2 * (16 * (t >> 1) + i) + (t & 1)) * 64 + k];
  }
  const int bo = threadIdx.x >> 4, bpart = threadIdx.x & 15;  // bias fold: 16 threads per output
  if (bn) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      wb[q] = a.tcn.w[bo * 64 + 4 * bpart + q];
      bb[q] = a.tcn.bn.beta[(4 * bpart + q) & 31];
    }
    t16_tcn_bn_finalize(a, tw, scratch);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e = threadIdx.x + 1024 * q, ti = e >> 6, k = e & 63, t = ti >> 4, i = ti & 15;
    float w = wr[q];
    if (bn) {
      w *= tw[TW_SCALE + (k & 31)];
      if (blockIdx.x == 0) a.tcn.bn.w_fold[(2 * (16 * (t >> 1) + i) + (t & 1)) * 64 + k] = w;
    }
    tw[ti * LDT_TCN + k] = w;
  }
  if (bn) {
    // b_fold[o] = b[o] + sum_k w[o][k] beta[k % 32]: 16 threads per output, 4 k each, fixed tree
    float acc = 0.0f;
#pragma unroll
    for (int q = 0; q < 4; ++q) acc = fmaf(wb[q], bb[q], acc);
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 16);
    if (bpart == 0) {
      const float b = a.tcn.b[bo] + acc;
      tw[TW_BIAS + bo] = b;
      if (blockIdx.x == 0) a.tcn.bn.b_fold[bo] = b;
    }
  } else {
    if (threadIdx.x < 32) tw[TW_MEAN + threadIdx.x] = a.tcn.mean ? a.tcn.mean[threadIdx.x] : 0.0f;
    if (threadIdx.x < 64) tw[TW_BIAS + threadIdx.x] = a.tcn.b[threadIdx.x];
  }
  if (threadIdx.x == 0) {
    TcnLds* t = (TcnLds*)(tw + TW_PAR);
    t->x = a.tcn.x; t->fg = a.tcn.fg; t->skip = a.tcn.skip; t->h = (float*)a.h;
    t->tap_rows = a.tcn.tap_rows; t->ld_skip = a.tcn.ld_skip; t->skip_row0 = a.tcn.skip_row0;
    t->x_bytes = (int)(a.tcn.x_rows * CH * 4); t->ld_h = (int)a.ld_h;
  }
}

// the unit's input rows: lane (g, j) loads node w0 + j's 16 channels of k-group g
__device__ __forceinline__ void t16_tcn_load(const TcnLds* tp, int s, int w0, int lane, int n, float4* xq) {
  const int g = lane >> 4, node = w0 + (lane & 15);
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void*)tcn_uniform(tp->x), (short)0, tcn_uniform(tp->x_bytes), 0x00020000);
  const long row = (long)s * n + node + (g >> 1) * tcn_uniform(tp->tap_rows);
  const int off = node < n ? (int)((row * CH + 16 * (g & 1)) * 4) : 0x7ffffff0;
#pragma unroll
  for (int q = 0; q < 4; ++q) xq[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 16 * q, 0));
  // all four in flight before the first use: left to the scheduler, each load was sunk next to
  // its first product behind its own vmcnt(0) -- four serial memory round trips per unit
  __builtin_amdgcn_sched_barrier(0);
}

// one unit: the products, the gate, the image rows (zero past n) and the global outputs
__device__ __forceinline__ void t16_tcn_unit(const float* tw, const float4* xq, float* img, int hs, int s, int w0,
                                             int lane, int n) {
  const TcnLds* tp = tcn_lds(tw);
  const int g = lane >> 4, j = lane & 15, node = w0 + j;
  const bool valid = node < n;
  const float* mu = tw + TW_MEAN + 16 * (g & 1);
  float xv[16];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 m = *(const float4*)(mu + 4 * q);
    xv[4 * q] = xq[q].x - m.x; xv[4 * q + 1] = xq[q].y - m.y;
    xv[4 * q + 2] = xq[q].z - m.z; xv[4 * q + 3] = xq[q].w - m.w;
  }
  const float* bias = tw + TW_BIAS;
  const long row = (long)s * n + node;
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    // the half's filter and gate tiles (t = 2 hf, 2 hf + 1), then its gate: one half live at a time
    f32x4v acc[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const float* wr = tw + (16 * (2 * hf + u) + j) * LDT_TCN + 16 * g;
      float wf[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = *(const float4*)(wr + 4 * q);
        wf[4 * q] = v.x; wf[4 * q + 1] = v.y; wf[4 * q + 2] = v.z; wf[4 * q + 3] = v.w;
      }
      acc[u] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[kk], xv[kk], acc[u], 0, 0, 0);
    }
    const int c0 = 16 * hf + 4 * g;
    f32x4v xg, f0, f1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float tf = gwn_gate_tanh(acc[0][r] + bias[2 * (c0 + r)]);
      const float sg = gwn_gate_sigmoid(acc[1][r] + bias[2 * (c0 + r) + 1]);
      xg[r] = tf * sg;
      if (r < 2) { f0[2 * r] = tf; f0[2 * r + 1] = sg; }
      else { f1[2 * r - 4] = tf; f1[2 * r - 3] = sg; }
    }
    *(f32x4v*)(img + hf * hs + node * 16 + 4 * g) = valid ? xg : f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
    if (valid) {
      __builtin_nontemporal_store(xg, (f32x4v*)(tcn_uniform(tp->h) + row * tcn_uniform(tp->ld_h) + c0));
      float* fg = tcn_uniform(tp->fg);
      if (fg) {
        __builtin_nontemporal_store(f0, (f32x4v*)(fg + row * 2 * CH + 2 * c0));
        __builtin_nontemporal_store(f1, (f32x4v*)(fg + row * 2 * CH + 2 * c0 + 4));
      }
      float* skip = tcn_uniform(tp->skip);
      const long srow0 = tcn_uniform(tp->skip_row0);
      if (skip && row >= srow0)
        __builtin_nontemporal_store(xg, (f32x4v*)(skip + (row - srow0) * tcn_uniform(tp->ld_skip) + c0));
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// a phase's slice images from the TCN: units (slice, 16-node group) dealt to the waves, each
// unit's rows loaded one unit ahead; the image rows past the last group are zeroed
__device__ __forceinline__ void t16_tcn_stage(int n, const float* tw, float* imgs, int imgf, int hs, int rows_img,
                                              int s0, int nsl, int lane, int wave, int nwaves) {
  const int nt = (n + 15) >> 4, units = nsl * nt;
  const TcnLds* tp = tcn_lds(tw);
  for (int u = wave; u < units; u += nwaves) {
    const int sl = u / nt, w0 = 16 * (u - sl * nt);
    float4 xq[4];
    t16_tcn_load(tp, s0 + sl, w0, lane, n, xq);
    t16_tcn_unit(tw, xq, imgs + sl * imgf, hs, s0 + sl, w0, lane, n);
  }
  const int pad = rows_img - 16 * nt;  // rows past the groups: zero (both halves)
  for (int e = threadIdx.x; e < nsl * pad * 8; e += blockDim.x) {
    const int sl = e / (pad * 8), rem = e - sl * pad * 8, w = 16 * nt + (rem >> 3), q = rem & 7;
    *(float4*)(imgs + sl * imgf + (q >> 2) * hs + w * 16 + 4 * (q & 3)) = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  }
}

// (Two slices per wave -- the same node column of two slices diffused against shared support
// fragments, the channel-map fragments shared by both mlps -- measured slower at every layer shape:
// 167 vs 159 us at 768 slices with 16 waves (51 registers spilled), 167 at 12 waves without spills;
// profiles/r05/spw.)
template <int MAXT>
__global__ __launch_bounds__(MAXT) void gcn_fwd_t16_kernel(const FusedFwd a, const PowSup p, const int maximg) {
  extern __shared__ float lds[];
  const int n = a.n;
  const int nt = (n + 15) >> 4;
  const int rows_img = t16_img_rows(n), hs = rows_img * 16, imgf = rows_img * CH;
  float* ws = lds;
  float* wpart = ws + (2 * a.nsup + 1) * CH * LDW16;
  const bool tcn = a.tcn.x != nullptr;
  float* imgs = wpart + t16_region(tcn);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  const int nwaves = blockDim.x >> 6;
  const long ldh = a.ld_h;
  const T16Range rg = t16_range(a.slices, nt);
  BnRun bn;
  bn_init(bn, wpart);
  t16_clock_start(a);
  const unsigned long long seed = t16_seed(a);
  // the phase's slices staged in one pass (stage_rows4; the channel maps inside its first round
  // trip), else slice by slice; with the fused TCN computed from its inputs (the TCN weights in
  // the BN partials' region until the final flush)
  const bool h16 = ((((uintptr_t)a.h) & 15) | (ldh & 3)) == 0;
  if (!h16 || tcn) t16_stage_maps(a.w_mlp, a.ld_w, false, 2 * a.nsup + 1, ws);
  if (tcn) t16_tcn_stage_weights(a, wpart, imgs);  // (the finalize's scratch: the free image space)
  // the residual's BatchNorm (the layer below's, finalized above when the TCN carries it: this
  // launch's workgroup 0 writes the global copies, so every workgroup reads its own)
  const bool bnk = tcn && a.tcn.bn.part != nullptr;
  const float* res_mean = bnk ? wpart + TW_MEAN : a.res_mean;
  const float* res_scale = bnk ? wpart + TW_SCALE : a.res_scale;
  for (long p0 = rg.tb; p0 < rg.te;) {
    const int s0 = (int)(p0 / nt);
    const long p1 = min(rg.te, (long)(s0 + maximg) * nt);
    const int s1 = (int)((p1 - 1) / nt);
    if (p0 != rg.tb || tcn) __syncthreads();  // the previous phase's images released (TCN: weights staged)
    if (tcn) {
      t16_tcn_stage(n, wpart, imgs, imgf, hs, rows_img, s0, s1 - s0 + 1, lane, wave, nwaves);
    } else if (h16) {
      const bool maps = p0 == rg.tb;
      stage_rows4<8>(
          a.h + (long)s0 * n * ldh, ldh, n, rows_img, s1 - s0 + 1,
          [&](int sl, int w, int q, float4 x) { *(float4*)(imgs + sl * imgf + (q >> 2) * hs + w * 16 + 4 * (q & 3)) = x; },
          [&] {
            if (maps) t16_stage_maps(a.w_mlp, a.ld_w, false, 2 * a.nsup + 1, ws);
          });
    } else {
      for (int s = s0; s <= s1; ++s) global_to_lds16(a.h + (long)s * n * ldh, ldh, n, rows_img, imgs + (s - s0) * imgf);
    }
    __syncthreads();
    const int span = (int)(p1 - p0);
    for (int tp = wave; tp < span; tp += nwaves) {
      const long t = p0 + tp;
      const int s = (int)(t / nt), tile = (int)(t - (long)s * nt);
      const float* xs = imgs + (s - s0) * imgf;
      const long row0 = (long)s * n;
      float* hs_out = (float*)a.h + row0 * ldh;
      const bool nt_ok = ((((uintptr_t)hs_out) & 15) | (ldh & 3)) == 0;
      const int w0 = 16 * tile;
      f32x4v hacc[2];
      hacc[0] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
      hacc[1] = hacc[0];
      {  // piece 0: the node features themselves
        f32x4v x0[2];
        t16_rows(xs, hs, w0, lane, x0);
        t16_mlp(ws, LDW16, x0, lane, hacc);
      }
      for (int k = 0; k < a.nsup; ++k) {
        f32x4v acc[2][2];  // [power][channel half]
        t16_diffuse(xs, hs, p.g4[2 * k], p.g4[2 * k + 1], n, tile, lane, acc);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          t16_mlp(ws + (1 + 2 * k + q) * CH * LDW16, LDW16, acc[q], lane, hacc);
          if (a.store_pieces && w0 + j < n) {
            float* dp = hs_out + (long)(w0 + j) * ldh + (1 + 2 * k + q) * CH + 4 * g;
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
              if (nt_ok) __builtin_nontemporal_store(acc[q][hf], (f32x4v*)(dp + 16 * hf));
              else {
#pragma unroll
                for (int e = 0; e < 4; ++e) dp[16 * hf + e] = acc[q][hf][e];
              }
            }
          }
        }
      }
      t16_epilogue(a, hacc, row0, w0, lane, n, bn, seed, res_mean, res_scale);
    }
    p0 = p1;
  }
  t16_bn_flush(a, bn, wpart);
  t16_clock_end(a);
}

// ---------------------------------------------------------------------------------------------
// bf16 operands (configs[2]'s mixed precision) on the 16-node tile forward: the diffusion on
// v_mfma_f32_16x16x32_bf16 (32 nodes per MFMA instead of 4), fp32 accumulation; the mlp, the hop
// pieces, z and the BN partials exactly as the f32 kernel (its accumulator layout is the same:
// lane l holds D[16 hf + 4 (l >> 4) + r][w0 + (l & 15)]).
//   A operand: the slice image in bf16, channel-major [32][s16] in LDS (s16 = 32 * nkg + 8: rows
//     >= n zero; the 8-element pad spreads the channel rows over the banks), lane l reading the 8
//     nodes 32 kg + 8 (l >> 4) .. of channel 16 hf + (l & 15) with one ds_read_b128;
//   B operand: gwn_support_g4_bf16's copy of the support, one 16-B load per lane per 32 nodes;
//   piece 0's mlp takes the tile's fp32 rows straight from HBM / L2 (no fp32 image in LDS).
typedef __bf16 bf16x8b __attribute__((ext_vector_type(8)));

__host__ __device__ inline int t16b_s16(int n) { return 32 * ((n + 31) / 32) + 8; }

size_t t16b_lds_bytes(int n, int nsup, int maximg) {
  return (size_t)((2 * nsup + 1) * CH * LDW16 + T16_WAVES * 3 * CH) * sizeof(float) +
         (size_t)maximg * CH * t16b_s16(n) * 2;
}

// channels 4q .. 4q+3 of node w into the channel-major bf16 image [32][s16]
__device__ __forceinline__ void put_bf16_cm(__bf16* img, int s16, int w, int q, float4 x) {
  img[(4 * q) * s16 + w] = (__bf16)x.x;
  img[(4 * q + 1) * s16 + w] = (__bf16)x.y;
  img[(4 * q + 2) * s16 + w] = (__bf16)x.z;
  img[(4 * q + 3) * s16 + w] = (__bf16)x.w;
}

typedef __bf16 bf16x8s __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4s __attribute__((ext_vector_type(4)));

// A phase's channel-major bf16 images (nsl slices, imgb bf16 apart, rows = s16 - 8 >= n, rows >= n
// zero) from fp32 rows (src: slice 0's row 0, slice stride n * ld floats, 16-B aligned, ld % 4 ==
// 0): work unit = (slice, 8 consecutive nodes, channel quad q), 8 row loads of 16 B (the 8 lanes of
// a node octet cover a whole 128-B row) then one 16-B LDS write per channel (8 nodes' bf16) --
// instead of one 2-B write per element (put_bf16_cm).  mid() runs with round 0's loads in flight.
template <typename Mid>
__device__ __forceinline__ void stage_bf16_octets(const float* src, long ld, int n, int s16, int nsl, __bf16* imgs,
                                                  int imgb, Mid mid) {
  const int rows = s16 - 8, per = rows, total = nsl * per;  // units per slice = (rows / 8) * 8
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)((long)nsl * n * ld * 4), 0x00020000);
  bool first = true;
  for (int u = threadIdx.x; u < total || first; u += blockDim.x) {
    const bool ok = u < total;
    const int sl = ok ? u / per : 0, rem = u - sl * per, k = rem >> 3, q = rem & 7;
    float4 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int w = 8 * k + i;
      const int off = (ok && w < n) ? (int)((((long)sl * n + w) * ld + 4 * q) * 4) : 0x7ffffff0;
      v[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
    }
    if (first) {
      mid();
      first = false;
    }
    if (!ok) continue;
    __bf16* img = imgs + (long)sl * imgb + 8 * k;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      bf16x8s o;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (__bf16)((const float*)&v[i])[e];
      *(bf16x8s*)(img + (4 * q + e) * s16) = o;
    }
  }
}

// a slice's node features (rows >= n zero) -> the channel-major bf16 image [32][s16]
__device__ __forceinline__ void global_to_lds16_bf16(const float* src, long ld, int n, __bf16* img) {
  const int s16 = t16b_s16(n), rows = s16 - 8;
  for (int e = threadIdx.x; e < rows * 8; e += blockDim.x) {
    const int v = e >> 3, q = e & 7;
    float4 x = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (v < n) x = *(const float4*)(src + (long)v * ld + 4 * q);
    img[(4 * q) * s16 + v] = (__bf16)x.x;
    img[(4 * q + 1) * s16 + v] = (__bf16)x.y;
    img[(4 * q + 2) * s16 + v] = (__bf16)x.z;
    img[(4 * q + 3) * s16 + v] = (__bf16)x.w;
  }
}

// support-fragment groups in flight ahead: one (two at 16 waves: PEMS 23.65k vs 23.79k samples/s;
// 12-wave workgroups with a ring 2-3 groups deep: slower again)
constexpr int T16B_AHEAD = 1;
// both powers of one support on bf16 operands (acc as t16_diffuse); G1 / G2: gwn_support_g4_bf16
// copies (block (kg, tile) = 64 lanes x 8 bf16)
template <int AH = T16B_AHEAD>
__device__ __forceinline__ void t16b_diffuse(const __bf16* img, const __bf16* G1, const __bf16* G2, int n, int tile,
                                             int lane, f32x4v (*acc)[2]) {
  const int g = lane >> 4, j = lane & 15;
  const int nt = (n + 15) >> 4, nkg = (n + 31) >> 5, s16 = t16b_s16(n);
  const int bytes = nkg * nt * 1024;
  const __amdgpu_buffer_rsrc_t r1 = __builtin_amdgcn_make_buffer_rsrc((void*)G1, (short)0, bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t r2 = __builtin_amdgcn_make_buffer_rsrc((void*)G2, (short)0, bytes, 0x00020000);
  auto off = [&](int kg) { return ((kg * nt + tile) * 64 + lane) * 16; };
  const __bf16* x0 = img + j * s16 + 8 * g;         // channel j (half 0)
  const __bf16* x1 = img + (16 + j) * s16 + 8 * g;  // channel 16 + j (half 1)
#pragma unroll
  for (int q = 0; q < 2; ++q) acc[q][0] = acc[q][1] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
  // support fragments T16B_AHEAD groups ahead (a group is only 4 MFMAs: one group ahead left the
  // L2 latency exposed); past the last group the offsets leave the range: zeros, no traffic
  auto ld = [&](const __amdgpu_buffer_rsrc_t& r, int kg) {
    return __builtin_bit_cast(bf16x8b, __builtin_amdgcn_raw_buffer_load_b128(r, off(kg), 0, 0));
  };
  bf16x8b b1 = ld(r1, 0), b2 = ld(r2, 0);
  bf16x8b c1 = AH > 1 ? ld(r1, 1) : b1, c2 = AH > 1 ? ld(r2, 1) : b2;
  bf16x8b d1 = AH > 2 ? ld(r1, 2) : b1, d2 = AH > 2 ? ld(r2, 2) : b2;
  bf16x8b a0 = *(const bf16x8b*)x0, a1 = *(const bf16x8b*)x1;
  for (int kg = 0; kg < nkg; ++kg) {
    const bf16x8b nb1 = ld(r1, kg + AH), nb2 = ld(r2, kg + AH);
    const int nx = kg + 1 < nkg ? 32 * (kg + 1) : 32 * kg;
    const bf16x8b na0 = *(const bf16x8b*)(x0 + nx), na1 = *(const bf16x8b*)(x1 + nx);
    acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b1, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b2, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b2, acc[1][1], 0, 0, 0);
    if (AH > 2) {
      b1 = c1; b2 = c2;
      c1 = d1; c2 = d2;
      d1 = nb1; d2 = nb2;
    } else if (AH > 1) {
      b1 = c1; b2 = c2;
      c1 = nb1; c2 = nb2;
    } else {
      b1 = nb1; b2 = nb2;
    }
    a0 = na0;
    a1 = na1;
  }
}

// the tile's fp32 node rows (piece 0 of the mlp) from global memory, in t16_rows' order
__device__ __forceinline__ void t16_rows_global(const float* src, long ld, int w0, int n, int lane, f32x4v* x) {
  const int g = lane >> 4, j = lane & 15;
  const int w = min(w0 + j, n - 1);
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    const float4 q = *(const float4*)(src + (long)w * ld + 16 * hf + 4 * g);
    x[hf] = w0 + j < n ? f32x4v{q.x, q.y, q.z, q.w} : f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
  }
}

template <int MAXT, bool MLPB = false>
__global__ __launch_bounds__(MAXT) void gcn_fwd_t16b_kernel(const FusedFwd a, const PowSup p, const int maximg) {
  extern __shared__ float lds[];
  const int n = a.n;
  const int nt = (n + 15) >> 4;
  const int s16 = t16b_s16(n), imgb = CH * s16;  // bf16 elements per image
  float* ws = lds;
  float* wpart = ws + (2 * a.nsup + 1) * CH * LDW16;
  __bf16* imgs = (__bf16*)(wpart + T16_WAVES * 3 * CH);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  const int nwaves = blockDim.x >> 6;
  const long ldh = a.ld_h;
  const T16Range rg = t16_range(a.slices, nt);
  BnRun bn;
  bn_init(bn, wpart);
  t16_clock_start(a);
  const unsigned long long seed = t16_seed(a);
  const bool h16 = ((((uintptr_t)a.h) & 15) | (ldh & 3)) == 0;
  // the channel maps: f32 for t16_mlp, or bf16 MFMA operands for t16_mlp_b (MLPB)
  auto stage_maps = [&] {
    if (MLPB) t16_stage_maps_bf16(a.w_mlp, a.ld_w, false, 2 * a.nsup + 1, (__bf16*)ws);
    else t16_stage_maps(a.w_mlp, a.ld_w, false, 2 * a.nsup + 1, ws);
  };
  auto mlp = [&](int piece, const f32x4v* x, f32x4v* out) {
    if (MLPB) t16_mlp_b((const __bf16*)ws, piece, x, lane, out);
    else t16_mlp(ws + piece * CH * LDW16, LDW16, x, lane, out);
  };
  if (!h16) stage_maps();
  for (long p0 = rg.tb; p0 < rg.te;) {
    const int s0 = (int)(p0 / nt);
    const long p1 = min(rg.te, (long)(s0 + maximg) * nt);
    const int s1 = (int)((p1 - 1) / nt);
    if (p0 != rg.tb) __syncthreads();  // the previous phase's images are released
    if (h16) {  // as the f32 kernel: the phase in one pass, the maps inside its first round trip
      const bool maps = p0 == rg.tb;
      stage_bf16_octets(a.h + (long)s0 * n * ldh, ldh, n, s16, s1 - s0 + 1, imgs, imgb, [&] {
        if (maps) stage_maps();
      });
    } else {
      for (int sl = s0; sl <= s1; ++sl) global_to_lds16_bf16(a.h + (long)sl * n * ldh, ldh, n, imgs + (sl - s0) * imgb);
    }
    __syncthreads();
    const int span = (int)(p1 - p0);
    for (int tp = wave; tp < span; tp += nwaves) {
      const long t = p0 + tp;
      const int sl = (int)(t / nt), tile = (int)(t - (long)sl * nt);
      const __bf16* xs = imgs + (sl - s0) * imgb;
      const long row0 = (long)sl * n;
      float* hs_out = (float*)a.h + row0 * ldh;
      const bool nt_ok = ((((uintptr_t)hs_out) & 15) | (ldh & 3)) == 0;
      const int w0 = 16 * tile;
      f32x4v hacc[2];
      hacc[0] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
      hacc[1] = hacc[0];
      if (MLPB) {  // piece 0 = bf16(g): the staged image's column, no global read
        const bf16x8m b0 = t16_img_col_b(xs, s16, w0, lane);
        t16_mlp_bp((const __bf16*)ws, 0, b0, lane, hacc);
        if (a.xg4)  // t16_store_g4's layout, already bf16
          *(bf16x8m*)((char*)a.xg4 + ((long)sl * nt + tile) * 1024 + lane * 16) = b0;
      } else {  // piece 0: the node features themselves (fp32)
        f32x4v x0[2];
        t16_rows_global(hs_out, ldh, w0, n, lane, x0);
        mlp(0, x0, hacc);
        if (a.xg4) t16_store_g4(a.xg4, 0, a.slices, sl, nt, tile, lane, x0);
      }
      for (int k = 0; k < a.nsup; ++k) {
        f32x4v acc[2][2];
        t16b_diffuse(xs, (const __bf16*)p.g4[2 * k], (const __bf16*)p.g4[2 * k + 1], n, tile, lane, acc);
        if (a.xg4 && k == a.xg4_k) t16_store_g4(a.xg4, 1, a.slices, sl, nt, tile, lane, acc[0]);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          if (MLPB) {  // one bf16 conversion for the mlp operand and the piece store
            const bf16x8m b = t16_pack_b(acc[q]);
            t16_mlp_bp((const __bf16*)ws, 1 + 2 * k + q, b, lane, hacc);
            if (a.store_pieces && a.pb && w0 + j < n) {
              __bf16* bp = (__bf16*)a.pb + (row0 + w0 + j) * a.ld_pb + (2 * k + q) * CH + 4 * g;
              // plain stores: write-back L2 merges a node's 8-B pieces into full lines (non-temporal:
              // 1.43x instead of 1.19x the algorithmic forward traffic at the same time)
              typedef __bf16 bf16x4p __attribute__((ext_vector_type(4)));
              *(bf16x4p*)bp = bf16x4p{b[0], b[1], b[2], b[3]};
              *(bf16x4p*)(bp + 16) = bf16x4p{b[4], b[5], b[6], b[7]};
              continue;
            }
          } else {
            mlp(1 + 2 * k + q, acc[q], hacc);
          }
          if (a.store_pieces && a.pb && w0 + j < n) {
            // bf16 pieces: node w0 + j, channels 16 hf + 4 g .. +3 as 8-B stores (non-temporal)
            __bf16* bp = (__bf16*)a.pb + (row0 + w0 + j) * a.ld_pb + (2 * k + q) * CH + 4 * g;
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
              typedef __bf16 bf16x4p __attribute__((ext_vector_type(4)));
              bf16x4p v;
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = (__bf16)acc[q][hf][e];
              __builtin_nontemporal_store(v, (bf16x4p*)(bp + 16 * hf));
            }
          } else if (a.store_pieces && w0 + j < n) {
            float* dp = hs_out + (long)(w0 + j) * ldh + (1 + 2 * k + q) * CH + 4 * g;
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
              if (nt_ok) __builtin_nontemporal_store(acc[q][hf], (f32x4v*)(dp + 16 * hf));
              else {
#pragma unroll
                for (int e = 0; e < 4; ++e) dp[16 * hf + e] = acc[q][hf][e];
              }
            }
          }
        }
      }
      t16_epilogue(a, hacc, row0, w0, lane, n, bn, seed);
    }
    p0 = p1;
  }
  t16_bn_flush(a, bn, wpart);
  t16_clock_end(a);
}

// Two slices per wave in the bf16-mlp forward (the same node column of slices 2q and 2q + 1): at
// N = 325 the single-slice kernel streams ~66 KB of support fragments per tile from L2 (~17 TB/s,
// the L2's shared-rows rate), so each fragment load here feeds both slices' MFMAs.
__device__ __forceinline__ void t16b_diffuse2(const __bf16* imgA, const __bf16* imgB, const __bf16* G1,
                                              const __bf16* G2, int n, int tile, int lane, f32x4v (*accA)[2],
                                              f32x4v (*accB)[2]) {
  const int g = lane >> 4, j = lane & 15;
  const int nt = (n + 15) >> 4, nkg = (n + 31) >> 5, s16 = t16b_s16(n);
  const int bytes = nkg * nt * 1024;
  const __amdgpu_buffer_rsrc_t r1 = __builtin_amdgcn_make_buffer_rsrc((void*)G1, (short)0, bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t r2 = __builtin_amdgcn_make_buffer_rsrc((void*)G2, (short)0, bytes, 0x00020000);
  auto off = [&](int kg) { return ((kg * nt + tile) * 64 + lane) * 16; };
  const __bf16* xa0 = imgA + j * s16 + 8 * g;
  const __bf16* xa1 = imgA + (16 + j) * s16 + 8 * g;
  const __bf16* xb0 = imgB + j * s16 + 8 * g;
  const __bf16* xb1 = imgB + (16 + j) * s16 + 8 * g;
#pragma unroll
  for (int q = 0; q < 2; ++q) accA[q][0] = accA[q][1] = accB[q][0] = accB[q][1] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
  auto ld = [&](const __amdgpu_buffer_rsrc_t& r, int kg) {
    return __builtin_bit_cast(bf16x8b, __builtin_amdgcn_raw_buffer_load_b128(r, off(kg), 0, 0));
  };
  bf16x8b b1 = ld(r1, 0), b2 = ld(r2, 0);
  for (int kg = 0; kg < nkg; ++kg) {
    const bf16x8b nb1 = ld(r1, kg + 1), nb2 = ld(r2, kg + 1);
    const bf16x8b pa0 = *(const bf16x8b*)(xa0 + 32 * kg), pa1 = *(const bf16x8b*)(xa1 + 32 * kg);
    const bf16x8b pb0 = *(const bf16x8b*)(xb0 + 32 * kg), pb1 = *(const bf16x8b*)(xb1 + 32 * kg);
    accA[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa0, b1, accA[0][0], 0, 0, 0);
    accA[0][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa1, b1, accA[0][1], 0, 0, 0);
    accB[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pb0, b1, accB[0][0], 0, 0, 0);
    accB[0][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pb1, b1, accB[0][1], 0, 0, 0);
    accA[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa0, b2, accA[1][0], 0, 0, 0);
    accA[1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa1, b2, accA[1][1], 0, 0, 0);
    accB[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pb0, b2, accB[1][0], 0, 0, 0);
    accB[1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pb1, b2, accB[1][1], 0, 0, 0);
    b1 = nb1;
    b2 = nb2;
  }
}

// t16_mlp_bp for two slices with one read of the map's A fragments
__device__ __forceinline__ void t16_mlp_bp2(const __bf16* maps, int p, const bf16x8m bA, const bf16x8m bB, int lane,
                                            f32x4v* haccA, f32x4v* haccB) {
  const bf16x8m a0 = *(const bf16x8m*)(maps + ((p * 2 + 0) * 64 + lane) * 8);
  const bf16x8m a1 = *(const bf16x8m*)(maps + ((p * 2 + 1) * 64 + lane) * 8);
  __builtin_amdgcn_sched_barrier(0);
  haccA[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bA, haccA[0], 0, 0, 0);
  haccB[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bB, haccB[0], 0, 0, 0);
  haccA[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bA, haccA[1], 0, 0, 0);
  haccB[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bB, haccB[1], 0, 0, 0);
}

// the bf16-mlp forward over slice pairs: units = (pair, node tile) in pair-major order, cut into
// equal ranges per CU; a phase holds maximg (even) slices
template <int MAXT>
__global__ __launch_bounds__(MAXT) void gcn_fwd_t16b2_kernel(const FusedFwd a, const PowSup p, const int maximg) {
  extern __shared__ float lds[];
  const int n = a.n;
  const int nt = (n + 15) >> 4;
  const int s16 = t16b_s16(n), imgb = CH * s16;
  float* ws = lds;
  float* wpart = ws + (2 * a.nsup + 1) * CH * LDW16;
  __bf16* imgs = (__bf16*)(wpart + T16_WAVES * 3 * CH);
  const __bf16* maps = (const __bf16*)ws;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  const int nwaves = blockDim.x >> 6;
  const long ldh = a.ld_h;
  const int pairs = (a.slices + 1) / 2;
  const T16Range rg = t16_range(pairs, nt);
  BnRun bn;
  bn_init(bn, wpart);
  t16_clock_start(a);
  const unsigned long long seed = t16_seed(a);
  for (long p0 = rg.tb; p0 < rg.te;) {
    const int q0 = (int)(p0 / nt);
    const long p1 = min(rg.te, (long)(q0 + maximg / 2) * nt);
    const int q1 = (int)((p1 - 1) / nt);
    const int s0 = 2 * q0, s1 = min(2 * q1 + 2, a.slices) - 1;
    if (p0 != rg.tb) __syncthreads();
    const bool first = p0 == rg.tb;
    stage_bf16_octets(a.h + (long)s0 * n * ldh, ldh, n, s16, s1 - s0 + 1, imgs, imgb, [&] {
      if (first) t16_stage_maps_bf16(a.w_mlp, a.ld_w, false, 2 * a.nsup + 1, (__bf16*)ws);
    });
    __syncthreads();
    const int span = (int)(p1 - p0);
    for (int tp = wave; tp < span; tp += nwaves) {
      const long t = p0 + tp;
      const int q = (int)(t / nt), tile = (int)(t - (long)q * nt);
      const int sA = 2 * q, sB = 2 * q + 1;
      const bool okB = sB < a.slices;  // an odd last slice: B diffuses A's image, stores nothing
      const __bf16* xsA = imgs + (sA - s0) * imgb;
      const __bf16* xsB = okB ? imgs + (sB - s0) * imgb : xsA;
      const long rowA = (long)sA * n, rowB = (long)sB * n;
      const int w0 = 16 * tile;
      f32x4v haccA[2], haccB[2];
      haccA[0] = haccA[1] = haccB[0] = haccB[1] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
      {
        const bf16x8m bA = t16_img_col_b(xsA, s16, w0, lane), bB = t16_img_col_b(xsB, s16, w0, lane);
        t16_mlp_bp2(maps, 0, bA, bB, lane, haccA, haccB);
        if (a.xg4) {
          *(bf16x8m*)((char*)a.xg4 + ((long)sA * nt + tile) * 1024 + lane * 16) = bA;
          if (okB) *(bf16x8m*)((char*)a.xg4 + ((long)sB * nt + tile) * 1024 + lane * 16) = bB;
        }
      }
      for (int k = 0; k < a.nsup; ++k) {
        f32x4v accA[2][2], accB[2][2];
        t16b_diffuse2(xsA, xsB, (const __bf16*)p.g4[2 * k], (const __bf16*)p.g4[2 * k + 1], n, tile, lane, accA, accB);
        if (a.xg4 && k == a.xg4_k) {
          t16_store_g4(a.xg4, 1, a.slices, sA, nt, tile, lane, accA[0]);
          if (okB) t16_store_g4(a.xg4, 1, a.slices, sB, nt, tile, lane, accB[0]);
        }
#pragma unroll
        for (int pw = 0; pw < 2; ++pw) {
          const bf16x8m bA = t16_pack_b(accA[pw]), bB = t16_pack_b(accB[pw]);
          t16_mlp_bp2(maps, 1 + 2 * k + pw, bA, bB, lane, haccA, haccB);
          if (a.store_pieces && a.pb && w0 + j < n) {
            typedef __bf16 bf16x4p __attribute__((ext_vector_type(4)));
            __bf16* bpA = (__bf16*)a.pb + (rowA + w0 + j) * a.ld_pb + (2 * k + pw) * CH + 4 * g;
            *(bf16x4p*)bpA = bf16x4p{bA[0], bA[1], bA[2], bA[3]};
            *(bf16x4p*)(bpA + 16) = bf16x4p{bA[4], bA[5], bA[6], bA[7]};
            if (okB) {
              __bf16* bpB = (__bf16*)a.pb + (rowB + w0 + j) * a.ld_pb + (2 * k + pw) * CH + 4 * g;
              *(bf16x4p*)bpB = bf16x4p{bB[0], bB[1], bB[2], bB[3]};
              *(bf16x4p*)(bpB + 16) = bf16x4p{bB[4], bB[5], bB[6], bB[7]};
            }
          } else if (a.store_pieces && w0 + j < n) {  // fp32 pieces into h
            float* dA = (float*)a.h + (rowA + w0 + j) * ldh + (1 + 2 * k + pw) * CH + 4 * g;
            float* dB = (float*)a.h + (rowB + w0 + j) * ldh + (1 + 2 * k + pw) * CH + 4 * g;
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
              __builtin_nontemporal_store(accA[pw][hf], (f32x4v*)(dA + 16 * hf));
              if (okB) __builtin_nontemporal_store(accB[pw][hf], (f32x4v*)(dB + 16 * hf));
            }
          }
        }
      }
      t16_epilogue(a, haccA, rowA, w0, lane, n, bn, seed);
      if (okB) t16_epilogue(a, haccB, rowB, w0, lane, n, bn, seed);
    }
    p0 = p1;
  }
  t16_bn_flush(a, bn, wpart);
  t16_clock_end(a);
}

// Backward on 16-node tiles: the forward's structure with the dh image (BN-backward prologue),
// the transposed supports A_k^T and (A_k^2)^T (so D = A dh, A^2 dh) and the channel map W^T:
//   dxg = W_0^T dh + sum_k W_{1+2k}^T (A_k dh) + W_{2+2k}^T (A_k^2 dh)
// (gcn_bwd_pow_kernel's schedule), t1 / t2 of the adaptive support, and the dxg store or the gate
// backward in the epilogue.  The prologue stages a whole slice's dh image; dres / dh_out rows are
// written for the workgroup's own tiles only [r0, r1).
// BF: the image is the bf16 channel-major one of the bf16 forward ([32][s16], rows = s16 - 8)
template <bool BF>
__device__ __forceinline__ void t16_bwd_put(float* img, int rows, int w, int q, float4 x) {
  if (BF) put_bf16_cm((__bf16*)img, rows + 8, w, q, x);
  else *(float4*)(img + (q >> 2) * rows * 16 + w * 16 + 4 * (q & 3)) = x;
}

// t16_bwd_stage's BatchNorm prologue into the bf16 channel-major images: work unit = (slice, 4
// consecutive nodes, channel quad), 4 dy / z row loads of 16 B, then dres / dh_out (the
// workgroup's own rows) as 16-B stores and one 8-B LDS write per channel (4 nodes' bf16).
// pair_shift 1: rg ranges over (slice pair, tile) units (gcn_bwd_t16b2_kernel), the own rows of
// slice s are its pair s >> 1's tiles in the range
template <typename Mid>
__device__ __forceinline__ void t16_bwd_stage_bn_bf16(const FusedBwd& a, __bf16* imgs, int imgb, int s0, int nsl,
                                                      const T16Range& rg, int nt, int n, int s16, Mid mid,
                                                      int pair_shift = 0) {
  const unsigned long long seed = a.seed_ptr ? *a.seed_ptr : 0ull;
  const float keep_scale = (a.drop_p > 0.0f) ? 1.0f / (1.0f - a.drop_p) : 1.0f;
  const int q = threadIdx.x & 7;  // blockDim % 8 == 0: every unit of a thread has channel quad q
  float mu[4], rs[4], gm[4], k1[4], k2[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = 4 * q + e;
    mu[e] = a.bn_mean[c]; rs[e] = a.bn_rstd[c]; gm[e] = a.bn_gamma[c];
    k1[e] = a.bn_sums[c] * a.inv_rows; k2[e] = a.bn_sums[CH + c] * a.inv_rows;
  }
  const long base = (long)s0 * n * CH;
  const int bytes = (int)((long)nsl * n * CH * 4);
  const __amdgpu_buffer_rsrc_t rdy = __builtin_amdgcn_make_buffer_rsrc((void*)(a.bn_dy + base), (short)0, bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc((void*)(a.bn_z + base), (short)0, bytes, 0x00020000);
  const int rows = s16 - 8, per = 2 * rows, total = nsl * per;  // units per slice = (rows / 4) * 8
  bool first = true;
  for (int u = threadIdx.x; u < total || first; u += blockDim.x) {
    const bool ok = u < total;
    const int sl = ok ? u / per : 0, rem = u - sl * per, k = rem >> 3;  // nodes 4k .. 4k + 3
    float4 dy[4], zv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int w = 4 * k + i;
      const int off = (ok && w < n) ? ((sl * n + w) * CH + 4 * q) * 4 : 0x7ffffff0;
      dy[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rdy, off, 0, 0));
      zv[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rz, off, 0, 0));
    }
    if (first) {
      mid();
      first = false;
    }
    if (!ok) continue;
    const long sb = (long)((s0 + sl) >> pair_shift) * nt;
    const long t0 = max(rg.tb - sb, 0l), t1 = min(rg.te - sb, (long)nt);
    float v[4][4];  // [node][channel]
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int w = 4 * k + i;
      const float dyv[4] = {dy[i].x, dy[i].y, dy[i].z, dy[i].w}, zz[4] = {zv[i].x, zv[i].y, zv[i].z, zv[i].w};
      float dz[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float xhat = (zz[c] - mu[c]) * rs[c];
        dz[c] = gm[c] * rs[c] * (dyv[c] - k1[c] - xhat * k2[c]);
        v[i][c] = dz[c];
      }
      if (w < n) {
        const long row = (long)(s0 + sl) * n + w;
        if (a.drop_p > 0.0f) {
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float uu = gwn_uniform(seed, a.salt, (unsigned long long)(row * CH + 4 * q + c));
            v[i][c] = (uu >= a.drop_p) ? v[i][c] * keep_scale : 0.0f;
          }
        }
        if (w >= 16 * t0 && w < 16 * t1) {
          t16_st4(a.dres + row * CH + 4 * q, make_float4(dz[0], dz[1], dz[2], dz[3]));
          t16_st4(a.dh_out + row * CH + 4 * q, make_float4(v[i][0], v[i][1], v[i][2], v[i][3]));
        }
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) v[i][c] = 0.0f;
      }
    }
    __bf16* img = imgs + (long)sl * imgb + 4 * k;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      bf16x4s o;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = (__bf16)v[i][c];
      *(bf16x4s*)(img + (4 * q + c) * s16) = o;
    }
  }
}

// A phase's dh images (slices s0 .. s0 + nsl - 1, imgf floats apart): dh itself, or with the
// BatchNorm-backward prologue dz = gamma*rstd*(dy - k1 - xhat*k2), dh = dropout'(dz), dres / dh_out
// written for the workgroup's own rows (its tiles [rg.tb, rg.te)).  Whole phase in rounds of U
// float4 per thread (stage_rows4's pattern: every load of a round before its first store); mid()
// with round 0's loads in flight.
// BF: the images are the bf16 channel-major ones of the bf16 forward ([32][s16], rows = s16 - 8)
template <bool BF, typename Mid>
__device__ __forceinline__ void t16_bwd_stage(const FusedBwd& a, float* imgs, int imgf, int s0, int nsl,
                                              const T16Range& rg, int nt, int n, int rows, Mid mid) {
  if (!a.bn_dy) {
    if (BF) stage_bf16_octets(a.dh + (long)s0 * n * CH, CH, n, rows + 8, nsl, (__bf16*)imgs, 2 * imgf, mid);
    else
      stage_rows4<8>(a.dh + (long)s0 * n * CH, CH, n, rows, nsl,
                     [&](int sl, int w, int q, float4 x) { t16_bwd_put<BF>(imgs + sl * imgf, rows, w, q, x); }, mid);
    return;
  }
  if (BF) {
    t16_bwd_stage_bn_bf16(a, (__bf16*)imgs, 2 * imgf, s0, nsl, rg, nt, n, rows + 8, mid);
    return;
  }
  constexpr int U = 4;
  const unsigned long long seed = a.seed_ptr ? *a.seed_ptr : 0ull;
  const float keep_scale = (a.drop_p > 0.0f) ? 1.0f / (1.0f - a.drop_p) : 1.0f;
  const int q = threadIdx.x & 7;  // blockDim % 8 == 0: every element of a thread has channel quad q
  float mu[4], rs[4], gm[4], k1[4], k2[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = 4 * q + e;
    mu[e] = a.bn_mean[c]; rs[e] = a.bn_rstd[c]; gm[e] = a.bn_gamma[c];
    k1[e] = a.bn_sums[c] * a.inv_rows; k2[e] = a.bn_sums[CH + c] * a.inv_rows;
  }
  const long base = (long)s0 * n * CH;  // first element of the phase
  const int bytes = (int)((long)nsl * n * CH * 4);
  const __amdgpu_buffer_rsrc_t rdy = __builtin_amdgcn_make_buffer_rsrc((void*)(a.bn_dy + base), (short)0, bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc((void*)(a.bn_z + base), (short)0, bytes, 0x00020000);
  const int per = rows * 8, total = nsl * per;
  bool first = true;
  for (int e0 = threadIdx.x; e0 < total || first; e0 += U * (int)blockDim.x) {
    float4 dy[U], zv[U];
#pragma unroll
    for (int i = 0; i < U; ++i) {
      const int e = e0 + i * (int)blockDim.x;
      const int sl = e / per, w = (e - sl * per) >> 3;
      const int off = (e < total && w < n) ? ((sl * n + w) * CH + 4 * q) * 4 : 0x7ffffff0;
      dy[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rdy, off, 0, 0));
      zv[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rz, off, 0, 0));
    }
    if (first) {
      mid();
      first = false;
    }
#pragma unroll
    for (int i = 0; i < U; ++i) {
      const int e = e0 + i * (int)blockDim.x;
      if (e >= total) break;
      const int sl = e / per, w = (e - sl * per) >> 3;
      float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if (w < n) {
        const long row = (long)(s0 + sl) * n + w;
        const float dyv[4] = {dy[i].x, dy[i].y, dy[i].z, dy[i].w}, zz[4] = {zv[i].x, zv[i].y, zv[i].z, zv[i].w};
        float dz[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float xhat = (zz[c] - mu[c]) * rs[c];
          dz[c] = gm[c] * rs[c] * (dyv[c] - k1[c] - xhat * k2[c]);
          v[c] = dz[c];
          if (a.drop_p > 0.0f) {
            const float u = gwn_uniform(seed, a.salt, (unsigned long long)(row * CH + 4 * q + c));
            v[c] = (u >= a.drop_p) ? v[c] * keep_scale : 0.0f;
          }
        }
        // this workgroup's rows of the slice: its tiles of it
        const long sb = (long)(s0 + sl) * nt;
        const long t0 = max(rg.tb - sb, 0l), t1 = min(rg.te - sb, (long)nt);
        if (w >= 16 * t0 && w < 16 * t1) {
          t16_st4(a.dres + row * CH + 4 * q, make_float4(dz[0], dz[1], dz[2], dz[3]));
          t16_st4(a.dh_out + row * CH + 4 * q, make_float4(v[0], v[1], v[2], v[3]));
        }
      }
      t16_bwd_put<BF>(imgs + sl * imgf, rows, w, q, make_float4(v[0], v[1], v[2], v[3]));
    }
  }
}

// rows of a [rows][ld] output from the t16 accumulator layout (lane: node w0 + j, channels
// 16 oh + 4 g .. + 3)
__device__ __forceinline__ void t16_store(float* out, long ld, const f32x4v* acc, int w0, int lane, int n) {
  const int g = lane >> 4, j = lane & 15;
  if (w0 + j >= n) return;
  float* p = out + (long)(w0 + j) * ld + 4 * g;
#pragma unroll
  for (int oh = 0; oh < 2; ++oh) t16_st4(p + 16 * oh, make_float4(acc[oh][0], acc[oh][1], acc[oh][2], acc[oh][3]));
}

// the tile epilogue's gate backward for node row m (lane group g: channels 16 oh + 4 g .. + 3):
// dfg = (g sigma (1 - f^2), g f sigma (1 - sigma)) with g = dx (+ dskip) and the saved (tanh f,
// sigmoid sigma) pairs.  Both channel halves' fg / dskip rows are requested before the first
// use: one memory round trip per tile instead of two.
__device__ __forceinline__ void t16_gate_bwd(const FusedBwd& a, const f32x4v* dx, long m, int g) {
  const bool sk = a.dskip && m >= a.skip_row0;
  float4 f0[2], f1[2], dq[2];
#pragma unroll
  for (int oh = 0; oh < 2; ++oh) {
    const int c0 = 16 * oh + 4 * g;
    f0[oh] = *(const float4*)(a.fg + m * 2 * CH + 2 * c0);
    f1[oh] = *(const float4*)(a.fg + m * 2 * CH + 2 * c0 + 4);
    dq[oh] = sk ? *(const float4*)(a.dskip + (m - a.skip_row0) * a.ld_dskip + c0) : make_float4(0, 0, 0, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int oh = 0; oh < 2; ++oh) {
    const int c0 = 16 * oh + 4 * g;
    const float fv[8] = {f0[oh].x, f0[oh].y, f0[oh].z, f0[oh].w, f1[oh].x, f1[oh].y, f1[oh].z, f1[oh].w};
    const float dv[4] = {dq[oh].x, dq[oh].y, dq[oh].z, dq[oh].w};
    float o[8];
#pragma unroll
    for (int e2 = 0; e2 < 4; ++e2) {
      const float gv = dx[oh][e2] + dv[e2];
      const float f = fv[2 * e2], sg = fv[2 * e2 + 1];
      o[2 * e2] = gv * sg * (1.0f - f * f);
      o[2 * e2 + 1] = gv * f * sg * (1.0f - sg);
    }
    t16_st4(a.dfg + m * 2 * CH + 2 * c0, make_float4(o[0], o[1], o[2], o[3]));
    t16_st4(a.dfg + m * 2 * CH + 2 * c0 + 4, make_float4(o[4], o[5], o[6], o[7]));
  }
}

// BF: bf16 operands in the diffusion (the bf16 forward's image / support layouts: sup_g4b_t), the
// tile's fp32 dh rows for the channel maps of piece 0 and t1 / t2 read back from dh_out (written by
// this workgroup's prologue for its own rows) or dh
template <int MAXT, bool BF, bool MLPB = false>
__global__ __launch_bounds__(MAXT) void gcn_bwd_t16_kernel(const FusedBwd a, const PowSup p, const int maximg) {
  extern __shared__ float lds[];
  const int n = a.n;
  const int nt = (n + 15) >> 4;
  const int rows_img = BF ? t16b_s16(n) - 8 : t16_img_rows(n), hs = rows_img * 16;
  const int imgf = BF ? CH * t16b_s16(n) / 2 : rows_img * CH;  // floats per image
  float* ws = lds;
  float* imgs = ws + (2 * a.nsup + 1) * CH * LDW16 + T16_WAVES * 3 * CH;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  const int nwaves = blockDim.x >> 6;
  auto mlp = [&](int piece, const f32x4v* x, f32x4v* out) {
    if (MLPB) t16_mlp_b((const __bf16*)ws, piece, x, lane, out);
    else t16_mlp(ws + piece * CH * LDW16, LDW16, x, lane, out);
  };
  const T16Range rg = t16_range(a.slices, nt);
  if (a.bn_dy && blockIdx.x == 0 && threadIdx.x < CH) {
    if (a.bn_dbeta) a.bn_dbeta[threadIdx.x] = a.bn_sums[threadIdx.x];
    if (a.bn_dgamma) a.bn_dgamma[threadIdx.x] = a.bn_sums[CH + threadIdx.x];
  }
  for (long p0 = rg.tb; p0 < rg.te;) {
    const int s0 = (int)(p0 / nt);
    const long p1 = min(rg.te, (long)(s0 + maximg) * nt);
    const int s1 = (int)((p1 - 1) / nt);
    if (p0 != rg.tb) __syncthreads();
    // the phase's dh images in one pass, the channel maps inside its first round trip
    const bool maps = p0 == rg.tb;
    t16_bwd_stage<BF>(a, imgs, imgf, s0, s1 - s0 + 1, rg, nt, n, rows_img, [&] {
      if (maps) {
        if (MLPB) t16_stage_maps_bf16(a.w_mlp, a.ld_w, true, 2 * a.nsup + 1, (__bf16*)ws);
        else t16_stage_maps(a.w_mlp, a.ld_w, true, 2 * a.nsup + 1, ws);
      }
    });
    __syncthreads();
    const int span = (int)(p1 - p0);
    for (int tp = wave; tp < span; tp += nwaves) {
      const long t = p0 + tp;
      const int s = (int)(t / nt), tile = (int)(t - (long)s * nt);
      const float* dhs = imgs + (s - s0) * imgf;
      const long row0 = (long)s * n;
      const int w0 = 16 * tile;
      f32x4v dx[2];
      dx[0] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
      dx[1] = dx[0];
      const float* dh_rows = (a.bn_dy ? a.dh_out : a.dh) + row0 * CH;  // (BF: the fp32 rows)
      // MLPB: the channel maps take bf16(dh), which is the staged image itself
      const int s16b = t16b_s16(n);
      if (MLPB) {
        t16_mlp_bp((const __bf16*)ws, 0, t16_img_col_b((const __bf16*)dhs, s16b, w0, lane), lane, dx);
      } else {
        f32x4v d0[2];
        if (BF) t16_rows_global(dh_rows, CH, w0, n, lane, d0);
        else t16_rows(dhs, hs, w0, lane, d0);
        mlp(0, d0, dx);
      }
      for (int k = 0; k < a.nsup; ++k) {
        f32x4v e[2][2];
        if (BF) t16b_diffuse((const __bf16*)dhs, (const __bf16*)p.g4[2 * k], (const __bf16*)p.g4[2 * k + 1], n, tile, lane, e);
        else t16_diffuse(dhs, hs, p.g4[2 * k], p.g4[2 * k + 1], n, tile, lane, e);
        mlp(1 + 2 * k, e[0], dx);
        mlp(2 + 2 * k, e[1], dx);
        if (k == a.adp_index) {  // t1 = W1^T dh + W2^T (A dh), t2 = W2^T dh
          f32x4v d0[2], tt[2];
          bf16x8m db;
          if (MLPB) db = t16_img_col_b((const __bf16*)dhs, s16b, w0, lane);
          else if (BF) t16_rows_global(dh_rows, CH, w0, n, lane, d0);
          else t16_rows(dhs, hs, w0, lane, d0);
          tt[0] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
          tt[1] = tt[0];
          if (MLPB) t16_mlp_bp((const __bf16*)ws, 1 + 2 * k, db, lane, tt);
          else mlp(1 + 2 * k, d0, tt);
          mlp(2 + 2 * k, e[0], tt);
          if (BF && a.tg4) t16_store_g4(a.tg4, 0, a.slices, s, nt, tile, lane, tt);
          else t16_store(a.t1 + row0 * a.ld_t, a.ld_t, tt, w0, lane, n);
          tt[0] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
          tt[1] = tt[0];
          if (MLPB) t16_mlp_bp((const __bf16*)ws, 2 + 2 * k, db, lane, tt);
          else mlp(2 + 2 * k, d0, tt);
          if (BF && a.tg4) t16_store_g4(a.tg4, 1, a.slices, s, nt, tile, lane, tt);
          else t16_store(a.t2 + row0 * a.ld_t, a.ld_t, tt, w0, lane, n);
        }
      }
      if (!a.dfg) {
        t16_store(a.dxg + row0 * a.ld_dxg, a.ld_dxg, dx, w0, lane, n);
        continue;
      }
      // gate backward (gate_bwd_kernel's arithmetic): g = dxg (+ dskip) -> dfg via (tanh f, sigmoid s)
      const int w = w0 + j;
      if (w >= n) continue;
      t16_gate_bwd(a, dx, row0 + w, g);
    }
    p0 = p1;
  }
}

// Two slices per wave in the bf16-mlp backward (gcn_fwd_t16b2_kernel's unit: slice pair 2q, 2q + 1
// x node tile): each transposed-support fragment feeds both slices' diffusion MFMAs and each
// channel-map fragment both mlps (W^T after diffusion, t1 / t2 of the adaptive support); the
// BN-backward prologue stages the pairs' dh images (dres / dh_out for the workgroup's own pair
// tiles), the epilogue is the gate backward (or the dxg store) of each slice.  12-wave workgroups
// (the forward pair kernel's register budget).  An odd last slice: B diffuses A's image and stores
// nothing.
template <int MAXT>
__global__ __launch_bounds__(MAXT) void gcn_bwd_t16b2_kernel(const FusedBwd a, const PowSup p, const int maximg) {
  extern __shared__ float lds[];
  const int n = a.n;
  const int nt = (n + 15) >> 4;
  const int s16 = t16b_s16(n), imgb = CH * s16;  // bf16 elements per image
  float* ws = lds;
  __bf16* imgs = (__bf16*)(ws + (2 * a.nsup + 1) * CH * LDW16 + T16_WAVES * 3 * CH);
  const __bf16* maps = (const __bf16*)ws;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  const int nwaves = blockDim.x >> 6;
  const int pairs = (a.slices + 1) / 2;
  const T16Range rg = t16_range(pairs, nt);
  if (a.bn_dy && blockIdx.x == 0 && threadIdx.x < CH) {
    if (a.bn_dbeta) a.bn_dbeta[threadIdx.x] = a.bn_sums[threadIdx.x];
    if (a.bn_dgamma) a.bn_dgamma[threadIdx.x] = a.bn_sums[CH + threadIdx.x];
  }
  for (long p0 = rg.tb; p0 < rg.te;) {
    const int q0 = (int)(p0 / nt);
    const long p1 = min(rg.te, (long)(q0 + maximg / 2) * nt);
    const int q1 = (int)((p1 - 1) / nt);
    const int s0 = 2 * q0, s1 = min(2 * q1 + 2, a.slices) - 1;
    if (p0 != rg.tb) __syncthreads();
    const bool first = p0 == rg.tb;
    auto mid = [&] {
      if (first) t16_stage_maps_bf16(a.w_mlp, a.ld_w, true, 2 * a.nsup + 1, (__bf16*)ws);
    };
    if (a.bn_dy) t16_bwd_stage_bn_bf16(a, imgs, imgb, s0, s1 - s0 + 1, rg, nt, n, s16, mid, 1);
    else stage_bf16_octets(a.dh + (long)s0 * n * CH, CH, n, s16, s1 - s0 + 1, imgs, imgb, mid);
    __syncthreads();
    const int span = (int)(p1 - p0);
    for (int tp = wave; tp < span; tp += nwaves) {
      const long t = p0 + tp;
      const int q = (int)(t / nt), tile = (int)(t - (long)q * nt);
      const int sA = 2 * q, sB = 2 * q + 1;
      const bool okB = sB < a.slices;
      const __bf16* xsA = imgs + (sA - s0) * imgb;
      const __bf16* xsB = okB ? imgs + (sB - s0) * imgb : xsA;
      const int w0 = 16 * tile;
      f32x4v dxA[2], dxB[2];
      dxA[0] = dxA[1] = dxB[0] = dxB[1] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
      // the channel maps take bf16(dh): the staged images' node columns
      const bf16x8m dbA = t16_img_col_b(xsA, s16, w0, lane), dbB = t16_img_col_b(xsB, s16, w0, lane);
      t16_mlp_bp2(maps, 0, dbA, dbB, lane, dxA, dxB);
      for (int k = 0; k < a.nsup; ++k) {
        f32x4v eA[2][2], eB[2][2];
        t16b_diffuse2(xsA, xsB, (const __bf16*)p.g4[2 * k], (const __bf16*)p.g4[2 * k + 1], n, tile, lane, eA, eB);
        const bf16x8m e1A = t16_pack_b(eA[0]), e1B = t16_pack_b(eB[0]);
        t16_mlp_bp2(maps, 1 + 2 * k, e1A, e1B, lane, dxA, dxB);
        t16_mlp_bp2(maps, 2 + 2 * k, t16_pack_b(eA[1]), t16_pack_b(eB[1]), lane, dxA, dxB);
        if (k == a.adp_index) {  // t1 = W1^T dh + W2^T (A dh), t2 = W2^T dh
          f32x4v tA[2], tB[2];
          tA[0] = tA[1] = tB[0] = tB[1] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
          t16_mlp_bp2(maps, 1 + 2 * k, dbA, dbB, lane, tA, tB);
          t16_mlp_bp2(maps, 2 + 2 * k, e1A, e1B, lane, tA, tB);
          if (a.tg4) {
            t16_store_g4(a.tg4, 0, a.slices, sA, nt, tile, lane, tA);
            if (okB) t16_store_g4(a.tg4, 0, a.slices, sB, nt, tile, lane, tB);
          } else {
            t16_store(a.t1 + (long)sA * n * a.ld_t, a.ld_t, tA, w0, lane, n);
            if (okB) t16_store(a.t1 + (long)sB * n * a.ld_t, a.ld_t, tB, w0, lane, n);
          }
          tA[0] = tA[1] = tB[0] = tB[1] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
          t16_mlp_bp2(maps, 2 + 2 * k, dbA, dbB, lane, tA, tB);
          if (a.tg4) {
            t16_store_g4(a.tg4, 1, a.slices, sA, nt, tile, lane, tA);
            if (okB) t16_store_g4(a.tg4, 1, a.slices, sB, nt, tile, lane, tB);
          } else {
            t16_store(a.t2 + (long)sA * n * a.ld_t, a.ld_t, tA, w0, lane, n);
            if (okB) t16_store(a.t2 + (long)sB * n * a.ld_t, a.ld_t, tB, w0, lane, n);
          }
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h == 1 && !okB) break;
        const long row0 = (long)(h ? sB : sA) * n;
        const f32x4v* dx = h ? dxB : dxA;
        if (!a.dfg) {
          t16_store(a.dxg + row0 * a.ld_dxg, a.ld_dxg, dx, w0, lane, n);
          continue;
        }
        // gate backward (gate_bwd_kernel's arithmetic): g = dxg (+ dskip) -> dfg via (tanh f, sigmoid s)
        const int w = w0 + j;
        if (w >= n) continue;
        t16_gate_bwd(a, dx, row0 + w, g);
      }
    }
    p0 = p1;
  }
}

// Support split policy.  Measured per layer (round 2, n = 207, B = 64, 256 CUs; fwd / bwd us,
// whole slices -> split): a unit costs about half a slice, not a third (it still stages the whole
// slice in LDS, hands off its partial sum and one of three runs the epilogue), so the split only pays
// where the whole-slice launch leaves most CUs idle: 64 slices 63.5 -> 37.8 (fwd); 192 slices
// 68 -> 78 / 67 -> 79; 448 slices 115 -> 147 / 111 -> 148; 640 slices 174 -> 212 / 167 -> 201.
// Split when every unit gets a CU of its own (slices * nsup <= CUs).
int ksplit_max_slices(int nsup) {
  static int v = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 0;
    return -cus;  // negative: a CU count, divided by nsup below
  }();
  return v >= 0 ? v : (-v) / nsup;
}

template <typename G>
int pick_ksplit(const G* g, int slices, int nwt) {
  if (!g->ksplit_ws || !g->ksplit_count || g->nsup < 2 || g->ksplit == 1 || g->sup_batch > 1 || nwt > 15)
    return 1;
  if (g->ksplit == g->nsup) return g->nsup;
  return slices <= ksplit_max_slices(g->nsup) ? g->nsup : 1;
}

}  // namespace


bool gwn_gcn_fused_eligible(int c, int n, int nsup, int ld_sup) {
  return c == CH && n > 0 && n <= 512 && nsup >= 0 && nsup <= 8 && ld_sup >= (n + 31) / 32 * 32;
}


// the 16-node tile kernels (GWN_GCN_T16=0 selects the 32-node tile power kernels)
constexpr int T16_LDS_MAX = 160 * 1024 - 1024;  // dynamic LDS of a t16 workgroup

static bool t16_enabled() {
  const char* e = getenv("GWN_GCN_T16");  // read per launch (tests switch it within one process)
  return !(e && e[0] == '0');
}

extern "C" int gwn_wall_clock_khz(void) {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess)
    return 0;
  return khz;
}

int gwn_device_cus() {
  static int v = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    return cus;
  }();
  return v;
}

long gwn_bn_part_slots(int slices) { return slices > gwn_device_cus() ? slices : gwn_device_cus(); }

namespace {

// Launch plan of the t16 kernels: one 16-wave workgroup per CU (at most one per tile), each over an
// equal contiguous range of the launch's tiles; the LDS holds the channel maps, the waves' BN
// partials and maximg slice images (as many as a range can touch, at most T16_MAXIMG and what
// fits), and never less than half a CU's LDS so that no two of them share a CU.
struct T16Plan {
  bool ok;
  int grid, maximg;
  size_t lds;
};
T16Plan t16_plan(int n, int nsup, int slices, bool tcn = false) {
  T16Plan pl{false, 0, 0, 0};
  const size_t fixed = t16_lds_bytes(n, nsup, 0, tcn), img = t16_lds_bytes(n, nsup, 1, tcn) - fixed;
  if (fixed + img > (size_t)T16_LDS_MAX || slices <= 0) return pl;
  const int nt = (n + 15) / 16;
  const long tiles = (long)slices * nt;
  pl.grid = (int)(tiles < gwn_device_cus() ? tiles : gwn_device_cus());
  const long per = (tiles + pl.grid - 1) / pl.grid;
  const int span = (int)((per - 1 + nt - 1) / nt) + 1;  // slices a range of `per` tiles can touch
  int maximg = (int)((T16_LDS_MAX - fixed) / img);
  maximg = maximg < T16_MAXIMG ? maximg : T16_MAXIMG;
  pl.maximg = maximg < span ? maximg : span;
  pl.lds = fixed + pl.maximg * img;
  if (pl.lds < 81 * 1024) pl.lds = 81 * 1024;
  pl.ok = true;
  return pl;
}
}  // namespace

// gwn_gcn_args.tcn runs inside the f32 16-node tile forward (else gwn_gcn_fwd issues it as its own
// launch first): c = 32, two taps, c_out = 32, xg = h's piece 0, 16-B aligned operands, the launch
// would take that kernel (with the TCN's LDS region), and it has at least a slice per CU: every
// workgroup computes the TCN of all the slices its tile range touches, so with less than a slice
// per CU most of that work is redundant (METR: the layers of 192 and 64 slices ran 4 and 1 us
// slower fused, those of >= 256 slices 2-6 us faster; step 25.04k -> 25.26k samples/s same-box,
// profiles/r05/tcn_fused)
// the in-kernel finalize's merge: 32 channels x (blockDim / 32) slot lanes, exchanged through the
// image space before the first phase is staged
constexpr size_t T16_BN_SCRATCH = 3 * (64 * T16_WAVES / 32) * CH * sizeof(double);
static bool bn_scratch_ok(int n, int nsup, int slices) {
  const T16Plan pl = t16_plan(n, nsup, slices, true);
  return pl.ok && pl.lds >= t16_lds_bytes(n, nsup, 0, true) + T16_BN_SCRATCH;
}
bool gwn_gcn_tcn_fusable(const gwn_gcn_args* g) {
  const gwn_tcn_args* t = g->tcn;
  if (!t) return false;
  auto al = [](const void* q) { return (((uintptr_t)q) & 15) == 0; };
  const int slices = g->rows / g->n, nwt = (g->n + 31) / 32;
  // (t16_tcn_load addresses the input rows with 32-bit byte offsets of one buffer resource)
  return t->c == CH && (t->ntaps == 0 || t->ntaps == 2) && (t->c_out == 0 || t->c_out == CH) &&
         (long long)t->t_in * t->P * CH * 4 < 0x7fff0000LL &&
         t->xg == g->h && t->ld_xg == g->ld_h && (long)(t->t_in - t->dilation) * t->P == g->rows && t->dilation > 0 &&
         al(t->x) && t->w_fg && t->b_fg && (!t->fg || al(t->fg)) &&
         (!t->skipcat || (al(t->skipcat) && (t->ld_skip & 3) == 0)) && g->c == CH &&
         (g->c_out == 0 || g->c_out == CH) && gwn_gcn_fused_eligible(g->c, g->n, g->nsup, g->ld_sup) &&
         al(g->h) && (g->ld_h & 3) == 0 && g->split_planes == 0 && g->sup_g4 && g->sup_batch <= 1 && g->nsup > 0 &&
         g->layout == 0 && t16_enabled() && (pick_ksplit(g, slices, nwt) <= 1 || g->ksplit != g->nsup) &&
         slices >= gwn_device_cus() && t16_plan(g->n, g->nsup, slices, true).ok &&
         (!t->bn || (t->bn_partials && t->bn_nparts > 0 && t->bn->w_next && t->bn->b_next && t->bn->w_fold &&
                     t->bn->b_fold && t->bn->gamma && t->bn->beta && t->bn->save_mean && t->bn->save_rstd &&
                     t->bn->scale && bn_scratch_ok(g->n, g->nsup, slices) &&
                     (!g->residual_mean || (g->residual_mean == t->bn->save_mean && g->residual_scale == t->bn->scale))));
}

extern "C" int gwn_gcn_tcn_fused(const gwn_gcn_args* a) { return a && a->tcn && gwn_gcn_tcn_fusable(a) ? 1 : 0; }

int gwn_gcn_fused_fwd_launch(const gwn_gcn_args* g, float* bn_part, hipStream_t s, int* used) {
  const int nwt = (g->n + 31) / 32;
  GWN_REQUIRE(g->ld_sup >= nwt * 32, "gcn_fwd (fused): supports must be padded to 32*ceil(n/32)");
  GWN_REQUIRE(g->layout == 0 || g->layout == 1, "gcn_fwd (fused): layout must be 0 or 1 (one wave per node tile)");
  FusedFwd a;
  a.h = g->h; a.ld_h = g->ld_h;
  for (int k = 0; k < 8; ++k) a.sup[k] = (k < g->nsup) ? g->sup[k] : nullptr;
  a.nsup = g->nsup; a.ld_sup = g->ld_sup;
  a.w_mlp = g->w_mlp; a.ld_w = (2 * g->nsup + 1) * CH; a.b_mlp = g->b_mlp; a.w_t = g->w_mlp_t;
  a.residual = g->residual; a.z = g->z; a.bn_part = bn_part;
  a.seed_ptr = g->seed_ptr; a.salt = g->salt; a.drop_p = g->drop_p;
  a.n = g->n;
  a.store_pieces = g->no_pieces ? 0 : 1;
  a.bn_rm = g->bn_running_mean; a.bn_rv = g->bn_running_var; a.bn_g = g->bn_weight; a.bn_b = g->bn_bias;
  a.bn_eps = g->bn_eps; a.x_out = g->bn_out;
  a.sup_bstride = g->sup_bstride; a.sup_batch = g->sup_batch;
  a.res_mean = g->residual_mean; a.res_scale = g->residual_scale; a.res_shift = g->residual_shift;
  a.ksplit = 1; a.slices = g->rows / g->n; a.kws = g->ksplit_ws; a.kcnt = g->ksplit_count; a.bn_slots = 0;
  a.xg4 = g->xg4; a.xg4_k = g->xg4_support;
  a.pb = g->pieces_bf16; a.ld_pb = g->ld_pb;
  a.tcn = {};
  a.clk = g->clock;
  GWN_REQUIRE(g->ksplit == 0 || g->ksplit == 1 || g->ksplit == g->nsup, "gcn_fwd: ksplit must be 0, 1 or nsup");
  GWN_REQUIRE(!a.res_scale == !a.res_shift && !a.res_scale == !a.res_mean,
              "gcn_fwd (fused): residual_mean, residual_scale and residual_shift go together");
  if (a.sup_batch > 1)
    GWN_REQUIRE(!g->split_planes && (g->rows / g->n) % a.sup_batch == 0,
                "gcn_fwd (per-sample supports): slices must be a multiple of sup_batch, no split path");
  if (a.x_out)
    GWN_REQUIRE(a.bn_rm && a.bn_rv && a.bn_g && a.bn_b && !bn_part,
                "gcn_fwd (fused): eval BatchNorm needs running mean / var, weight, bias (and no BN partials)");
  else
    GWN_REQUIRE(a.z != nullptr, "gcn_fwd (fused): z is required");
  GWN_REQUIRE(g->split_planes >= 0 && g->split_planes <= 2, "gcn_fwd: split_planes must be a gwn_dtype (0, 1, 2)");
  if (g->split_planes >= 1 && g->sup_g4b && a.sup_batch <= 1 && g->nsup > 0 && g->layout == 0 && t16_enabled() &&
      g->ksplit != g->nsup) {
    const int slices = g->rows / g->n;
    const size_t fixed = t16b_lds_bytes(g->n, g->nsup, 0), img = t16b_lds_bytes(g->n, g->nsup, 1) - fixed;
    if (fixed + img <= (size_t)T16_LDS_MAX) {
      GWN_REQUIRE(g->w_mlp_t, "gcn_fwd (16-node tiles, bf16): w_mlp_t is required with sup_g4b");
      GWN_REQUIRE(!g->pieces_bf16 || (g->ld_pb >= 2L * g->nsup * CH && g->ld_pb % 4 == 0 &&
                                      ((uintptr_t)g->pieces_bf16 & 7) == 0),
                  "gcn_fwd (bf16 pieces): ld_pb >= 2*nsup*c, a multiple of 4, 8-B aligned pieces_bf16");
      static bool attr_b = false;
      if (!attr_b) {
        (void)hipFuncSetAttribute((const void*)gcn_fwd_t16b_kernel<1024>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  T16_LDS_MAX);
        (void)hipFuncSetAttribute((const void*)gcn_fwd_t16b_kernel<1024, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, T16_LDS_MAX);
        attr_b = true;
      }
      const int nt = (g->n + 15) / 16;
      const long tiles = (long)slices * nt;
      const int grid = (int)(tiles < gwn_device_cus() ? tiles : gwn_device_cus());
      const long per = (tiles + grid - 1) / grid;
      int maximg = (int)((T16_LDS_MAX - fixed) / img);
      maximg = maximg < T16_MAXIMG ? maximg : T16_MAXIMG;
      const int span = (int)((per - 1 + nt - 1) / nt) + 1;
      maximg = maximg < span ? maximg : span;
      size_t lds = fixed + maximg * img;
      if (lds < 81 * 1024) lds = 81 * 1024;
      PowSup p = {};
      for (int k = 0; k < 2 * g->nsup; ++k) p.g4[k] = (const float*)g->sup_g4b[k];
      a.ksplit = 1;
      a.bn_slots = (int)gwn_bn_part_slots(slices);
      // the bf16-mlp forward takes two slices per wave (12-wave workgroups, 168 registers): PEMS
      // forward 63 -> 58 us per launch, 25.8k -> 26.4k samples/s (profiles/r05/welford_hash); with
      // 16 waves it spills (76 us)
      const int slices2 = (slices + 1) / 2;
      const long units2 = (long)slices2 * nt;
      const int grid2 = (int)(units2 < gwn_device_cus() ? units2 : gwn_device_cus());
      const long per2 = (units2 + grid2 - 1) / grid2;
      int gmax2 = (int)((T16_LDS_MAX - fixed) / (2 * img));
      gmax2 = gmax2 < T16_MAXIMG / 2 ? gmax2 : T16_MAXIMG / 2;
      const int span2 = (int)((per2 - 1 + nt - 1) / nt) + 1;
      const int maximg2 = 2 * (gmax2 < span2 ? gmax2 : span2);
      const bool h16 = ((((uintptr_t)a.h) & 15) | (a.ld_h & 3)) == 0;
      // (pairs from ~10 units per CU, as the backward: PEMS' 64-slice layer ran 25.2 us paired
      // against 23.6 us with single slices)
      if (g->split_planes == 2 && gmax2 >= 1 && h16 && units2 >= 10L * grid2) {
        static bool attr2 = false;
        if (!attr2) {
          (void)hipFuncSetAttribute((const void*)gcn_fwd_t16b2_kernel<768>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    T16_LDS_MAX);
          attr2 = true;
        }
        size_t lds2 = fixed + maximg2 * img;
        if (lds2 < 81 * 1024) lds2 = 81 * 1024;
        gcn_fwd_t16b2_kernel<768><<<grid2, 768, lds2, s>>>(a, p, maximg2);
        if (used) *used = grid2;
      } else {
        if (g->split_planes == 2) gcn_fwd_t16b_kernel<1024, true><<<grid, 64 * T16_WAVES, lds, s>>>(a, p, maximg);
        else gcn_fwd_t16b_kernel<1024><<<grid, 64 * T16_WAVES, lds, s>>>(a, p, maximg);
        if (used) *used = grid;
      }
      GWN_CHECK_LAUNCH();
      return GWN_OK;
    }
  }
  GWN_REQUIRE(!g->xg4 && !g->pieces_bf16,
              "gcn_fwd: xg4 / pieces_bf16 are written by the bf16 16-node tile kernel only (sup_g4b, layout 0)");
  GWN_REQUIRE(!g->split_planes,
              "gcn_fwd: bf16 operands (split_planes 1) run on the 16-node tile kernel only: sup_g4b, layout 0, shared "
              "supports, no forced support split, gwn_gcn_t16b_supported(n, nsup)");
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gcn_fwd_t16_kernel<1024>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              T16_LDS_MAX);
    attr_set = true;
  }
  const int slices = g->rows / g->n;
  a.ksplit = pick_ksplit(g, slices, nwt);
  const int grid = a.ksplit > 1 ? (slices + 7) / 8 * 8 * a.ksplit : slices;
  const bool tcn = g->tcn != nullptr;
  GWN_REQUIRE(!tcn || gwn_gcn_tcn_fusable(g), "gcn_fwd (fused): tcn given where it cannot be fused");
  const T16Plan pl = t16_plan(g->n, g->nsup, slices, tcn);
  // (the t16 ranges already cut small launches finely: the support split runs only when forced)
  if (g->sup_g4 && a.sup_batch <= 1 && g->nsup > 0 && (a.ksplit <= 1 || g->ksplit != g->nsup) && g->layout == 0 &&
      t16_enabled() && pl.ok) {
    GWN_REQUIRE(g->w_mlp_t, "gcn_fwd (16-node tiles): w_mlp_t (the transposed mlp weights) is required with sup_g4");
    if (tcn) {
      const gwn_tcn_args* t = g->tcn;
      a.tcn.x = t->x; a.tcn.mean = t->x_mean; a.tcn.w = t->w_fg; a.tcn.b = t->b_fg; a.tcn.fg = t->fg;
      a.tcn.skip = t->skipcat; a.tcn.ld_skip = t->ld_skip; a.tcn.skip_row0 = t->skip_row0;
      a.tcn.tap_rows = (long)t->dilation * t->P; a.tcn.x_rows = (long)t->t_in * t->P;
      if (t->bn) {  // the layer below's BatchNorm finalized in the launch (raw weights folded there)
        const gwn_bn_fold* f = t->bn;
        a.tcn.mean = nullptr; a.tcn.w = f->w_next; a.tcn.b = f->b_next;
        a.tcn.bn = {t->bn_partials, t->bn_nparts, f->gamma, f->beta, f->running_mean, f->running_var, f->momentum,
                    f->eps, f->save_mean, f->save_rstd, f->scale, f->w_fold, f->b_fold, f->num_batches_tracked};
      }
    }
    PowSup p = {};
    for (int k = 0; k < 2 * g->nsup; ++k) p.g4[k] = g->sup_g4[k];
    a.ksplit = 1;
    // 16-node tile waves, one workgroup per CU over an equal tile range; it writes every BN
    // partial slot (gwn_bn_part_slots)
    a.bn_slots = (int)gwn_bn_part_slots(slices);
    gcn_fwd_t16_kernel<1024><<<pl.grid, 64 * T16_WAVES, pl.lds, s>>>(a, p, pl.maximg);
    if (used) *used = pl.grid;
    GWN_CHECK_LAUNCH();
    return GWN_OK;
  }
  return slice_fwd_launch(g, a, bn_part, grid, s);  // the whole-slice schedules (gcn_slice.hip)
}

int gwn_gcn_fused_bwd_launch(const gwn_gcn_bwd_args* g, const float* const* supT, float* dxg, long ld_dxg,
                             float* t1, float* t2, long ld_t, hipStream_t s) {
  const int nwt = (g->n + 31) / 32;
  GWN_REQUIRE(g->ld_sup >= nwt * 32, "gcn_bwd (fused): supports must be padded to 32*ceil(n/32)");
  GWN_REQUIRE(g->layout == 0 || g->layout == 1, "gcn_bwd (fused): layout must be 0 or 1 (one wave per node tile)");
  FusedBwd a;
  a.dh = g->dh;
  for (int k = 0; k < 8; ++k) a.supT[k] = (k < g->nsup) ? supT[k] : nullptr;
  a.nsup = g->nsup; a.ld_sup = g->ld_sup;
  a.w_mlp = g->w_mlp; a.ld_w = (2 * g->nsup + 1) * CH;
  a.dxg = dxg; a.ld_dxg = ld_dxg;
  a.t1 = t1; a.t2 = t2; a.ld_t = ld_t; a.adp_index = g->adp_index;
  a.n = g->n;
  a.bn_dy = g->bn_dy; a.bn_z = g->bn_z; a.bn_gamma = g->bn_gamma; a.bn_mean = g->bn_mean;
  a.bn_rstd = g->bn_rstd; a.bn_sums = g->bn_sums; a.bn_dgamma = g->bn_dgamma; a.bn_dbeta = g->bn_dbeta;
  a.dres = g->dres; a.dh_out = g->dh_out;
  a.seed_ptr = g->seed_ptr; a.salt = g->salt; a.drop_p = g->drop_p; a.inv_rows = 1.0f / (float)g->rows;
  a.fg = g->fg; a.dskip = g->dskip; a.ld_dskip = g->ld_dskip; a.skip_row0 = g->skip_row0; a.dfg = g->dfg;
  a.sup_bstride = g->sup_bstride; a.sup_batch = g->sup_batch;
  a.ksplit = 1; a.slices = g->rows / g->n; a.kws = g->ksplit_ws; a.kcnt = g->ksplit_count;
  a.tg4 = g->tg4;
  GWN_REQUIRE(g->ksplit == 0 || g->ksplit == 1 || g->ksplit == g->nsup, "gcn_bwd: ksplit must be 0, 1 or nsup");
  if (a.sup_batch > 1)
    GWN_REQUIRE((g->rows / g->n) % a.sup_batch == 0 && g->adp_index < 0,
                "gcn_bwd (per-sample supports): slices must be a multiple of sup_batch, adp_index -1");
  if (a.bn_dy)
    GWN_REQUIRE(a.bn_z && a.bn_gamma && a.bn_mean && a.bn_rstd && a.bn_sums && a.dres && a.dh_out,
                "gcn_bwd (fused): BN prologue needs bn_z, gamma, mean, rstd, sums, dres and dh_out");
  else
    GWN_REQUIRE(a.dh != nullptr, "gcn_bwd (fused): dh is required without the BN prologue");
  if (a.dfg) GWN_REQUIRE(a.fg != nullptr, "gcn_bwd (fused): the gate epilogue needs fg");
  // the t16 backward stages dh (or dy / z, writing dres / dh_out) as 16-B rows
  const auto a16 = [](const void* ptr) { return ((uintptr_t)ptr & 15) == 0; };
  const bool t16_rows16 = a.bn_dy ? a16(a.bn_dy) && a16(a.bn_z) && a16(a.dres) && a16(a.dh_out) : a16(a.dh);
  GWN_REQUIRE(g->split_planes >= 0 && g->split_planes <= 2, "gcn_bwd: split_planes must be a gwn_dtype (0, 1, 2)");
  if (g->split_planes >= 1 && g->sup_g4b_t && a.sup_batch <= 1 && g->nsup > 0 && g->layout == 0 && t16_enabled() &&
      g->ksplit != g->nsup) {
    GWN_REQUIRE(t16_rows16, "gcn_bwd (16-node tiles, bf16): dh, or bn_dy / bn_z / dres / dh_out, must be 16-B aligned");
    const int slices = g->rows / g->n;
    const size_t fixed = t16b_lds_bytes(g->n, g->nsup, 0), img = t16b_lds_bytes(g->n, g->nsup, 1) - fixed;
    if (fixed + img <= (size_t)T16_LDS_MAX) {
      static bool attr_b = false;
      if (!attr_b) {
        (void)hipFuncSetAttribute((const void*)gcn_bwd_t16_kernel<1024, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, T16_LDS_MAX);
        (void)hipFuncSetAttribute((const void*)gcn_bwd_t16_kernel<1024, true, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, T16_LDS_MAX);
        attr_b = true;
      }
      const int nt = (g->n + 15) / 16;
      const long tiles = (long)slices * nt;
      const int grid = (int)(tiles < gwn_device_cus() ? tiles : gwn_device_cus());
      const long per = (tiles + grid - 1) / grid;
      int maximg = (int)((T16_LDS_MAX - fixed) / img);
      maximg = maximg < T16_MAXIMG ? maximg : T16_MAXIMG;
      const int span = (int)((per - 1 + nt - 1) / nt) + 1;
      maximg = maximg < span ? maximg : span;
      size_t lds = fixed + maximg * img;
      if (lds < 81 * 1024) lds = 81 * 1024;
      PowSup p = {};
      for (int k = 0; k < 2 * g->nsup; ++k) p.g4[k] = (const float*)g->sup_g4b_t[k];
      a.ksplit = 1;
      // the bf16-mlp backward takes two slices per wave (gcn_bwd_t16b2_kernel, 12-wave workgroups)
      const int pairs = (slices + 1) / 2;
      const long units2 = (long)pairs * nt;
      const int grid2 = (int)(units2 < gwn_device_cus() ? units2 : gwn_device_cus());
      const long per2 = (units2 + grid2 - 1) / grid2;
      int gmax2 = (int)((T16_LDS_MAX - fixed) / (2 * img));
      gmax2 = gmax2 < T16_MAXIMG / 2 ? gmax2 : T16_MAXIMG / 2;
      const int span2 = (int)((per2 - 1 + nt - 1) / nt) + 1;
      const int maximg2 = 2 * (gmax2 < span2 ? gmax2 : span2);
      // (pairs only from ~10 units per CU: at PEMS' 192-slice layer, 7.9 per CU, the pair kernel's
      // 12 waves were 44.0 against 42.6 us; 256 slices 38.9 vs 42.8, 768 slices 92.8 vs 98.8)
      if (g->split_planes == 2 && gmax2 >= 1 && units2 >= 10L * grid2) {
        static bool attr2 = false;
        if (!attr2) {
          (void)hipFuncSetAttribute((const void*)gcn_bwd_t16b2_kernel<768>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    T16_LDS_MAX);
          attr2 = true;
        }
        size_t lds2 = fixed + maximg2 * img;
        if (lds2 < 81 * 1024) lds2 = 81 * 1024;
        gcn_bwd_t16b2_kernel<768><<<grid2, 768, lds2, s>>>(a, p, maximg2);
      } else if (g->split_planes == 2) {
        gcn_bwd_t16_kernel<1024, true, true><<<grid, 64 * T16_WAVES, lds, s>>>(a, p, maximg);
      } else {
        gcn_bwd_t16_kernel<1024, true><<<grid, 64 * T16_WAVES, lds, s>>>(a, p, maximg);
      }
      GWN_CHECK_LAUNCH();
      return GWN_OK;
    }
  }
  GWN_REQUIRE(!g->tg4, "gcn_bwd: tg4 is written by the bf16 16-node tile kernel only (sup_g4b_t, layout 0)");
  GWN_REQUIRE(!g->split_planes,
              "gcn_bwd: bf16 operands (split_planes 1) run on the 16-node tile kernel only: sup_g4b_t, layout 0, "
              "shared supports, no forced support split, gwn_gcn_t16b_supported(n, nsup)");
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gcn_bwd_t16_kernel<1024, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              T16_LDS_MAX);
    (void)hipFuncSetAttribute((const void*)gcn_bwd_t16_kernel<1024, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              T16_LDS_MAX);
    attr_set = true;
  }
  const int slices = g->rows / g->n;
  a.ksplit = pick_ksplit(g, slices, nwt);
  const int grid = a.ksplit > 1 ? (slices + 7) / 8 * 8 * a.ksplit : slices;
  const T16Plan pl = t16_plan(g->n, g->nsup, slices);
  if (g->sup_g4_t && a.sup_batch <= 1 && g->nsup > 0 && (a.ksplit <= 1 || g->ksplit != g->nsup) && g->layout == 0 &&
      t16_enabled() && pl.ok && t16_rows16) {
    PowSup p = {};
    for (int k = 0; k < 2 * g->nsup; ++k) p.g4[k] = g->sup_g4_t[k];
    a.ksplit = 1;
    gcn_bwd_t16_kernel<1024, false><<<pl.grid, 64 * T16_WAVES, pl.lds, s>>>(a, p, pl.maximg);
    GWN_CHECK_LAUNCH();
    return GWN_OK;
  }
  return slice_bwd_launch(g, a, grid, s);  // the whole-slice schedules (gcn_slice.hip)
}

extern "C" long gwn_gcn_bn_partial_count(int rows, int n, int c, int nsup, int ld_sup) {
  (void)c; (void)nsup; (void)ld_sup;
  if (rows <= 0 || n <= 0 || rows % n) return 0;
  return gwn_bn_part_slots(rows / n);  // max(slices, CUs): every path writes all of them
}

// the bf16 16-node tile kernels run for (n, nsup) (c == 32, sup_g4b / sup_g4b_t given, layout 0)
extern "C" int gwn_gcn_t16b_supported(int n, int nsup) {
  return n > 0 && nsup > 0 && t16_enabled() && t16b_lds_bytes(n, nsup, 1) <= (size_t)T16_LDS_MAX ? 1 : 0;
}
