// Fused diffusion graph convolution (gcn.forward, reference model.py:41-55, + residual model.py:234)
// and its backward, for C = 32 channels and N <= 512 nodes.
//
// One workgroup = one slice (a (t, b) pair: N nodes x 32 channels, contiguous rows of the
// channels-last activation).  All products run on v_mfma_f32_32x32x2_f32 in the transposed
// orientation
//     D'[c][w] = sum_v X[v][c] * G[v][w]            (M = channel, N = node, K = node)
// so that
//   * the A operand X[v][c] is an LDS row read (conflict-free, rows padded to 33 floats),
//   * the B operand G[v][w] is a coalesced 128-B buffer_load of the (L2-resident) support with a
//     scalar row offset (1 VGPR of addressing for the whole K loop), rolled 16 k-steps ahead,
//   * the accumulator D'[c][w] (channel on registers, node on lanes) is directly the B operand
//     of the next product that contracts over channels (the 1x1 mlp): no lane shuffles.
// The node features never leave LDS between hops; only the pieces needed by the backward
// (x1, x2 per support) and the layer output are written to HBM, as full coalesced rows.
//
// Two wave layouts of the same schedule:
//   * 225 <= n <= 256 ("4-wave"; selectable for any n <= 256): 256 threads = one wave per SIMD; wave v owns the node tiles
//     {v, v + 4}.  Every LDS A value feeds two MFMAs, every wave runs two independent accumulator
//     chains, and the W fragments of the mlp are loaded once for both tiles.  A tile slot beyond
//     the last node tile (e.g. tile 7 for n <= 224) is computed on finite don't-care columns and
//     never stored, so the four waves run the same instruction stream (no divergent barriers).
//   * otherwise ("tile-wave"): one wave per 32-node tile (up to 16 waves, n <= 512).  At n = 207
//     (7 tiles) it beats the 4-wave layout by 10-23 % (tools/bench_gcn.py, round 1).
//
// Contract on the supports: [np][ld] with np = 32*ceil(n/32) <= ld, ZERO outside [n][n]
// (the executor keeps padded copies), so the K loop runs whole 32-node batches unguarded.
#include "gwn_internal.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int CH = 32;   // channels (one MFMA tile)
constexpr int LDR = 33;  // LDS row stride (floats): conflict-free row and column reads
constexpr int KB = 16;   // k-steps (32 nodes) per batch of the K loop
constexpr int EPT = 16;  // tile-wave epilogue elements per thread: np*32 / (64*np/32) = 16 for every n
constexpr int EPT4 = 32; // 4-wave epilogue elements per thread: covers np <= 256 with 256 threads
constexpr int TPW = 2;   // node tiles per wave in the 4-wave layout

struct FusedFwd {
  const float* h; long ld_h;
  const float* sup[8]; int nsup, ld_sup;
  const float* w_mlp; int ld_w; const float* b_mlp;
  const float* residual; float* z; float* bn_part;
  const unsigned long long* seed_ptr; unsigned long long salt; float drop_p;
  int n;
  int store_pieces;  // 0: hop outputs not written to h (inference: no backward follows)
  // eval BatchNorm folded into the epilogue (running statistics): x_out = bn(z); z not written
  const float* bn_rm; const float* bn_rv; const float* bn_g; const float* bn_b; float bn_eps; float* x_out;
  long sup_bstride; int sup_batch;  // per-sample supports (sup_batch > 1): sample b = slice % sup_batch
  const float* res_mean; const float* res_scale; const float* res_shift;  // (residual - mean) * scale + shift
  int ksplit, slices; float* kws; int* kcnt;  // support split (ksplit > 1): see unit_of()
};

struct FusedBwd {
  const float* dh;
  const float* supT[8]; int nsup, ld_sup;
  const float* w_mlp; int ld_w;
  float* dxg; long ld_dxg;
  float* t1; float* t2; long ld_t; int adp_index;
  int n;
  // optional BatchNorm-backward prologue (dh computed from the BN output gradient)
  const float* bn_dy; const float* bn_z; const float* bn_gamma; const float* bn_mean; const float* bn_rstd;
  const float* bn_sums; float* bn_dgamma; float* bn_dbeta; float* dres; float* dh_out;
  const unsigned long long* seed_ptr; unsigned long long salt; float drop_p; float inv_rows;
  // optional gate-backward epilogue (dfg instead of dxg)
  const float* fg; const float* dskip; long ld_dskip; long skip_row0; float* dfg;
  long sup_bstride; int sup_batch;  // per-sample supports, as FusedFwd
  int ksplit, slices; float* kws; int* kcnt;  // support split, as FusedFwd
};

// support k of this workgroup's slice (per-sample supports: sample = slice % sup_batch)
template <typename Args>
__device__ __forceinline__ const float* slice_sup(const Args& a, const float* base) {
  return a.sup_batch > 1 ? base + (long)(blockIdx.x % a.sup_batch) * a.sup_bstride : base;
}

__device__ __forceinline__ int crow(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }

// Work unit of this workgroup: a whole slice (ksplit <= 1), or support k0 of a slice (ksplit = nsup
// workgroups per slice).  The ksplit units of a slice are blockIdx i, i + 8, i + 16, ...: with the
// round-robin workgroup-to-XCD dispatch they share one XCD's L2 (partial sums written and read
// there).  Returns false for the padding workgroups of the last group of 8 slices.
struct Unit {
  int slice, k0, k1;
};
template <typename Args>
__device__ __forceinline__ bool unit_of(const Args& a, Unit& u) {
  if (a.ksplit <= 1) {
    u.slice = blockIdx.x; u.k0 = 0; u.k1 = a.nsup;
    return true;
  }
  const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
  u.k0 = j % a.ksplit; u.k1 = u.k0 + 1;
  u.slice = (j / a.ksplit) * 8 + x;
  return u.slice < a.slices;
}

// Support split hand-off (MI355X_MICROARCH.md, inter-workgroup visibility: write-through payload,
// counter add behind a barrier, write-through loads by the last arriver; no L2 write-back fence --
// an agent release per unit, i.e. a buffer_wbl2 of the XCD's L2 full of fresh hop pieces, cost
// ~50 us per launch).  cache-policy aux 16 = sc1 (write-through store / L1-bypassing load).
constexpr int SC1 = 16;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// partial D'[c][w] tile -> rows w of part [n][32] as 16-B sc1 stores (rows >= n dropped by the
// buffer range)
__device__ __forceinline__ void acc_to_part(float* part, int n, const f32x16& d, int w0, int lane) {
  const int half = lane >> 5, col = lane & 31;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)part, (short)0, n * CH * 4, 0x00020000);
  const int voff = (w0 + col) * CH * 4;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    // (hipcc 7.2 splats {bit_cast(unsigned, d[i]), ...} to d[0]: go through float4)
    const float4 v = make_float4(d[4 * g], d[4 * g + 1], d[4 * g + 2], d[4 * g + 3]);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, voff + crow(4 * g, half) * 4, 0, SC1);
  }
}

// count this unit's (already stored) partial; true in the slice's last unit to arrive, which also
// resets the counter for the next launch
__device__ __forceinline__ bool split_arrive(int* cnt, int parts, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's partial stores have completed
  __syncthreads();
  if (threadIdx.x == 0) *flag = (atomicAdd(cnt, 1) == parts - 1);
  __syncthreads();
  if (!*flag) return false;
  if (threadIdx.x == 0) atomicExch(cnt, 0);
  return true;
}

// sum of the parts partials [parts][np][32] of a slice, in part order, into LDS rows [n][LDR]
// (16-B sc1 loads)
__device__ __forceinline__ void split_sum_to_lds(const float* part, int parts, int n, int np, float* buf) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void*)part, (short)0, parts * np * CH * 4, 0x00020000);
  for (int e = threadIdx.x; e < n * 8; e += blockDim.x) {
    float4 v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, e * 16, 0, SC1));
    for (int p = 1; p < parts; ++p) {
      const float4 q = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, e * 16, p * np * CH * 4, SC1));
      v.x += q.x; v.y += q.y; v.z += q.z; v.w += q.w;
    }
    float* b = buf + (e >> 3) * LDR + 4 * (e & 7);
    b[0] = v.x; b[1] = v.y; b[2] = v.z; b[3] = v.w;
  }
}


// bf16 kernels: support batches prefetched ahead of their MFMAs (whole hop up to this many)
#ifndef GWN_BF16_PD
#define GWN_BF16_PD 11
#endif
#ifndef GWN_EXP
// kernel experiments (timing only; 1-16 give wrong results): 1 no G loads, 2 no LDS A reads,
// 4 no W loads, 16 no phase barriers (forward); 32 = forward hop pieces stored straight from the
// accumulators by the compute waves instead of by a store wave through LDS (correct, slower);
// 256 = clock diagnostic (per-workgroup cycles / real-time ticks after the BN partials,
// tools/clock_gcn.py)
#define GWN_EXP 0
#endif

__device__ __forceinline__ float bload(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
#if GWN_EXP & 1
  return (float)(voff + soff) * 1e-9f;
#else
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
#endif
}

// the last 32-node K batch holds at most 16 real nodes: its upper 8 k-steps (2 nodes each) only
// multiply zero rows of the padded support and are skipped (n = 207: nodes 192..206)
__host__ __device__ constexpr bool half_last_batch(int n) { return n - 32 * ((n + 31) / 32 - 1) <= 16; }

struct GBatch {
  float v[KB];
};

// first K batch (32 nodes) of G's B-operand fragments; issued a phase ahead of its diffusion
__device__ __forceinline__ GBatch g_first(const float* G, int ld, int nkb, int w0, int lane) {
  const int half = lane >> 5, col = lane & 31;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)G, (short)0, nkb * 32 * ld * 4, 0x00020000);
  const int voff = (half * ld + w0 + col) * 4;
  GBatch g;
#pragma unroll
  for (int j = 0; j < KB; ++j) g.v[j] = bload(rs, voff, j * 2 * ld * 4);
  return g;
}

// W fragments for mlp_from_acc (A operand W[c'=col][off + crow(s, half)]); issued ahead
__device__ __forceinline__ GBatch w_frags(const float* W, int ld_w, int off, int lane) {
  const int half = lane >> 5, col = lane & 31;
  const float* wp = W + (long)col * ld_w + off;
  GBatch f;
#pragma unroll
  for (int s = 0; s < 16; ++s) {
#if GWN_EXP & 4
    f.v[s] = (float)(off + s) * 1e-6f + (float)lane * 1e-9f;
#else
    f.v[s] = wp[crow(s, half)];
#endif
  }
  return f;
}

// D'[c][w0+col] += sum_v buf[v][c] * G[v][w0+col];  g0 = g_first(G, ...) (consumed)
template <bool HL>
__device__ __forceinline__ f32x16 diffuse(const float* buf, const float* G, int ld, int nkb, int w0,
                                          int lane, f32x16 acc, const GBatch& g0) {
  const int half = lane >> 5, col = lane & 31;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)G, (short)0, nkb * 32 * ld * 4, 0x00020000);
  const int voff = (half * ld + w0 + col) * 4;
  const int rowb = 2 * ld * 4;  // bytes between k-steps (2 nodes)
  // Two register sets ga / gb (no write-after-read between a batch's MFMAs and the next batch's
  // loads): the loads of batch b+1 issue at the top of batch b, 16 MFMAs ahead of their use.
  // The loop body has no branch around a load, so hipcc keeps the waits counted (vmcnt(N)).
  float ga[KB], gb[KB];
#pragma unroll
  for (int j = 0; j < KB; ++j) ga[j] = g0.v[j];
  auto lds_batch = [&](int kb, float* av) {
    const float* bp = buf + (32 * kb + half) * LDR + col;
#pragma unroll
    for (int j = 0; j < KB; ++j) {
#if GWN_EXP & 2
      av[j] = (float)(kb * KB + j) * 1e-9f + (float)lane * 1e-12f + bp[0] * 1e-30f;
#else
      av[j] = bp[2 * j * LDR];
#endif
    }
  };
  auto g_batch = [&](int kb, float* g) {
#pragma unroll
    for (int j = 0; j < KB; ++j) g[j] = bload(rs, voff, (kb * KB + j) * rowb);
  };
  auto mfma_batch = [&](const float* av, const float* g) {
#pragma unroll
    for (int j = 0; j < KB; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j], g[j], acc, 0, 0, 0);
  };
  // k-step j of a batch covers nodes 32 kb + 2 j + {0, 1}: when the last batch holds at most 16
  // real nodes (n = 207: nodes 192..206) its upper 8 k-steps multiply zero rows and are skipped
  // (HL = half_last_batch(n), a kernel template flag; 7 % of the diffusion MFMAs at n = 207)
  auto last_batch = [&](int kb, const float* g) {
    const float* bp = buf + (32 * kb + half) * LDR + col;
    float av[KB];
    if (HL) {
#pragma unroll
      for (int j = 0; j < KB / 2; ++j) av[j] = bp[2 * j * LDR];
#pragma unroll
      for (int j = 0; j < KB / 2; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j], g[j], acc, 0, 0, 0);
    } else {
      lds_batch(kb, av);
      mfma_batch(av, g);
    }
  };
  int kb = 0;
  for (; kb + 2 < nkb; kb += 2) {
    float av[KB];
    g_batch(kb + 1, gb);
    lds_batch(kb, av);
    mfma_batch(av, ga);
    g_batch(kb + 2, ga);
    lds_batch(kb + 1, av);
    mfma_batch(av, gb);
  }
  if (kb + 1 < nkb) {  // two batches left
    float av[KB];
    g_batch(kb + 1, gb);
    lds_batch(kb, av);
    mfma_batch(av, ga);
    last_batch(kb + 1, gb);
  } else {             // one batch left
    last_batch(kb, ga);
  }
  return acc;
}

// acc_out[c'][w] += sum_c W[c'][off + c] * D'[c][w]   with D' = the accumulator `d`, wf = w_frags(off)
__device__ __forceinline__ f32x16 mlp_from_acc(const GBatch& wf, const f32x16& d, f32x16 acc) {
#pragma unroll
  for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wf.v[s], d[s], acc, 0, 0, 0);
  return acc;
}

// acc[c'][w] += sum_c W[c'][off + c] * buf[w][c]      (buf = LDS rows)
__device__ __forceinline__ f32x16 mlp_from_lds(const float* W, int ld_w, int off, const float* buf,
                                               int w0, int lane, f32x16 acc) {
  const int half = lane >> 5, col = lane & 31;
  const float* wp = W + (long)col * ld_w + off;
  const float* bp = buf + (w0 + col) * LDR;
#pragma unroll
  for (int s = 0; s < 16; ++s)
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wp[2 * s + half], bp[2 * s + half], acc, 0, 0, 0);
  return acc;
}

// acc[c][w] += sum_c' W[c'][off + c] * buf[w][c']      (transposed weights: dP = W^T dh)
__device__ __forceinline__ f32x16 mlpT_from_lds(const float* W, int ld_w, int off, const float* buf,
                                                int w0, int lane, f32x16 acc) {
  const int half = lane >> 5, col = lane & 31;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, CH * ld_w * 4, 0x00020000);
  const int voff = (half * ld_w + off + col) * 4;
  const float* bp = buf + (w0 + col) * LDR;
  float wf[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) wf[s] = bload(rs, voff, 2 * s * ld_w * 4);
#pragma unroll
  for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wf[s], bp[2 * s + half], acc, 0, 0, 0);
  return acc;
}

__device__ __forceinline__ void acc_to_lds(float* buf, const f32x16& d, int w0, int lane) {
  const int half = lane >> 5, col = lane & 31;
  float* bp = buf + (w0 + col) * LDR;
#pragma unroll
  for (int r = 0; r < 16; ++r) bp[crow(r, half)] = d[r];
}

// Tile D'[c][w] straight from the accumulator to rows w of dst: each store instruction writes
// 2 channels of 32 rows; the 16 instructions of a wave cover its 32 full 128-B row segments, which
// L2 merges before write-back.  No LDS round trip and no barrier.
// A lane's 16 accumulator rows are 4 runs of 4 consecutive channels (crow(4g..4g+3, half) =
// 8g + 4h + 0..3), so with a 16-B aligned row base they go out as 4 dwordx4 stores: a quarter of
// the write requests of 16 dword stores (measured: the scalar form cost 20 % of the forward at
// T = 12, where every CU streams hop pieces out at once).
__device__ __forceinline__ void acc_to_global(float* dst, long ld, const f32x16& d, int w0, int lane, int n) {
  const int half = lane >> 5, col = lane & 31;
  if (w0 + col >= n) return;
  float* p = dst + (long)(w0 + col) * ld;
  if ((((uintptr_t)dst & 15) | (ld & 3)) == 0) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *(float4*)(p + crow(4 * g, half)) = make_float4(d[4 * g], d[4 * g + 1], d[4 * g + 2], d[4 * g + 3]);
  } else {
#pragma unroll
    for (int r = 0; r < 16; ++r) p[crow(r, half)] = d[r];
  }
}

// LDS image index of (row w, channel c): padded rows [np][LDR], or (PL, the balanced layout)
// channel-half planes [2][np][16]
template <bool PL>
__device__ __forceinline__ int img_idx(int w, int c, int np) {
  return PL ? ((c >> 4) * np + w) * 16 + (c & 15) : w * LDR + c;
}

template <bool PL = false>
__device__ __forceinline__ void global_to_lds(const float* src, long ld, int n, int np, float* buf) {
  if ((((uintptr_t)src) & 15) == 0 && (ld & 3) == 0) {
    // 16-B buffer loads, four per thread in flight before its first LDS write (the element loop
    // below compiles to load -> s_waitcnt vmcnt(0) -> write per element: one memory round trip per
    // element, 14 per thread for a 207-node slice); rows >= n read zeros (out of range)
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)((long)n * ld * 4), 0x00020000);
    const int total = np * 8;  // float4s of the [np][32] image
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
        if (e < total) {
          const int w = e >> 3, c = 4 * (e & 7);
          buf[img_idx<PL>(w, c, np)] = v[i].x;
          buf[img_idx<PL>(w, c + 1, np)] = v[i].y;
          buf[img_idx<PL>(w, c + 2, np)] = v[i].z;
          buf[img_idx<PL>(w, c + 3, np)] = v[i].w;
        }
      }
    }
    return;
  }
  for (int e = threadIdx.x; e < np * CH; e += blockDim.x) {
    const int w = e >> 5, c = e & 31;
    buf[img_idx<PL>(w, c, np)] = (w < n) ? src[(long)w * ld + c] : 0.0f;
  }
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.0f;
  return z;
}

// ---------------------------------------------------------------------------------------------
// Shared prologue / epilogue bodies (NEPT rows-per-thread bound: wb + i*ws covers np rows)

// forward epilogue on the mlp output in ys: bias, dropout (same counter hash as the GEMM
// epilogue: index m*32 + c), residual -> z (+ per-slice BN partials), or -> bn(z) in eval mode
template <int NEPT>
__device__ __forceinline__ void fwd_epilogue(const FusedFwd& a, float* ys, float* red0, float* red1, long row0,
                                             int n, int slice) {
  const unsigned long long seed = a.seed_ptr ? *a.seed_ptr : 0ull;
  const float keep_scale = (a.drop_p > 0.0f) ? 1.0f / (1.0f - a.drop_p) : 1.0f;
  const int c = threadIdx.x & 31, wb = threadIdx.x >> 5, ws = blockDim.x >> 5;
  const float bias = a.b_mlp[c];
  float bmu = 0.0f, brs = 1.0f, bg = 1.0f, bb = 0.0f;
  // the layer below's BatchNorm applied to the residual on load (gwn_batchnorm_fwd_fold)
  const bool raff = a.res_scale != nullptr;
  const float rmu = raff ? a.res_mean[c] : 0.0f;
  const float rsc = raff ? a.res_scale[c] : 1.0f, rsh = raff ? a.res_shift[c] : 0.0f;
  if (a.x_out) {  // eval BatchNorm, the arithmetic of bn_apply_kernel (ops.hip)
    bmu = a.bn_rm[c];
    brs = 1.0f / sqrtf(a.bn_rv[c] + a.bn_eps);
    bg = a.bn_g[c];
    bb = a.bn_b[c];
  }
  // all residual loads are issued before the first store (the compiler cannot reorder loads
  // across possibly aliasing stores itself)
  float res[NEPT];
#pragma unroll
  for (int i = 0; i < NEPT; ++i) {
    const int w = min(wb + i * ws, n - 1);
    res[i] = a.residual[(row0 + w) * CH + c];
  }
#pragma unroll
  for (int i = 0; i < NEPT; ++i) {
    const int w = wb + i * ws;
    if (w < n) {
      const long m = row0 + w;
      float v = ys[w * LDR + c] + bias;
      if (a.drop_p > 0.0f) {
        const float u = gwn_uniform(seed, a.salt, (unsigned long long)m * CH + c);
        v = (u >= a.drop_p) ? v * keep_scale : 0.0f;
      }
      v += raff ? fmaf(res[i] - rmu, rsc, rsh) : res[i];
      if (a.x_out) {
        a.x_out[m * CH + c] = (v - bmu) * brs * bg + bb;
      } else {
        a.z[m * CH + c] = v;
        ys[w * LDR + c] = v;
      }
    }
  }
  if (a.bn_part == nullptr || a.x_out) return;
  __syncthreads();
  // per-slice BN partials (count, mean, M2) per channel, fixed order
  const int ngroups = blockDim.x >> 5;
  const int g = threadIdx.x >> 5;
  float s = 0.0f;
  for (int w = g; w < n; w += ngroups) s += ys[w * LDR + c];
  red0[threadIdx.x] = s;
  __syncthreads();
  float mean = 0.0f;
  for (int i = 0; i < ngroups; ++i) mean += red0[i * 32 + c];
  mean /= (float)n;
  float q = 0.0f;
  for (int w = g; w < n; w += ngroups) {
    const float dlt = ys[w * LDR + c] - mean;
    q += dlt * dlt;
  }
  red1[threadIdx.x] = q;
  __syncthreads();
  if (threadIdx.x < 32) {
    float m2 = 0.0f;
    for (int i = 0; i < ngroups; ++i) m2 += red1[i * 32 + c];
    float* pp = a.bn_part + (long)slice * 3 * CH;
    pp[c] = (float)n;
    pp[CH + c] = mean;
    pp[2 * CH + c] = m2;
  }
}

// backward prologue: dh of the slice into LDS (rows >= n zero), either loaded or computed by the
// BatchNorm backward of this layer's output (same arithmetic as bn_bwd_apply_kernel, ops.hip):
//   dz = gamma*rstd*(dy - k1 - xhat*k2) -> residual gradient dres; dropout'(dz) -> dh (LDS + HBM)
template <int NEPT, bool PL = false>
__device__ __forceinline__ void bwd_prologue(const FusedBwd& a, float* dhs, long row0, int n, int np,
                                             bool lead = true, bool first = blockIdx.x == 0) {
  if (!a.bn_dy) {
    global_to_lds<PL>(a.dh + row0 * CH, CH, n, np, dhs);
    return;
  }
  if (first && threadIdx.x < CH) {
    if (a.bn_dbeta) a.bn_dbeta[threadIdx.x] = a.bn_sums[threadIdx.x];
    if (a.bn_dgamma) a.bn_dgamma[threadIdx.x] = a.bn_sums[CH + threadIdx.x];
  }
  const unsigned long long seed = a.seed_ptr ? *a.seed_ptr : 0ull;
  const float keep_scale = (a.drop_p > 0.0f) ? 1.0f / (1.0f - a.drop_p) : 1.0f;
  const int c = threadIdx.x & 31, wb = threadIdx.x >> 5, ws = blockDim.x >> 5;
  const float mu = a.bn_mean[c], rs = a.bn_rstd[c], gm = a.bn_gamma[c];
  const float k1 = a.bn_sums[c] * a.inv_rows, k2 = a.bn_sums[CH + c] * a.inv_rows;
  float dy[NEPT], zv[NEPT];  // all loads before the first store (see fwd_epilogue)
#pragma unroll
  for (int i = 0; i < NEPT; ++i) {
    const long idx = (row0 + min(wb + i * ws, n - 1)) * CH + c;
    dy[i] = a.bn_dy[idx];
    zv[i] = a.bn_z[idx];
  }
#pragma unroll
  for (int i = 0; i < NEPT; ++i) {
    const int w = wb + i * ws;
    float v = 0.0f;
    if (w < n) {
      const long idx = (row0 + w) * CH + c;
      const float xhat = (zv[i] - mu) * rs;
      const float dz = gm * rs * (dy[i] - k1 - xhat * k2);
      if (lead) a.dres[idx] = dz;
      v = dz;
      if (a.drop_p > 0.0f) {
        const float u = gwn_uniform(seed, a.salt, (unsigned long long)idx);
        v = (u >= a.drop_p) ? v * keep_scale : 0.0f;
      }
      if (lead) a.dh_out[idx] = v;
    }
    if (w < np) dhs[img_idx<PL>(w, c, np)] = v;
  }
}

// gate backward (gate_bwd_kernel, ops.hip) on dxg staged in buf: g = dxg (+ dskip) -> dfg through
// the saved (tanh f, sigmoid s) pairs; the fg / dfg rows move as coalesced float2s
template <int NEPT>
__device__ __forceinline__ void bwd_gate_epilogue(const FusedBwd& a, const float* buf, long row0, int n) {
  const int c = threadIdx.x & 31, wb = threadIdx.x >> 5, ws = blockDim.x >> 5;
  float2 fs[NEPT];
  float dsk[NEPT];
#pragma unroll
  for (int i = 0; i < NEPT; ++i) {
    const long m = row0 + min(wb + i * ws, n - 1);
    fs[i] = *(const float2*)(a.fg + m * 2 * CH + 2 * c);
    dsk[i] = (a.dskip && m >= a.skip_row0) ? a.dskip[(m - a.skip_row0) * a.ld_dskip + c] : 0.0f;
  }
#pragma unroll
  for (int i = 0; i < NEPT; ++i) {
    const int w = wb + i * ws;
    if (w < n) {
      const long m = row0 + w;
      const float g = buf[w * LDR + c] + dsk[i];
      const float f = fs[i].x, sg = fs[i].y;
      float2 o;
      o.x = g * sg * (1.0f - f * f);
      o.y = g * f * sg * (1.0f - sg);
      *(float2*)(a.dfg + m * 2 * CH + 2 * c) = o;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// tile-wave layout: one wave per 32-node tile

// With one wave more than node tiles (blockDim = 64 * (nkb + 1), the launcher's choice whenever the
// hop pieces are stored), the last wave is a store wave: it copies each hop piece from the LDS
// image to h as whole 128-B rows while the compute waves run the next diffusion.  gfx950 counts
// stores in vmcnt, in order with loads, so a compute wave that stored a piece would wait for those
// writes to complete at its next G-fragment wait; the store wave takes them off that path (and
// lands on the SIMD that hosts one compute wave, 2,2,2,1 -> 2,2,2,2).
template <int MAXT, bool HL>
__global__ __launch_bounds__(MAXT, 4) void gcn_fwd_fused_kernel(const FusedFwd a) {
  extern __shared__ float lds[];
  __shared__ float red[2][MAXT];
  __shared__ int last_unit;
  Unit u;
  if (!unit_of(a, u)) return;
  const int n = a.n;
  const int nkb = (n + 31) >> 5;
  const int np = nkb * 32;
  float* xs = lds;
  float* ys = lds + np * LDR;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, w0 = wave * 32;
  const bool compute = wave < nkb;
  const bool store_wave = (int)(blockDim.x >> 6) > nkb;  // block-uniform
  const long row0 = (long)u.slice * n;
  const long ldh = a.ld_h, pstride = CH;  // piece p of row w at hs + w*ldh + p*pstride
  const float* hs = a.h + row0 * ldh;
  // hop pieces: by the store wave (whole rows through LDS), else straight from the accumulators
  auto piece_rows = [&](int piece) {  // store wave only
    const float* src = ys;
    float* dst = (float*)hs + piece * pstride;
    for (int e = lane; e < n * 8; e += 64) {
      const int w = e >> 3, q = e & 7;
      const float* b = src + w * LDR + 4 * q;
      // write-once data the backward reads after the whole forward: non-temporal
      typedef float f32x4_t __attribute__((ext_vector_type(4)));
      const f32x4_t v = {b[0], b[1], b[2], b[3]};
      __builtin_nontemporal_store(v, (f32x4_t*)(dst + (long)w * ldh + 4 * q));
    }
  };

#if GWN_EXP & 256
  // clock diagnostic: shader cycles and 100 MHz real-time ticks over the workgroup's life
  const unsigned long long t_cyc0 = __builtin_amdgcn_s_memtime(), t_real0 = __builtin_amdgcn_s_memrealtime();
#endif
  // software pipeline: every G first batch / W fragment set is issued one phase before use
  GBatch g0 = (u.k1 > u.k0 && compute) ? g_first(slice_sup(a, a.sup[u.k0]), a.ld_sup, nkb, w0, lane) : GBatch{};
  global_to_lds(hs, ldh, n, np, xs);
  __syncthreads();
  f32x16 hacc = zero16();
  if (compute && u.k0 == 0) hacc = mlp_from_lds(a.w_mlp, a.ld_w, 0, xs, w0, lane, zero16());
  for (int k = u.k0; k < u.k1; ++k) {
    const float* G = slice_sup(a, a.sup[k]);
    f32x16 d = zero16();
    if (compute) {
      d = diffuse<HL>(xs, G, a.ld_sup, nkb, w0, lane, zero16(), g0);
      g0 = g_first(G, a.ld_sup, nkb, w0, lane);  // hop 2 re-reads the same support
      GBatch wf = w_frags(a.w_mlp, a.ld_w, (1 + 2 * k) * CH, lane);
      hacc = mlp_from_acc(wf, d, hacc);
    }
#if !(GWN_EXP & 16)
    __syncthreads();  // ys is free: every wave finished the previous support's hop 2 (and its store)
#endif
    if (compute) {
      acc_to_lds(ys, d, w0, lane);
      if (a.store_pieces && !store_wave) acc_to_global((float*)hs + (1 + 2 * k) * pstride, ldh, d, w0, lane, n);
    }
#if !(GWN_EXP & 16)
    __syncthreads();
#endif
    if (compute) {
      d = diffuse<HL>(ys, G, a.ld_sup, nkb, w0, lane, zero16(), g0);
      if (k + 1 < u.k1) g0 = g_first(slice_sup(a, a.sup[k + 1]), a.ld_sup, nkb, w0, lane);
      GBatch wf = w_frags(a.w_mlp, a.ld_w, (2 + 2 * k) * CH, lane);
      hacc = mlp_from_acc(wf, d, hacc);
      if (a.store_pieces && !store_wave) acc_to_global((float*)hs + (2 + 2 * k) * pstride, ldh, d, w0, lane, n);
    } else if (a.store_pieces) {
      piece_rows(1 + 2 * k);  // x1 (in ys) while the compute waves run hop 2
    }
    if (a.store_pieces && store_wave) {  // x2 through ys as well
      __syncthreads();
      if (compute) acc_to_lds(ys, d, w0, lane);
      __syncthreads();
      if (!compute) piece_rows(2 + 2 * k);  // while the compute waves run the next hop 1
    }
  }
  __syncthreads();
  if (a.ksplit > 1) {  // partial mlp sum of this support; the slice's last unit runs the epilogue
    float* part = a.kws + (long)u.slice * a.ksplit * np * CH;
    if (compute) acc_to_part(part + (long)u.k0 * np * CH, n, hacc, w0, lane);
    if (!split_arrive(a.kcnt + u.slice, a.ksplit, &last_unit)) return;
    split_sum_to_lds(part, a.ksplit, n, np, ys);
  } else if (compute) {
    acc_to_lds(ys, hacc, w0, lane);
  }
  __syncthreads();
  fwd_epilogue<EPT>(a, ys, red[0], red[1], row0, n, u.slice);
#if GWN_EXP & 256
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    // past the per-slice BN partials: [slices][3][32] floats, then 4 floats per workgroup
    float* dg = a.bn_part + (long)gridDim.x * 3 * CH + 4 * blockIdx.x;
    dg[0] = (float)(c1 - t_cyc0);
    dg[1] = (float)(r1 - t_real0);
    dg[2] = (float)(t_real0 & 0xffffffull);  // start tick (low 24 bits)
    dg[3] = (float)__smid();
  }
#endif
}

template <int MAXT, bool HL>
__global__ __launch_bounds__(MAXT, 4) void gcn_bwd_fused_kernel(const FusedBwd a) {
  extern __shared__ float lds[];
  __shared__ int last_unit;
  Unit un;
  if (!unit_of(a, un)) return;
  const int n = a.n;
  const int nkb = (int)(blockDim.x >> 6);
  const int np = nkb * 32;
  float* dhs = lds;
  float* buf = lds + np * LDR;
  const int lane = threadIdx.x & 63, w0 = (threadIdx.x >> 6) * 32;
  const long row0 = (long)un.slice * n;

  GBatch g0 = (un.k1 > un.k0) ? g_first(slice_sup(a, a.supT[un.k0]), a.ld_sup, nkb, w0, lane) : GBatch{};
  // the BN-backward prologue's HBM outputs (dres, dh, BN dgamma / dbeta) come from support 0's unit
  bwd_prologue<EPT>(a, dhs, row0, n, np, un.k0 == 0, un.slice == 0 && un.k0 == 0);
  __syncthreads();
  f32x16 dx = (un.k0 == 0) ? mlpT_from_lds(a.w_mlp, a.ld_w, 0, dhs, w0, lane, zero16()) : zero16();
  for (int k = un.k0; k < un.k1; ++k) {
    const float* GT = slice_sup(a, a.supT[k]);
    {
      const f32x16 u = mlpT_from_lds(a.w_mlp, a.ld_w, (2 + 2 * k) * CH, dhs, w0, lane, zero16());
      __syncthreads();
      acc_to_lds(buf, u, w0, lane);
      if (k == a.adp_index) acc_to_global(a.t2 + row0 * a.ld_t, a.ld_t, u, w0, lane, n);
    }
    __syncthreads();
    f32x16 t = mlpT_from_lds(a.w_mlp, a.ld_w, (1 + 2 * k) * CH, dhs, w0, lane, zero16());
    t = diffuse<HL>(buf, GT, a.ld_sup, nkb, w0, lane, t, g0);  // dx1 = dP_x1 + A dP_x2
    g0 = g_first(GT, a.ld_sup, nkb, w0, lane);
    __syncthreads();
    acc_to_lds(buf, t, w0, lane);
    if (k == a.adp_index) acc_to_global(a.t1 + row0 * a.ld_t, a.ld_t, t, w0, lane, n);
    __syncthreads();
    dx = diffuse<HL>(buf, GT, a.ld_sup, nkb, w0, lane, dx, g0);  // dxg += A dx1
    if (k + 1 < un.k1) g0 = g_first(slice_sup(a, a.supT[k + 1]), a.ld_sup, nkb, w0, lane);
  }
  if (a.ksplit > 1) {  // partial input gradient of this support; the slice's last unit finishes
    float* part = a.kws + (long)un.slice * a.ksplit * np * CH;
    acc_to_part(part + (long)un.k0 * np * CH, n, dx, w0, lane);
    if (!split_arrive(a.kcnt + un.slice, a.ksplit, &last_unit)) return;
    split_sum_to_lds(part, a.ksplit, n, np, buf);
    __syncthreads();
    if (a.dfg) {
      bwd_gate_epilogue<EPT>(a, buf, row0, n);
    } else {
      for (int e = threadIdx.x; e < n * CH; e += blockDim.x)
        a.dxg[(row0 + (e >> 5)) * a.ld_dxg + (e & 31)] = buf[(e >> 5) * LDR + (e & 31)];
    }
    return;
  }
  if (!a.dfg) {
    acc_to_global(a.dxg + row0 * a.ld_dxg, a.ld_dxg, dx, w0, lane, n);
    return;
  }
  __syncthreads();  // every wave finished reading buf
  acc_to_lds(buf, dx, w0, lane);
  __syncthreads();
  bwd_gate_epilogue<EPT>(a, buf, row0, n);
}

// ---------------------------------------------------------------------------------------------
// 4-wave layout (n <= 256): wave v owns node tiles {v, v + 4}

struct GBatch2 {
  float v[TPW][KB];
};

__device__ __forceinline__ GBatch2 g_first2(const float* G, int ld, int nkb, const int* w0, int lane) {
  GBatch2 g;
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const GBatch b = g_first(G, ld, nkb, w0[i], lane);
#pragma unroll
    for (int j = 0; j < KB; ++j) g.v[i][j] = b.v[j];
  }
  return g;
}

// acc[i] += D' of tile i (diffuse() for TPW tiles sharing every A operand); g0 = g_first2(G, ...)
__device__ __forceinline__ void diffuse2(const float* buf, const float* G, int ld, int nkb, const int* w0,
                                         int lane, f32x16* acc, const GBatch2& g0) {
  const int half = lane >> 5, col = lane & 31;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)G, (short)0, nkb * 32 * ld * 4, 0x00020000);
  int voff[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) voff[i] = (half * ld + w0[i] + col) * 4;
  const int rowb = 2 * ld * 4;
  float ga[TPW][KB], gb[TPW][KB];
#pragma unroll
  for (int i = 0; i < TPW; ++i)
#pragma unroll
    for (int j = 0; j < KB; ++j) ga[i][j] = g0.v[i][j];
  auto lds_batch = [&](int kb, float* av) {
    const float* bp = buf + (32 * kb + half) * LDR + col;
#pragma unroll
    for (int j = 0; j < KB; ++j) av[j] = bp[2 * j * LDR];
  };
  auto g_batch = [&](int kb, float (*g)[KB]) {
#pragma unroll
    for (int i = 0; i < TPW; ++i)
#pragma unroll
      for (int j = 0; j < KB; ++j) g[i][j] = bload(rs, voff[i], (kb * KB + j) * rowb);
  };
  auto mfma_batch = [&](const float* av, float (*g)[KB]) {
#pragma unroll
    for (int j = 0; j < KB; ++j)
#pragma unroll
      for (int i = 0; i < TPW; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j], g[i][j], acc[i], 0, 0, 0);
  };
  int kb = 0;
  for (; kb + 2 < nkb; kb += 2) {
    float av[KB];
    g_batch(kb + 1, gb);
    lds_batch(kb, av);
    mfma_batch(av, ga);
    g_batch(kb + 2, ga);
    lds_batch(kb + 1, av);
    mfma_batch(av, gb);
  }
  float av[KB];
  if (kb + 1 < nkb) {
    g_batch(kb + 1, gb);
    lds_batch(kb, av);
    mfma_batch(av, ga);
    lds_batch(kb + 1, av);
    mfma_batch(av, gb);
  } else {
    lds_batch(kb, av);
    mfma_batch(av, ga);
  }
}

__device__ __forceinline__ void mlp_from_lds2(const float* W, int ld_w, int off, const float* buf, const int* w0,
                                              int lane, f32x16* acc) {
  const int half = lane >> 5, col = lane & 31;
  const float* wp = W + (long)col * ld_w + off;
  float wf[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) wf[s] = wp[2 * s + half];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const float* bp = buf + (w0[i] + col) * LDR;
#pragma unroll
    for (int s = 0; s < 16; ++s) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(wf[s], bp[2 * s + half], acc[i], 0, 0, 0);
  }
}

__device__ __forceinline__ void mlpT_from_lds2(const float* W, int ld_w, int off, const float* buf, const int* w0,
                                               int lane, f32x16* acc) {
  const int half = lane >> 5, col = lane & 31;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, CH * ld_w * 4, 0x00020000);
  const int voff = (half * ld_w + off + col) * 4;
  float wf[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) wf[s] = bload(rs, voff, 2 * s * ld_w * 4);
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const float* bp = buf + (w0[i] + col) * LDR;
#pragma unroll
    for (int s = 0; s < 16; ++s) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(wf[s], bp[2 * s + half], acc[i], 0, 0, 0);
  }
}

// launch bounds (256 threads, >= 2 waves per SIMD): <= 256 VGPRs, two workgroups per CU
__global__ __launch_bounds__(256, 2) void gcn_fwd_fused4_kernel(const FusedFwd a) {
  extern __shared__ float lds[];
  __shared__ float red[2][256];
  const int n = a.n;
  const int nkb = (n + 31) >> 5;
  const int np = nkb * 32;
  float* xs = lds;
  float* ys = lds + np * LDR;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long row0 = (long)blockIdx.x * n;
  const float* hs = a.h + row0 * a.ld_h;
  int w0[TPW];
  bool tv[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    w0[i] = 32 * (wv + 4 * i);
    tv[i] = wv + 4 * i < nkb;
  }

  GBatch2 g0 = (a.nsup > 0) ? g_first2(slice_sup(a, a.sup[0]), a.ld_sup, nkb, w0, lane) : GBatch2{};
  global_to_lds(hs, a.ld_h, n, np, xs);
  __syncthreads();
  f32x16 hacc[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) hacc[i] = zero16();
  mlp_from_lds2(a.w_mlp, a.ld_w, 0, xs, w0, lane, hacc);
  for (int k = 0; k < a.nsup; ++k) {
    const float* G = slice_sup(a, a.sup[k]);
    f32x16 d[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) d[i] = zero16();
    diffuse2(xs, G, a.ld_sup, nkb, w0, lane, d, g0);
    g0 = g_first2(G, a.ld_sup, nkb, w0, lane);  // hop 2 re-reads the same support
    {
      const GBatch wf = w_frags(a.w_mlp, a.ld_w, (1 + 2 * k) * CH, lane);
#pragma unroll
      for (int i = 0; i < TPW; ++i) hacc[i] = mlp_from_acc(wf, d[i], hacc[i]);
    }
    __syncthreads();  // ys is free once every wave finished the previous support's hop 2
#pragma unroll
    for (int i = 0; i < TPW; ++i)
      if (tv[i]) acc_to_lds(ys, d[i], w0[i], lane);
    if (a.store_pieces) {
#pragma unroll
      for (int i = 0; i < TPW; ++i) acc_to_global((float*)hs + (1 + 2 * k) * CH, a.ld_h, d[i], w0[i], lane, n);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < TPW; ++i) d[i] = zero16();
    diffuse2(ys, G, a.ld_sup, nkb, w0, lane, d, g0);
    if (k + 1 < a.nsup) g0 = g_first2(slice_sup(a, a.sup[k + 1]), a.ld_sup, nkb, w0, lane);
    {
      const GBatch wf = w_frags(a.w_mlp, a.ld_w, (2 + 2 * k) * CH, lane);
#pragma unroll
      for (int i = 0; i < TPW; ++i) hacc[i] = mlp_from_acc(wf, d[i], hacc[i]);
    }
    if (a.store_pieces) {
#pragma unroll
      for (int i = 0; i < TPW; ++i) acc_to_global((float*)hs + (2 + 2 * k) * CH, a.ld_h, d[i], w0[i], lane, n);
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < TPW; ++i)
    if (tv[i]) acc_to_lds(ys, hacc[i], w0[i], lane);
  __syncthreads();
  fwd_epilogue<EPT4>(a, ys, red[0], red[1], row0, n, blockIdx.x);
}

__global__ __launch_bounds__(256, 2) void gcn_bwd_fused4_kernel(const FusedBwd a) {
  extern __shared__ float lds[];
  const int n = a.n;
  const int nkb = (n + 31) >> 5;
  const int np = nkb * 32;
  float* dhs = lds;
  float* buf = lds + np * LDR;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long row0 = (long)blockIdx.x * n;
  int w0[TPW];
  bool tv[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    w0[i] = 32 * (wv + 4 * i);
    tv[i] = wv + 4 * i < nkb;
  }

  GBatch2 g0 = (a.nsup > 0) ? g_first2(slice_sup(a, a.supT[0]), a.ld_sup, nkb, w0, lane) : GBatch2{};
  bwd_prologue<EPT4>(a, dhs, row0, n, np);
  __syncthreads();
  f32x16 dx[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) dx[i] = zero16();
  mlpT_from_lds2(a.w_mlp, a.ld_w, 0, dhs, w0, lane, dx);
  for (int k = 0; k < a.nsup; ++k) {
    const float* GT = slice_sup(a, a.supT[k]);
    {
      f32x16 u[TPW];
#pragma unroll
      for (int i = 0; i < TPW; ++i) u[i] = zero16();
      mlpT_from_lds2(a.w_mlp, a.ld_w, (2 + 2 * k) * CH, dhs, w0, lane, u);
      __syncthreads();
#pragma unroll
      for (int i = 0; i < TPW; ++i)
        if (tv[i]) acc_to_lds(buf, u[i], w0[i], lane);
      if (k == a.adp_index) {
#pragma unroll
        for (int i = 0; i < TPW; ++i) acc_to_global(a.t2 + row0 * a.ld_t, a.ld_t, u[i], w0[i], lane, n);
      }
    }
    __syncthreads();
    f32x16 t[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) t[i] = zero16();
    mlpT_from_lds2(a.w_mlp, a.ld_w, (1 + 2 * k) * CH, dhs, w0, lane, t);
    diffuse2(buf, GT, a.ld_sup, nkb, w0, lane, t, g0);  // dx1 = dP_x1 + A dP_x2
    g0 = g_first2(GT, a.ld_sup, nkb, w0, lane);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < TPW; ++i)
      if (tv[i]) acc_to_lds(buf, t[i], w0[i], lane);
    if (k == a.adp_index) {
#pragma unroll
      for (int i = 0; i < TPW; ++i) acc_to_global(a.t1 + row0 * a.ld_t, a.ld_t, t[i], w0[i], lane, n);
    }
    __syncthreads();
    diffuse2(buf, GT, a.ld_sup, nkb, w0, lane, dx, g0);  // dxg += A dx1
    if (k + 1 < a.nsup) g0 = g_first2(slice_sup(a, a.supT[k + 1]), a.ld_sup, nkb, w0, lane);
  }
  if (!a.dfg) {
#pragma unroll
    for (int i = 0; i < TPW; ++i) acc_to_global(a.dxg + row0 * a.ld_dxg, a.ld_dxg, dx[i], w0[i], lane, n);
    return;
  }
  __syncthreads();  // every wave finished reading buf
#pragma unroll
  for (int i = 0; i < TPW; ++i)
    if (tv[i]) acc_to_lds(buf, dx[i], w0[i], lane);
  __syncthreads();
  bwd_gate_epilogue<EPT4>(a, buf, row0, n);
}

// ---------------------------------------------------------------------------------------------
// Balanced layout (v_mfma_f32_16x16x4_f32), n <= 256: four waves, one per SIMD, equal work.
//
// The 32x32 tile-wave layout lands 7 node tiles (n = 207) on the 4 SIMDs as 2,2,2,1, so the busiest
// SIMD carries 2/7 of the slice instead of 1/4, and a lone workgroup (the last round of a layer,
// or the small T = 1 layers) leaves three SIMDs mostly idle.  Here every product D'[c][w] of the
// slice is cut in four equal quarters: wave (hc, hw) owns channels 16hc..16hc+15 of the 16*NKB
// nodes from hw*16*NKB (NKB 16x16 tiles; np = 32*NKB).  The costs: a support fragment feeds one
// channel half (each G element is loaded twice per slice, ~32 B/clk/CU of L2 at full MFMA rate),
// and the forward mlp's contraction over channels is split between the two channel-half waves,
// whose partial outputs are summed once per slice, in a fixed order, before the epilogue.
// LDS images are channel-half planes [2][np][16] (img_idx<true>): the A fragment of a k-step
// (4 rows x 16 channels) is 256 contiguous bytes, and an accumulator tile (4 consecutive channels
// of 16 rows per lane group) is written back as one ds_write_b128 per lane.
//
// 16x16x4 f32 operand layout (lane l = 16 g + i, i = l & 15, g = l >> 4):
//   A[m = i][k = g], B[k = g][n = i], D register r: D[m = 4 g + r][n = i].
// The mlp contracts over channels straight from the accumulator: k-slot g of MFMA step j is channel
// 4g + j of the half (register j of the accumulator), with the weights indexed to match.
//
// Measured (tools/bench_gcn.py, n = 207, round 2): 5 % slower than the tile-wave layout at T = 12
// and 11-27 % slower at T = 7 / T = 1 (forward and backward), although its busiest SIMD carries
// 13 % fewer MFMA cycles.  Each 32-cycle 16x16x4 MFMA needs a 4-row x 64-B support fragment (four
// cache lines) where the 64-cycle 32x32x2 needs two: four times the L1 line rate per MFMA cycle,
// and a single wave per SIMD when one workgroup per CU is left.  Selectable (layout 3), never
// auto-selected; parity-tested with the other layouts.

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 zero4() {
  f32x4 z = {0.0f, 0.0f, 0.0f, 0.0f};
  return z;
}

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// acc[t][c][w] += sum_v img[v][c] * G[v][w] over the wave's quarter, v < 16 * nb16
template <int NKB>
__device__ __forceinline__ void bal_diffuse(const float* img, const float* G, int ld, int np, int nb16, int hc,
                                            int hw, int lane, f32x4 (&acc)[NKB]) {
  const int g = lane >> 4, i = lane & 15;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)G, (short)0, np * ld * 4, 0x00020000);
  const int voff = (g * ld + hw * 16 * NKB + i) * 4;
  const float* ap = img + (hc * np + g) * 16 + i;
  // batch b = nodes 16b..16b+15 = 4 k-steps; two register sets, batch b+1 loads issued before
  // batch b's MFMAs (a third set, two batches ahead, measured 25 % slower: register pressure)
  float ga[4][NKB], gb[4][NKB];
  auto gload = [&](int b, float (&gr)[4][NKB]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < NKB; ++t) gr[j][t] = bload(rs, voff + 64 * t, (16 * b + 4 * j) * ld * 4);
  };
  auto step = [&](int b, float (&gr)[4][NKB]) {
    float av[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) av[j] = ap[(16 * b + 4 * j) * 16];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < NKB; ++t) acc[t] = mfma4(av[j], gr[j][t], acc[t]);
  };
  gload(0, ga);
  int b = 0;
  for (; b + 2 < nb16; b += 2) {
    gload(b + 1, gb);
    step(b, ga);
    gload(b + 2, ga);
    step(b + 1, gb);
  }
  if (b + 1 < nb16) {
    gload(b + 1, gb);
    step(b, ga);
    step(b + 1, gb);
  } else {
    step(b, ga);
  }
}

// hacc[hp][t][c'][w] += sum_{c in half hc} W[16hp + c'][off + c] * d[t][c][w]
template <int NKB>
__device__ __forceinline__ void bal_mlp(const float* W, int ld_w, int off, int hc, int lane, const f32x4 (&d)[NKB],
                                        f32x4 (&hacc)[2][NKB]) {
  const int g = lane >> 4, i = lane & 15;
  float wf[2][4];
#pragma unroll
  for (int hp = 0; hp < 2; ++hp)
#pragma unroll
    for (int j = 0; j < 4; ++j) wf[hp][j] = W[(long)(16 * hp + i) * ld_w + off + 16 * hc + 4 * g + j];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int hp = 0; hp < 2; ++hp)
#pragma unroll
      for (int t = 0; t < NKB; ++t) hacc[hp][t] = mfma4(wf[hp][j], d[t][j], hacc[hp][t]);
}

// acc[t][c][w] += sum_{c'} W[c'][off + c] * dimg[w][c']     (dP = W^T dh, dimg in planes)
template <int NKB>
__device__ __forceinline__ void bal_mlpT(const float* W, int ld_w, int off, const float* dimg, int np, int hc, int hw,
                                         int lane, f32x4 (&acc)[NKB]) {
  const int g = lane >> 4, i = lane & 15;
  float wa[2][4];
#pragma unroll
  for (int hp = 0; hp < 2; ++hp)
#pragma unroll
    for (int j = 0; j < 4; ++j) wa[hp][j] = W[(long)(16 * hp + 4 * g + j) * ld_w + off + 16 * hc + i];
#pragma unroll
  for (int hp = 0; hp < 2; ++hp) {
    f32x4 bv[NKB];
#pragma unroll
    for (int t = 0; t < NKB; ++t) bv[t] = *(const f32x4*)(dimg + (hp * np + 16 * (hw * NKB + t) + i) * 16 + 4 * g);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < NKB; ++t) acc[t] = mfma4(wa[hp][j], bv[t][j], acc[t]);
  }
}

// the wave's quarter of D'[c][w] into a plane image / into rows w < n of dst (16-B aligned rows)
template <int NKB>
__device__ __forceinline__ void bal_to_img(float* img, const f32x4 (&d)[NKB], int np, int hc, int hw, int lane) {
  const int g = lane >> 4, i = lane & 15;
#pragma unroll
  for (int t = 0; t < NKB; ++t) *(f32x4*)(img + (hc * np + 16 * (hw * NKB + t) + i) * 16 + 4 * g) = d[t];
}

template <int NKB, bool NT>
__device__ __forceinline__ void bal_to_global(float* dst, long ld, const f32x4 (&d)[NKB], int hc, int hw, int lane,
                                              int n) {
  const int g = lane >> 4, i = lane & 15;
#pragma unroll
  for (int t = 0; t < NKB; ++t) {
    const int w = 16 * (hw * NKB + t) + i;
    if (w < n) {
      f32x4* p = (f32x4*)(dst + (long)w * ld + 16 * hc + 4 * g);
      if (NT) __builtin_nontemporal_store(d[t], p);
      else *p = d[t];
    }
  }
}

// the wave's quarter of D'[c][w] (c in half hc, or c' = 16hp + ... for the mlp halves) into padded
// rows S[w][LDR]; ADD: S = d + S
template <int NKB, bool ADD>
__device__ __forceinline__ void bal_to_rows(float* S, const f32x4 (&d)[NKB], int c0, int hw, int lane) {
  const int g = lane >> 4, i = lane & 15;
#pragma unroll
  for (int t = 0; t < NKB; ++t) {
    float* p = S + (16 * (hw * NKB + t) + i) * LDR + c0 + 4 * g;
#pragma unroll
    for (int r = 0; r < 4; ++r) p[r] = ADD ? d[t][r] + p[r] : d[t][r];
  }
}

template <int NKB>
__device__ __forceinline__ void bal_zero(f32x4 (&d)[NKB]) {
#pragma unroll
  for (int t = 0; t < NKB; ++t) d[t] = zero4();
}

template <int NKB>
__global__ __launch_bounds__(256, 2) void gcn_fwd_bal_kernel(const FusedFwd a) {
  extern __shared__ float lds[];
  __shared__ float red[2][256];
  constexpr int np = 32 * NKB;
  const int n = a.n, nb16 = (n + 15) >> 4;
  float* xs = lds;            // x (piece 0), planes
  float* ys = lds + np * CH;  // hop-1 output, planes
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hc = wave & 1, hw = wave >> 1;
  const long row0 = (long)blockIdx.x * n;
  float* hs = (float*)a.h + row0 * a.ld_h;
  for (int e = threadIdx.x; e < np * 8; e += 256) {  // x rows as float4s, rows >= n zero
    const int w = e >> 3, q = e & 7;
    f32x4 v = zero4();
    if (w < n) v = *(const f32x4*)(hs + (long)w * a.ld_h + 4 * q);
    *(f32x4*)(xs + ((q >> 2) * np + w) * 16 + 4 * (q & 3)) = v;
  }
  __syncthreads();
  f32x4 hacc[2][NKB];
  bal_zero(hacc[0]);
  bal_zero(hacc[1]);
  {
    f32x4 x[NKB];
    const int g = lane >> 4, i = lane & 15;
#pragma unroll
    for (int t = 0; t < NKB; ++t) x[t] = *(const f32x4*)(xs + (hc * np + 16 * (hw * NKB + t) + i) * 16 + 4 * g);
    bal_mlp(a.w_mlp, a.ld_w, 0, hc, lane, x, hacc);
  }
  for (int k = 0; k < a.nsup; ++k) {
    const float* G = slice_sup(a, a.sup[k]);
    f32x4 d[NKB];
    bal_zero(d);
    bal_diffuse(xs, G, a.ld_sup, np, nb16, hc, hw, lane, d);
    bal_mlp(a.w_mlp, a.ld_w, (1 + 2 * k) * CH, hc, lane, d, hacc);
    if (a.store_pieces) bal_to_global<NKB, true>(hs + (1 + 2 * k) * CH, a.ld_h, d, hc, hw, lane, n);
    __syncthreads();  // ys is free: every wave finished the previous support's hop 2
    bal_to_img(ys, d, np, hc, hw, lane);
    __syncthreads();
    bal_zero(d);
    bal_diffuse(ys, G, a.ld_sup, np, nb16, hc, hw, lane, d);
    bal_mlp(a.w_mlp, a.ld_w, (2 + 2 * k) * CH, hc, lane, d, hacc);
    if (a.store_pieces) bal_to_global<NKB, true>(hs + (2 + 2 * k) * CH, a.ld_h, d, hc, hw, lane, n);
  }
  // mlp output = channel-half-0 partial + channel-half-1 partial (fixed order), rows [np][LDR]
  float* S = lds;
  __syncthreads();
  if (hc == 1) {
    bal_to_rows<NKB, false>(S, hacc[0], 0, hw, lane);
    bal_to_rows<NKB, false>(S, hacc[1], 16, hw, lane);
  }
  __syncthreads();
  if (hc == 0) {
    bal_to_rows<NKB, true>(S, hacc[0], 0, hw, lane);
    bal_to_rows<NKB, true>(S, hacc[1], 16, hw, lane);
  }
  __syncthreads();
  fwd_epilogue<4 * NKB>(a, S, red[0], red[1], row0, n, blockIdx.x);
}

template <int NKB>
__global__ __launch_bounds__(256, 2) void gcn_bwd_bal_kernel(const FusedBwd a) {
  extern __shared__ float lds[];
  constexpr int np = 32 * NKB;
  const int n = a.n, nb16 = (n + 15) >> 4;
  float* dhs = lds;            // dh, planes
  float* buf = lds + np * CH;  // dP_x2 / dx1, planes
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hc = wave & 1, hw = wave >> 1;
  const long row0 = (long)blockIdx.x * n;

  bwd_prologue<4 * NKB, true>(a, dhs, row0, n, np);
  __syncthreads();
  f32x4 dx[NKB];
  bal_zero(dx);
  bal_mlpT(a.w_mlp, a.ld_w, 0, dhs, np, hc, hw, lane, dx);
  for (int k = 0; k < a.nsup; ++k) {
    const float* GT = slice_sup(a, a.supT[k]);
    {
      f32x4 u[NKB];
      bal_zero(u);
      bal_mlpT(a.w_mlp, a.ld_w, (2 + 2 * k) * CH, dhs, np, hc, hw, lane, u);
      __syncthreads();
      bal_to_img(buf, u, np, hc, hw, lane);
      if (k == a.adp_index) bal_to_global<NKB, false>(a.t2 + row0 * a.ld_t, a.ld_t, u, hc, hw, lane, n);
    }
    __syncthreads();
    f32x4 t[NKB];
    bal_zero(t);
    bal_mlpT(a.w_mlp, a.ld_w, (1 + 2 * k) * CH, dhs, np, hc, hw, lane, t);
    bal_diffuse(buf, GT, a.ld_sup, np, nb16, hc, hw, lane, t);  // dx1 = dP_x1 + A dP_x2
    __syncthreads();
    bal_to_img(buf, t, np, hc, hw, lane);
    if (k == a.adp_index) bal_to_global<NKB, false>(a.t1 + row0 * a.ld_t, a.ld_t, t, hc, hw, lane, n);
    __syncthreads();
    bal_diffuse(buf, GT, a.ld_sup, np, nb16, hc, hw, lane, dx);  // dxg += A dx1
  }
  if (!a.dfg) {
    bal_to_global<NKB, false>(a.dxg + row0 * a.ld_dxg, a.ld_dxg, dx, hc, hw, lane, n);
    return;
  }
  __syncthreads();  // every wave finished reading dhs / buf
  bal_to_rows<NKB, false>(lds, dx, 16 * hc, hw, lane);
  __syncthreads();
  bwd_gate_epilogue<4 * NKB>(a, lds, row0, n);
}

// dst (padded [np][ld_dst], zero outside n x n) = src or src^T
__global__ void pad_copy_kernel(const float* src, int n, int ld_src, float* dst, int ld_dst, int np,
                                int transpose, long src_bstride = 0, long dst_bstride = 0) {
  __shared__ float tile[32][33];
  src += blockIdx.z * src_bstride;  // batched: blockIdx.z walks the matrices
  dst += blockIdx.z * dst_bstride;
  const int bx = blockIdx.x * 32, by = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 8 rows per pass
  for (int r = ty; r < 32; r += 8) {
    const int i = by + r, j = bx + tx;
    tile[r][tx] = (i < n && j < n) ? src[(long)i * ld_src + j] : 0.0f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    if (transpose) {
      const int i = bx + r, j = by + tx;
      if (i < np && j < np) dst[(long)i * ld_dst + j] = tile[tx][r];
    } else {
      const int i = by + r, j = bx + tx;
      if (i < np && j < np) dst[(long)i * ld_dst + j] = tile[r][tx];
    }
  }
}

size_t fused_lds_bytes(int n) {
  const int np = (n + 31) / 32 * 32;
  return (size_t)2 * np * LDR * sizeof(float);
}

template <typename K>
void ensure_lds_attr(K kern) {
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)fused_lds_bytes(512));
}

// layout: 0 = auto, 1 = tile-wave, 2 = 4-wave.  Auto picks the tile-wave layout: measured at
// METR-LA shape (n = 207, 7 tiles) the 4-wave kernel is 10-23 % slower (fewer waves to hide the
// operand latency, plus the dead 8th tile slot); it is only auto-selected when all 8 slots are real.
bool use_4wave(int layout, int nwt) { return layout == 2 || (layout == 0 && nwt == 8); }

inline bool al16(const void* q, long ld) { return ((((uintptr_t)q) & 15) | (ld & 3)) == 0; }

// layout 0 (auto) resolves through GWN_GCN_LAYOUT when set (measurements), else the default below
int auto_layout() {
  static int v = [] {
    const char* e = getenv("GWN_GCN_LAYOUT");
    return e ? atoi(e) : 0;
  }();
  return v;
}

#define GWN_BAL_CASE(K, N) \
  case N: K<N><<<slices, 256, lds, s>>>(a); break;
#define GWN_BAL_SWITCH(K)                                                                    \
  switch (nwt) {                                                                             \
    GWN_BAL_CASE(K, 1) GWN_BAL_CASE(K, 2) GWN_BAL_CASE(K, 3) GWN_BAL_CASE(K, 4)             \
    GWN_BAL_CASE(K, 5) GWN_BAL_CASE(K, 6) GWN_BAL_CASE(K, 7) GWN_BAL_CASE(K, 8)             \
    default: break;                                                                          \
  }

// Support split policy.  Measured per layer (round 2, n = 207, B = 64, 256 CUs; fwd / bwd us,
// whole slices -> split): a unit costs about half a slice, not a third (it still stages the whole
// slice in LDS, hands off its partial sum and one of three runs the epilogue), so the split only pays
// where the whole-slice launch leaves most CUs idle: 64 slices 63.5 -> 37.8 (fwd); 192 slices
// 68 -> 78 / 67 -> 79; 448 slices 115 -> 147 / 111 -> 148; 640 slices 174 -> 212 / 167 -> 201.
// Default: split when every unit gets a CU of its own (slices * nsup <= CUs); GWN_KSPLIT_SLICES
// overrides with a slice-count threshold (0 = never split).
int ksplit_max_slices(int nsup) {
  static int v = [] {
    const char* e = getenv("GWN_KSPLIT_SLICES");
    if (e) return atoi(e);
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

bool gwn_gcn_split_eligible(int c, int n, int planes);
int gwn_gcn_split_fwd_launch(const gwn_gcn_args* g, const FusedFwd& a, hipStream_t s);
int gwn_gcn_bf16_bwd_launch(const gwn_gcn_bwd_args* g, const FusedBwd& a, hipStream_t s);

int gwn_gcn_fused_fwd_launch(const gwn_gcn_args* g, float* bn_part, hipStream_t s) {
  const int nwt = (g->n + 31) / 32;
  GWN_REQUIRE(g->ld_sup >= nwt * 32, "gcn_fwd (fused): supports must be padded to 32*ceil(n/32)");
  GWN_REQUIRE(g->layout >= 0 && g->layout <= 3 && !(g->layout >= 2 && nwt > 8),
              "gcn_fwd (fused): layouts 2 (4-wave) and 3 (balanced) need n <= 256");
  FusedFwd a;
  a.h = g->h; a.ld_h = g->ld_h;
  for (int k = 0; k < 8; ++k) a.sup[k] = (k < g->nsup) ? g->sup[k] : nullptr;
  a.nsup = g->nsup; a.ld_sup = g->ld_sup;
  a.w_mlp = g->w_mlp; a.ld_w = (2 * g->nsup + 1) * CH; a.b_mlp = g->b_mlp;
  a.residual = g->residual; a.z = g->z; a.bn_part = bn_part;
  a.seed_ptr = g->seed_ptr; a.salt = g->salt; a.drop_p = g->drop_p;
  a.n = g->n;
  a.store_pieces = g->no_pieces ? 0 : 1;
  a.bn_rm = g->bn_running_mean; a.bn_rv = g->bn_running_var; a.bn_g = g->bn_weight; a.bn_b = g->bn_bias;
  a.bn_eps = g->bn_eps; a.x_out = g->bn_out;
  a.sup_bstride = g->sup_bstride; a.sup_batch = g->sup_batch;
  a.res_mean = g->residual_mean; a.res_scale = g->residual_scale; a.res_shift = g->residual_shift;
  a.ksplit = 1; a.slices = g->rows / g->n; a.kws = g->ksplit_ws; a.kcnt = g->ksplit_count;
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
  if (g->split_planes) {
    GWN_REQUIRE(gwn_gcn_split_eligible(g->c, g->n, g->split_planes) && g->sup_split && g->w_split && g->nsup > 0,
                "gcn_fwd (split): needs c == 32, an instantiated node-tile count, split supports and weights");
    return gwn_gcn_split_fwd_launch(g, a, s);
  }
  const size_t lds = fused_lds_bytes(g->n);
  static bool attr_set = false;
  if (!attr_set) {
    ensure_lds_attr(gcn_fwd_fused_kernel<512, false>);
    ensure_lds_attr(gcn_fwd_fused_kernel<512, true>);
    ensure_lds_attr(gcn_fwd_fused_kernel<1024, false>);
    ensure_lds_attr(gcn_fwd_fused_kernel<1024, true>);
    ensure_lds_attr(gcn_fwd_fused4_kernel);
    attr_set = true;
  }
  const int slices = g->rows / g->n;
  const int layout = g->layout ? g->layout : auto_layout();
  if (layout == 3) {
    GWN_REQUIRE(nwt <= 8 && al16(a.h, a.ld_h), "gcn_fwd (fused): layout 3 (balanced) needs n <= 256 and 16-B rows of h");
    GWN_BAL_SWITCH(gcn_fwd_bal_kernel)
  } else if (use_4wave(layout, nwt)) gcn_fwd_fused4_kernel<<<slices, 256, lds, s>>>(a);
  else {
    // + one store wave when hop pieces are stored through LDS rows (h 16-B aligned, ld % 4 == 0)
    const bool rows_ok = !(GWN_EXP & 32) && ((((uintptr_t)a.h) & 15) | (a.ld_h & 3)) == 0;
    const int waves = nwt + ((a.store_pieces && rows_ok && nwt < 16) ? 1 : 0);
    a.ksplit = pick_ksplit(g, slices, nwt);
    const int grid = a.ksplit > 1 ? (slices + 7) / 8 * 8 * a.ksplit : slices;
    if (half_last_batch(g->n)) {
      if (waves <= 8) gcn_fwd_fused_kernel<512, true><<<grid, 64 * waves, lds, s>>>(a);
      else gcn_fwd_fused_kernel<1024, true><<<grid, 64 * waves, lds, s>>>(a);
    } else {
      if (waves <= 8) gcn_fwd_fused_kernel<512, false><<<grid, 64 * waves, lds, s>>>(a);
      else gcn_fwd_fused_kernel<1024, false><<<grid, 64 * waves, lds, s>>>(a);
    }
  }
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

int gwn_gcn_fused_bwd_launch(const gwn_gcn_bwd_args* g, const float* const* supT, float* dxg, long ld_dxg,
                             float* t1, float* t2, long ld_t, hipStream_t s) {
  const int nwt = (g->n + 31) / 32;
  GWN_REQUIRE(g->ld_sup >= nwt * 32, "gcn_bwd (fused): supports must be padded to 32*ceil(n/32)");
  GWN_REQUIRE(g->layout >= 0 && g->layout <= 3 && !(g->layout >= 2 && nwt > 8),
              "gcn_bwd (fused): layouts 2 (4-wave) and 3 (balanced) need n <= 256");
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
  if (g->split_planes == 1) return gwn_gcn_bf16_bwd_launch(g, a, s);
  GWN_REQUIRE(g->split_planes == 0, "gcn_bwd (fused): split_planes must be 0 (f32) or 1 (bf16)");
  static bool attr_set = false;
  if (!attr_set) {
    ensure_lds_attr(gcn_bwd_fused_kernel<512, false>);
    ensure_lds_attr(gcn_bwd_fused_kernel<512, true>);
    ensure_lds_attr(gcn_bwd_fused_kernel<1024, false>);
    ensure_lds_attr(gcn_bwd_fused_kernel<1024, true>);
    ensure_lds_attr(gcn_bwd_fused4_kernel);
    attr_set = true;
  }
  const size_t lds = fused_lds_bytes(g->n);
  const int slices = g->rows / g->n;
  const int layout = g->layout ? g->layout : auto_layout();
  if (layout == 3) {
    GWN_REQUIRE(nwt <= 8 && (a.dfg || al16(a.dxg, a.ld_dxg)) &&
                    (a.adp_index < 0 || (al16(a.t1, a.ld_t) && al16(a.t2, a.ld_t))),
                "gcn_bwd (fused): layout 3 (balanced) needs n <= 256 and 16-B rows of dxg / t1 / t2");
    GWN_BAL_SWITCH(gcn_bwd_bal_kernel)
  } else if (use_4wave(layout, nwt)) gcn_bwd_fused4_kernel<<<slices, 256, lds, s>>>(a);
  else {
    a.ksplit = pick_ksplit(g, slices, nwt);
    const int grid = a.ksplit > 1 ? (slices + 7) / 8 * 8 * a.ksplit : slices;
    if (half_last_batch(g->n)) {
      if (nwt <= 8) gcn_bwd_fused_kernel<512, true><<<grid, 64 * nwt, lds, s>>>(a);
      else gcn_bwd_fused_kernel<1024, true><<<grid, 64 * nwt, lds, s>>>(a);
    } else {
      if (nwt <= 8) gcn_bwd_fused_kernel<512, false><<<grid, 64 * nwt, lds, s>>>(a);
      else gcn_bwd_fused_kernel<1024, false><<<grid, 64 * nwt, lds, s>>>(a);
    }
  }
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

// diagnostics: resident workgroups per CU of the fused kernels for n nodes (HIP occupancy API),
// for the layout the launchers pick by default
extern "C" int gwn_fused_occupancy(int n, int backward) {
  const int nwt = (n + 31) / 32;
  const size_t lds = fused_lds_bytes(n);
  int blocks = -1;
  hipError_t e;
  if (use_4wave(0, nwt)) {
    if (backward) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, gcn_bwd_fused4_kernel, 256, lds);
    else e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, gcn_fwd_fused4_kernel, 256, lds);
  } else if (backward) {
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, gcn_bwd_fused_kernel<1024, false>, 64 * nwt, lds);
  } else {
    // training forward: the compute waves plus the store wave
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, gcn_fwd_fused_kernel<1024, false>,
                                                     64 * (nwt < 16 ? nwt + 1 : nwt), lds);
  }
  return e == hipSuccess ? blocks : -(int)e;
}

extern "C" int gwn_transpose(const float* src, int n, int ld_src, float* dst, int ld_dst, hipStream_t s) {
  GWN_REQUIRE(n > 0, "transpose: bad shape");
  dim3 grid((n + 31) / 32, (n + 31) / 32);
  pad_copy_kernel<<<grid, 256, 0, s>>>(src, n, ld_src, dst, ld_dst, n, 1);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

extern "C" int gwn_pad_square(const float* src, int n, int ld_src, float* dst, int np, int ld_dst, int transpose,
                              hipStream_t s) {
  GWN_REQUIRE(n > 0 && np >= n && ld_dst >= np, "pad_square: bad shape");
  dim3 grid((np + 31) / 32, (np + 31) / 32);
  pad_copy_kernel<<<grid, 256, 0, s>>>(src, n, ld_src, dst, ld_dst, np, transpose);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

extern "C" int gwn_pad_square_batched(const float* src, int batch, long src_bstride, int n, int ld_src, float* dst,
                                      int np, int ld_dst, long dst_bstride, int transpose, hipStream_t s) {
  GWN_REQUIRE(n > 0 && np >= n && ld_dst >= np && batch > 0 && batch <= 65535 && src_bstride >= (long)n * ld_src &&
                  dst_bstride >= (long)np * ld_dst,
              "pad_square_batched: bad shape");
  dim3 grid((np + 31) / 32, (np + 31) / 32, batch);
  pad_copy_kernel<<<grid, 256, 0, s>>>(src, n, ld_src, dst, ld_dst, np, transpose, src_bstride, dst_bstride);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

// =============================================================================================
// Split-bf16 forward (the same schedule as gcn_fwd_fused_kernel on v_mfma_f32_32x32x16_bf16).
//
// Every fp32 operand x is carried as P bf16 pieces x = x_0 + x_1 (+ x_2) + r (x_0 = bf16(x),
// x_1 = bf16(x - x_0), ...; each difference is exact in fp32), and a product a*b is the sum of
// the piece products a_i*b_j with i + j < P, accumulated in fp32.  P = 3 (6 products) leaves a
// representation error of 2^-24 relative per operand: the results stay at fp32 accuracy (the
// tests hold it to the fp32 path's tolerances), at 6 x 32 cycles per 16-deep K step against
// 8 x 64 cycles for the f32 MFMA: 2.67x the matrix throughput.  P = 2 (3 products, ~1e-5
// relative) is kept for measurements only.
//
// Operand images:
//   * node features (A operand, LDS): P planes of [channel][node] bf16, row stride SB bytes
//     (SB = 16 mod 256: the 16 lanes of a ds_read_b128 group hit 16 distinct 16-B bank slots);
//   * supports (B operand, global / L2): P planes of G^T [w][v] bf16 (gwn_split_supports), read as
//     two 16-B buffer loads per lane per 32-node K batch;
//   * mlp weights (A operand of the channel contraction): P planes [piece][c'][32], the 32 inputs of
//     each piece in "lane order" j = 16 s + 8 h + i (gwn_split_mlp_weights): for pieces >= 1 that
//     is the MFMA accumulator row order crow(8 s + i, h), so the hop accumulator is the B operand
//     as it stands (K permuted consistently on both sides); for piece 0 it is the channel order.
// K permutation of the diffusion: K step j of batch b, lane half h, element i is node
// 32 b + 16 h + 8 j + i, so each lane reads 32 contiguous bytes of a G^T row / LDS plane row.

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int split_row_bytes(int np) { return ((2 * np - 16 + 255) / 256) * 256 + 16; }
constexpr int cmax(int a, int b) { return a > b ? a : b; }
// bytes of the forward kernel's first LDS region: the P node-feature planes, and the fp32
// [np][LDR] rows the epilogue stages there (the larger of the two for P = 1)
constexpr int split_xs_bytes(int np, int P) { return cmax(P * 32 * split_row_bytes(np), np * LDR * 4); }

template <int P>
__device__ __forceinline__ void split8(const float* x, bf16x8* out) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    float r = x[i];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const __bf16 h = (__bf16)r;
      out[p][i] = h;
      if (p + 1 < P) r -= (float)h;
    }
  }
}

// acc += sum_{i+j<P} a_i b_j, smallest terms first
template <int P>
__device__ __forceinline__ f32x16 mfma_split(const bf16x8* a, const bf16x8* b, f32x16 acc) {
#pragma unroll
  for (int s = P - 1; s >= 0; --s)
#pragma unroll
    for (int i = 0; i <= s; ++i) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[s - i], acc, 0, 0, 0);
  return acc;
}

template <int P, int PD>
struct SplitPre {
  i32x4 v[PD][P][2];
};

struct SplitG {
  __amdgpu_buffer_rsrc_t rs;
  int voff;    // this lane's byte offset in a plane: row w, K half
  int planeb;  // bytes per plane
};

__device__ __forceinline__ SplitG split_g(const void* gs, int np, int ldg, int P, int w, int half) {
  SplitG g;
  g.planeb = np * ldg * 2;
  g.rs = __builtin_amdgcn_make_buffer_rsrc((void*)gs, (short)0, P * g.planeb, 0x00020000);
  g.voff = (w * ldg + 16 * half) * 2;
  return g;
}

__device__ __forceinline__ i32x4 gload16(const SplitG& g, int extra, int soff) {
  return __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(g.rs, g.voff + extra, soff, 0));
}

template <int P, int PD>
__device__ __forceinline__ SplitPre<P, PD> split_pre(const SplitG& g) {
  SplitPre<P, PD> s;
#pragma unroll
  for (int b = 0; b < PD; ++b)
#pragma unroll
    for (int p = 0; p < P; ++p) {
      s.v[b][p][0] = gload16(g, 0, p * g.planeb + b * 64);
      s.v[b][p][1] = gload16(g, 16, p * g.planeb + b * 64);
    }
  return s;
}

// acc[c][w] += sum_v img[v][c] * G[v][w]: img = LDS planes, G = split support (first PD batches in g0)
template <int NKB, int P, int PD>
__device__ __forceinline__ f32x16 diffuse_split(const char* img, const SplitG& g, int lane, f32x16 acc,
                                                const SplitPre<P, PD>& g0) {
  constexpr int SB = split_row_bytes(NKB * 32);
  constexpr int PLX = 32 * SB;
  const int col = lane & 31, half = lane >> 5;
  const char* ab = img + col * SB + half * 32;
  i32x4 gv[NKB][P][2];
#pragma unroll
  for (int b = 0; b < PD && b < NKB; ++b)
#pragma unroll
    for (int p = 0; p < P; ++p) {
      gv[b][p][0] = g0.v[b][p][0];
      gv[b][p][1] = g0.v[b][p][1];
    }
#pragma unroll
  for (int b = 0; b < NKB; ++b) {
    if (b + PD < NKB) {
#pragma unroll
      for (int p = 0; p < P; ++p) {
        gv[b + PD][p][0] = gload16(g, 0, p * g.planeb + (b + PD) * 64);
        gv[b + PD][p][1] = gload16(g, 16, p * g.planeb + (b + PD) * 64);
      }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      bf16x8 av[P], bv[P];
#pragma unroll
      for (int p = 0; p < P; ++p) {
        av[p] = *(const bf16x8*)(ab + p * PLX + b * 64 + j * 16);
        bv[p] = __builtin_bit_cast(bf16x8, gv[b][p][j]);
      }
      acc = mfma_split<P>(av, bv, acc);
    }
  }
  return acc;
}

template <int P>
struct SplitW {
  bf16x8 v[2][P];
};

// weight fragments of mlp piece `piece` (A operand: row c' = lane & 31, lane-order inputs)
template <int P>
__device__ __forceinline__ SplitW<P> split_w(const void* ws, int piece, int lane) {
  const int col = lane & 31, half = lane >> 5;
  SplitW<P> f;
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int p = 0; p < P; ++p)
      f.v[s][p] = *((const bf16x8*)ws + ((piece * P + p) * 32 + col) * 4 + s * 2 + half);
  return f;
}

// acc[c'][w] += sum_c W[c'][c] * D[c][w] with D = the hop accumulator (rows in crow order)
template <int P>
__device__ __forceinline__ f32x16 mlp_acc_split(const SplitW<P>& wf, const f32x16& d, f32x16 acc) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    float x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = d[8 * s + i];
    bf16x8 bv[P];
    split8<P>(x, bv);
    acc = mfma_split<P>(wf.v[s], bv, acc);
  }
  return acc;
}

// hop accumulator D[c][w] -> the LDS planes [c][w] (the next hop's A operand)
template <int NKB, int P>
__device__ __forceinline__ void acc_to_planes(char* img, const f32x16& d, int w0, int lane) {
  constexpr int SB = split_row_bytes(NKB * 32);
  constexpr int PLX = 32 * SB;
  const int col = lane & 31, half = lane >> 5;
  char* base = img + (w0 + col) * 2;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float v = d[r];
    const int c = crow(r, half);
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const __bf16 h = (__bf16)v;
      *(__bf16*)(base + p * PLX + c * SB) = h;
      if (p + 1 < P) v -= (float)h;
    }
  }
}

template <int NKB, int P, int PD>
__global__ __launch_bounds__(64 * NKB) void gcn_fwd_split_kernel(const FusedFwd a, const void* gsplit,
                                                                 long gstride, int ldg, const void* wsplit) {
  constexpr int NP = NKB * 32;
  constexpr int SB = split_row_bytes(NP);
  extern __shared__ float lds[];
  __shared__ float red[2][64 * NKB];
  char* xs = (char*)lds;
  char* ys = xs + split_xs_bytes(NP, P);  // the first region also stages the fp32 epilogue rows
  const int n = a.n;
  const int lane = threadIdx.x & 63, w0 = (threadIdx.x >> 6) * 32;
  const int col = lane & 31, half = lane >> 5;
  const long row0 = (long)blockIdx.x * n;
  const float* hs = a.h + row0 * a.ld_h;

  SplitG g = split_g(gsplit, NP, ldg, P, w0 + col, half);
  SplitPre<P, PD> g0{};
  if (a.nsup > 0) g0 = split_pre<P, PD>(g);
  SplitW<P> wf = split_w<P>(wsplit, 0, lane);
  // stage the node features as P planes [c][v] (rows >= n zero)
  for (int e = threadIdx.x; e < NP * CH; e += blockDim.x) {
    const int w = e >> 5, c = e & 31;
    float v = (w < n) ? hs[(long)w * a.ld_h + c] : 0.0f;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const __bf16 h = (__bf16)v;
      *(__bf16*)(xs + p * 32 * SB + c * SB + w * 2) = h;
      if (p + 1 < P) v -= (float)h;
    }
  }
  // mlp piece 0 straight from the rows of h (B operand: row w, channels 16 s + 8 h + i)
  f32x16 hacc = zero16();
  {
    const int w = w0 + col;
    const float* xr = hs + (long)min(w, n - 1) * a.ld_h + 8 * half;
    const float keep = (w < n) ? 1.0f : 0.0f;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const float4 q0 = *(const float4*)(xr + 16 * s);
      const float4 q1 = *(const float4*)(xr + 16 * s + 4);
      float x[8] = {q0.x * keep, q0.y * keep, q0.z * keep, q0.w * keep,
                    q1.x * keep, q1.y * keep, q1.z * keep, q1.w * keep};
      bf16x8 bv[P];
      split8<P>(x, bv);
      hacc = mfma_split<P>(wf.v[s], bv, hacc);
    }
  }
  __syncthreads();
  for (int k = 0; k < a.nsup; ++k) {
    wf = split_w<P>(wsplit, 1 + 2 * k, lane);
    f32x16 d = diffuse_split<NKB, P, PD>(xs, g, lane, zero16(), g0);
    g0 = split_pre<P, PD>(g);  // hop 2 re-reads the same support
    hacc = mlp_acc_split<P>(wf, d, hacc);
    wf = split_w<P>(wsplit, 2 + 2 * k, lane);
    __syncthreads();  // ys is free once every wave finished the previous support's hop 2
    acc_to_planes<NKB, P>(ys, d, w0, lane);
    if (a.store_pieces) acc_to_global((float*)hs + (1 + 2 * k) * CH, a.ld_h, d, w0, lane, n);
    __syncthreads();
    d = diffuse_split<NKB, P, PD>(ys, g, lane, zero16(), g0);
    if (k + 1 < a.nsup) {
      g = split_g((const char*)gsplit + (k + 1) * gstride * 2, NP, ldg, P, w0 + col, half);
      g0 = split_pre<P, PD>(g);
    }
    hacc = mlp_acc_split<P>(wf, d, hacc);
    if (a.store_pieces) acc_to_global((float*)hs + (2 + 2 * k) * CH, a.ld_h, d, w0, lane, n);
  }
  __syncthreads();
  acc_to_lds((float*)xs, hacc, w0, lane);
  __syncthreads();
  fwd_epilogue<EPT>(a, (float*)xs, red[0], red[1], row0, n, blockIdx.x);
}

// dst[s][p][w][v] (bf16, [np][ld_dst] per plane) = piece p of G_s^T, G_s = padded support [np][ld_src]
struct SplitSupArgs {
  const float* src[8];
};

template <int P>
__global__ void split_supports_kernel(SplitSupArgs sa, int np, int ld_src, __bf16* dst, long sup_stride,
                                      int ld_dst) {
  __shared__ float tile[32][33];
  const float* src = sa.src[blockIdx.z];
  __bf16* out = dst + blockIdx.z * sup_stride;
  const long plane = (long)np * ld_dst;
  const int bx = blockIdx.x * 32, by = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int r = ty; r < 32; r += 8) tile[r][tx] = src[(long)(by + r) * ld_src + bx + tx];  // G[v = by+r][w = bx+tx]
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    float v = tile[tx][r];  // G[by + tx][bx + r] -> G^T[w = bx + r][v = by + tx]
    __bf16* o = out + (long)(bx + r) * ld_dst + by + tx;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const __bf16 h = (__bf16)v;
      o[p * plane] = h;
      if (p + 1 < P) v -= (float)h;
    }
  }
}

struct SplitWArgs {
  const float* w[16];
};

// dst[l][piece][p][c'][j] = piece p of W_l[c'][piece*32 + ch(j)], j = 16 s + 8 h + i in lane order
template <int P>
__global__ void split_mlp_kernel(SplitWArgs wa, int width, __bf16* dst, long layer_stride) {
  const int l = blockIdx.y;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;  // over pieces * 32 * 32
  const int npieces = width / CH;
  if (e >= npieces * CH * CH) return;
  const int j = e & 31, cp = (e >> 5) & 31, piece = e >> 10;
  const int s = j >> 4, h = (j >> 3) & 1, i = j & 7;
  const int ch = (piece == 0) ? j : crow(8 * s + i, h);
  float v = wa.w[l][(long)cp * width + piece * CH + ch];
  __bf16* o = dst + l * layer_stride + ((long)(piece * P) * CH + cp) * CH + j;
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const __bf16 hh = (__bf16)v;
    o[(long)p * CH * CH] = hh;
    if (p + 1 < P) v -= (float)hh;
  }
}

// dst[l][piece][c][c'] (bf16) = W_l[c'][piece*32 + c]: the A operand of the backward's channel
// contraction dP = W^T dh (row c, inputs c' in plain order, matching the dh image rows)
__global__ void mlpT_bf16_kernel(SplitWArgs wa, int width, __bf16* dst, long layer_stride) {
  const int l = blockIdx.y;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;  // over pieces * 32 * 32
  const int npieces = width / CH;
  if (e >= npieces * CH * CH) return;
  const int cp = e & 31, c = (e >> 5) & 31, piece = e >> 10;
  dst[l * layer_stride + e] = (__bf16)wa.w[l][(long)cp * width + piece * CH + c];
}

// ---------------------------------------------------------------------------------------------
// bf16 backward (the schedule of gcn_bwd_fused_kernel with bf16 operands, fp32 accumulation):
//   dh image: LDS rows [w][32 c'] bf16 (row stride DHB), the B operand of dP = W^T dh;
//   hop image: one bf16 plane [c][v] (the A operand of the diffusions through G^T);
//   supports: gwn_split_supports(planes = 1) of the TRANSPOSED supports, i.e. planes of A [w][v].
constexpr int DHB = 80;  // 64 B of bf16 + 16: the 16 lanes of a ds_read_b128 group hit distinct bank slots

__device__ __forceinline__ f32x16 mlpT_bf16(const void* wt, int piece, const char* dhimg, int w0, int lane,
                                            f32x16 acc) {
  const int col = lane & 31, half = lane >> 5;
  const bf16x8* wp = (const bf16x8*)wt + (piece * CH + col) * 4 + half;  // row c = col, inputs 8h + 16s
  const char* bp = dhimg + (w0 + col) * DHB + half * 16;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const bf16x8 a = wp[2 * s];
    const bf16x8 b = *(const bf16x8*)(bp + 32 * s);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  }
  return acc;
}

template <int NKB, int PD>
__global__ __launch_bounds__(64 * NKB) void gcn_bwd_bf16_kernel(const FusedBwd a, const void* gsplit, long gstride,
                                                                int ldg, const void* wtsplit) {
  constexpr int NP = NKB * 32;
  constexpr int DHI = NP * DHB;        // bf16 dh image; the fp32 rows [w][LDR] of the prologue dh
                                       // and the epilogue dx are staged at the base as well
  extern __shared__ float lds[];
  char* dhimg = (char*)lds;            // aliases the prologue staging (converted in registers)
  char* img = dhimg + DHI;
  float* stg = lds;
  const int n = a.n;
  const int lane = threadIdx.x & 63, w0 = (threadIdx.x >> 6) * 32;
  const int col = lane & 31, half = lane >> 5;
  const long row0 = (long)blockIdx.x * n;

  SplitG g = split_g(gsplit, NP, ldg, 1, w0 + col, half);
  SplitPre<1, PD> g0{};
  if (a.nsup > 0) g0 = split_pre<1, PD>(g);
  bwd_prologue<EPT>(a, stg, row0, n, NP);  // dh (fp32) for rows < np, zero beyond n
  __syncthreads();
  {
    // fp32 staging -> bf16 dh image (each thread converts the same 16 elements it reads)
    float v[EPT];
    const int c = threadIdx.x & 31, wb = threadIdx.x >> 5, ws = blockDim.x >> 5;
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int w = wb + i * ws;
      v[i] = (w < NP) ? stg[w * LDR + c] : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int w = wb + i * ws;
      if (w < NP) *(__bf16*)(dhimg + w * DHB + c * 2) = (__bf16)v[i];
    }
  }
  __syncthreads();
  f32x16 dx = mlpT_bf16(wtsplit, 0, dhimg, w0, lane, zero16());
  for (int k = 0; k < a.nsup; ++k) {
    const f32x16 u = mlpT_bf16(wtsplit, 2 + 2 * k, dhimg, w0, lane, zero16());
    __syncthreads();  // img free: every wave finished the previous diffusion
    acc_to_planes<NKB, 1>(img, u, w0, lane);
    if (k == a.adp_index) acc_to_global(a.t2 + row0 * a.ld_t, a.ld_t, u, w0, lane, n);
    __syncthreads();
    f32x16 t = mlpT_bf16(wtsplit, 1 + 2 * k, dhimg, w0, lane, zero16());
    t = diffuse_split<NKB, 1, PD>(img, g, lane, t, g0);  // dx1 = dP_x1 + A dP_x2
    g0 = split_pre<1, PD>(g);
    __syncthreads();
    acc_to_planes<NKB, 1>(img, t, w0, lane);
    if (k == a.adp_index) acc_to_global(a.t1 + row0 * a.ld_t, a.ld_t, t, w0, lane, n);
    __syncthreads();
    dx = diffuse_split<NKB, 1, PD>(img, g, lane, dx, g0);  // dxg += A dx1
    if (k + 1 < a.nsup) {
      g = split_g((const char*)gsplit + (k + 1) * gstride * 2, NP, ldg, 1, w0 + col, half);
      g0 = split_pre<1, PD>(g);
    }
  }
  if (!a.dfg) {
    acc_to_global(a.dxg + row0 * a.ld_dxg, a.ld_dxg, dx, w0, lane, n);
    return;
  }
  __syncthreads();  // every wave finished reading the images
  acc_to_lds(stg, dx, w0, lane);
  __syncthreads();
  bwd_gate_epilogue<EPT>(a, stg, row0, n);
}

template <int NKB>
void launch_bf16_bwd(const FusedBwd& a, const gwn_gcn_bwd_args* g, int slices, hipStream_t s) {
  constexpr int NP = NKB * 32;
  // whole-hop prefetch where a workgroup holds a CU on its own anyway (9+ node tiles); below that
  // its extra registers would cost the second co-resident workgroup (N=207: 144 vs 104 VGPRs)
  constexpr int PD = NKB >= 9 ? (NKB < GWN_BF16_PD ? NKB : GWN_BF16_PD) : (NKB > 1 ? 2 : 1);
  const size_t lds = (size_t)cmax(NP * LDR * 4, NP * DHB + 32 * split_row_bytes(NP));
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gcn_bwd_bf16_kernel<NKB, PD>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    attr_set = true;
  }
  gcn_bwd_bf16_kernel<NKB, PD><<<slices, 64 * NKB, lds, s>>>(a, g->supT_split, g->sup_split_stride, g->ld_split,
                                                             g->wT_split);
}

template <int NKB, int P, int PD>
void launch_split(const FusedFwd& a, const gwn_gcn_args* g, int slices, hipStream_t s) {
  constexpr int NP = NKB * 32;
  const size_t lds = (size_t)split_xs_bytes(NP, P) + P * 32 * split_row_bytes(NP);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gcn_fwd_split_kernel<NKB, P, PD>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  gcn_fwd_split_kernel<NKB, P, PD><<<slices, 64 * NKB, lds, s>>>(a, g->sup_split, g->sup_split_stride,
                                                                  g->ld_split, g->w_split);
}

}  // namespace

bool gwn_gcn_split_eligible(int c, int n, int planes) {
  const int nkb = (n + 31) / 32;
  return c == CH && n > 0 && ((planes == 1 && nkb <= 16) || (planes == 3 && (nkb == 1 || nkb == 7 || nkb == 11)) ||
                              (planes == 2 && nkb == 7));
}

// bf16 operands (planes = 1): one instantiation per node-tile count
// The whole hop's support fragments (NKB batches x 32 B per lane) are issued one phase ahead of
// the hop: with bf16 operands a batch is 2 MFMAs (64 cycles), far shorter than an L2 round trip,
// so a short prefetch distance leaves every batch waiting on its loads
template <int NKB>
void launch_bf16_fwd(const FusedFwd& a, const gwn_gcn_args* g, int slices, hipStream_t s) {
  launch_split<NKB, 1, (NKB < GWN_BF16_PD ? NKB : GWN_BF16_PD)>(a, g, slices, s);
}

int gwn_gcn_split_fwd_launch(const gwn_gcn_args* g, const FusedFwd& a, hipStream_t s) {
  const int nkb = (g->n + 31) / 32;
  const int slices = g->rows / g->n;
  GWN_REQUIRE(g->ld_split >= nkb * 32 && g->sup_split_stride % 8 == 0 && g->ld_split % 8 == 0,
              "gcn_fwd (split): bad split-support layout");
  if (g->split_planes == 1) {
    switch (nkb) {
      case 1: launch_bf16_fwd<1>(a, g, slices, s); break;
      case 2: launch_bf16_fwd<2>(a, g, slices, s); break;
      case 3: launch_bf16_fwd<3>(a, g, slices, s); break;
      case 4: launch_bf16_fwd<4>(a, g, slices, s); break;
      case 5: launch_bf16_fwd<5>(a, g, slices, s); break;
      case 6: launch_bf16_fwd<6>(a, g, slices, s); break;
      case 7: launch_bf16_fwd<7>(a, g, slices, s); break;
      case 8: launch_bf16_fwd<8>(a, g, slices, s); break;
      case 9: launch_bf16_fwd<9>(a, g, slices, s); break;
      case 10: launch_bf16_fwd<10>(a, g, slices, s); break;
      case 11: launch_bf16_fwd<11>(a, g, slices, s); break;
      case 12: launch_bf16_fwd<12>(a, g, slices, s); break;
      case 13: launch_bf16_fwd<13>(a, g, slices, s); break;
      case 14: launch_bf16_fwd<14>(a, g, slices, s); break;
      case 15: launch_bf16_fwd<15>(a, g, slices, s); break;
      default: launch_bf16_fwd<16>(a, g, slices, s); break;
    }
  } else if (g->split_planes == 3) {
    if (nkb == 7) launch_split<7, 3, 2>(a, g, slices, s);
    else if (nkb == 11) launch_split<11, 3, 2>(a, g, slices, s);
    else launch_split<1, 3, 1>(a, g, slices, s);
  } else {
    launch_split<7, 2, 2>(a, g, slices, s);
  }
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

int gwn_gcn_bf16_bwd_launch(const gwn_gcn_bwd_args* g, const FusedBwd& a, hipStream_t s) {
  const int nkb = (g->n + 31) / 32;
  const int slices = g->rows / g->n;
  GWN_REQUIRE(gwn_gcn_split_eligible(g->c, g->n, 1) && g->supT_split && g->wT_split && g->nsup > 0 &&
                  g->ld_split >= nkb * 32 && g->sup_split_stride % 8 == 0 && g->ld_split % 8 == 0 && a.sup_batch <= 1,
              "gcn_bwd (bf16): needs c == 32, n <= 512, nsup >= 1, split transposed supports and weights");
  switch (nkb) {
    case 1: launch_bf16_bwd<1>(a, g, slices, s); break;
    case 2: launch_bf16_bwd<2>(a, g, slices, s); break;
    case 3: launch_bf16_bwd<3>(a, g, slices, s); break;
    case 4: launch_bf16_bwd<4>(a, g, slices, s); break;
    case 5: launch_bf16_bwd<5>(a, g, slices, s); break;
    case 6: launch_bf16_bwd<6>(a, g, slices, s); break;
    case 7: launch_bf16_bwd<7>(a, g, slices, s); break;
    case 8: launch_bf16_bwd<8>(a, g, slices, s); break;
    case 9: launch_bf16_bwd<9>(a, g, slices, s); break;
    case 10: launch_bf16_bwd<10>(a, g, slices, s); break;
    case 11: launch_bf16_bwd<11>(a, g, slices, s); break;
    case 12: launch_bf16_bwd<12>(a, g, slices, s); break;
    case 13: launch_bf16_bwd<13>(a, g, slices, s); break;
    case 14: launch_bf16_bwd<14>(a, g, slices, s); break;
    case 15: launch_bf16_bwd<15>(a, g, slices, s); break;
    default: launch_bf16_bwd<16>(a, g, slices, s); break;
  }
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

extern "C" int gwn_gcn_split_supported(int c, int n, int planes) { return gwn_gcn_split_eligible(c, n, planes) ? 1 : 0; }

extern "C" long gwn_split_support_elems(int n, int planes) {
  const long np = (n + 31) / 32 * 32;
  return (long)planes * np * np;
}

extern "C" int gwn_split_supports(const float* const* sup, int nsup, int n, int ld_sup, int planes, void* dst,
                                  long sup_stride_elems, int ld_dst, hipStream_t s) {
  const int np = (n + 31) / 32 * 32;
  GWN_REQUIRE(nsup >= 1 && nsup <= 8 && planes >= 1 && planes <= 3 && ld_sup >= np && ld_dst >= np &&
                  sup_stride_elems >= (long)planes * np * ld_dst,
              "split_supports: bad shape");
  SplitSupArgs sa;
  for (int k = 0; k < 8; ++k) sa.src[k] = k < nsup ? sup[k] : nullptr;
  dim3 grid(np / 32, np / 32, nsup);
  if (planes == 3) split_supports_kernel<3><<<grid, 256, 0, s>>>(sa, np, ld_sup, (__bf16*)dst, sup_stride_elems, ld_dst);
  else if (planes == 2) split_supports_kernel<2><<<grid, 256, 0, s>>>(sa, np, ld_sup, (__bf16*)dst, sup_stride_elems, ld_dst);
  else split_supports_kernel<1><<<grid, 256, 0, s>>>(sa, np, ld_sup, (__bf16*)dst, sup_stride_elems, ld_dst);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

extern "C" long gwn_split_mlp_elems(int nsup, int planes) { return (long)(2 * nsup + 1) * planes * CH * CH; }

extern "C" int gwn_split_mlp_weights(const float* const* w, int nlayers, int nsup, int planes, void* dst,
                                     long layer_stride_elems, hipStream_t s) {
  const int width = (2 * nsup + 1) * CH;
  GWN_REQUIRE(nlayers >= 1 && nlayers <= 16 && nsup >= 0 && planes >= 1 && planes <= 3 &&
                  layer_stride_elems >= gwn_split_mlp_elems(nsup, planes),
              "split_mlp_weights: bad shape");
  SplitWArgs wa;
  for (int l = 0; l < 16; ++l) wa.w[l] = l < nlayers ? w[l] : nullptr;
  const int total = (2 * nsup + 1) * CH * CH;
  dim3 grid((total + 255) / 256, nlayers);
  if (planes == 3) split_mlp_kernel<3><<<grid, 256, 0, s>>>(wa, width, (__bf16*)dst, layer_stride_elems);
  else if (planes == 2) split_mlp_kernel<2><<<grid, 256, 0, s>>>(wa, width, (__bf16*)dst, layer_stride_elems);
  else split_mlp_kernel<1><<<grid, 256, 0, s>>>(wa, width, (__bf16*)dst, layer_stride_elems);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

extern "C" long gwn_bf16_mlpT_elems(int nsup) { return (long)(2 * nsup + 1) * CH * CH; }

extern "C" int gwn_bf16_mlpT_weights(const float* const* w, int nlayers, int nsup, void* dst, long layer_stride_elems,
                                     hipStream_t s) {
  const int width = (2 * nsup + 1) * CH;
  GWN_REQUIRE(nlayers >= 1 && nlayers <= 16 && nsup >= 0 && layer_stride_elems >= gwn_bf16_mlpT_elems(nsup),
              "bf16_mlpT_weights: bad shape");
  SplitWArgs wa;
  for (int l = 0; l < 16; ++l) wa.w[l] = l < nlayers ? w[l] : nullptr;
  const int total = (2 * nsup + 1) * CH * CH;
  dim3 grid((total + 255) / 256, nlayers);
  mlpT_bf16_kernel<<<grid, 256, 0, s>>>(wa, width, (__bf16*)dst, layer_stride_elems);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}
