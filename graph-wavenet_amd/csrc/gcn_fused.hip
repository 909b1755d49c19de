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
// Wave layout: one wave per 32-node tile (up to 16 waves, n <= 512).
//
// Two schedules of the diffusion chain:
//   * "power" (gcn_fwd_pow_kernel / gcn_bwd_pow_kernel, shared supports with their squares given):
//     both hops of a support come from the node features in ONE pass over the LDS image, against
//     A_k and A_k^2 (two accumulators per A-operand read), so the waves of a slice never wait on
//     each other between hops; the backward diffuses dh through A_k^T and (A_k^2)^T and applies
//     the transposed mlp per node (dx = W0^T dh + sum_k W1k^T A_k^T dh + W2k^T (A_k^2)^T dh).
//   * "chain" (gcn_fwd_fused_kernel / gcn_bwd_fused_kernel): hop 2 diffuses hop 1's output,
//     staged through LDS between barriers (per-sample supports, or no squares given).
//
// Contract on the supports: [np][ld] with np = 32*ceil(n/32) <= ld, ZERO outside [n][n]
// (the executor keeps padded copies), so the K loop runs whole 32-node batches unguarded.
#include "gwn_internal.h"
#include <type_traits>

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int CH = 32;   // channels (one MFMA tile)
constexpr int LDR = 33;  // LDS row stride (floats): conflict-free row and column reads
constexpr int KB = 16;   // k-steps (32 nodes) per batch of the K loop
constexpr int EPT = 16;  // tile-wave epilogue elements per thread: np*32 / (64*np/32) = 16 for every n

struct FusedFwd {
  const float* h; long ld_h;
  const float* sup[8]; int nsup, ld_sup;
  const float* w_mlp; int ld_w; const float* b_mlp;
  const float* w_t;  // w_mlp transposed [ld_w][32] (power forward: coalesced fragment rows)
  const float* residual; float* z; float* bn_part;
  const unsigned long long* seed_ptr; unsigned long long salt; float drop_p;
  int n;
  int store_pieces;  // 0: hop outputs not written to h (inference: no backward follows)
  // eval BatchNorm folded into the epilogue (running statistics): x_out = bn(z); z not written
  const float* bn_rm; const float* bn_rv; const float* bn_g; const float* bn_b; float bn_eps; float* x_out;
  long sup_bstride; int sup_batch;  // per-sample supports (sup_batch > 1): sample b = slice % sup_batch
  const float* res_mean; const float* res_scale; const float* res_shift;  // (residual - mean) * scale + shift
  int ksplit, slices; float* kws; int* kcnt;  // support split (ksplit > 1): see unit_of()
  int bn_slots;  // t16 kernels: BN partial slots to write (those past the grid get count 0)
  void* xg4; int xg4_k;  // bf16 t16 kernel: X and support xg4_k's hop 1 in the tiled activation layout
  void* pb; long ld_pb;  // bf16 t16 kernel: the hop pieces as bf16 [rows][ld_pb] instead of h's columns
  // f32 t16 forward: the layer's gated TCN computed in the phase staging (gwn_gcn_args.tcn; x NULL =
  // off): xg = tanh(f) sigmoid(g) of taps x[r], x[r + tap_rows] (minus mean) straight into the
  // slice images, and to h's piece 0, fg and the skip rows
  // with bn (bn.part != NULL): x is the layer below's pre-BN z and its BatchNorm is finalized
  // from bn.part in every workgroup (gwn_tcn_args.bn): w / b are then the raw weights
  struct {
    const float* x; const float* mean; const float* w; const float* b; float* fg; float* skip;
    long tap_rows, x_rows, ld_skip, skip_row0;
    struct {
      const float* part; int nparts; const float* gamma; const float* beta; float* rm; float* rv; float mom, eps;
      float* save_mean; float* save_rstd; float* scale; float* w_fold; float* b_fold; long long* nbt;
    } bn;
  } tcn;
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
  void* tg4;  // bf16 t16 kernel: t1 / t2 in the tiled activation layout instead of dhcat's columns
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
  // the partials are read with sc1 loads (L1 bypass); the agent-scope acquire additionally
  // invalidates this CU's L1, so the hand-off does not rest on the load policy alone
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
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

__device__ __forceinline__ float bload(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
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
  for (int s = 0; s < 16; ++s) f.v[s] = wp[crow(s, half)];
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
    for (int j = 0; j < KB; ++j) av[j] = bp[2 * j * LDR];
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

// the same as 4 non-temporal 16-B stores per lane (hop pieces: written once, read by the backward
// after the whole forward -- kept out of the L2 the supports live in); dst 16-B aligned, ld % 4 == 0
__device__ __forceinline__ void acc_to_global_nt(float* dst, long ld, const f32x16& d, int w0, int lane, int n) {
  typedef float f32x4_t __attribute__((ext_vector_type(4)));
  const int half = lane >> 5, col = lane & 31;
  if (w0 + col >= n) return;
  float* p = dst + (long)(w0 + col) * ld;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const f32x4_t v = {d[4 * g], d[4 * g + 1], d[4 * g + 2], d[4 * g + 3]};
    __builtin_nontemporal_store(v, (f32x4_t*)(p + crow(4 * g, half)));
  }
}

// LDS image index of (row w, channel c): padded rows [np][LDR]
__device__ __forceinline__ int img_idx(int w, int c) { return w * LDR + c; }

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
          buf[img_idx(w, c)] = v[i].x;
          buf[img_idx(w, c + 1)] = v[i].y;
          buf[img_idx(w, c + 2)] = v[i].z;
          buf[img_idx(w, c + 3)] = v[i].w;
        }
      }
    }
    return;
  }
  for (int e = threadIdx.x; e < np * CH; e += blockDim.x) {
    const int w = e >> 5, c = e & 31;
    buf[img_idx(w, c)] = (w < n) ? src[(long)w * ld + c] : 0.0f;
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
template <int NEPT>
__device__ __forceinline__ void bwd_prologue(const FusedBwd& a, float* dhs, long row0, int n, int np,
                                             bool lead = true, bool first = blockIdx.x == 0) {
  if (!a.bn_dy) {
    global_to_lds(a.dh + row0 * CH, CH, n, np, dhs);
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
    if (w < np) dhs[img_idx(w, c)] = v;
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
    __syncthreads();  // ys is free: every wave finished the previous support's hop 2 (and its store)
    if (compute) {
      acc_to_lds(ys, d, w0, lane);
      if (a.store_pieces && !store_wave) acc_to_global((float*)hs + (1 + 2 * k) * pstride, ldh, d, w0, lane, n);
    }
    __syncthreads();
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
// "power" schedule: both hops of a support in one pass over the LDS image, and every wave on its
// own from the staging barrier to its end.
//
// D1'[c][w] = sum_v img[v][c] G1[v][w],  D2'[c][w] = sum_v img[v][c] G2[v][w]   (G2 = G1^2)
// K runs in 8-node batches of KP = 4 k-steps (k-step j of batch b: nodes 8 b + 2 j + {0, 1}, the
// lane half picks one); one LDS A-operand read feeds the two MFMAs of a k-step (two independent
// accumulator chains).  The B fragments of both supports run RING - 1 = 3 batches (24 MFMAs) ahead
// of their MFMAs in a 4-deep register ring, and the A operands of the next batch are read before
// the current batch's MFMAs: a wave alone on its SIMD otherwise waits for its operands (per-wave
// stamps of the one-batch look-ahead form: 68k cycles for 47k cycles of MFMA work).  Loads past the
// padded support (np rows) return zeros (buffer range) and the LDS image carries 16 spare rows, so
// the loop has no branch around a load.  nb = ceil(n / 8) batches: the MFMAs stop at the last
// 8-node group holding a real node (n = 207: 104 of 112 k-steps).
constexpr int KP = 4;
constexpr int RING = 4;

struct GPair {
  float a[KP], b[KP];
};

struct GPairSrc {
  __amdgpu_buffer_rsrc_t r1, r2;
  int voff, rowb;
};

__device__ __forceinline__ GPairSrc gp_src(const float* G1, const float* G2, int ld, int np, int w0, int lane) {
  GPairSrc s;
  s.r1 = __builtin_amdgcn_make_buffer_rsrc((void*)G1, (short)0, np * ld * 4, 0x00020000);
  s.r2 = __builtin_amdgcn_make_buffer_rsrc((void*)G2, (short)0, np * ld * 4, 0x00020000);
  s.voff = ((lane >> 5) * ld + w0 + (lane & 31)) * 4;
  s.rowb = 2 * ld * 4;
  return s;
}

__device__ __forceinline__ GPair gp_load(const GPairSrc& s, int batch) {
  GPair g;
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    g.a[j] = bload(s.r1, s.voff, (batch * KP + j) * s.rowb);
    g.b[j] = bload(s.r2, s.voff, (batch * KP + j) * s.rowb);
  }
  return g;
}

// rows of the LDS image of the power kernels: np + 16 (the A operands of one batch past the last
// are read ahead)
__host__ __device__ constexpr int pow_img_rows(int np) { return np + 16; }

// the W fragments of an mlp product on a diffusion accumulator (forward: W[c'][off + crow(s)],
// the channel contraction W D; backward: W[crow(s)][off + c], the transposed W^T E)
struct WFrag {
  float v[16];
};

template <bool TRANSPOSED>
__device__ __forceinline__ WFrag wfrag_load(const float* W, int ld_w, int off, int lane) {
  const int half = lane >> 5, col = lane & 31;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, CH * ld_w * 4, 0x00020000);
  WFrag w;
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int c = crow(s, half);
    w.v[s] = TRANSPOSED ? bload(rs, (c * ld_w + off + col) * 4, 0) : bload(rs, (col * ld_w + off + c) * 4, 0);
  }
  return w;
}

__device__ __forceinline__ f32x16 mlp_frag(const WFrag& w, const f32x16& d, f32x16 acc) {
#pragma unroll
  for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w.v[s], d[s], acc, 0, 0, 0);
  return acc;
}

// acc1 += img * G1, acc2 += img * G2 over n nodes; q0 = gp_load(src, 0), issued by the caller a
// phase ahead (batches 1 .. RING - 2 are issued here).  The first mlp product's W fragments
// (offset off1 of W [32][ld_w]) are issued after the last support batch, ahead of the tail's MFMAs.
template <bool TRANSPOSED>
__device__ __forceinline__ void diffuse_pair(const float* img, const GPairSrc& src, int n, int lane, f32x16& acc1,
                                             f32x16& acc2, const GPair& q0, const float* W, int ld_w, int off1,
                                             WFrag& w1, const float* tail_rows = nullptr, float4* tail = nullptr) {
  const int nb = (n + 7) >> 3;
  const float* bp = img + (lane >> 5) * LDR + (lane & 31);
  auto lds = [&](int b, float* v) {
#pragma unroll
    for (int j = 0; j < KP; ++j) v[j] = bp[(8 * b + 2 * j) * LDR];
  };
  auto mfma = [&](const float* v, const GPair& g) {
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(v[j], g.a[j], acc1, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(v[j], g.b[j], acc2, 0, 0, 0);
    }
  };
  GPair q[RING];
  q[0] = q0;
#pragma unroll
  for (int r = 1; r < RING - 1; ++r) q[r] = gp_load(src, r);
  float av[KP];
  lds(0, av);
  int b = 0;
  for (; b + RING <= nb; b += RING) {
#pragma unroll
    for (int r = 0; r < RING; ++r) {
      // batch b + r: issue batch b + r + RING - 1 into the slot batch b + r - 1 freed, read batch
      // b + r + 1's A operands, then b + r's MFMAs.  sched_barrier pins that order: left alone, the
      // machine scheduler sinks the loads next to their first use and the waits then expose the
      // full L2 latency every batch (seen in the ISA: vmcnt(3..5) waits inside the loop)
      q[(r + RING - 1) % RING] = gp_load(src, b + r + RING - 1);
      __builtin_amdgcn_sched_barrier(0);
      float an[KP];
      lds(b + r + 1, an);
      __builtin_amdgcn_sched_barrier(0);
      mfma(av, q[r]);
#pragma unroll
      for (int j = 0; j < KP; ++j) av[j] = an[j];
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  w1 = wfrag_load<TRANSPOSED>(W, ld_w, off1, lane);
  if (tail_rows) {  // the epilogue's rows (4 x 16 B per lane), behind the last support batch
#pragma unroll
    for (int g = 0; g < 4; ++g) tail[g] = *(const float4*)(tail_rows + 8 * g);
  }
  __builtin_amdgcn_sched_barrier(0);
  // fewer than RING batches left, all already in flight
#pragma unroll
  for (int r = 0; r < RING - 1; ++r) {
    if (b + r < nb) {
      float an[KP];
      lds(b + r + 1, an);
      mfma(av, q[r]);
#pragma unroll
      for (int j = 0; j < KP; ++j) av[j] = an[j];
    }
  }
}

// x[r] <- sum of x[r] over the 32 lanes of this lane's half, for 16 registers at once: within each
// 16-lane row by DPP (xor 1, xor 2 by quad_perm, then row rotations by 4 and 8), across the two
// rows of the half by one ds_swizzle (xor 16).  Fixed order: deterministic (the lanes of a row may
// differ in the last bit; callers take lane 0's).
__device__ __forceinline__ float dpp_add(float x, int ctrl) {
  int v = __builtin_bit_cast(int, x);
  int y;
  switch (ctrl) {  // (the dpp control must be a compile-time constant)
    case 0: y = __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false); break;   // quad_perm [1,0,3,2]
    case 1: y = __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false); break;   // quad_perm [2,3,0,1]
    case 2: y = __builtin_amdgcn_update_dpp(0, v, 0x124, 0xF, 0xF, false); break;  // row_ror 4
    default: y = __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false); break; // row_ror 8
  }
  return x + __builtin_bit_cast(float, y);
}

__device__ __forceinline__ void half_sums16(float* x) {
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) x[r] = dpp_add(x[r], c);
#pragma unroll
  for (int r = 0; r < 16; ++r)
    x[r] += __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, x[r]), 0x401F));
}

// Forward epilogue of one wave's 32-node tile, straight from the mlp accumulator (lane = node
// w0 + col, register r = channel crow(r, half)): bias, dropout (the chain kernel's counter hash,
// index m*32 + c), residual (optionally BatchNorm-on-load), z (4 x 16-B stores per lane), and the
// tile's BN partial (count, mean, M2 per channel; butterfly sums over the lanes of a half) in slot
// (slice, tile) -- or, eval mode, bn(z) to x_out.  `res` = the residual rows, loaded ahead.
__device__ __forceinline__ void fwd_tile_epilogue(const FusedFwd& a, const f32x16& hacc, const float4* res,
                                                  long row0, int w0, int lane, int n, int slice, int tile, int nkb,
                                                  float* tpart, int* tiles_done) {
  const int half = lane >> 5, col = lane & 31;
  const int w = w0 + col;
  const bool valid = w < n;
  const long m = row0 + min(w, n - 1);
  const unsigned long long seed = a.seed_ptr ? *a.seed_ptr : 0ull;
  const float keep_scale = (a.drop_p > 0.0f) ? 1.0f / (1.0f - a.drop_p) : 1.0f;
  float* dst = a.x_out ? a.x_out : a.z;
  float v[16];
  // channels 8g + 4 half + e of group g: per-channel vectors as float4s, one group at a time
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int c0 = 8 * g + 4 * half;
    const float4 bq = *(const float4*)(a.b_mlp + c0);
    const float* bias = (const float*)&bq;
    const float* rv = (const float*)&res[g];
    float4 mq, sq, hq;
    if (a.res_scale) {
      mq = *(const float4*)(a.res_mean + c0);
      sq = *(const float4*)(a.res_scale + c0);
      hq = *(const float4*)(a.res_shift + c0);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = 4 * g + e;
      float x = hacc[r] + bias[e];
      if (a.drop_p > 0.0f) {
        const float u = gwn_uniform(seed, a.salt, (unsigned long long)m * CH + c0 + e);
        x = (u >= a.drop_p) ? x * keep_scale : 0.0f;
      }
      // residual, or bn(z_prev) applied on load: (z - mean) * scale + shift
      x += a.res_scale ? fmaf(rv[e] - ((const float*)&mq)[e], ((const float*)&sq)[e], ((const float*)&hq)[e]) : rv[e];
      v[r] = x;
    }
    if (a.x_out) {  // eval BatchNorm, the arithmetic of bn_apply_kernel (ops.hip)
      const float4 rm = *(const float4*)(a.bn_rm + c0), rvv = *(const float4*)(a.bn_rv + c0);
      const float4 gq = *(const float4*)(a.bn_g + c0), bb = *(const float4*)(a.bn_b + c0);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        v[4 * g + e] = (v[4 * g + e] - ((const float*)&rm)[e]) * (1.0f / sqrtf(((const float*)&rvv)[e] + a.bn_eps)) *
                           ((const float*)&gq)[e] + ((const float*)&bb)[e];
    }
    if (valid) *(float4*)(dst + m * CH + c0) = make_float4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
  }
  if (a.bn_part == nullptr || a.x_out) return;
  // the tile's BN partial: count, mean and M2 per channel over its real nodes (two butterfly sums)
  const int cnt = min(32, n - w0);
  const float inv = 1.0f / (float)cnt;
  float* pp = tpart + tile * 3 * CH;
  float sm[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) sm[r] = valid ? v[r] : 0.0f;
  half_sums16(sm);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    sm[r] *= inv;  // mean
    const float d = valid ? v[r] - sm[r] : 0.0f;
    v[r] = d * d;
  }
  half_sums16(v);
  if (col == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int c = crow(r, half);
      pp[c] = (float)cnt;
      pp[CH + c] = sm[r];
      pp[2 * CH + c] = v[r];
    }
  }
  // the slice's partial: the last wave of the workgroup to get here merges the tiles' partials in
  // tile order (Chan's formula; LDS counter, no barrier) -- one partial per slice for the finalize
  __threadfence_block();
  int last = 0;
  if (lane == 0) last = atomicAdd(tiles_done, 1) == nkb - 1;
  last = __shfl(last, 0, 64);
  if (!last) return;
  __threadfence_block();
  if (lane < CH) {
    float nn = 0.0f, mean = 0.0f, m2 = 0.0f;
    for (int t = 0; t < nkb; ++t) {
      const float nb = tpart[t * 3 * CH + lane], mb = tpart[t * 3 * CH + CH + lane];
      const float qb = tpart[t * 3 * CH + 2 * CH + lane];
      const float tot = nn + nb;
      const float d = mb - mean;
      mean += d * (nb / tot);
      m2 += qb + d * d * (nn * nb / tot);
      nn = tot;
    }
    float* sp = a.bn_part + (long)slice * 3 * CH;
    sp[lane] = nn;
    sp[CH + lane] = mean;
    sp[2 * CH + lane] = m2;
  }
}

struct PowSup {
  const float* g2[8];   // forward: A_k^2; backward: (A_k^2)^T
  const float* g4[16];  // t16 kernels: [2k] A_k, [2k + 1] A_k^2 (backward: transposed) in gwn_support_g4's layout
};

// Forward: h pieces 1 + 2k, 2 + 2k = A_k^T-diffused xg and (A_k^2)^T-diffused xg (the reference's
// x1 = nconv(x, A), x2 = nconv(x1, A) up to fp32 reassociation), mlp, epilogue per wave
// (fwd_tile_epilogue).  One barrier: the staging one.  Hop pieces leave straight from the
// accumulators (4 x 16-B stores per lane).  The support split (ksplit > 1) keeps the chain
// kernel's whole-slice epilogue after the in-launch combine.
template <int MAXT>
__global__ __launch_bounds__(MAXT, 4) void gcn_fwd_pow_kernel(const FusedFwd a, const PowSup p) {
  extern __shared__ float lds[];
  __shared__ float red[2][MAXT];  // whole-slice epilogue (support split); tile partials otherwise
  __shared__ int last_unit;
  __shared__ int tiles_done;
  Unit u;
  if (!unit_of(a, u)) return;
  const int n = a.n;
  const int nkb = (n + 31) >> 5;
  const int np = nkb * 32;
  float* xs = lds;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, w0 = wave * 32;
  const long row0 = (long)u.slice * n;
  const long ldh = a.ld_h;
  float* hs = (float*)a.h + row0 * ldh;

  const int k0 = u.k0 < u.k1 ? u.k0 : 0;
  GPairSrc src = gp_src(a.sup[k0], p.g2[k0], a.ld_sup, np, w0, lane);
  GPair q0 = (u.k1 > u.k0) ? gp_load(src, 0) : GPair{};
  // piece 0's W fragments (A operand W[c'][c] = W^T[c][c'], K pairs in natural order; rows of W^T
  // are coalesced) land during the staging
  float w0f[16];
  if (u.k0 == 0) {
    const float* wp = a.w_t + (lane >> 5) * CH + (lane & 31);
#pragma unroll
    for (int s = 0; s < 16; ++s) w0f[s] = wp[2 * s * CH];
  }
  if (threadIdx.x == 0) tiles_done = 0;
  global_to_lds(hs, ldh, n, pow_img_rows(np), xs);
  __syncthreads();
  f32x16 hacc = zero16();
  if (u.k0 == 0) {
    const float* bp = xs + (w0 + (lane & 31)) * LDR + (lane >> 5);
#pragma unroll
    for (int s = 0; s < 16; ++s) hacc = __builtin_amdgcn_mfma_f32_32x32x2f32(w0f[s], bp[2 * s], hacc, 0, 0, 0);
  }
  // the epilogue's residual rows: prefetched in the last support's tail
  const bool tile_epi = a.ksplit <= 1;
  float4 res[4];
  const float* res_rows = a.residual + (row0 + min(w0 + (lane & 31), n - 1)) * CH + 4 * (lane >> 5);
  const bool nt_ok = ((((uintptr_t)hs) & 15) | (ldh & 3)) == 0;
  // one support: both hops, the two mlp products, the hop pieces; LAST (the residual prefetch of
  // the epilogue rides in its tail) is a separate instantiation so that the residual registers are
  // not live through the other supports
  auto support = [&](int k, auto last_tag) {
    constexpr bool LAST = decltype(last_tag)::value;
    f32x16 d1 = zero16(), d2 = zero16();
    WFrag w1;
    // W[c'][off + c] = W^T[off + c][c']: the transposed-read form on W^T's piece block
    diffuse_pair<true>(xs, src, n, lane, d1, d2, q0, a.w_t + (1 + 2 * k) * CH * CH, CH, 0, w1,
                       LAST ? res_rows : nullptr, res);
    if (!LAST && k + 1 < u.k1) {
      src = gp_src(a.sup[k + 1], p.g2[k + 1], a.ld_sup, np, w0, lane);
      q0 = gp_load(src, 0);
    }
    const WFrag w2 = wfrag_load<true>(a.w_t + (2 + 2 * k) * CH * CH, CH, 0, lane);
    hacc = mlp_frag(w1, d1, hacc);
    hacc = mlp_frag(w2, d2, hacc);
    if (a.store_pieces) {
      if (nt_ok) {
        acc_to_global_nt(hs + (1 + 2 * k) * CH, ldh, d1, w0, lane, n);
        acc_to_global_nt(hs + (2 + 2 * k) * CH, ldh, d2, w0, lane, n);
      } else {
        acc_to_global(hs + (1 + 2 * k) * CH, ldh, d1, w0, lane, n);
        acc_to_global(hs + (2 + 2 * k) * CH, ldh, d2, w0, lane, n);
      }
    }
  };
  if (u.k1 > u.k0) {
    for (int k = u.k0; k + 1 < u.k1; ++k) support(k, std::false_type());
    if (tile_epi) support(u.k1 - 1, std::true_type());
    else support(u.k1 - 1, std::integral_constant<bool, false>());
  }
  if (tile_epi) {
    fwd_tile_epilogue(a, hacc, res, row0, w0, lane, n, u.slice, wave, nkb, &red[0][0], &tiles_done);
    return;
  }
  __syncthreads();  // every wave is done with the node image: it stages the combined mlp output now
  float* part = a.kws + (long)u.slice * a.ksplit * np * CH;
  acc_to_part(part + (long)u.k0 * np * CH, n, hacc, w0, lane);
  if (!split_arrive(a.kcnt + u.slice, a.ksplit, &last_unit)) return;
  split_sum_to_lds(part, a.ksplit, n, np, xs);
  __syncthreads();
  fwd_epilogue<EPT>(a, xs, red[0], red[1], row0, n, u.slice);
}

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
__device__ __forceinline__ void t16_epilogue(const FusedFwd& a, const f32x4v* hacc, long row0, int w0, int lane,
                                             int n, BnRun& bn, const float* res_mean = nullptr,
                                             const float* res_scale = nullptr) {
  if (!res_mean) res_mean = a.res_mean;
  if (!res_scale) res_scale = a.res_scale;
  const int g = lane >> 4, j = lane & 15;
  const int w = w0 + j;
  const bool valid = w < n;
  const long m = row0 + min(w, n - 1);
  const unsigned long long seed = a.seed_ptr ? *a.seed_ptr : 0ull;
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
  double n = 0.0, mean = 0.0, m2 = 0.0;
  auto merge = [&](double nb, double mb, double qb) {
    if (nb <= 0.0) return;
    const double nn = n + nb, d = mb - mean, w = nb / nn;
    mean += d * w;
    m2 += qb + d * d * n * w;
    n = nn;
  };
  constexpr int U = 4;
  for (int i0 = sub; i0 < f.nparts; i0 += U * nsub) {
    float nb[U], mb[U], qb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * nsub;
      const float* pp = f.part + (long)(i < f.nparts ? i : 0) * 3 * CH;
      nb[u] = i < f.nparts ? pp[c] : 0.0f;
      mb[u] = pp[CH + c];
      qb[u] = pp[2 * CH + c];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) merge(nb[u], mb[u], qb[u]);
  }
  scratch[(sub * 3) * CH + c] = (float)n;
  scratch[(sub * 3 + 1) * CH + c] = (float)mean;
  scratch[(sub * 3 + 2) * CH + c] = (float)m2;
  __syncthreads();
  if (threadIdx.x < CH) {
    n = mean = m2 = 0.0;
    for (int q = 0; q < nsub; ++q) merge(scratch[(q * 3) * CH + c], scratch[(q * 3 + 1) * CH + c], scratch[(q * 3 + 2) * CH + c]);
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
      t16_epilogue(a, hacc, row0, w0, lane, n, bn, res_mean, res_scale);
    }
    p0 = p1;
  }
  t16_bn_flush(a, bn, wpart);
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
      t16_epilogue(a, hacc, row0, w0, lane, n, bn);
    }
    p0 = p1;
  }
  t16_bn_flush(a, bn, wpart);
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
      t16_epilogue(a, haccA, rowA, w0, lane, n, bn);
      if (okB) t16_epilogue(a, haccB, rowB, w0, lane, n, bn);
    }
    p0 = p1;
  }
  t16_bn_flush(a, bn, wpart);
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
// workgroup's own rows) as 16-B stores and one 8-B LDS write per channel (4 nodes' bf16)
template <typename Mid>
__device__ __forceinline__ void t16_bwd_stage_bn_bf16(const FusedBwd& a, __bf16* imgs, int imgb, int s0, int nsl,
                                                      const T16Range& rg, int nt, int n, int s16, Mid mid) {
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
    const long sb = (long)(s0 + sl) * nt;
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
      const long m = row0 + w;
      const bool sk = a.dskip && m >= a.skip_row0;
#pragma unroll
      for (int oh = 0; oh < 2; ++oh) {
        const int c0 = 16 * oh + 4 * g;
        const float4 f0 = *(const float4*)(a.fg + m * 2 * CH + 2 * c0);
        const float4 f1 = *(const float4*)(a.fg + m * 2 * CH + 2 * c0 + 4);
        const float4 dq = sk ? *(const float4*)(a.dskip + (m - a.skip_row0) * a.ld_dskip + c0) : make_float4(0, 0, 0, 0);
        const float fv[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
        const float dv[4] = {dq.x, dq.y, dq.z, dq.w};
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
    p0 = p1;
  }
}

// Backward gate epilogue of one wave's tile from the input-gradient accumulator (lane = node,
// register r = channel crow(r, half)): g = dxg (+ dskip) -> dfg through the saved (tanh f,
// sigmoid s) pairs (gate_bwd_kernel's arithmetic), 16-B loads / stores.
__device__ __forceinline__ void bwd_gate_tile(const FusedBwd& a, const f32x16& dx, long row0, int w0, int lane, int n) {
  const int half = lane >> 5, col = lane & 31;
  const int w = w0 + col;
  if (w >= n) return;
  const long m = row0 + w;
  float4 fs[8], ds[4];
  const float* fp = a.fg + m * 2 * CH + 8 * half;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    fs[2 * g] = *(const float4*)(fp + 16 * g);
    fs[2 * g + 1] = *(const float4*)(fp + 16 * g + 4);
  }
  const bool sk = a.dskip && m >= a.skip_row0;
#pragma unroll
  for (int g = 0; g < 4; ++g)
    ds[g] = sk ? *(const float4*)(a.dskip + (m - a.skip_row0) * a.ld_dskip + 8 * g + 4 * half) : make_float4(0, 0, 0, 0);
  float* op = a.dfg + m * 2 * CH + 8 * half;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float* f8 = (const float*)&fs[2 * g];  // (f, s) of channels 8g + 4h + 0..3
    const float* d4 = (const float*)&ds[g];
    float o[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float gv = dx[4 * g + e] + d4[e];
      const float f = f8[2 * e], sg = f8[2 * e + 1];
      o[2 * e] = gv * sg * (1.0f - f * f);
      o[2 * e + 1] = gv * f * sg * (1.0f - sg);
    }
    *(float4*)(op + 16 * g) = make_float4(o[0], o[1], o[2], o[3]);
    *(float4*)(op + 16 * g + 4) = make_float4(o[4], o[5], o[6], o[7]);
  }
}

// Backward: dx = W0^T dh + sum_k [W_{1+2k}^T (A_k dh) + W_{2+2k}^T (A_k^2 dh)] (node-wise mlp
// commutes with the node diffusion), with A_k dh read as the transposed support.  For the
// adaptive support the gram's operands t2 = W_2^T dh and t1 = W_1^T dh + W_2^T (A dh) come from
// the same accumulators.  Prologue (BN backward, whole slice) as the chain kernel's; the gate
// epilogue (or the dxg store) runs per wave from the accumulator.
template <int MAXT>
__global__ __launch_bounds__(MAXT, 4) void gcn_bwd_pow_kernel(const FusedBwd a, const PowSup p) {
  extern __shared__ float lds[];
  __shared__ int last_unit;
  Unit un;
  if (!unit_of(a, un)) return;
  const int n = a.n;
  const int nkb = (int)(blockDim.x >> 6);
  const int np = nkb * 32;
  float* dhs = lds;
  const int lane = threadIdx.x & 63, w0 = (threadIdx.x >> 6) * 32;
  const long row0 = (long)un.slice * n;

  const int k0 = un.k0 < un.k1 ? un.k0 : 0;
  GPairSrc src = gp_src(a.supT[k0], p.g2[k0], a.ld_sup, np, w0, lane);
  GPair q0 = (un.k1 > un.k0) ? gp_load(src, 0) : GPair{};
  bwd_prologue<EPT>(a, dhs, row0, n, pow_img_rows(np), un.k0 == 0, un.slice == 0 && un.k0 == 0);
  __syncthreads();
  f32x16 dx = (un.k0 == 0) ? mlpT_from_lds(a.w_mlp, a.ld_w, 0, dhs, w0, lane, zero16()) : zero16();
  for (int k = un.k0; k < un.k1; ++k) {
    f32x16 e1 = zero16(), e2 = zero16();
    WFrag w1;
    diffuse_pair<true>(dhs, src, n, lane, e1, e2, q0, a.w_mlp, a.ld_w, (1 + 2 * k) * CH, w1);
    if (k + 1 < un.k1) {
      src = gp_src(a.supT[k + 1], p.g2[k + 1], a.ld_sup, np, w0, lane);
      q0 = gp_load(src, 0);
    }
    const WFrag w2 = wfrag_load<true>(a.w_mlp, a.ld_w, (2 + 2 * k) * CH, lane);
    dx = mlp_frag(w1, e1, dx);
    dx = mlp_frag(w2, e2, dx);
    if (k == a.adp_index) {
      __builtin_amdgcn_sched_barrier(0);  // (register pressure: keep the gram operands after dx)
      f32x16 t1 = mlpT_from_lds(a.w_mlp, a.ld_w, (1 + 2 * k) * CH, dhs, w0, lane, zero16());
      t1 = mlp_frag(w2, e1, t1);
      acc_to_global(a.t1 + row0 * a.ld_t, a.ld_t, t1, w0, lane, n);
      __builtin_amdgcn_sched_barrier(0);
      const f32x16 t2 = mlpT_from_lds(a.w_mlp, a.ld_w, (2 + 2 * k) * CH, dhs, w0, lane, zero16());
      acc_to_global(a.t2 + row0 * a.ld_t, a.ld_t, t2, w0, lane, n);
    }
  }
  if (a.ksplit > 1) {  // partial input gradient of this support; the slice's last unit finishes
    float* part = a.kws + (long)un.slice * a.ksplit * np * CH;
    acc_to_part(part + (long)un.k0 * np * CH, n, dx, w0, lane);
    if (!split_arrive(a.kcnt + un.slice, a.ksplit, &last_unit)) return;
    split_sum_to_lds(part, a.ksplit, n, np, dhs);
    __syncthreads();
    if (a.dfg) {
      bwd_gate_epilogue<EPT>(a, dhs, row0, n);
    } else {
      for (int e = threadIdx.x; e < n * CH; e += blockDim.x)
        a.dxg[(row0 + (e >> 5)) * a.ld_dxg + (e & 31)] = dhs[(e >> 5) * LDR + (e & 31)];
    }
    return;
  }
  if (a.dfg) bwd_gate_tile(a, dx, row0, w0, lane, n);
  else acc_to_global(a.dxg + row0 * a.ld_dxg, a.ld_dxg, dx, w0, lane, n);
}

size_t fused_lds_bytes(int n) {
  const int np = (n + 31) / 32 * 32;
  return (size_t)2 * np * LDR * sizeof(float);
}

// the power schedule keeps one image (node features forward, dh backward) of np + 16 rows
size_t pow_lds_bytes(int n) {
  const int np = (n + 31) / 32 * 32;
  return (size_t)pow_img_rows(np) * LDR * sizeof(float);
}

template <typename K>
void ensure_lds_attr(K kern) {
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)fused_lds_bytes(512));
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

// zero the BN partial slots [written, gwn_bn_part_slots(slices)) that a whole-slice kernel leaves
int bn_part_tail(float* bn_part, int slices, int c, hipStream_t s) {
  const long slots = gwn_bn_part_slots(slices);
  if (!bn_part || slots <= slices) return GWN_OK;
  return hipMemsetAsync(bn_part + (long)slices * 3 * c, 0, (size_t)(slots - slices) * 3 * c * sizeof(float), s) ==
                 hipSuccess
             ? GWN_OK
             : gwn_set_error(GWN_ERR_HIP, "gcn_fwd: BN partial tail memset failed");
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
constexpr size_t T16_BN_SCRATCH = 3 * (64 * T16_WAVES / 32) * CH * sizeof(float);
static bool bn_scratch_ok(int n, int nsup, int slices) {
  const T16Plan pl = t16_plan(n, nsup, slices, true);
  return pl.ok && pl.lds >= t16_lds_bytes(n, nsup, 0, true) + T16_BN_SCRATCH;
}
bool gwn_gcn_tcn_fusable(const gwn_gcn_args* g) {
  const gwn_tcn_args* t = g->tcn;
  if (!t) return false;
  auto al = [](const void* q) { return (((uintptr_t)q) & 15) == 0; };
  const int slices = g->rows / g->n, nwt = (g->n + 31) / 32;
  return t->c == CH && (t->ntaps == 0 || t->ntaps == 2) && (t->c_out == 0 || t->c_out == CH) &&
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

int gwn_gcn_fused_fwd_launch(const gwn_gcn_args* g, float* bn_part, hipStream_t s) {
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
      if (g->split_planes == 2 && gmax2 >= 1 && h16) {
        static bool attr2 = false;
        if (!attr2) {
          (void)hipFuncSetAttribute((const void*)gcn_fwd_t16b2_kernel<768>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    T16_LDS_MAX);
          attr2 = true;
        }
        size_t lds2 = fixed + maximg2 * img;
        if (lds2 < 81 * 1024) lds2 = 81 * 1024;
        gcn_fwd_t16b2_kernel<768><<<grid2, 768, lds2, s>>>(a, p, maximg2);
      } else if (g->split_planes == 2)
        gcn_fwd_t16b_kernel<1024, true><<<grid, 64 * T16_WAVES, lds, s>>>(a, p, maximg);
      else gcn_fwd_t16b_kernel<1024><<<grid, 64 * T16_WAVES, lds, s>>>(a, p, maximg);
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
    ensure_lds_attr(gcn_fwd_fused_kernel<512, false>);
    ensure_lds_attr(gcn_fwd_fused_kernel<512, true>);
    ensure_lds_attr(gcn_fwd_fused_kernel<1024, false>);
    ensure_lds_attr(gcn_fwd_fused_kernel<1024, true>);
    ensure_lds_attr(gcn_fwd_pow_kernel<512>);
    ensure_lds_attr(gcn_fwd_pow_kernel<1024>);
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
    GWN_CHECK_LAUNCH();
    return GWN_OK;
  }
  if (g->sup2 && a.sup_batch <= 1 && g->nsup > 0) {
    GWN_REQUIRE(g->w_mlp_t, "gcn_fwd (power schedule): w_mlp_t (the transposed mlp weights) is required with sup2");
    PowSup p = {};
    for (int k = 0; k < 8; ++k) p.g2[k] = (k < g->nsup) ? g->sup2[k] : nullptr;
    const size_t lds = pow_lds_bytes(g->n);
    if (nwt <= 8) gcn_fwd_pow_kernel<512><<<grid, 64 * nwt, lds, s>>>(a, p);
    else gcn_fwd_pow_kernel<1024><<<grid, 64 * nwt, lds, s>>>(a, p);
  } else {
    // + one store wave when hop pieces are stored through LDS rows (h 16-B aligned, ld % 4 == 0)
    const size_t lds = fused_lds_bytes(g->n);
    const bool rows_ok = ((((uintptr_t)a.h) & 15) | (a.ld_h & 3)) == 0;
    const int waves = nwt + ((a.store_pieces && rows_ok && nwt < 16) ? 1 : 0);
    if (half_last_batch(g->n)) {
      if (waves <= 8) gcn_fwd_fused_kernel<512, true><<<grid, 64 * waves, lds, s>>>(a);
      else gcn_fwd_fused_kernel<1024, true><<<grid, 64 * waves, lds, s>>>(a);
    } else {
      if (waves <= 8) gcn_fwd_fused_kernel<512, false><<<grid, 64 * waves, lds, s>>>(a);
      else gcn_fwd_fused_kernel<1024, false><<<grid, 64 * waves, lds, s>>>(a);
    }
  }
  GWN_CHECK_LAUNCH();
  return bn_part_tail(a.x_out ? nullptr : bn_part, slices, CH, s);
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
      if (g->split_planes == 2) gcn_bwd_t16_kernel<1024, true, true><<<grid, 64 * T16_WAVES, lds, s>>>(a, p, maximg);
      else gcn_bwd_t16_kernel<1024, true><<<grid, 64 * T16_WAVES, lds, s>>>(a, p, maximg);
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
    ensure_lds_attr(gcn_bwd_fused_kernel<512, false>);
    ensure_lds_attr(gcn_bwd_fused_kernel<512, true>);
    ensure_lds_attr(gcn_bwd_fused_kernel<1024, false>);
    ensure_lds_attr(gcn_bwd_fused_kernel<1024, true>);
    ensure_lds_attr(gcn_bwd_pow_kernel<512>);
    ensure_lds_attr(gcn_bwd_pow_kernel<1024>);
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
  if (g->sup2_t && a.sup_batch <= 1 && g->nsup > 0) {
    PowSup p = {};
    for (int k = 0; k < 8; ++k) p.g2[k] = (k < g->nsup) ? g->sup2_t[k] : nullptr;
    const size_t lds = pow_lds_bytes(g->n);
    if (nwt <= 8) gcn_bwd_pow_kernel<512><<<grid, 64 * nwt, lds, s>>>(a, p);
    else gcn_bwd_pow_kernel<1024><<<grid, 64 * nwt, lds, s>>>(a, p);
  } else {
    const size_t lds = fused_lds_bytes(g->n);
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

// diagnostics: resident workgroups per CU of the fused kernels for n nodes (HIP occupancy API):
// the power schedule the executor uses for shared supports (pow = 1) or the chain schedule
extern "C" int gwn_fused_occupancy(int n, int backward, int pow) {
  const int nwt = (n + 31) / 32;
  int blocks = -1;
  hipError_t e;
  if (pow) {
    const size_t lds = pow_lds_bytes(n);
    if (backward) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, gcn_bwd_pow_kernel<1024>, 64 * nwt, lds);
    else e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, gcn_fwd_pow_kernel<1024>, 64 * nwt, lds);
  } else if (backward) {
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, gcn_bwd_fused_kernel<1024, false>, 64 * nwt,
                                                     fused_lds_bytes(n));
  } else {
    // training forward: the compute waves plus the store wave
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, gcn_fwd_fused_kernel<1024, false>,
                                                     64 * (nwt < 16 ? nwt + 1 : nwt), fused_lds_bytes(n));
  }
  return e == hipSuccess ? blocks : -(int)e;
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
