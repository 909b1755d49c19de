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
#include "gcn_common.h"
#include <type_traits>

using namespace gcnk;

namespace {

// support k of this workgroup's slice (per-sample supports: sample = slice % sup_batch)
template <typename Args>
__device__ __forceinline__ const float* slice_sup(const Args& a, const float* base) {
  return a.sup_batch > 1 ? base + (long)(blockIdx.x % a.sup_batch) * a.sup_bstride : base;
}


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

namespace gcnk {

int slice_fwd_launch(const gwn_gcn_args* g, FusedFwd& a, float* bn_part, int grid, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    ensure_lds_attr(gcn_fwd_fused_kernel<512, false>);
    ensure_lds_attr(gcn_fwd_fused_kernel<512, true>);
    ensure_lds_attr(gcn_fwd_fused_kernel<1024, false>);
    ensure_lds_attr(gcn_fwd_fused_kernel<1024, true>);
    ensure_lds_attr(gcn_fwd_pow_kernel<512>);
    ensure_lds_attr(gcn_fwd_pow_kernel<1024>);
    attr_set = true;
  }
  const int nwt = (g->n + 31) / 32, slices = g->rows / g->n;
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

int slice_bwd_launch(const gwn_gcn_bwd_args* g, FusedBwd& a, int grid, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    ensure_lds_attr(gcn_bwd_fused_kernel<512, false>);
    ensure_lds_attr(gcn_bwd_fused_kernel<512, true>);
    ensure_lds_attr(gcn_bwd_fused_kernel<1024, false>);
    ensure_lds_attr(gcn_bwd_fused_kernel<1024, true>);
    ensure_lds_attr(gcn_bwd_pow_kernel<512>);
    ensure_lds_attr(gcn_bwd_pow_kernel<1024>);
    attr_set = true;
  }
  const int nwt = (g->n + 31) / 32;
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

}  // namespace gcnk

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
