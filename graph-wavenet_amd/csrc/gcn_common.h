// Shared definitions of the fused diffusion graph convolution (gcn.forward, reference
// model.py:41-55, + residual model.py:234) for C = 32 channels and N <= 512 nodes: the launch
// arguments of the forward / backward kernels, and the entry points of the whole-slice schedules.
//   gcn_fused.hip: the persistent 16-node tile kernels (f32 / bf16 operands), their launch plans
//                  and the gwn_gcn_fwd / gwn_gcn_bwd dispatch;
//   gcn_slice.hip: the whole-slice schedules (one workgroup per slice, 32-node tile waves): the
//                  chained hops (per-sample supports) and the 32-node power schedule, with the
//                  support split.
#pragma once
#include "gwn_internal.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace gcnk {

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
  unsigned long long* clk;  // gwn_gcn_args.clock (NULL: off)
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

struct PowSup {
  const float* g2[8];   // forward: A_k^2; backward: (A_k^2)^T
  const float* g4[16];  // t16 kernels: [2k] A_k, [2k + 1] A_k^2 (backward: transposed) in gwn_support_g4's layout
};

// accumulator register r of v_mfma_f32_32x32x2 in lane half `half`: row crow(r, half) of the tile
__device__ __forceinline__ int crow(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }

// the whole-slice schedules (gcn_slice.hip): gwn_gcn_fwd / gwn_gcn_bwd where the 16-node tile
// kernels do not run; a.ksplit and grid (slices, or the support split's units) already chosen
int slice_fwd_launch(const gwn_gcn_args* g, FusedFwd& a, float* bn_part, int grid, hipStream_t s);
int slice_bwd_launch(const gwn_gcn_bwd_args* g, FusedBwd& a, int grid, hipStream_t s);

}  // namespace gcnk
