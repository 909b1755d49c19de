/*
 * libgwn — MI355X (gfx950) native kernels for the Graph WaveNet gwnet.forward()/backward hot path.
 *
 * C-ABI only: plain device pointers, sizes and a hipStream_t; no torch types.  Every entry point
 * is asynchronous on the given stream, never allocates, never synchronises the host, and keeps
 * no mutable global state besides a thread-local error string.  Workspaces are owned by the
 * caller (see the *_workspace_floats queries).  Return value: 0 on success, otherwise a GWN_ERR_*
 * code; gwn_last_error() gives the message.  All arithmetic is fp32 with fixed-order reductions
 * (bitwise reproducible run to run).
 *
 * Internal activation layout ("slab-major, channels-last"): a tensor that the reference holds as
 * NCHW [B, C, N, T] (model.py:175-241) is held as [T][B][N][C], i.e. a row-major matrix with
 * rows = T*B*N positions and C contiguous channels.  One time step is a "slab" of P = B*N rows;
 * one (t, b) pair is a "slice" of N consecutive rows (the operand of one diffusion step).
 *
 * The reference (sklin93/Graph-WaveNet) is pure Python with no FFI; each entry below names the
 * reference function whose arithmetic it replaces (file:line in the reference tree).
 */
#ifndef GWN_H_
#define GWN_H_

#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GWN_OK 0
#define GWN_ERR_ARG 1
#define GWN_ERR_HIP 2

int gwn_version(void);

/* Arithmetic (MFMA operand) precision of the diffusion / mlp products.  Storage stays fp32 in
 * every mode (activations, weights, gradients, optimizer state); accumulation is always fp32. */
typedef enum gwn_dtype {
  GWN_DTYPE_F32 = 0,     /* v_mfma_f32_32x32x2_f32: exact fp32 products (the reference's arithmetic) */
  GWN_DTYPE_BF16 = 1,    /* bf16 operands, fp32 accumulation (mixed precision, configs[2]) */
  GWN_DTYPE_BF16_MLP = 2 /* GWN_DTYPE_BF16 plus the gcn's 1x1 mlp (and its transpose in the
                            backward) on bf16 operands, fp32 accumulation: the bf16 mode's default */
} gwn_dtype;
/* debugging aid: 1 = synchronise the device after every kernel launch and report a fault at the
 * kernel's source line (also enabled by GWN_SYNC_CHECK=1 in the environment), 2 = suspended (while
 * a stream is being captured into a graph), 0 = off (default) */
void gwn_set_sync_check(int mode);
const char* gwn_last_error(void);
/* sizeof of the argument structs below, for bindings that mirror them (ctypes, cgo):
 * "gwn_gemm_desc", "gwn_tcn_args", "gwn_tcn_bwd_args", "gwn_gcn_args", "gwn_gcn_bwd_args",
 * "gwn_reduce_seg", "gwn_wgrad_problem", "gwn_gram_layer", "gwn_bn_fold";
 * -1 for an unknown name */
long gwn_abi_sizeof(const char* struct_name);

/* ---------------------------------------------------------------------------------------------
 * Generic fp32 MFMA GEMM:  C(m,n) = epi(alpha * sum_k A(m,k) * B(k,n)).
 * Used for the 1x1 / dilated convolutions (model.py:102-104, 135-151, 161-169, 27) and their
 * gradients.  Index maps (two-level so one launch can walk strided slices):
 *   A(m,k): ko=k/a_kin, ki=k%a_kin, row=m+ko*a_row_shift (0<=row<a_rows else 0)
 *           -> A[row*lda_m + ki*lda_k + ko*a_ko_stride]
 *   B(k,n): kb=k/b_kin, kj=k%b_kin, no=n/b_nin, ni=n%b_nin
 *           -> B[kj*ldb_k + kb*b_ko_stride + ni*ldb_n + no*b_no_stride]
 *   C(m,n): no=n/c_nin, ni=n%c_nin -> C[m*ldc_m + ni*ldc_n + no*c_no_stride] (C0 alike)
 * epi: 0 = store (+bias_n, relu, dropout, +beta*C0); 1 = gated tanh*sigmoid (columns 2c+g);
 *      2 = relu-backward mask (keep where mask(m,n) > 0).
 * ksplit > 1 splits K over blocks; the partial sums go to `part` ([ksplit][M][N] floats, see
 * gwn_gemm_workspace_floats) and are reduced in a fixed order.
 * ------------------------------------------------------------------------------------------- */
typedef struct gwn_gemm_desc {
  const float* A; long lda_m, lda_k, a_ko_stride; int a_kin, a_row_shift, a_rows;
  const float* B; long ldb_k, ldb_n, b_ko_stride, b_no_stride; int b_kin, b_nin;
  float* C; long ldc_m, ldc_n, c_no_stride; int c_nin;
  const float* C0; long ldc0_m, ldc0_n, c0_no_stride; float beta;
  const float* bias_n;
  const float* mask; long ldmask_m;
  int M, N, K;
  float alpha;
  int epi, relu;
  float* aux; long ld_aux;
  float* aux2; long ld_aux2; int aux2_row0;
  const unsigned long long* seed_ptr; unsigned long long seed_salt; float drop_p;
  int ksplit, kchunk; float* part;
  /* optional: ones_out[m] = alpha * sum_k A(m,k) (B extended by a column of ones).  In a weight
   * gradient dW = dY^T X this is the bias gradient sum_r dY[r][m], for free.  With split-K the
   * partial buffer holds ksplit*(M*N + M) floats (gwn_gemm_workspace_floats covers it). */
  float* ones_out;
  /* optional batch (batch <= 1 = none): blockIdx.z walks `batch` independent GEMMs whose A, B, C
   * (and C0) start a_bstride, b_bstride, c_bstride floats apart.  Needs ksplit == 1, epi 0, no
   * ones_out / mask (the per-sample nconv2, model.py:20-22). */
  int batch; long a_bstride, b_bstride, c_bstride;
} gwn_gemm_desc;

int gwn_gemm(const gwn_gemm_desc* desc, hipStream_t stream);
long gwn_gemm_workspace_floats(int M, int N, int ksplit);

/* Row-tile "NT" GEMM for 1x1 convs over channels-last rows (the output head, model.py:216-222,
 * 238-240, and with a transposed weight their input gradients):
 *   C[m][n] = epi( sum_k A[m][k] * B[n][k] ),  epi: + bias[n] (NULL = none), relu (0/1), then
 *   mask: v = (mask[m][ldmask] > 0) ? v : 0 (NULL = none; the relu backward).
 * A [M][lda], B [N][ldb] K-contiguous, K / lda / ldb multiples of 4, A and B 16-B aligned. */
int gwn_gemm_nt(const float* A, long lda, const float* B, long ldb, float* C, long ldc, int M, int N, int K,
                const float* bias, int relu, const float* mask, long ldmask, hipStream_t stream);
/* gwn_gemm_nt on bf16 operands (the bf16 compute mode's head, configs[2]): A and B rounded to bf16
 * (round to nearest even) as they are read, products summed in fp32; fp32 in and out, the same
 * epilogue.  N a multiple of 64. */
int gwn_gemm_nt_bf16(const float* A, long lda, const float* B, long ldb, float* C, long ldc, int M, int N, int K,
                     const float* bias, int relu, const float* mask, long ldmask, hipStream_t stream);

/* ---------------------------------------------------------------------------------------------
 * nconv (model.py:12-14): einsum('ncvl,vw->ncwl', x, A), i.e. for every slice s
 *   y_s[w][c] = sum_v A[v][w] * x_s[v][c]            (transpose_a = 1, the forward)
 *   y_s[v][c] = sum_w A[v][w] * x_s[w][c]            (transpose_a = 0, its input gradient)
 * plus an optional addend y0 (may alias y).  A is [n][lda]; slices are `slices` blocks of n rows
 * of C channels, row stride ldx / ldy / ldy0 (floats), consecutive slices n rows apart.
 * ------------------------------------------------------------------------------------------- */
int gwn_nconv(const float* A, int lda, int transpose_a, const float* x, long ldx, float* y,
              long ldy, const float* y0, long ldy0, int n, int c, int slices, hipStream_t stream);

/* Adjacency gradient of nconv (the backward of model.py:13 w.r.t. A, used for the adaptive
 * support): dA[v][w] (+)= sum_{s,c} x_s[v][c] * dy_s[w][c].  `accumulate` adds to dA.  Needs
 * gwn_nconv_adj_grad_workspace_floats(n, slices*c) floats of workspace. */
int gwn_nconv_adj_grad(const float* x, long ldx, const float* dy, long lddy, int n, int c,
                       int slices, float* dA, int ld_dA, int accumulate, float* workspace,
                       hipStream_t stream);
long gwn_nconv_adj_grad_workspace_floats(int n, int c, int slices);

/* Per-sample diffusion nconv2 (model.py:16-22): einsum('ncvl,nvw->ncwl', x, A) with one support
 * per batch element b: A_b = A + b*a_bstride ([n][lda]); x / y hold `batch` groups of `slices`
 * slices (n rows of c floats each, row stride ldx / ldy), group b at b*slices*n rows.  One launch.
 *   y_s[w][:] = sum_v A_b[v][w] x_s[v][:]   (transpose_a = 1, the forward)
 *   y_s[v][:] = sum_w A_b[v][w] x_s[w][:]   (transpose_a = 0, its input gradient) */
int gwn_nconv2(const float* A, int lda, long a_bstride, int transpose_a, const float* x, long ldx, float* y,
               long ldy, int n, int c, int slices, int batch, hipStream_t stream);
/* Its support gradient: dA_b[v][w] (+)= sum_{s in group b} sum_c x_s[v][c] dy_s[w][c]; dA_b at
 * dA + b*dA_bstride ([n][ld_dA]).  One launch, no workspace. */
int gwn_nconv2_adj_grad(const float* x, long ldx, const float* dy, long lddy, int n, int c, int slices,
                        int batch, float* dA, int ld_dA, long dA_bstride, int accumulate, hipStream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Adaptive adjacency (model.py:185-188): adp = softmax(relu(E1 @ E2), dim=1), E1 [n][d],
 * E2 [d][n]; adp is written as [n][ld_adp].  Backward (autograd of the same expression):
 * given dadp [n][ld_adp] -> dE1 [n][d], dE2 [d][n]; workspace = n*ld_adp floats.
 * ------------------------------------------------------------------------------------------- */
int gwn_adaptive_adj_fwd(const float* e1, const float* e2, int n, int d, float* adp, int ld_adp,
                         hipStream_t stream);
int gwn_adaptive_adj_bwd(const float* e1, const float* e2, const float* adp, const float* dadp,
                         int n, int d, int ld_adp, float* de1, float* de2, float* workspace,
                         hipStream_t stream);
/* per-sample adaptive adjacencies of gwnet_diff_G (model.py:342-344: softmax(relu(E1_b @ E2_b),
 * dim=2) with E1 [batch][n][d], E2 [batch][d][n]); sample b written at adp + b*adp_bstride as
 * [n][ld_adp] (columns >= n zero).  Forward only: the reference draws these embeddings afresh
 * per call (model.py:324-329) and never trains them. */
int gwn_adaptive_adj_fwd_batched(const float* e1, const float* e2, int batch, int n, int d, float* adp,
                                 int ld_adp, long adp_bstride, hipStream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Input padding + start_conv (model.py:176-181): x is the reference NCHW input [B][cin][n][t]
 * given by element strides (may be a non-contiguous transpose view, train.py:245); it is
 * left-padded with zeros to t0 >= t steps and mapped 1x1 cin -> c:
 *   out[(tt*B + b)*n + v][co] = bias[co] + sum_ci W[co][ci] * xpad[b][ci][v][tt]
 * xin (optional, [t0*B*n][cin]) receives the padded input channels-last (for the weight grad).
 * ------------------------------------------------------------------------------------------- */
int gwn_start_conv_fwd(const float* x, long sb, long sc, long sn, long st, int B, int cin, int n,
                       int t, int t0, const float* W, const float* bias, int c, float* out,
                       float* xin, hipStream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Gated dilated TCN (model.py:206-212; filter_convs Conv2d 135-137, gate_convs legacy Conv1d
 * 139-141):  for output row r (t < t_out = t_in - dilation):
 *   f = Wf0 x[r] + Wf1 x[r + d*P] + bf,  g = Wg0 x[r] + Wg1 x[r + d*P] + bg,
 *   xg[r] = tanh(f) * sigmoid(g)
 * w_fg is the packed [2c][2c] matrix (row 2co+gate, column tap*c+ci), b_fg [2c] interleaved the
 * same way.  fg [rows][2c] receives (tanh f, sigmoid g) for the backward.  xg is written with
 * row stride ld_xg (it is piece 0 of the gcn concat, model.py:42).  skipcat (optional) receives
 * the rows >= skip_row0 at column offset given by its pointer (the skip path only reads the last
 * T_final steps, model.py:216-222).
 * ------------------------------------------------------------------------------------------- */
typedef struct gwn_tcn_args {
  const float* x; int t_in, P, c, dilation;
  const float* w_fg; const float* b_fg;
  float* xg; long ld_xg;
  float* fg;
  float* skipcat; long ld_skip; int skip_row0;
  /* x_mean [c] (c == 32 row-GEMM path): x holds the PRE-BatchNorm z of the layer below and the
   * input used is x - x_mean; w_fg / b_fg are then the folded weights of gwn_batchnorm_fwd_fold
   * (BatchNorm applied on load, centred before any product). */
  const float* x_mean;
  /* kernel taps and output (dilation) channels (model.py:135-141 kernel_size, dilation_channels):
   * ntaps taps t, t+d, ..., t+(ntaps-1)d, so t_out = t_in - (ntaps-1)*dilation; w_fg is then
   * [2*c_out][ntaps*c] (row 2co+gate, column tap*c+ci), b_fg [2*c_out], xg / fg / skipcat carry
   * c_out (resp. 2*c_out) channels.  0 = the defaults ntaps 2, c_out c.  Non-default values run
   * the generic GEMM path (no x_mean fold). */
  int ntaps, c_out;
  /* bn (optional, c == 32 row-GEMM / fused path, training): x holds the PRE-BatchNorm z of the
   * layer below and its BatchNorm is finalized by this call -- bn_partials [bn_nparts][3][c]
   * (gwn_gcn_fwd's partials of that layer) merged into the statistics, and every output of
   * gwn_batchnorm_fwd_fold written (save_mean / save_rstd / scale, the running statistics,
   * num_batches_tracked advanced once, w_fold / b_fold from bn->w_next / b_next = this TCN's raw
   * weights) -- then the TCN applied with them (x_mean, w_fg and b_fg are ignored).  Inside the
   * f32 16-node tile forward (gwn_gcn_args.tcn) every workgroup merges the partials itself: no
   * finalize launch; elsewhere gwn_batchnorm_fwd_fold runs first as its own launch. */
  const struct gwn_bn_fold* bn; const float* bn_partials; int bn_nparts;
} gwn_tcn_args;
/* fg may be NULL when no backward follows (inference; c == 32 row-GEMM path): the (tanh, sigmoid)
 * pairs are then not stored. */
int gwn_gated_tcn_fwd(const gwn_tcn_args* a, hipStream_t stream);

/* Backward: dxg [rows][ld_dxg] (NULL = zero) (+ dskip [rows-skip_row0][ld_dskip] for rows >= skip_row0) ->
 *   dfg (scratch [rows][2c]), dW_fg [2c][2c] (packed like w_fg), db_fg [2c],
 *   dx [t_in*P][c]  (+)= tap-0 rows and tap-1 rows (accumulate_dx adds to existing content).
 * workspace: gwn_gated_tcn_bwd_workspace_floats(...) floats. */
typedef struct gwn_tcn_bwd_args {
  const float* x; int t_in, P, c, dilation;
  const float* w_fg; const float* fg;
  const float* dxg; long ld_dxg;
  const float* dskip; long ld_dskip; int skip_row0;
  float* dfg;
  float* dw_fg; float* db_fg;
  float* dx; int accumulate_dx;
  float* workspace;
  /* 1 = data path only (dfg, dx); dW_fg / db_fg are left to a gwn_wgrad call of the caller
   * (e.g. on a second stream) */
  int skip_weight_grads;
  /* --- optional fusions of the c == 32 row-GEMM path (zero / NULL = off) ---
   * dfg_ready: dfg already holds the gate gradient (gwn_gcn_bwd's fused epilogue wrote it); the
   *   element-wise gate backward is skipped and dxg / dskip are ignored.
   * acc_row0: with accumulate_dx, dx rows < acc_row0 are overwritten rather than accumulated
   *   (their residual part is zero, so nobody has to clear them first).
   * bn_z / bn_mean / bn_rstd / bn_sums: BatchNorm-backward statistics of the layer below over the
   *   FINAL dx (which is that BatchNorm's output gradient), from the same launch:
   *   bn_sums[j] = sum_r dx[r][j],  bn_sums[c + j] = sum_r dx[r][j] * (bn_z[r][j] - mean[j]) * rstd[j]
   *   (fixed-order partials in the workspace, then an in-order merge). */
  int dfg_ready; long acc_row0;
  const float* bn_z; const float* bn_mean; const float* bn_rstd; float* bn_sums;
  /* x_mean / x_scale / x_shift [c]: x holds the PRE-BatchNorm z of the layer below and the TCN
   * input is (z - x_mean[ci]) * x_scale[ci] + x_shift[ci] (gwn_batchnorm_fwd_fold; the weight
   * gradient applies it on load).  c % 32 == 0 path only. */
  const float* x_mean; const float* x_scale; const float* x_shift;
  /* taps / output channels as gwn_tcn_args (0 = 2 / c): dfg, fg [rows][2*c_out], dxg c_out
   * channels, dW_fg [2*c_out][ntaps*c], dx [t_in*P][c] */
  int ntaps, c_out;
} gwn_tcn_bwd_args;
int gwn_gated_tcn_bwd(const gwn_tcn_bwd_args* a, hipStream_t stream);
long gwn_gated_tcn_bwd_workspace_floats(int t_in, int P, int c, int dilation);
/* the same for ntaps taps and c_out output channels (gwn_tcn_bwd_args.ntaps / .c_out) */
long gwn_gated_tcn_bwd_workspace_floats_ex(int t_in, int P, int c, int dilation, int ntaps, int c_out);

/* ---------------------------------------------------------------------------------------------
 * Graph convolution + residual (gcn.forward model.py:41-55 and model.py:234):
 *   h = [xg, A1^T xg, (A1^T)^2 xg, ..., AK^T xg, (AK^T)^2 xg]  (piece-major concat, order=2)
 *   z = dropout(W_mlp h + b_mlp) + residual[rows shifted by d*P]
 * h is a [rows][(2K+1)c] buffer whose piece 0 already holds xg (written by the TCN);
 * supports [K] point to [n][ld_sup] matrices (the adaptive one included).  If nsup == 0 the
 * residual_convs 1x1 conv (model.py:232) is applied instead: z = W xg + b + residual.
 * Dropout keeps h(m, c) iff hash(*seed, salt, m*c_out + c) >= p, scaled by 1/(1-p)
 * (train mode only; p = 0 disables).
 * ------------------------------------------------------------------------------------------- */
typedef struct gwn_gcn_args {
  int rows, n, c, nsup;
  const float* const* sup; int ld_sup;
  float* h; long ld_h;
  const float* w_mlp; const float* b_mlp;
  const float* residual;
  float* z;
  const unsigned long long* seed_ptr; unsigned long long salt; float drop_p;
  /* optional: per-slice BatchNorm partials [rows/n][3][c] (count, mean, M2) of z,
   * written by the fused path (c == 32, n <= 512) for gwn_batchnorm_fwd_partials / _fold; NULL =
   * not wanted.  When the generic path runs instead, they are computed from z by a separate pass. */
  float* bn_partials;
  /* --- optional (zero / NULL = off), fused path only ---
   * no_pieces: the hop outputs (pieces 1..2K of h) are not stored: an inference forward that no
   *   backward follows; h then only needs piece 0 (ld_h may be c).
   * eval BatchNorm (model.py:236 with the module in eval mode) folded into the epilogue: with
   *   bn_out != NULL, bn_out[r][j] = (z - running_mean[j]) / sqrt(running_var[j] + bn_eps) *
   *   weight[j] + bias[j] is written instead of z (z may be NULL, bn_partials must be NULL).
   * layout: wave layout of the fused kernels: 0 = the persistent 16-node tile kernels where they
   *   apply (sup_g4 given, shared supports; GWN_GCN_T16=0 disables them), else one wave per
   *   32-node tile; 1 = one wave per 32-node tile always.  Other values are rejected. */
  int no_pieces;
  const float* bn_running_mean; const float* bn_running_var; const float* bn_weight; const float* bn_bias;
  float bn_eps; float* bn_out;
  int layout;
  /* operand precision of the diffusion products (gwn_dtype; 0 = GWN_DTYPE_F32, the f32-MFMA
   * kernels): GWN_DTYPE_BF16 (1): bf16 operands, fp32 accumulation (v_mfma_f32_16x16x32_bf16) on the
   * 16-node tile kernel -- the mixed-precision path of configs[2].  Needs c == 32, nsup >= 1,
   * sup_g4b, layout 0, shared supports and gwn_gcn_t16b_supported(n, nsup); GWN_ERR_ARG otherwise.
   * The mlp operands, z and the BN partials stay fp32; the hop pieces are fp32 columns of h, or
   * bf16 in pieces_bf16 when given.  GWN_DTYPE_BF16_MLP (2): the same, and the mlp takes bf16
   * operands too (the pieces and W rounded to bf16, fp32 accumulation). */
  int split_planes;
  /* per-sample supports (the per-sample-graph variant, gcn2 model.py:57-80; sup_batch <= 1 = shared):
   * slice s = t*sup_batch + b diffuses with support k at sup[k] + b*sup_bstride (floats), same
   * padded [np][ld_sup] layout.  Fused path only (c == 32, n <= 512), f32 MFMA (split_planes 0). */
  long sup_bstride; int sup_batch;
  /* residual_mean / residual_scale / residual_shift [c] (fused path): residual holds the
   * PRE-BatchNorm z of the layer below; the residual added is
   * (residual - residual_mean[j]) * residual_scale[j] + residual_shift[j]
   * (BatchNorm applied on load with gwn_batchnorm_fwd_fold's mean / scale and the BN bias). */
  const float* residual_mean; const float* residual_scale; const float* residual_shift;
  /* support split (fused tile-wave path, shared supports, nsup >= 2): each slice becomes nsup
   * workgroups, one per support (its two hops + its share of the mlp, piece 0 with support 0),
   * whose partial mlp sums [np][c] go to ksplit_ws; the last of them to finish (ksplit_count[slice],
   * a device counter that is zero on entry and left zero) adds them in support order and runs the
   * epilogue.  Finer work units for layers with too few slices to occupy the chip (a unit costs
   * about half a slice, so auto splits only when slices * nsup <= CUs; with sup_g4 given the persistent 16-node tile kernels, which already cut
   * every launch into equal per-CU tile ranges, take precedence over the auto split).  ksplit: 0 = auto,
   * 1 = off, nsup = always.  ksplit_ws: gwn_gcn_ksplit_ws_floats(rows, n, nsup) floats,
   * ksplit_count: rows / n ints; NULL = no split. */
  int ksplit; float* ksplit_ws; int* ksplit_count;
  /* sup2 [nsup] (optional, f32 fused path with shared supports): the squared supports A_k A_k in
   * the same padded layout (gwn_support_square).  Given, hop piece 2 + 2k is computed as
   * (A_k^2)^T xg in the same pass over the node features as piece 1 + 2k (no hop-to-hop
   * dependency inside a slice) -- equal to A_k^T (A_k^T xg) up to fp32 reassociation.  NULL = the
   * chained hops. */
  const float* const* sup2;
  /* w_mlp_t: w_mlp transposed, [(2*nsup+1)*c][c] (required with sup2: the power forward reads the
   * mlp's MFMA fragments as coalesced rows of it) */
  const float* w_mlp_t;
  /* c_out: output channels (model.py:152 gcn(dilation_channels, residual_channels)): the pieces
   * of h carry c channels, w_mlp is [c_out][(2K+1)c], b_mlp / residual / z / bn_partials carry
   * c_out.  0 = c.  c_out != c runs the generic path. */
  int c_out;
  /* sup_g4 [2*nsup] (optional, f32 fused path, shared supports): A_k (index 2k) and A_k^2 (2k+1) in
   * the 16-node k-interleaved layout of gwn_support_g4.  Given (layout 0, GWN_GCN_T16 not 0), the
   * persistent 16-node tile kernels run: one 16-wave workgroup per CU over an equal range of the
   * launch's 16-node tiles, each support fragment a 16-B load of four k-steps. */
  const float* const* sup_g4;
  /* sup_g4b [2*nsup] (optional, bf16 operands: split_planes >= 1): A_k and A_k^2 as
   * gwn_support_g4_bf16 copies.  Given, the 16-node tile forward runs with the diffusion on bf16
   * MFMA operands (fp32 accumulation; the mlp on bf16 operands with GWN_DTYPE_BF16_MLP, else fp32;
   * the hop pieces fp32 in h or bf16 in pieces_bf16; z and BN partials fp32). */
  const void* const* sup_g4b;
  /* xg4 (optional, the bf16 16-node tile kernel only: gwn_gcn_t16b_supported): X (the node
   * features, piece 0) and support xg4_support's hop-1 piece also written as bf16 in
   * gwn_gram_g4_bf16's tiled activation layout, X in the first slices*ceil(n/16) KiB, the hop piece
   * in the next (the adaptive-support gram's operands) */
  void* xg4; int xg4_support;
  /* pieces_bf16 (optional, the bf16 16-node tile kernel only): the hop pieces 1 .. 2*nsup written
   * as bf16 to pieces_bf16[row * ld_pb + (piece - 1) * c + ch] INSTEAD of h's fp32 columns c .. (their
   * only reader in the bf16 training step is the mlp weight gradient, gwn_wgrad_problem.Xb) */
  void* pieces_bf16; long ld_pb;
  /* bn_fold (optional, train mode, c == 32, bn_partials given): gwn_batchnorm_fwd_fold on this
   * launch's partials, issued by gwn_gcn_fwd itself (a second launch on the same stream); the
   * caller then does not call gwn_batchnorm_fwd_fold. */
  const struct gwn_bn_fold* bn_fold;
  /* tcn (optional): the layer's gated TCN (gwn_gated_tcn_fwd's arguments, its xg = h and ld_xg =
   * ld_h: the TCN writes piece 0 of h) run by this call before the diffusion.  When the f32 16-node
   * tile forward runs (c == 32, two taps, c_out == c, 16-B aligned x / h / fg / skipcat, split_planes
   * 0, sup_g4 given) it is computed inside that kernel's staging -- the slice images come straight
   * from x, and xg, fg and the skip rows are written from there -- otherwise it is issued as its own
   * launch first.  The caller then does not call gwn_gated_tcn_fwd. */
  const struct gwn_tcn_args* tcn;
  /* clock (optional, instrumentation): the 16-node tile forward kernels store each workgroup's
   * device wall clock (gwn_wall_clock_khz ticks) at its start and end, clock[2*wg] and
   * clock[2*wg + 1] (wg < CUs: one workgroup per CU); each launch overwrites the previous one's.
   * Other forward paths write nothing (the caller zeroes it first to tell). */
  unsigned long long* clock;
  /* bn_slots_used (optional, host int): set by gwn_gcn_fwd to the number of leading BN partial slots
   * that can hold rows -- the 16-node tile kernels' workgroup count, else gwn_gcn_bn_partial_count's
   * -- a consumer may pass it as nparts instead (the slots past it are zero-count) */
  int* bn_slots_used;
} gwn_gcn_args;
/* gwn_batchnorm_fwd_fold's arguments (same meaning) for gwn_gcn_args.bn_fold */
typedef struct gwn_bn_fold {
  const float* gamma; const float* beta; float* running_mean; float* running_var;
  float momentum; float eps;
  float* save_mean; float* save_rstd; float* scale;
  const float* w_next; const float* b_next; float* w_fold; float* b_fold;
  long long* num_batches_tracked;
} gwn_bn_fold;
/* c == 32, n <= 512 and ld_sup >= np = 32*ceil(n/32): one fused launch (gcn_fused.hip: node
 * features LDS-resident through the whole diffusion chain, mlp accumulated from the MFMA
 * accumulators, residual + dropout + BN partials in the epilogue).  In that case the supports
 * must be [np][ld_sup] and ZERO outside [n][n] (gwn_pad_square makes such copies).
 * Otherwise: 2K nconv GEMMs + one mlp GEMM. */
int gwn_gcn_fwd(const gwn_gcn_args* a, hipStream_t stream);
/* 1 iff gwn_gcn_fwd runs a->tcn (and its BatchNorm finalize, tcn->bn) inside its own kernel, 0 when
 * it issues them as separate launches first (or a->tcn is NULL) */
int gwn_gcn_tcn_fused(const gwn_gcn_args* a);
/* the device wall clock's rate (kHz) that gwn_gcn_args.clock counts in */
int gwn_wall_clock_khz(void);
/* number of BatchNorm partial slots gwn_gcn_fwd writes to bn_partials ([slots][3][c]):
 * max(rows/n, CUs of the device).  Every path writes all of them (slots that hold no rows get
 * count 0): the whole-slice kernels one per slice, the persistent 16-node tile kernels one per
 * workgroup (one workgroup per CU, each over an equal tile range).  The consumer
 * (gwn_batchnorm_fwd_fold / _partials) takes this as nparts. */
long gwn_gcn_bn_partial_count(int rows, int n, int c, int nsup, int ld_sup);

/* 1 iff the bf16 16-node tile gcn kernels (sup_g4b / sup_g4b_t) run for n nodes and nsup supports
 * (c == 32, their LDS fits, the t16 kernels not disabled by GWN_GCN_T16=0): the condition for
 * split_planes >= 1 and for requesting xg4 / tg4 */
int gwn_gcn_t16b_supported(int n, int nsup);

/* Backward of gwn_gcn_fwd given dh (gradient w.r.t. the dropout output, i.e. dz with the
 * dropout mask and scale already applied).  Produces dW_mlp [c][(2K+1)c], db_mlp [c], the
 * concat gradient dhcat [rows][ld_dhcat] whose piece 0 (columns 0..c) ends up holding dxg, and,
 * for support `adp_index` (-1 = none), the adjacency gradient dadp [n][ld_sup].  Workspace
 * floats from gwn_gcn_bwd_workspace_floats. */
typedef struct gwn_gcn_bwd_args {
  int rows, n, c, nsup;
  const float* const* sup; int ld_sup;
  const float* h; long ld_h;
  const float* w_mlp;
  const float* dh;
  float* dhcat; long ld_dhcat;
  float* dw_mlp; float* db_mlp;
  int adp_index; float* dadp; int accumulate_dadp;
  float* workspace;
  /* optional transposed supports (gwn_transpose) enabling the fused backward (c == 32,
   * n <= 512); NULL = generic path */
  const float* const* sup_t;
  /* 1 = data path only (dhcat); dW_mlp / db_mlp / dadp are left to gwn_wgrad / gwn_gram calls of
   * the caller (e.g. on a second stream) */
  int skip_weight_grads;
  /* --- optional fusions of the fused path (sup_t given, c == 32, n <= 512; NULL = off) ---
   * BatchNorm backward prologue (replaces gwn_batchnorm_bwd for this layer): with bn_dy != NULL,
   * dh is not read but computed per slice from the BN output gradient bn_dy [rows][c], the BN
   * input bn_z [rows][c], its saved mean / rstd, gamma and bn_sums [2c] (sum dy, sum dy*xhat,
   * e.g. gwn_gated_tcn_bwd's bn_sums):
   *   dz = gamma*rstd*(dy - sums[j]/rows - xhat*sums[c+j]/rows),  dres[r][j] = dz,
   *   dh_out[r][j] = dropout'(dz) (mask hash(seed, salt, r*c + j) >= drop_p, scale 1/(1-p)),
   *   bn_dbeta = sums[0..c), bn_dgamma = sums[c..2c)           (identical to gwn_batchnorm_bwd) */
  const float* bn_dy; const float* bn_z; const float* bn_gamma; const float* bn_mean;
  const float* bn_rstd; const float* bn_sums; float* bn_dgamma; float* bn_dbeta;
  float* dres; float* dh_out;
  const unsigned long long* seed_ptr; unsigned long long salt; float drop_p;
  /* gate backward epilogue (replaces the element-wise part of gwn_gated_tcn_bwd): with dfg != NULL
   * the input gradient dxg is not stored to dhcat piece 0; instead, with g = dxg + dskip (dskip
   * [rows - skip_row0][ld_dskip] for rows >= skip_row0, NULL = none) and fg = (tanh f, sigmoid s)
   * interleaved [rows][2c]:  dfg[r][2j] = g*s*(1 - f^2),  dfg[r][2j+1] = g*f*s*(1 - s). */
  const float* fg; const float* dskip; long ld_dskip; int skip_row0; float* dfg;
  /* wave layout of the fused kernel, as gwn_gcn_args.layout */
  int layout;
  /* per-sample supports, as gwn_gcn_args (sup and sup_t alike); needs the fused path and
   * adp_index = -1 (the per-sample variant's supports are inputs: no adjacency gradient) */
  long sup_bstride; int sup_batch;
  /* operand precision of the fused backward's diffusion products (gwn_dtype): GWN_DTYPE_F32 (0) or
   * GWN_DTYPE_BF16 (1: v_mfma_f32_16x16x32_bf16, fp32 accumulation) on the 16-node tile kernel, which
   * needs sup_g4b_t (as gwn_gcn_args.split_planes); GWN_DTYPE_BF16_MLP (2): the W^T products too */
  int split_planes;
  /* support split of the fused f32 backward, as gwn_gcn_args (partial input gradients, the last
   * workgroup of a slice adds them in support order and runs the store / gate epilogue) */
  int ksplit; float* ksplit_ws; int* ksplit_count;
  /* sup2_t [nsup] (optional, f32 fused path, shared supports): the transposed squared supports
   * (A_k^2)^T (gwn_support_square).  Given, the input gradient is computed as
   * W0^T dh + sum_k W_{1+2k}^T (A_k dh) + W_{2+2k}^T (A_k^2 dh) with every diffusion reading dh
   * (no hop-to-hop dependency).  NULL = the chained (Horner) backward. */
  const float* const* sup2_t;
  /* output channels as gwn_gcn_args.c_out (0 = c): dh [rows][c_out], dW_mlp [c_out][(2K+1)c] */
  int c_out;
  /* sup_g4_t [2*nsup] (optional): A_k^T (index 2k) and (A_k^2)^T (2k+1) in the layout of
   * gwn_support_g4: the persistent 16-node tile backward, as gwn_gcn_args.sup_g4 */
  const float* const* sup_g4_t;
  /* sup_g4b_t [2*nsup] (optional, bf16 operands: split_planes >= 1): A_k^T and (A_k^2)^T as
   * gwn_support_g4_bf16 copies: the bf16 16-node tile backward (as sup_g4b of gwn_gcn_args) */
  const void* const* sup_g4b_t;
  /* tg4 (optional, the bf16 16-node tile kernel only): t1 / t2 of the adaptive support as bf16
   * in gwn_gram_g4_bf16's tiled activation layout (t1 in the first slices*ceil(n/16) KiB, t2 in the
   * next) INSTEAD of dhcat's columns c .. 3c.  Requires skip_weight_grads (or no dadp / adp_index
   * < 0): the in-library adjacency gram reads dhcat's columns, so the caller runs
   * gwn_gram_g4_bf16 on tg4 itself; GWN_ERR_ARG otherwise */
  void* tg4;
} gwn_gcn_bwd_args;
int gwn_gcn_bwd(const gwn_gcn_bwd_args* a, hipStream_t stream);
long gwn_gcn_bwd_workspace_floats(int rows, int n, int c, int nsup);
long gwn_gcn_bwd_workspace_floats_ex(int rows, int n, int c, int nsup, int c_out);
/* partial-sum floats of the support split (gwn_gcn_args.ksplit_ws / gwn_gcn_bwd_args.ksplit_ws):
 * (rows / n) * nsup * 32*ceil(n/32) * 32 */
long gwn_gcn_ksplit_ws_floats(int rows, int n, int nsup);

/* ---------------------------------------------------------------------------------------------
 * Weight + bias gradients of a channels-last 1x1 / dilated conv, the row reduction
 *   dW[j][k] = sum_{r<R} dY[r][j] * X[r + (k / Kt) * shift][k % Kt]   (j < J, k < Kt * ntaps)
 *   db[j]    = sum_{r<R} dY[r][j]                                      (db may be NULL)
 * J and Kt multiples of 32, (J/32)*(Kt*ntaps/32) <= 16; X has x_rows >= R + (ntaps-1)*shift rows.
 * gcn mlp: J = c, X = h, Kt = (2K+1)c, ntaps = 1.  gated TCN: J = 2c, X = x, Kt = c, ntaps = 2,
 * shift = dilation*P.  Deterministic (fixed-order partial sums).
 * ------------------------------------------------------------------------------------------- */
int gwn_wgrad(const float* dY, long ldy, int J, const float* X, long ldx, long x_rows, int Kt, int ntaps,
              long shift, int R, float* dW, long ld_w, float* db, float* workspace, hipStream_t stream);
long gwn_wgrad_workspace_floats(int R, int J, int Kc);
/* the same with X = (Xz - x_mean[k % Kt]) * x_scale[k % Kt] + x_shift[k % Kt] applied on load
 * (Xz = the pre-BatchNorm z of gwn_batchnorm_fwd_fold; rows past R carry dY = 0, so zero-padded
 * rows never reach dW) */
int gwn_wgrad_bn(const float* dY, long ldy, int J, const float* X, long ldx, long x_rows, int Kt, int ntaps,
                 long shift, int R, const float* x_mean, const float* x_scale, const float* x_shift, float* dW,
                 long ld_w, float* db, float* workspace, hipStream_t stream);

/* Deferred reduction (one launch for the weight gradients of a whole backward):
 * gwn_wgrad_partials writes the gwn_wgrad_partial_count(R, J, Kc) workgroup partials
 * [count][J*Kc + J] of a gwn_wgrad_bn problem without reducing them (also for narrow 1x1 inputs,
 * Kc <= 4 with J | 256: the start conv); gwn_reduce_partials then sums
 * every segment's partials in a fixed order (deterministic) in ONE launch: out [J][ld_out] = dW,
 * out2 [J] = db (may be NULL).  At most 32 segments per call. */
typedef struct gwn_reduce_seg {
  const float* part; int nparts; long part_stride;  /* partial p at part + p * part_stride */
  int J, Kc;                                        /* rows / columns written (J <= the problem's) */
  float* out; long ld_out; float* out2;
  long db_off;  /* offset of db within a partial (0 = J*Kc; a problem computed with more rows than
                 * are written, e.g. a 12-row weight from a 32-row padded gradient: J_pad * Kc) */
} gwn_reduce_seg;
int gwn_wgrad_partial_count(int R, int J, int Kc);
int gwn_wgrad_partials(const float* dY, long ldy, int J, const float* X, long ldx, long x_rows, int Kt, int ntaps,
                       long shift, int R, const float* x_mean, const float* x_scale, const float* x_shift, float* part,
                       hipStream_t stream);
int gwn_reduce_partials(const gwn_reduce_seg* segs, int nseg, hipStream_t stream);
/* Weight-gradient partials on bf16 operands (the bf16 compute mode's head, end_conv_1 and the skip
 * convs): part[c][j*Kc + k] = sum over chunk c's rows r of bf16(dY[r][j]) bf16(X[r][k]) (fp32 sums),
 * part[c][J*Kc + j] = sum_r dY[r][j] (fp32), for the gwn_wgrad_bf16_partial_count(R, J, Kc) row
 * chunks; gwn_reduce_partials sums them (part_stride J*Kc + J).  J, Kc multiples of 128. */
int gwn_wgrad_bf16_partial_count(int R, int J, int Kc);
int gwn_wgrad_bf16_partials(const float* dY, long ldy, int J, const float* X, long ldx, int Kc, int R, float* part,
                            hipStream_t stream);

/* Grouped weight gradients: the gwn_wgrad_bn problem for the same weight shape of up to 8 layers
 * in ONE launch (the deferred gcn-mlp or gated-TCN weight gradients of a whole backward).  Problem
 * p writes nparts[p] partials [nparts][J*Kc + J] (bias last) at its `part`, where nparts comes from
 * gwn_wgrad_group_plan (the device's CUs dealt to the problems in proportion to R; the return value
 * is their sum, 0 for an unsupported shape); gwn_reduce_partials then sums them (a segment per
 * problem).  Built shapes (gwn_wgrad_group_supported): (J, Kt, ntaps) = (32, 224, 1) the gcn mlp
 * with 3 supports, (64, 32, 2) the gated TCN, (32, 512, 1) end_conv_2 on its 32-row padded
 * gradient.  x_mean / x_scale / x_shift: all three for every problem, or for none.  dY, X 16-B
 * aligned, ldy / ldx multiples of 4.  Deterministic (fixed-order sums, no float atomics). */
typedef struct gwn_wgrad_problem {
  const float* dY; long ldy;
  const float* X; long ldx; long x_rows; long shift;
  const float* x_mean; const float* x_scale; const float* x_shift;
  float* part;
  int R;
  /* Xb (optional, the gcn-mlp shape only): columns 32 .. Kc of X come from this bf16 matrix
   * (Xb[r * ldxb + k - 32], gwn_gcn_args.pieces_bf16) and only columns 0 .. 32 from X: the bf16
   * mode's hop pieces.  For every problem of the launch or for none. */
  const void* Xb; long ldxb;
} gwn_wgrad_problem;
int gwn_wgrad_group_supported(int J, int Kt, int ntaps);
int gwn_wgrad_group_plan(const int* R, int nprob, int J, int Kt, int ntaps, int* nparts);
int gwn_wgrad_group(const gwn_wgrad_problem* problems, int nprob, int J, int Kt, int ntaps, hipStream_t stream);

/* Adjacency gradient of order-2 diffusion over all slices (c = 32 channels per row):
 *   dA[v][w] (+)= sum_s sum_c X1[s*n + v][c] T1[s*n + w][c]  (+ same for X2, T2 when non-NULL)
 * i.e. both pairs (xg, dx1) and (x1, dx2) of gcn.forward's adaptive support in one launch. */
int gwn_gram(const float* x1, const float* t1, const float* x2, const float* t2, long ldx, long ldt, int n,
             int slices, float* dA, int ld_dA, int accumulate, float* workspace, hipStream_t stream);
/* The same for the adaptive support of up to 8 layers in ONE launch (+ one reduction), every layer's
 * both pairs summed into dA: layer l contributes sum over its slices of x1^T t1 + x2^T t2 (its own
 * operand pointers, common ldx / ldt, c = 32).  Workspace: gwn_gram_group_workspace_floats(n,
 * slices[], nlayers) floats.  fp32 operands (the f32 mode's training step). */
typedef struct gwn_gram_layer {
  const float* x1; const float* t1; const float* x2; const float* t2;
  int slices;
} gwn_gram_layer;
long gwn_gram_group_workspace_floats(int n, const int* slices, int nlayers);
int gwn_gram_group(const gwn_gram_layer* layers, int nlayers, long ldx, long ldt, int n, float* dA, int ld_dA,
                   int accumulate, float* workspace, hipStream_t stream);
/* gwn_gram on bf16 MFMA operands with fp32 accumulation (the bf16 mode, gwn_dtype BF16) */
int gwn_gram_bf16(const float* x1, const float* t1, const float* x2, const float* t2, long ldx, long ldt, int n,
                  int slices, float* dA, int ld_dA, int accumulate, float* workspace, hipStream_t stream);
/* workspace for any gwn_gram launch over AT MOST `slices` slices (non-decreasing in slices, so one
 * query at a schedule's largest layer covers every layer) */
long gwn_gram_workspace_floats(int n, int slices);
/* gwn_gram_bf16 on bf16 operands in the 16-node tiled activation layout (written by gwn_gcn_fwd's
 * xg4 and gwn_gcn_bwd's tg4): X[s][16 vt + j][c] at byte ((s*nt + vt)*64 + 16 g + j)*16 + 2 e for
 * c = 4 g + e (e < 4) and c = 16 + 4 g + e - 4 (e >= 4), nt = ceil(n/16), nodes >= n zero.
 * dA (+)= sum_s X1_s T1_s^T (+ X2_s T2_s^T) with fp32 accumulation; ws holds
 * gwn_gram_g4_workspace_floats(n, slices) floats (a bound for every smaller launch). */
int gwn_gram_g4_bf16(const void* x1, const void* t1, const void* x2, const void* t2, int n, int slices,
                     float* dA, int ld_dA, int accumulate, float* ws, hipStream_t stream);
long gwn_gram_g4_workspace_floats(int n, int slices);
/* gwn_gram_g4_bf16 of up to 8 layers in ONE launch (+ one reduction): each gwn_gram_layer's x1 / t1
 * point to that layer's bf16 tiled buffers (the pointer type is nominal here), x2 / t2 must be
 * x1 / t1 + slices*ceil(n/16) KiB (the xg4 / tg4 layout).  One workgroup pair per two CUs splits
 * the output rows, each walking an equal share of every layer's (slice, pair) steps with the
 * operands staged once per step in LDS.  Workspace: gwn_gram_g4_group_workspace_floats floats
 * (0: n > 368, not supported -- use gwn_gram_g4_bf16 per layer). */
long gwn_gram_g4_group_workspace_floats(int n, const int* slices, int nlayers);
int gwn_gram_g4_group(const gwn_gram_layer* layers, int nlayers, int n, float* dA, int ld_dA, int accumulate,
                      float* workspace, hipStream_t stream);

/* ---------------------------------------------------------------------------------------------
 * BatchNorm2d (model.py:236, bn = nn.BatchNorm2d(c) model.py:152) over the rows of z [rows][c].
 * train: batch mean / biased variance (eps), running stats updated with `momentum` and the
 * unbiased variance; mean/rstd saved for the backward.  eval: running stats (and, when save_mean /
 * save_rstd are given, the running mean and 1/sqrt(running_var + eps) saved for an eval backward).
 * ------------------------------------------------------------------------------------------- */
int gwn_batchnorm_fwd(const float* z, int rows, int c, const float* gamma, const float* beta,
                      float* running_mean, float* running_var, float momentum, float eps,
                      int training, float* out, float* save_mean, float* save_rstd,
                      float* workspace, hipStream_t stream);
long gwn_batchnorm_workspace_floats(int rows, int c);
/* train-mode BN from precomputed partials [nparts][3][c] (count, mean, M2), e.g. written by the
 * fused gwn_gcn_fwd: merge (fixed order), update running stats, normalise z into out. */
int gwn_batchnorm_fwd_partials(const float* z, int rows, int c, const float* partials, int nparts,
                               const float* gamma, const float* beta, float* running_mean,
                               float* running_var, float momentum, float eps, float* out,
                               float* save_mean, float* save_rstd, long long* num_batches_tracked,
                               hipStream_t stream);
/* num_batches_tracked (here and in gwn_batchnorm_fwd_fold; NULL = none): the module's counter,
 * advanced by one by the same launch (BatchNorm2d's train-mode forward, model.py:236) */
/* BatchNorm applied on load instead of a normalised copy (train mode, c == 32): merge the partials
 * and update the running statistics as gwn_batchnorm_fwd_partials; instead of writing bn(z), emit
 * scale[j] = gamma[j] * rstd[j] (bn(z) = (z - mean) * scale + beta) and fold it into the NEXT
 * layer's gated TCN (its only matrix consumer, model.py:206-212), which then reads z - mean:
 *   w_fold[n][tap*c + ci] = w_next[n][tap*c + ci] * scale[ci],
 *   b_fold[n] = b_next[n] + sum_{tap,ci} w_next[n][tap*c + ci] * beta[ci].
 * The residual add (gwn_gcn_args.residual_*) and the TCN weight gradient (gwn_tcn_bwd_args.x_*)
 * apply (z - mean) * scale + beta on load.  Centring first keeps the products as well
 * conditioned as on bn(z) itself.  w_next == NULL: statistics and scale only. */
int gwn_batchnorm_fwd_fold(const float* partials, int nparts, int c, const float* gamma, const float* beta,
                           float* running_mean, float* running_var, float momentum, float eps, float* save_mean,
                           float* save_rstd, float* scale, const float* w_next, const float* b_next, float* w_fold,
                           float* b_fold, long long* num_batches_tracked, hipStream_t stream);
/* dst[j][i] = src[i][j] for an n x n matrix (supports for the fused backward) */
int gwn_transpose(const float* src, int n, int ld_src, float* dst, int ld_dst, hipStream_t stream);
/* diagnostics: resident workgroups per CU of the fused gcn kernel (forward, or backward != 0;
 * pow != 0: the power schedule of shared supports, else the chained one) */
int gwn_fused_occupancy(int n, int backward, int pow);
/* Squared support for the power schedule of gwn_gcn_fwd / gwn_gcn_bwd (sup2 / sup2_t):
 * a2 = a a, a2_t = (a a)^T, and a_t = a^T when a_t != NULL, all [np][ld] like a (a padded support,
 * zero outside [n][n]; np a multiple of 32).  One launch (f32 MFMA). */
int gwn_support_square(const float* a, int np, int ld, float* a2, float* a2_t, float* a_t, hipStream_t stream);
/* gwn_support_square that also writes the gwn_support_g4 copies (g4_stride floats apart) of A and
 * A^2 (copies 0, 1) and, with g4_count == 4, of A^T and (A^2)^T (copies 2, 3): the adaptive
 * support's per-step preparation for the 16-node tile kernels in one launch (n <= np) */
int gwn_support_square_g4(const float* a, int np, int ld, float* a2, float* a2_t, float* a_t, int n, float* g4,
                          long g4_stride, int g4_count, hipStream_t stream);
/* 16-node k-interleaved copies of `count` padded [np][ld] supports src[c] (zero outside [n][n]) for
 * the 16-node tile kernels (gwn_gcn_args.sup_g4): with nt = ceil(n/16) column tiles and
 * nkg = ceil(n/16) groups of four 4-row k-steps,
 *   dst[c*dst_stride + ((kg*nt + t)*64 + 16*g + j)*4 + i] = src[c][16*kg + 4*i + g][16*t + j]
 * (one 1-KiB block per (k-group, tile): a wave's 16-B load per lane holds four k-steps).
 * gwn_support_g4_floats(n) = nkg*nt*256, the floats of one copy (dst_stride >= it). */
long gwn_support_g4_floats(int n);
/* the bf16 form for the bf16 16-node tile forward (gwn_gcn_args.sup_g4b): with nkg = ceil(n/32)
 * groups of 32 rows, dst[c*dst_stride + ((kg*nt + t)*64 + 16*g + j)*8 + i] =
 * bf16(src[c][32*kg + 8*g + i][16*t + j]); gwn_support_g4_bf16_elems(n) = nkg*nt*512 bf16 per copy */
long gwn_support_g4_bf16_elems(int n);
int gwn_support_g4_bf16(const float* const* src, int count, int n, int ld, void* dst, long dst_stride,
                        hipStream_t stream);
int gwn_support_g4(const float* const* src, int count, int n, int ld, float* dst, long dst_stride,
                   hipStream_t stream);
/* dst [np][ld_dst] = src (or src^T if transpose) inside [n][n], zero elsewhere (np >= n) */
int gwn_pad_square(const float* src, int n, int ld_src, float* dst, int np, int ld_dst, int transpose,
                   hipStream_t stream);
/* the same for `batch` matrices src + b*src_bstride -> dst + b*dst_bstride (per-sample supports of
 * gwnet_diff_G, model.py:244-407) */
int gwn_pad_square_batched(const float* src, int batch, long src_bstride, int n, int ld_src, float* dst, int np,
                           int ld_dst, long dst_bstride, int transpose, hipStream_t stream);

/* BN backward fused with the residual split and the dropout backward of the same layer:
 *   batch_stats != 0 (train-mode forward):  dz = gamma*rstd*(dy - mean(dy) - xhat*mean(dy*xhat))
 *   batch_stats == 0 (eval-mode forward, running statistics):  dz = gamma*rstd*dy
 *   dgamma = sum dy*xhat, dbeta = sum dy
 *   dres[r + res_row0] = dz[r]   (the residual path, model.py:234; rows < res_row0 zeroed)
 *   dh[r] = dz[r] * mask(r) / (1-p)   (dropout backward, model.py:54)  */
int gwn_batchnorm_bwd(const float* dy, const float* z, int rows, int c, const float* gamma,
                      const float* save_mean, const float* save_rstd, float* dgamma,
                      float* dbeta, float* dres, int res_row0, float* dh,
                      const unsigned long long* seed_ptr, unsigned long long salt,
                      float drop_p, int batch_stats, float* workspace, hipStream_t stream);

/* Column sums db[j] = sum_r dy[r][j] (bias gradients), fixed order. */
int gwn_colsum(const float* dy, int rows, int ncol, long ld, float* out, int accumulate,
               float* workspace, hipStream_t stream);
long gwn_colsum_workspace_floats(int rows, int ncol);

/* ---------------------------------------------------------------------------------------------
 * Masked metrics + loss gradient (engine.py:46-58, util.py:510-552 with null_val = 0):
 *   pred[b][t][v][o] = out[b][o][v][t] * std + mean,   real[b][v][o] broadcast over t
 *   metrics[0..2] = masked MAE, MAPE, RMSE;  dout = d(MAE)/d(out) (if dout != NULL)
 * ------------------------------------------------------------------------------------------- */
int gwn_masked_loss(const float* out, const float* real, long rsb, long rsn, long rso, int B,
                    int o, int n, int tf, float mean, float std, float* metrics, float* dout,
                    float* workspace, hipStream_t stream);
long gwn_masked_loss_workspace_floats(int B, int o, int n, int tf);
/* gwn_masked_loss on the head's own row layout (the fused training step: no NCHW copy of the
 * output and none of its gradient): prediction (b, oo, v, t) at y[((t*B + b)*n + v)*ld_y + oo],
 * its gradient written to dy[((t*B + b)*n + v)*ld_dy + oo] (columns o .. ld_dy zeroed; dy NULL =
 * metrics only).  Same metrics (summed in another order), same workspace. */
int gwn_masked_loss_rows(const float* y, int ld_y, const float* real, long rsb, long rsn, long rso, int B, int o,
                         int n, int tf, float mean, float std, float* metrics, float* dy, int ld_dy,
                         float* workspace, hipStream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Optimiser tail (engine.py:53-55): clip_grad_norm_(max_norm) over the listed ranges of the flat
 * gradient buffer, then torch.optim.Adam (L2 weight decay, bias correction) on the same ranges.
 * range_lo / range_hi: DEVICE arrays of nranges [lo, hi) element ranges; `total` = the number of
 * elements they cover.  step_ptr: device int64 step counter (incremented before use).
 * ------------------------------------------------------------------------------------------- */
int gwn_clip_adam(float* params, float* grads, float* exp_avg, float* exp_avg_sq,
                  const long* range_lo, const long* range_hi, int nranges, long total,
                  float max_norm, float lr, float beta1, float beta2, float eps,
                  float weight_decay, long long* step_ptr, float* workspace,
                  float* total_norm_out, hipStream_t stream);
/* workspace floats of gwn_clip_adam / gwn_adam_clipped (the 512 partials and an arrival counter that
 * the partial-sum pass -- gwn_sqnorm_partials / gwn_gather_sqnorm / gwn_clip_adam's own -- resets) */
long gwn_clip_adam_workspace_floats(long total);
/* The same update in ONE launch when the clip norm's partial sums are already in workspace[0 ..
 * 512) (gwn_gather_sqnorm): every block derives the clip coefficient from them, reads the step, and
 * the last block to finish advances *step_ptr and, when seed != NULL, the dropout counter
 * (*seed += seed_inc) -- clip_grad_norm_ + Adam + the step's counter bookkeeping (engine.py:53-55). */
int gwn_adam_clipped(float* params, float* grads, float* exp_avg, float* exp_avg_sq,
                     const long* range_lo, const long* range_hi, int nranges, long total,
                     float max_norm, float lr, float beta1, float beta2, float eps, float weight_decay,
                     long long* step_ptr, float* workspace, float* total_norm_out,
                     unsigned long long* seed, unsigned long long seed_inc, hipStream_t stream);
/* the 512 partial sums of grads^2 over the ranges into workspace[0 .. 512) (for gwn_adam_clipped) */
int gwn_sqnorm_partials(const float* grads, const long* range_lo, const long* range_hi, int nranges, long total,
                        float* workspace, hipStream_t stream);
/* gwn_gather plus the 512 partial sums of dst[i]^2 into workspace[0 .. 512) (the flat gradient's
 * unpack and its clip-norm partials in one pass; entries gathered from a zero slot add nothing) */
int gwn_gather_sqnorm(const float* src, const int* idx, float* dst, long count, float* workspace,
                      hipStream_t stream);

/* dst[i] = src[idx[i]] (parameter repacking into kernel layouts and back). */
int gwn_gather(const float* src, const int* idx, float* dst, long count, hipStream_t stream);
/* gwn_gather, except that dst[sum_dst .. sum_dst + len) receives the sum of the nvec gathered
 * vectors at sum_src + v*len (v in order): the parameter packing with the skip convs' summed bias
 * (model.py:216-222 adds every layer's skip bias into one sum) in one launch */
int gwn_gather_sum(const float* src, const int* idx, float* dst, long count, long sum_src, int nvec, int len,
                   long sum_dst, hipStream_t stream);
/* out[b][o][v][t] = y[(t*B + b)*n + v][o]  (head output back to the reference NCHW layout) */
int gwn_to_nchw(const float* y, int B, int o, int n, int t, float* out, hipStream_t stream);
/* dy[(t*B + b)*n + v][o] = dout[b][o][v][t] */
int gwn_from_nchw(const float* dout, int B, int o, int n, int t, float* dy, hipStream_t stream);
/* the same into rows of ld_dy >= o floats, columns o .. ld_dy-1 zeroed (a 32-wide padded gradient) */
int gwn_from_nchw_ld(const float* dout, int B, int o, int n, int t, float* dy, int ld_dy, hipStream_t stream);
/* sum of `count` vectors of length len spaced by stride: out[j] = sum_i x[i*stride + j] */
int gwn_sum_vectors(const float* x, int count, int len, long stride, float* out,
                    hipStream_t stream);
/* (*counter) += inc  on the device (dropout seed / step bookkeeping inside graphs) */
int gwn_increment_u64(unsigned long long* counter, unsigned long long inc, hipStream_t stream);


/* ---------------------------------------------------------------------------------------------
 * Evaluation and data ingestion (infer.hip)
 *
 * util.metric(scaler.inverse_transform(yhat[:, :, h]), real[:, :, h]) for every horizon h
 * (train.py:392-400, test.py:76-85; util.py:510-559 with null_val 0): out[h] = (mae, mape, rmse).
 * yhat / real are [S][N][H] addressed by element strides (s, h, n); pred = yhat * std + mean.
 * Workspace: gwn_horizon_metrics_workspace_floats(H) floats.  Fixed-order reductions. */
int gwn_horizon_metrics(const float* yhat, long ps, long ph, long pn, const float* real, long rs, long rh,
                        long rn, int S, int H, int N, float mean, float std, float* out, float* workspace,
                        hipStream_t stream);
long gwn_horizon_metrics_workspace_floats(int H);
/* dst[i][:] = src[idx[i]][:] for i < count, rows of row_floats floats (a shuffled mini-batch from
 * an HBM-resident sample array, util.py:36-51) */
int gwn_gather_rows(const float* src, long row_floats, const long long* idx, int count, float* dst,
                    hipStream_t stream);
/* Mini-batch of sliding windows (generate_training_data.py:28-49) straight from the raw series
 * [T][N] (fp64): for b < B, x[b][l][n] = (series[t + xoff[l]][n] (- mean) / std if scale_x,
 * computed in fp64), tod[t'] and dow[t'] appended as channels when non-NULL; y[b][l][n] the same
 * with yoff and no scaling; t = t_last[b].  x, y fp32 [B][LX or LY][N][cin]. */
int gwn_window_batch(const double* series, const double* tod, const double* dow, int N,
                     const long long* t_last, int B, const int* xoff, int LX, const int* yoff, int LY,
                     double mean, double std, int scale_x, float* x, float* y, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* GWN_H_ */
