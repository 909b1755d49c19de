// Internal helpers shared by the HIP translation units of libgwn (not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/gwn.h"

// After every launch: the launch status; with GWN_SYNC_CHECK=1 in the environment (debugging
// only) also a device synchronise, so an asynchronous fault is reported at file:line of its kernel.
int gwn_launch_status(const char* file, int line);
// GWN_SYNC_CHECK only: [p, p + bytes) must lie inside one device allocation (else an error code)
int gwn_debug_range(const void* p, long bytes, const char* what);
#define GWN_DEBUG_RANGE(p, bytes, what)                        \
  do {                                                         \
    const int rr_ = gwn_debug_range((p), (bytes), (what));     \
    if (rr_) return rr_;                                       \
  } while (0)
#define GWN_CHECK_LAUNCH()                                   \
  do {                                                       \
    const int rc_ = gwn_launch_status(__FILE__, __LINE__);   \
    if (rc_) return rc_;                                     \
  } while (0)

#define GWN_REQUIRE(cond, msg)                                \
  do {                                                        \
    if (!(cond)) return gwn_set_error(GWN_ERR_ARG, msg);      \
  } while (0)

int gwn_set_error(int code, const char* msg);

// ---------------------------------------------------------------------------------------------
// Generic fp32 MFMA GEMM (gemm.hip).  C(m,n) = epi(alpha * sum_k A(m,k) B(k,n)).
//
// Two-level indices let one launch walk "slices" that are not a single stride apart:
//   A(m,k): ko = k / a_kin, ki = k % a_kin; src_row = m + ko*a_row_shift (valid iff
//           0 <= src_row < a_rows); addr = A + src_row*lda_m + ki*lda_k + ko*a_ko_stride
//   B(k,n): kb = k / b_kin, kj = k % b_kin; no = n / b_nin, ni = n % b_nin;
//           addr = B + kj*ldb_k + kb*b_ko_stride + ni*ldb_n + no*b_no_stride
//   C(m,n): no = n / c_nin, ni = n % c_nin; addr = C + m*ldc_m + ni*ldc_n + no*c_no_stride
// a_kin / b_kin must be multiples of 16 (or >= K); b_nin / c_nin multiples of 32 (or >= N).
// ---------------------------------------------------------------------------------------------
enum GemmEpi {
  EPI_STORE = 0,      // v = alpha*acc + bias_n[n] (+relu) (+dropout) + beta*C0
  EPI_GATE = 1,       // n = 2c+g: (tanh(f) * sigmoid(g)) -> C[m][c]; aux = (tanh f, sigmoid g); aux2 dual store
  EPI_MASKGRAD = 2,   // v = alpha*acc * (mask[m][n] > 0) + beta*C0   (relu backward)
};

typedef gwn_gemm_desc GemmParams;

int gwn_gemm_launch(const GemmParams& p, hipStream_t stream);

// Fused diffusion GCN (gcn_fused.hip)
bool gwn_gcn_fused_eligible(int c, int n, int nsup, int ld_sup);
// *folded: the launch also ran g->bn_fold (the 16-node tile kernels' last-workgroup finalize)
// *used (optional): the leading BN partial slots that can hold rows (the t16 kernels' grid; else
// gwn_bn_part_slots: the slots past it are written as zeros either way)
int gwn_gcn_fused_fwd_launch(const gwn_gcn_args* g, float* bn_part, hipStream_t s, int* used = nullptr);
bool gwn_gcn_tcn_fusable(const gwn_gcn_args* g);
int gwn_device_cus();  // compute units of the current device (cached)
// BatchNorm partial slots of a gwn_gcn_fwd launch over `slices` slices (every slot written)
long gwn_bn_part_slots(int slices);
int gwn_gcn_fused_bwd_launch(const gwn_gcn_bwd_args* g, const float* const* supT, float* dxg, long ld_dxg,
                             float* t1, float* t2, long ld_t, hipStream_t s);

// Large-graph diffusion (bigdiff.hip): y_s = G^T x_s (+ y0) over all slices, n > 512, c = 32
bool gwn_bigdiff_eligible(int n, int c, const float* G, int ldg, const float* x, long ldx, const float* y, long ldy,
                          const float* y0, long ldy0);
int gwn_bigdiff(const float* G, int ldg, const float* x, long ldx, float* y, long ldy, const float* y0, long ldy0,
                int n, int slices, hipStream_t s);

// gwn_gram with the operand precision of the bf16 mode (bf16 != 0: bf16 MFMA operands, fp32 sums)
int gwn_gram_dtype(const float* x1, const float* t1, const float* x2, const float* t2, long ldx, long ldt, int n,
                   int slices, float* dA, int ld_dA, int accumulate, float* ws, int bf16, hipStream_t s);

// Weight-stationary row GEMMs of the gated TCN (rowgemm.hip), c = 32
int gwn_rowgemm_tcn_fwd(const gwn_tcn_args* a, hipStream_t s);
int gwn_rowgemm_tcn_bwd_data(const gwn_tcn_bwd_args* a, hipStream_t s);
int gwn_rowgemm_tcn_bwd_nparts(const gwn_tcn_bwd_args* a);
constexpr int GWN_ROWGEMM_MAX_PARTS = 2048;  // waves of one rowgemm launch (8 per CU)

// Deterministic counter-based dropout RNG, identical in every kernel that applies or
// differentiates the same mask: a 32-bit key of (seed, salt) (uniform per launch), then per element
// the lowbias32 finaliser (two multiplies) of idx * phi + key -- 32-bit arithmetic throughout (the
// splitmix64 form it replaces spent ~30 VALU ops per element on 64-bit multiplies).  idx < 2^32.
// Branch-free gate nonlinearities of the gated TCN (model.py:206-212) on v_exp_f32 / v_rcp_f32:
// absolute error ~1e-7 (a few ulp of 1); the row-GEMM TCN and the gcn-fused TCN share them.
__device__ __forceinline__ float gwn_gate_sigmoid(float x) { return __frcp_rn(1.0f + __expf(-x)); }
__device__ __forceinline__ float gwn_gate_tanh(float x) { return 1.0f - 2.0f * __frcp_rn(__expf(2.0f * x) + 1.0f); }

__host__ __device__ inline unsigned gwn_mix32(unsigned h) {
  h ^= h >> 16;
  h *= 0x7FEB352Du;
  h ^= h >> 15;
  h *= 0x846CA68Bu;
  h ^= h >> 16;
  return h;
}
// idx < 2^32: the launches that apply dropout check rows * channels < 2^32 on the host
// (gwn_gcn_fwd / gwn_gcn_bwd / gwn_batchnorm_bwd), so a mask never repeats within a tensor.
__host__ __device__ inline float gwn_uniform(unsigned long long seed, unsigned long long salt,
                                             unsigned long long idx) {
  const unsigned key = gwn_mix32((unsigned)seed ^ gwn_mix32((unsigned)(seed >> 32) + 0x9E3779B9u * ((unsigned)salt + 1u)));
  return (float)(gwn_mix32((unsigned)idx * 0x9E3779B1u + key) >> 8) * (1.0f / 16777216.0f);
}
