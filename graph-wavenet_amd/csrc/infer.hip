// Inference-side kernels of libgwn (the reference's evaluation path, train.py:377-404 and
// test.py:58-87, and its data ingestion, Utils/util.py:14-54 + generate_training_data.py:12-49):
//
//  * gwn_horizon_metrics — util.metric(pred, real) (util.py:510-559, null_val 0) for every horizon
//    of a whole test-set prediction in two launches (per-block partials, fixed-order final), where
//    the reference loops over 12 horizons with 3 masked-metric calls and 3 host syncs each.
//  * gwn_gather_rows — mini-batch assembly from an HBM-resident sample array by an index vector
//    (util.DataLoader's shuffle + slicing, with the dataset uploaded once).
//  * gwn_window_batch — mini-batch assembly straight from the raw sensor series (one copy of the
//    readings in HBM instead of the 12x-duplicated sliding-window arrays): sample t gets
//    x = series[t + x_offsets] (channel 0 scaled in fp64 like StandardScaler on the host's float64
//    arrays, then rounded to fp32), time-of-day (and day-of-week) channels; y unscaled.
#include "gwn_internal.h"

namespace {

constexpr int HM_BLOCKS = 64;  // partial blocks per horizon (fixed -> fixed summation order)

template <int NT>
__device__ float bsum(float v, float* sh) {
  sh[threadIdx.x] = v;
  __syncthreads();
#pragma unroll
  for (int s = NT / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) sh[threadIdx.x] += sh[threadIdx.x + s];
    __syncthreads();
  }
  const float r = sh[0];
  __syncthreads();
  return r;
}

// partial[h][blk][4] = (count, sum |d|, sum |d| / y, sum d^2) over labels y != 0, d = pred - y,
// pred = yhat * std + mean (StandardScaler.inverse_transform)
__global__ void horizon_partial_kernel(const float* yhat, long ps, long ph, long pn, const float* real, long rs,
                                       long rh, long rn, int S, int N, float mean, float std, float* part) {
  __shared__ float sh[256];
  const int h = blockIdx.y, blk = blockIdx.x;
  const long total = (long)S * N;
  float c = 0.0f, a = 0.0f, p = 0.0f, q = 0.0f;
  for (long i = (long)blk * 256 + threadIdx.x; i < total; i += 256L * HM_BLOCKS) {
    const long s = i / N;
    const int n = (int)(i - s * N);
    const float y = real[s * rs + h * rh + n * rn];
    if (y != 0.0f) {
      const float pred = yhat[s * ps + h * ph + n * pn] * std + mean;
      const float d = pred - y;
      c += 1.0f;
      a += fabsf(d);
      p += fabsf(d) / y;
      q += d * d;
    }
  }
  c = bsum<256>(c, sh);
  a = bsum<256>(a, sh);
  p = bsum<256>(p, sh);
  q = bsum<256>(q, sh);
  if (threadIdx.x == 0) {
    float* o = part + ((long)h * HM_BLOCKS + blk) * 4;
    o[0] = c; o[1] = a; o[2] = p; o[3] = q;
  }
}

__global__ void horizon_final_kernel(const float* part, int H, float* out) {
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= H) return;
  double c = 0.0, a = 0.0, p = 0.0, q = 0.0;
  for (int b = 0; b < HM_BLOCKS; ++b) {
    const float* o = part + ((long)h * HM_BLOCKS + b) * 4;
    c += o[0]; a += o[1]; p += o[2]; q += o[3];
  }
  // reference: mask / mean(mask) with the mean over all S*N labels and the loss mean over S*N,
  // i.e. sum / count; no labels: the NaN mask is zeroed and every metric is 0
  out[3 * h] = c > 0.0 ? (float)(a / c) : 0.0f;
  out[3 * h + 1] = c > 0.0 ? (float)(p / c) : 0.0f;
  out[3 * h + 2] = c > 0.0 ? (float)sqrt(q / c) : 0.0f;
}

// dst[i][:] = src[idx[i]][:] (row_floats per row, 16-B quads when aligned)
__global__ void gather_rows_kernel(const float* src, long row_floats, const long long* idx, int count, float* dst,
                                   int vec) {
  const long per = vec ? row_floats / 4 : row_floats;
  const long total = per * count;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long i = e / per, j = e - i * per;
    const long r = idx[i];
    if (vec) ((float4*)dst)[i * per + j] = ((const float4*)src)[r * per + j];
    else dst[i * row_floats + j] = src[r * row_floats + j];
  }
}

// x [B][LX][N][cin], y [B][LY][N][cin] (cin = 1 + has_tod + has_dow) from series [T][N] (fp64),
// tod [T], dow [T] (fp64); sample b is the window whose last observation is t_last[b]
__global__ void window_batch_kernel(const double* series, const double* tod, const double* dow, int N,
                                    const long long* t_last, int B, const int* xoff, int LX, const int* yoff,
                                    int LY, double mean, double std, int scale_x, int cin, float* x, float* y) {
  const long xtot = (long)B * LX * N, ytot = (long)B * LY * N;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < xtot + ytot; e += (long)gridDim.x * blockDim.x) {
    const bool isx = e < xtot;
    const long f = isx ? e : e - xtot;
    const int L = isx ? LX : LY;
    const int n = (int)(f % N);
    const long bl = f / N;
    const int l = (int)(bl % L);
    const int b = (int)(bl / L);
    const long t = t_last[b] + (isx ? xoff[l] : yoff[l]);
    double v = series[t * N + n];
    if (isx && scale_x) v = (v - mean) / std;
    float* o = (isx ? x : y) + f * cin;
    o[0] = (float)v;
    int k = 1;
    if (tod) o[k++] = (float)tod[t];
    if (dow) o[k++] = (float)dow[t];
  }
}

inline unsigned grid_for(long n) {
  long g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace

extern "C" {

long gwn_horizon_metrics_workspace_floats(int H) { return (long)H * HM_BLOCKS * 4; }

int gwn_horizon_metrics(const float* yhat, long ps, long ph, long pn, const float* real, long rs, long rh, long rn,
                        int S, int H, int N, float mean, float std, float* out, float* ws, hipStream_t s) {
  GWN_REQUIRE(yhat && real && out && ws && S > 0 && H > 0 && N > 0 && H <= 65535, "horizon_metrics: bad arguments");
  horizon_partial_kernel<<<dim3(HM_BLOCKS, H), 256, 0, s>>>(yhat, ps, ph, pn, real, rs, rh, rn, S, N, mean, std, ws);
  GWN_CHECK_LAUNCH();
  horizon_final_kernel<<<(H + 63) / 64, 64, 0, s>>>(ws, H, out);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

int gwn_gather_rows(const float* src, long row_floats, const long long* idx, int count, float* dst, hipStream_t s) {
  GWN_REQUIRE(src && idx && dst && row_floats > 0 && count > 0, "gather_rows: bad arguments");
  const int vec = (row_floats % 4 == 0) && ((uintptr_t)src % 16 == 0) && ((uintptr_t)dst % 16 == 0);
  gather_rows_kernel<<<grid_for(count * (vec ? row_floats / 4 : row_floats)), 256, 0, s>>>(src, row_floats, idx,
                                                                                          count, dst, vec);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

int gwn_window_batch(const double* series, const double* tod, const double* dow, int N, const long long* t_last,
                     int B, const int* xoff, int LX, const int* yoff, int LY, double mean, double std, int scale_x,
                     float* x, float* y, hipStream_t s) {
  GWN_REQUIRE(series && t_last && xoff && yoff && x && y && N > 0 && B > 0 && LX > 0 && LY > 0 && std != 0.0,
              "window_batch: bad arguments");
  const int cin = 1 + (tod ? 1 : 0) + (dow ? 1 : 0);
  window_batch_kernel<<<grid_for((long)B * (LX + LY) * N), 256, 0, s>>>(series, tod, dow, N, t_last, B, xoff, LX,
                                                                         yoff, LY, mean, std, scale_x, cin, x, y);
  GWN_CHECK_LAUNCH();
  return GWN_OK;
}

}  // extern "C"
