// Batched StandardScaler fit + transform (SURVEY.md §2.3 K2 col_moments; reference
// train_ensemble_public.py:44 make_pipeline(StandardScaler(), SVC(...)) fitted once per stacking
// fold): K row subsets of one f64 matrix X [n][F] (the 5 fold-training sets + the full set).
//
//  scaler_sums  : grid (K, splits) — per (subset, split) partial Σx, then (second launch, given the
//                 means) partial Σ(x − mean)²; 256 threads = 4 row lanes × 64 columns, rows of the
//                 subset read through its index list (one coalesced row per 64 threads)
//  scaler_apply : mean, population variance and scale (0 → 1, sklearn 0.23.2) from the partials,
//                 summed in split order (deterministic), and Z[off_k + i] = (X[rows_k[i]] − mean_k) /
//                 scale_k into ONE concatenated output — every fold's scaled matrix in one launch.
// The two-pass form (mean, then Σ(x − mean)²) keeps the variance free of E[x²] − mean² cancellation.
#include "common.h"

namespace hfens {

constexpr int kScThreads = 256;
constexpr int kScCols = 64;                       // F ≤ 64
constexpr int kScLanes = kScThreads / kScCols;    // row lanes per block

// pass 0: part[k][s][c] = Σ x ; pass 1: part[k][s][c] = Σ (x − mean_k[c])²  (mean from pass-0 partials)
__global__ __launch_bounds__(kScThreads) void scaler_sums_kernel(const double* __restrict__ X, int F,
                                                                 const long long* __restrict__ rows,
                                                                 const long long* __restrict__ offs, int S,
                                                                 const double* __restrict__ part0, double* __restrict__ part) {
  __shared__ double red[kScLanes][kScCols];
  __shared__ double mean[kScCols];
  const int k = blockIdx.x, s = blockIdx.y;
  const int c = threadIdx.x % kScCols, rl = threadIdx.x / kScCols;
  const long long o0 = offs[k], o1 = offs[k + 1], nk = o1 - o0;
  if (part0 != nullptr && threadIdx.x < kScCols) {
    double t = 0.0;
    for (int q = 0; q < S; ++q) t += part0[((size_t)k * S + q) * kScCols + threadIdx.x];
    mean[threadIdx.x] = nk > 0 ? t / (double)nk : 0.0;
  }
  __syncthreads();
  const long long per = (nk + S - 1) / S;
  const long long b = o0 + (long long)s * per, e = min(o1, b + per);
  double acc = 0.0;
  if (c < F) {
    const double mc = part0 != nullptr ? mean[c] : 0.0;
    for (long long i = b + rl; i < e; i += kScLanes) {
      const double x = X[rows[i] * F + c];
      if (part0 != nullptr) {
        const double d = x - mc;
        acc = fma(d, d, acc);
      } else {
        acc += x;
      }
    }
  }
  red[rl][c] = acc;
  __syncthreads();
  if (threadIdx.x < kScCols) {
    double t = 0.0;
    for (int q = 0; q < kScLanes; ++q) t += red[q][threadIdx.x];
    part[((size_t)k * S + s) * kScCols + threadIdx.x] = t;
  }
}

__global__ __launch_bounds__(kScThreads) void scaler_apply_kernel(const double* __restrict__ X, int F,
                                                                  const long long* __restrict__ rows,
                                                                  const long long* __restrict__ offs, int S,
                                                                  const double* __restrict__ p_sum,
                                                                  const double* __restrict__ p_m2,
                                                                  double* __restrict__ mean_out,
                                                                  double* __restrict__ var_out,
                                                                  double* __restrict__ Z, int row_blocks) {
  __shared__ double mean[kScCols], scale[kScCols];
  const int k = blockIdx.x;
  const long long o0 = offs[k], o1 = offs[k + 1], nk = o1 - o0;
  if (threadIdx.x < kScCols) {
    double t = 0.0, m2 = 0.0;
    for (int q = 0; q < S; ++q) {
      t += p_sum[((size_t)k * S + q) * kScCols + threadIdx.x];
      m2 += p_m2[((size_t)k * S + q) * kScCols + threadIdx.x];
    }
    const double m = nk > 0 ? t / (double)nk : 0.0;
    const double v = nk > 0 ? m2 / (double)nk : 0.0;
    const double sd = sqrt(v);
    mean[threadIdx.x] = m;
    scale[threadIdx.x] = sd == 0.0 ? 1.0 : sd;
    if (blockIdx.y == 0 && threadIdx.x < F) {
      mean_out[(size_t)k * F + threadIdx.x] = m;
      var_out[(size_t)k * F + threadIdx.x] = v;
    }
  }
  __syncthreads();
  const int c = threadIdx.x % kScCols, rl = threadIdx.x / kScCols;
  if (c >= F) return;
  const double mc = mean[c], sc = scale[c];
  for (long long i = o0 + (long long)blockIdx.y * kScLanes + rl; i < o1; i += (long long)row_blocks * kScLanes)
    Z[i * F + c] = (X[rows[i] * F + c] - mc) / sc;
}

void scaler_batch(uintptr_t X, long long n, int F, uintptr_t rows, uintptr_t offs, int K, long long max_rows,
                  uintptr_t part, uintptr_t mean, uintptr_t var, uintptr_t Z, uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F <= kScCols && K >= 1 && n >= 1, "scaler_batch: 1 <= F <= 64, K >= 1");
  hipStream_t st = as_stream(stream);
  // ≥ 1024 rows per split, ≤ 64 splits: ≈ K·S blocks of partial sums
  int S = (int)((max_rows + 1023) / 1024);
  S = S < 1 ? 1 : (S > 64 ? 64 : S);
  double* p_sum = (double*)part;
  double* p_m2 = p_sum + (size_t)K * S * kScCols;
  const auto* Xp = (const double*)X;
  const auto* rp = (const long long*)rows;
  const auto* op = (const long long*)offs;
  hipLaunchKernelGGL(scaler_sums_kernel, dim3(K, S), dim3(kScThreads), 0, st, Xp, F, rp, op, S, nullptr, p_sum);
  launch_check();
  hipLaunchKernelGGL(scaler_sums_kernel, dim3(K, S), dim3(kScThreads), 0, st, Xp, F, rp, op, S, p_sum, p_m2);
  launch_check();
  const int rb = (int)((max_rows + 4 * kScLanes - 1) / (4 * kScLanes)) > 256 ? 256
                 : (int)((max_rows + 4 * kScLanes - 1) / (4 * kScLanes));
  hipLaunchKernelGGL(scaler_apply_kernel, dim3(K, rb < 1 ? 1 : rb), dim3(kScThreads), 0, st, Xp, F, rp, op, S,
                     p_sum, p_m2, (double*)mean, (double*)var, (double*)Z, rb < 1 ? 1 : rb);
  launch_check();
}

}  // namespace hfens
