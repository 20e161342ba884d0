// Device-side pieces of the stacking fit that used to need the host between the base fits and the
// meta model (reference train_ensemble_public.py:43-48,61; sklearn StackingClassifier.fit =
// refit every base model + cross_val_predict(method='predict_proba') → final LR):
//
//   gbdt_ranks_dev : sklearn BestSplitter's root feature-visit order of every stump of every model
//                    (host.hip sklearn_stump_ranks), with each model's constant features found on
//                    the device from its rows' bins — no host read of the masks' min / max bins;
//   oof_trees      : out-of-fold P(class 1) of a batch of GBDT fold models straight from their
//                    device node tables (f64, sklearn's rule float32(x) ≤ threshold, trees added in
//                    order: ops/reference.py tree_raw), written into the meta-feature column;
//   oof_linear     : the same for a batch of logistic regressions from the solver's device
//                    coefficients (x·w + b, features in order).
// One launch each; the stacking trainer (models/stack_trainer.py) queues them on the base models'
// stream right behind the solves, so the meta model can be launched before any host read.
#include "common.h"

namespace hfens {

constexpr int kRkThreads = 256;
constexpr int kRkMaxF = 128;

__device__ __forceinline__ unsigned sk_rand_r_dev(unsigned* s) {
  if (*s == 0u) *s = 1u;
  *s ^= *s << 13;
  *s ^= *s >> 17;
  *s ^= *s << 5;
  return *s % (2147483647u + 1u);
}

// grid B (one workgroup per model), block 256.  bins [F][ldb] u8, w [B][n] (> 0: the model's row),
// seeds [B][T] (the trees' rand_r states), ranks out [T][B][F] (visit position, F for constants).
__global__ __launch_bounds__(kRkThreads) void gbdt_ranks_dev_kernel(int T, int B, int F, int n,
                                                                    const unsigned char* __restrict__ bins,
                                                                    long long ldb, const float* __restrict__ w,
                                                                    const long long* __restrict__ seeds,
                                                                    int* __restrict__ ranks) {
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ unsigned char cst[kRkMaxF];
  __shared__ int red[2][kRkThreads / 64];
  __shared__ unsigned char feats[kRkThreads * kRkMaxF];   // one Fisher-Yates array per thread
  const float* wb = w + (size_t)b * n;
  for (int f = 0; f < F; ++f) {
    const unsigned char* bf = bins + (size_t)f * ldb;
    int mn = 256, mx = -1;
    for (int r = tid; r < n; r += kRkThreads) {
      if (wb[r] > 0.f) {
        const int v = bf[r];
        mn = min(mn, v);
        mx = max(mx, v);
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      mn = min(mn, __shfl_xor(mn, o, kWave));
      mx = max(mx, __shfl_xor(mx, o, kWave));
    }
    if (lane == 0) { red[0][wave] = mn; red[1][wave] = mx; }
    __syncthreads();
    if (tid == 0) {
      int a = red[0][0], c = red[1][0];
      for (int k = 1; k < kRkThreads / 64; ++k) { a = min(a, red[0][k]); c = max(c, red[1][k]); }
      cst[f] = (unsigned char)(c <= a);   // one occupied bin (or no rows): constant, never visited
    }
    __syncthreads();
  }
  unsigned char* fs = feats + (size_t)tid * kRkMaxF;
  for (int t = tid; t < T; t += kRkThreads) {
    unsigned st = (unsigned)seeds[(size_t)b * T + t];
    int* rk = ranks + ((size_t)t * B + b) * F;
    for (int f = 0; f < F; ++f) { fs[f] = (unsigned char)f; rk[f] = F; }
    int f_i = F, n_found = 0, n_total = 0, visited = 0, pos = 0;
    while (f_i > n_total && (visited < F || visited <= n_found)) {
      ++visited;
      const int f_j = (int)(sk_rand_r_dev(&st) % (unsigned)(f_i - n_found)) + n_found;
      const int cur = fs[f_j];
      if (cst[cur]) {
        fs[f_j] = fs[n_total];
        fs[n_total] = (unsigned char)cur;
        ++n_found;
        ++n_total;
        continue;
      }
      --f_i;
      fs[f_j] = fs[f_i];
      fs[f_i] = (unsigned char)cur;
      rk[cur] = pos++;
    }
  }
}

void gbdt_ranks_dev(int T, int B, int F, int n, uintptr_t bins, long long ldb, uintptr_t w, uintptr_t seeds,
                    uintptr_t ranks, uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F <= kRkMaxF && B >= 1 && T >= 1 && n >= 0 && ldb >= n,
                "gbdt_ranks_dev: 1 <= F <= 128, B, T >= 1, ldb >= n");
  hipLaunchKernelGGL(gbdt_ranks_dev_kernel, dim3(B), dim3(kRkThreads), 0, as_stream(stream), T, B, F, n,
                     (const unsigned char*)bins, ldb, (const float*)w, (const long long*)seeds, (int*)ranks);
  launch_check();
}

__device__ __forceinline__ double sigmoid_f64(double z) { return 1.0 / (1.0 + exp(-z)); }

// One thread per listed row.  rows [m] (row of X), model [m] (which fold model predicts it);
// tree tables [T][B][NN] in heap layout (children of node k: 2k+1, 2k+2; feat < 0: leaf);
// init [B] raw prior log-odds.  meta[row·ld + col] = σ(init + Σ_t lr·v_t) added tree by tree.
__global__ __launch_bounds__(256) void oof_trees_kernel(const double* __restrict__ X, int F,
                                                        const long long* __restrict__ rows,
                                                        const int* __restrict__ model, long long m, int T, int B,
                                                        int NN, const int* __restrict__ feat,
                                                        const double* __restrict__ thr,
                                                        const double* __restrict__ value,
                                                        const double* __restrict__ init, double lr,
                                                        double* __restrict__ meta, int ld, int col) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const long long r = rows[i];
  const int b = model[i];
  const double* x = X + (size_t)r * F;
  double raw = init[b];
  for (int t = 0; t < T; ++t) {
    const size_t base = ((size_t)t * B + b) * NN;
    int k = 0;
    for (int d = 0; d < 32; ++d) {   // depth ≤ 5 in practice; bounded walk
      const int f = feat[base + k];
      if (f < 0) break;
      const double xv = (double)(float)x[f];
      k = xv <= thr[base + k] ? 2 * k + 1 : 2 * k + 2;
      if (k >= NN) { k = (k - 1) / 2; break; }   // (malformed table: stay at the parent)
    }
    raw = __dadd_rn(raw, __dmul_rn(lr, value[base + k]));
  }
  meta[(size_t)r * ld + col] = sigmoid_f64(raw);
}

void oof_trees(uintptr_t X, int F, uintptr_t rows, uintptr_t model, long long m, int T, int B, int NN, uintptr_t feat,
               uintptr_t thr, uintptr_t value, uintptr_t init, double lr, uintptr_t meta, int ld, int col,
               uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && T >= 1 && B >= 1 && NN >= 1 && col >= 0 && col < ld, "oof_trees: bad shape");
  if (m == 0) return;
  hipLaunchKernelGGL(oof_trees_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, as_stream(stream),
                     (const double*)X, F, (const long long*)rows, (const int*)model, m, T, B, NN, (const int*)feat,
                     (const double*)thr, (const double*)value, (const double*)init, lr, (double*)meta, ld, col);
  launch_check();
}

// W [B][F1] (coefficients, then the intercept column when has_icpt, scaled by icpt_scale).
__global__ __launch_bounds__(256) void oof_linear_kernel(const double* __restrict__ X, int F,
                                                         const long long* __restrict__ rows,
                                                         const int* __restrict__ model, long long m,
                                                         const double* __restrict__ W, int F1, int has_icpt,
                                                         double icpt_scale, double* __restrict__ meta, int ld,
                                                         int col) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const long long r = rows[i];
  const double* x = X + (size_t)r * F;
  const double* wb = W + (size_t)model[i] * F1;
  double z = 0.0;
  for (int f = 0; f < F; ++f) z = __dadd_rn(z, __dmul_rn(x[f], wb[f]));
  if (has_icpt) z = __dadd_rn(z, __dmul_rn(wb[F], icpt_scale));
  meta[(size_t)r * ld + col] = sigmoid_f64(z);
}

void oof_linear(uintptr_t X, int F, uintptr_t rows, uintptr_t model, long long m, uintptr_t W, int F1, int has_icpt,
                double icpt_scale, uintptr_t meta, int ld, int col, uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F1 >= F && F1 <= F + 1 && col >= 0 && col < ld, "oof_linear: bad shape");
  if (m == 0) return;
  hipLaunchKernelGGL(oof_linear_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, as_stream(stream),
                     (const double*)X, F, (const long long*)rows, (const int*)model, m, (const double*)W, F1,
                     has_icpt, icpt_scale, (double*)meta, ld, col);
  launch_check();
}

}  // namespace hfens
