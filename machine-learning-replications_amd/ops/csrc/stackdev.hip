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

constexpr int kRkThreads = 1024;
constexpr int kRkMaxF = 128;

__device__ __forceinline__ unsigned sk_rand_r_dev(unsigned* s) {
  if (*s == 0u) *s = 1u;
  *s ^= *s << 13;
  *s ^= *s >> 17;
  *s ^= *s << 5;
  return *s % (2147483647u + 1u);
}

// grid B (one workgroup per model), block 1024.  bins [F][ldb] u8, w [B][n] (> 0: the model's row),
// seeds [B][T] (the trees' rand_r states), ranks out [T][B][F] (visit position, F for constants).
// Constant features: wave v scans features v, v + 16, … over all rows (4 rows per lane and load
// when the rows are 4-aligned), min / max occupied bin by DPP-free xor shuffles, no barrier per
// feature; then thread t walks tree t's Fisher-Yates draw.
__global__ __launch_bounds__(kRkThreads) void gbdt_ranks_dev_kernel(int T, int B, int F, int n,
                                                                    const unsigned char* __restrict__ bins,
                                                                    long long ldb, const float* __restrict__ w,
                                                                    const long long* __restrict__ seeds,
                                                                    int* __restrict__ ranks) {
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int kW = kRkThreads / 64;
  __shared__ unsigned char cst[kRkMaxF];
  __shared__ unsigned char feats[kRkThreads / 4 * kRkMaxF];   // Fisher-Yates arrays (threads < T ≤ 256 used)
  const float* wb = w + (size_t)b * n;
  const bool vec = (n % 4) == 0 && (ldb % 4) == 0 && ((uintptr_t)bins % 4) == 0 && ((uintptr_t)w % 16) == 0;
  for (int f = wave; f < F; f += kW) {
    const unsigned char* bf = bins + (size_t)f * ldb;
    int mn = 256, mx = -1;
    if (vec) {
#pragma unroll 4
      for (int r = 4 * lane; r < n; r += 256) {
        const unsigned bv = *reinterpret_cast<const unsigned*>(bf + r);
        const float4 wv = *reinterpret_cast<const float4*>(wb + r);
        const float ww[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int v = (int)((bv >> (8 * q)) & 0xFFu);
          mn = ww[q] > 0.f ? min(mn, v) : mn;
          mx = ww[q] > 0.f ? max(mx, v) : mx;
        }
      }
    } else {
      for (int r = lane; r < n; r += 64) {
        if (wb[r] > 0.f) {
          const int v = bf[r];
          mn = min(mn, v);
          mx = max(mx, v);
        }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      mn = min(mn, __shfl_xor(mn, o, kWave));
      mx = max(mx, __shfl_xor(mx, o, kWave));
    }
    if (lane == 0) cst[f] = (unsigned char)(mx <= mn);   // one occupied bin (or no rows): constant
  }
  __syncthreads();
  if (tid >= kRkThreads / 4) return;
  unsigned char* fs = feats + (size_t)tid * kRkMaxF;
  for (int t = tid; t < T; t += kRkThreads / 4) {
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

// ---- SVC γ on the device (gamma='scale' = 1 / (F · Var(Z)), sklearn svm/_base.py) ---------------
// One workgroup per fit over its scaled rows Z [l_f][F] (f64, rows offs[f] … offs[f+1] of one
// concatenated matrix): two passes (mean, then Σ(z − mean)²) in a fixed order (deterministic).
// gamma[f] f64 (NaN when Z has a non-finite value: raised by the host where it reads γ), and
// ngl2e[f] = f32(−γ·log2 e), the field the SVC kernels' problem records carry.  With this the
// stacking trainer enqueues the whole SVC batch (problem records patched on the device, below)
// before the selected columns are even known on the host.
constexpr int kGmThreads = 1024;

__device__ __forceinline__ double block_sum_gm(double v, double* sh) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  double r = 0.0;
  for (int w = 0; w < kGmThreads / 64; ++w) r += sh[w];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(kGmThreads) void svm_gamma_kernel(const double* __restrict__ Z, const long long* __restrict__ offs,
                                                               int F, double* __restrict__ gamma,
                                                               float* __restrict__ ngl2e) {
  __shared__ double sh[kGmThreads / 64];
  const int f = blockIdx.x;
  const long long b = offs[f] * F, e = offs[f + 1] * F;
  const double cnt = (double)(e - b);
  double s = 0.0;
  bool fin = true;
  for (long long i = b + threadIdx.x; i < e; i += kGmThreads) {
    const double z = Z[i];
    fin = fin && isfinite(z);
    s += z;
  }
  const double tot = block_sum_gm(s, sh);
  const double bad = block_sum_gm(fin ? 0.0 : 1.0, sh);
  const double mean = cnt > 0 ? tot / cnt : 0.0;
  double q = 0.0;
  for (long long i = b + threadIdx.x; i < e; i += kGmThreads) {
    const double d = Z[i] - mean;
    q += d * d;
  }
  const double var = cnt > 0 ? block_sum_gm(q, sh) / cnt : 0.0;
  if (threadIdx.x == 0) {
    double g = var != 0.0 ? 1.0 / ((double)F * var) : 1.0;
    if (bad != 0.0 || !isfinite(var)) g = __longlong_as_double(0x7ff8000000000000LL);   // NaN
    gamma[f] = g;
    ngl2e[f] = (float)(-g * 1.4426950408889634);
  }
}

void svm_gamma(uintptr_t Z, uintptr_t offs, int K, int F, uintptr_t gamma, uintptr_t ngl2e, uintptr_t stream) {
  HFENS_REQUIRE(K >= 1 && F >= 1, "svm_gamma: K, F >= 1");
  hipLaunchKernelGGL(svm_gamma_kernel, dim3(K), dim3(kGmThreads), 0, as_stream(stream), (const double*)Z,
                     (const long long*)offs, F, (double*)gamma, (float*)ngl2e);
  launch_check();
}

// record i of an array of `count` structs (stride bytes): its f32 field at byte `off` ← src[fit_of[i]]
__global__ void svm_patch_f32_kernel(unsigned char* __restrict__ base, int stride, int off, int count,
                                     const int* __restrict__ fit_of, const float* __restrict__ src) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) *reinterpret_cast<float*>(base + (size_t)i * stride + off) = src[fit_of[i]];
}

void svm_patch_f32(uintptr_t base, int stride, int off, int count, uintptr_t fit_of, uintptr_t src, uintptr_t stream) {
  HFENS_REQUIRE(stride > 0 && off >= 0 && off + 4 <= stride && (off % 4) == 0 && count >= 0, "svm_patch_f32: bad layout");
  if (count == 0) return;
  hipLaunchKernelGGL(svm_patch_f32_kernel, dim3((count + 255) / 256), dim3(256), 0, as_stream(stream),
                     (unsigned char*)base, stride, off, count, (const int*)fit_of, (const float*)src);
  launch_check();
}

// Cascade parts of the working-set SMO (models/smo.py _cascade_seed): part q of a parent problem
// (points [0, npos) positive, then negative) holds the parent's positives j, j+P, … then its
// negatives npos+j, npos+j+P, …; where[start_q + t] = the parent's absolute point index of the
// part's t-th point.  tab: [Q][7] int64 {start, len, aoff, P, j, npos, cp}; grid (x: points, y: parts).
__global__ void cascade_where_kernel(const long long* __restrict__ tab, long long* __restrict__ where) {
  const long long* r = tab + 7 * (size_t)blockIdx.y;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= r[1]) return;
  const long long P = r[3], j = r[4], npos = r[5], cp = r[6];
  const long long pos = t < cp ? j + t * P : npos + j + (t - cp) * P;
  where[r[0] + t] = r[2] + pos;
}

void cascade_where(uintptr_t tab, int Q, long long max_len, uintptr_t where, uintptr_t stream) {
  HFENS_REQUIRE(Q >= 0 && max_len >= 0 && Q <= 65535, "cascade_where: 0 <= parts <= 65535");
  if (Q == 0 || max_len == 0) return;
  hipLaunchKernelGGL(cascade_where_kernel, dim3((unsigned)((max_len + 255) / 256), Q), dim3(256), 0, as_stream(stream),
                     (const long long*)tab, (long long*)where);
  launch_check();
}

}  // namespace hfens
