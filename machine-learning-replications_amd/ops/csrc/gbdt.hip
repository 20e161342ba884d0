// Histogram GBDT training for binomial deviance (reference model
// GradientBoostingClassifier(100 stumps), train_ensemble_public.py:45).
//
// B independent models (CV folds + full refit, or seeds) train together on one binned matrix;
// model b sees rows with weight w[b][i] > 0.  Trees grow level-wise in heap layout (node k →
// children 2k+1, 2k+2).  Per boosting stage:
//   gbdt_apply_prep : route rows through the previous tree's last level, add lr·leaf value to
//                     raw (f64), accumulate that tree's leaf Σw·r² (impurity) and the training
//                     deviance, then compute this stage's residual g = w(y−p) and hessian
//                     h = w·p(1−p) (f32) and reset every row to the root.
//   gbdt_hist       : per (model, node, feature, bin) sums of (g, h, w) in FIXED POINT (int64,
//                     scale 2^shift).  Integer sums are exact and order-independent, so the
//                     histogram is bit-identical for any launch geometry, any atomics order and
//                     any data-parallel sharding (RCCL all-reduce of int64 SUM is exact).
//                     Low-cardinality features (≤ 8 bins, 80 % of the HF columns) accumulate in
//                     registers over a whole row chunk and reduce once per chunk; others use an
//                     LDS histogram with ds_add_u64 and one global flush per workgroup.
//   gbdt_split      : per (model, node): prefix scan over bins, friedman_mse proxy
//                     (w_r·S_l − w_l·S_r)²/(w_l·w_r), deterministic tie-break (lowest feature,
//                     lowest bin), threshold = midpoint of the adjacent *non-empty* bins' values
//                     (= sklearn's exact splitter on the model's own training rows), Newton leaf
//                     values Σr/Σh for children of the last level.
//   gbdt_route      : move rows of split nodes one level down, accumulating child Σw·r².
#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace hfens {

struct GbdtShape {
  int B, n, F, NN;  // models, rows, features, heap nodes per tree
};

// rint(v·scale) as int64 for |v·scale| < 2^51 (every fixed-point use here: |g|, h, w ≤ 1 at scale
// ≤ 2^40, deviance terms at 2^26): adding 1.5·2^52 rounds to nearest-even in the FPU and leaves
// the integer in the low mantissa bits — 2 VALU ops instead of the f64→i64 conversion sequence.
__device__ __forceinline__ long long q_of(double v, double scale) {
  const double t = v * scale + 6755399441055744.0;
  return (long long)__double_as_longlong(t) - 0x4338000000000000LL;
}

__device__ __forceinline__ long long wave_sum_i64(long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Stochastic gradient boosting (subsample < 1): row i of model b is in stage t's bag iff
// splitmix64(seed_b ⊕ splitmix64(t, global row)) < subsample·2^64 (top 24 bits compared).
// Counter-based: no RNG state, identical for any launch geometry and any row sharding.
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__device__ __forceinline__ bool gb_in_bag(unsigned long long seed, int stage, long long gi, unsigned thr24) {
  const unsigned long long k = splitmix64(((unsigned long long)stage << 40) ^ (unsigned long long)gi);
  return (unsigned)(splitmix64(seed ^ k) >> 40) < thr24;
}

struct GbdtBag {
  float* wt;                        // [B][n] this stage's in-bag weights (written when active)
  const unsigned long long* seeds;  // [B]
  long long row_off;                // global index of local row 0 (data-parallel shards)
  unsigned thr24;                   // subsample·2^24
  int stage;                        // current stage t
  int active;                       // subsample < 1
};

// ------------------------------------------------------------------------------------------
// A: apply previous tree (one pending routing level + leaf values) and prepare this stage.
// prev_* are the previous tree's tables [B][NN] (heap), or nullptr for the first stage.
__global__ __launch_bounds__(256) void gbdt_apply_prep_kernel(
    GbdtShape S, const unsigned char* __restrict__ bins, const float* __restrict__ y,
    const float* __restrict__ w, double* __restrict__ raw, float* __restrict__ g,
    float* __restrict__ h, int* __restrict__ node, const int* __restrict__ prev_feat,
    const int* __restrict__ prev_blo, const double* __restrict__ prev_value,
    long long* __restrict__ prev_r2 /*[B][NN] previous tree Σw r²*/, long long* __restrict__ dev_acc /*[B]*/,
    long long* __restrict__ cur_r2 /*[B][NN] this tree (root slot)*/, double lr, double qscale,
    double dscale, GbdtBag bag) {
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63;
  long long dev_q = 0, r2_q = 0;
  // per-node Σw r² of the previous tree: block-local LDS accumulation, one global atomic per
  // (block, node) — a direct global atomic per row serialises on ~3 hot addresses per model
  __shared__ long long nacc[64];
  if (threadIdx.x < 64) nacc[threadIdx.x] = 0;
  __syncthreads();
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < S.n; i += gridDim.x * blockDim.x) {
    const size_t bi = (size_t)b * S.n + i;
    const float w0 = w[bi];
    float wi = w0, wp = w0;   // this stage's / the previous stage's in-bag weight
    if (bag.active) {
      const unsigned long long sd = bag.seeds[b];
      wi = gb_in_bag(sd, bag.stage, bag.row_off + i, bag.thr24) ? w0 : 0.f;
      wp = (prev_feat != nullptr && gb_in_bag(sd, bag.stage - 1, bag.row_off + i, bag.thr24)) ? w0 : 0.f;
      bag.wt[bi] = wi;
    }
    double rw = raw[bi];
    const double yi = y[i];
    if (prev_feat != nullptr) {
      int nd = node[bi];
      const int f = prev_feat[b * S.NN + nd];
      if (f >= 0) {  // pending split at the last level
        const int side = bins[(size_t)f * S.n + i] <= prev_blo[b * S.NN + nd] ? 1 : 2;
        nd = 2 * nd + side;
      }
      if (wp > 0.f) {
        const double p0 = 1.0 / (1.0 + exp(-rw));
        const double r0 = yi - p0;
        atomicAdd((unsigned long long*)&nacc[nd], (unsigned long long)q_of(wp * r0 * r0, qscale));
      }
      rw += lr * prev_value[b * S.NN + nd];
      raw[bi] = rw;
    }
    const double p = 1.0 / (1.0 + exp(-rw));
    const double r = yi - p;
    const float gi = (float)(wi * r);
    const float hi = (float)(wi * p * (1.0 - p));
    g[bi] = gi;
    h[bi] = hi;
    node[bi] = 0;
    if (wp > 0.f) {
      // binomial deviance −2(y·raw − log(1+e^raw)) of the previous stage's bag, after its update
      // (sklearn BinomialDeviance; train_score_ with subsample = in-bag loss)
      const double l1p = rw > 0 ? rw + log1p(exp(-rw)) : log1p(exp(rw));
      dev_q += q_of(wp * (-2.0) * (yi * rw - l1p), dscale);
    }
    if (wi > 0.f) r2_q += q_of(wi * r * r, qscale);
  }
  dev_q = wave_sum_i64(dev_q);
  r2_q = wave_sum_i64(r2_q);
  if (lane == 0) {
    if (prev_feat != nullptr && dev_q != 0) atomicAdd((unsigned long long*)&dev_acc[b], (unsigned long long)dev_q);
    if (r2_q != 0) atomicAdd((unsigned long long*)&cur_r2[(size_t)b * S.NN], (unsigned long long)r2_q);
  }
  __syncthreads();
  if (prev_feat != nullptr && threadIdx.x < S.NN && nacc[threadIdx.x] != 0)
    atomicAdd((unsigned long long*)&prev_r2[(size_t)b * S.NN + threadIdx.x],
              (unsigned long long)nacc[threadIdx.x]);
}

// ------------------------------------------------------------------------------------------
// B: histograms.  grid = (row chunks, F, B).  hist layout [B][NL][F][256][3] int64 where the
// level's nodes are heap indices node0 .. node0+NL-1.
template <int C>
__device__ void hist_registers(const unsigned char* __restrict__ col, const float* __restrict__ g,
                               const float* __restrict__ h, const float* __restrict__ w,
                               const int* __restrict__ node, int node0, int r0, int r1,
                               double qscale, long long* __restrict__ out /*[256][3]*/) {
  long long ag[C], ah[C], aw[C];
#pragma unroll
  for (int c = 0; c < C; ++c) { ag[c] = 0; ah[c] = 0; aw[c] = 0; }
  for (int i = r0 + threadIdx.x; i < r1; i += blockDim.x) {
    if (node[i] != node0) continue;
    const float wi = w[i];
    if (!(wi > 0.f)) continue;
    const int bb = col[i];
    const long long qg = q_of(g[i], qscale), qh = q_of(h[i], qscale), qw = q_of(wi, qscale);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const bool m = (bb == c);
      ag[c] += m ? qg : 0;
      ah[c] += m ? qh : 0;
      aw[c] += m ? qw : 0;
    }
  }
  __shared__ long long red[4][C * 3];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    long long a = wave_sum_i64(ag[c]), b2 = wave_sum_i64(ah[c]), c2 = wave_sum_i64(aw[c]);
    if (lane == 0) { red[wave][3 * c] = a; red[wave][3 * c + 1] = b2; red[wave][3 * c + 2] = c2; }
  }
  __syncthreads();
  if (threadIdx.x < C * 3) {
    long long s = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) s += red[k][threadIdx.x];
    if (s != 0) atomicAdd((unsigned long long*)&out[threadIdx.x], (unsigned long long)s);
  }
}

__global__ __launch_bounds__(256) void gbdt_hist_kernel(
    GbdtShape S, const unsigned char* __restrict__ bins, const int* __restrict__ nbins,
    const float* __restrict__ g, const float* __restrict__ h, const float* __restrict__ w,
    const int* __restrict__ node, int node0, int NL, int chunk, long long* __restrict__ hist,
    double qscale) {
  const int f = blockIdx.y;
  const int b = blockIdx.z;
  const int r0 = blockIdx.x * chunk;
  const int r1 = min(S.n, r0 + chunk);
  const size_t boff = (size_t)b * S.n;
  const unsigned char* col = bins + (size_t)f * S.n;
  const int nb = nbins[f];
  long long* hb = hist + (size_t)b * NL * S.F * 768;
  if (NL == 1) {
    long long* out = hb + (size_t)f * 768;
    if (nb <= 2) return hist_registers<2>(col, g + boff, h + boff, w + boff, node + boff, node0, r0, r1, qscale, out);
    if (nb <= 4) return hist_registers<4>(col, g + boff, h + boff, w + boff, node + boff, node0, r0, r1, qscale, out);
    if (nb <= 8) return hist_registers<8>(col, g + boff, h + boff, w + boff, node + boff, node0, r0, r1, qscale, out);
  }
  // LDS path: NL ≤ 16 nodes × 256 bins × 3 stats × 8 B = up to 96 KiB
  extern __shared__ __attribute__((aligned(16))) long long lh[];
  const int tot = NL * nb * 3;
  for (int k = threadIdx.x; k < tot; k += blockDim.x) lh[k] = 0;
  __syncthreads();
  for (int i = r0 + threadIdx.x; i < r1; i += blockDim.x) {
    const int nd = node[boff + i] - node0;
    if (nd < 0 || nd >= NL) continue;
    const float wi = w[boff + i];
    if (!(wi > 0.f)) continue;
    const int bb = col[i];
    long long* cell = lh + ((size_t)nd * nb + bb) * 3;
    atomicAdd((unsigned long long*)&cell[0], (unsigned long long)q_of(g[boff + i], qscale));
    atomicAdd((unsigned long long*)&cell[1], (unsigned long long)q_of(h[boff + i], qscale));
    atomicAdd((unsigned long long*)&cell[2], (unsigned long long)q_of(wi, qscale));
  }
  __syncthreads();
  for (int k = threadIdx.x; k < tot; k += blockDim.x) {
    const long long v = lh[k];
    if (v == 0) continue;
    const int s = k % 3, bb = (k / 3) % nb, nd = k / (3 * nb);
    atomicAdd((unsigned long long*)&hb[(((size_t)nd * S.F + f) * 256 + bb) * 3 + s],
              (unsigned long long)v);
  }
}

// ------------------------------------------------------------------------------------------
// C: split finding.  grid = (NL, B), 256 threads (4 waves; wave ↔ features f ≡ wave mod 4).
struct SplitOut {
  int* feat;          // [B][NN]  split feature, -2 leaf
  int* blo;           // [B][NN]  last bin going left
  double* thr;        // [B][NN]
  double* value;      // [B][NN]  node value (mean residual for internal, Newton for leaves)
  long long* stats;   // [B][NN][4] Σw, Σr, Σh, (unused)   (fixed point)
  const long long* r2;  // [B][NN] Σw r² (filled by apply_prep / route)
};

__device__ __forceinline__ void scan_feature(const long long* __restrict__ hf, int nb, int lane,
                                             long long tw, long long tg, double min_leaf_q,
                                             double& best_gain, int& best_bin) {
  // lane owns bins 4·lane .. 4·lane+3; exclusive prefix across lanes via shuffles
  long long pw[4], pg[4];
  long long sw = 0, sg = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int bb = 4 * lane + j;
    const long long gw = bb < nb ? hf[bb * 3 + 2] : 0;
    const long long gg = bb < nb ? hf[bb * 3 + 0] : 0;
    sw += gw; sg += gg;
    pw[j] = sw; pg[j] = sg;
  }
  long long xw = sw, xg = sg;  // inclusive scan of lane totals
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    long long tw2 = __shfl_up(xw, o, kWave), tg2 = __shfl_up(xg, o, kWave);
    if (lane >= o) { xw += tw2; xg += tg2; }
  }
  const long long ew = xw - sw, eg = xg - sg;
  best_gain = -1.0;
  best_bin = 0x7fffffff;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int bb = 4 * lane + j;
    if (bb >= nb - 1) continue;
    const long long lw = ew + pw[j], lg = eg + pg[j];
    const long long rw = tw - lw, rg = tg - lg;
    if ((double)lw < min_leaf_q || (double)rw < min_leaf_q) continue;
    const double dlw = (double)lw, drw = (double)rw;
    const double diff = drw * (double)lg - dlw * (double)rg;
    const double gain = diff / dlw * diff / drw;
    if (gain > best_gain) { best_gain = gain; best_bin = bb; }
  }
  // wave argmax, lowest bin on ties
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    double og = __shfl_xor(best_gain, o, kWave);
    int ob = __shfl_xor(best_bin, o, kWave);
    if (og > best_gain || (og == best_gain && ob < best_bin)) { best_gain = og; best_bin = ob; }
  }
}

// scan_feature for nb ≤ 4 bins (binary and small features: every bin is lane 0's in scan_feature):
// each lane computes lane 0's result itself from the same (broadcast) reads — no cross-lane scan and
// no argmax shuffles; same arithmetic in the same order, so the same (gain, bin).
__device__ __forceinline__ void scan_feature_small(const long long* hf, int nb, long long tw, long long tg,
                                                   double min_leaf_q, double& best_gain, int& best_bin) {
  best_gain = -1.0;
  best_bin = 0x7fffffff;
  long long lw = 0, lg = 0;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    if (j >= nb - 1) break;
    lw += hf[j * 3 + 2];
    lg += hf[j * 3 + 0];
    const long long rw = tw - lw, rg = tg - lg;
    if ((double)lw < min_leaf_q || (double)rw < min_leaf_q) continue;
    const double dlw = (double)lw, drw = (double)rw;
    const double diff = drw * (double)lg - dlw * (double)rg;
    const double gain = diff / dlw * diff / drw;
    if (gain > best_gain) { best_gain = gain; best_bin = j; }
  }
}

__global__ __launch_bounds__(256) void gbdt_split_kernel(
    GbdtShape S, const long long* __restrict__ hist, const int* __restrict__ nbins,
    const double* __restrict__ lo_val, const double* __restrict__ hi_val, int node0, int NL,
    int last_level, double min_leaf_q, double min_split_q, double qscale, SplitOut o) {
  const int nd = blockIdx.x;      // node within level
  const int b = blockIdx.y;
  const int hn = node0 + nd;      // heap index
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long* hb = hist + ((size_t)b * NL + nd) * S.F * 768;
  long long* st = o.stats + ((size_t)b * S.NN + hn) * 4;
  // node totals from feature 0's bins
  __shared__ long long tot[3];
  __shared__ double wg[4];
  __shared__ int wf[4], wbin[4];
  if (wave == 0) {
    long long a = 0, c = 0, d = 0;
    const int nb0 = nbins[0];
    for (int bb = lane; bb < nb0; bb += 64) { a += hb[bb * 3]; c += hb[bb * 3 + 1]; d += hb[bb * 3 + 2]; }
    a = wave_sum_i64(a); c = wave_sum_i64(c); d = wave_sum_i64(d);
    if (lane == 0) { tot[0] = a; tot[1] = c; tot[2] = d; }
  }
  __syncthreads();
  const long long tg = tot[0], th = tot[1], tw = tot[2];
  if (tw <= 0) {  // unreachable / empty node
    if (threadIdx.x == 0) { o.feat[b * S.NN + hn] = -3; }
    return;
  }
  double bg = -1.0;
  int bf = 0x7fffffff, bbin = 0;
  if ((double)tw >= min_split_q) {
    for (int f = wave; f < S.F; f += 4) {
      double gg;
      int gb;
      scan_feature(hb + (size_t)f * 768, nbins[f], lane, tw, tg, min_leaf_q, gg, gb);
      if (gg > bg) { bg = gg; bf = f; bbin = gb; }  // f ascending within a wave
    }
  }
  if (lane == 0) { wg[wave] = bg; wf[wave] = bf; wbin[wave] = bbin; }
  __syncthreads();
  if (threadIdx.x != 0) return;
  bg = wg[0]; bf = wf[0]; bbin = wbin[0];
  for (int k = 1; k < 4; ++k)
    if (wg[k] > bg || (wg[k] == bg && wf[k] < bf)) { bg = wg[k]; bf = wf[k]; bbin = wbin[k]; }
  // node record
  st[0] = tw; st[1] = tg; st[2] = th;
  const double inv = 1.0 / qscale;
  // impurity==0 ⇒ leaf (sklearn: impurity <= EPSILON); impurity from Σw r² (st[3], filled by prep/route)
  const double dw = tw * inv, dg = tg * inv;
  const double imp = o.r2[(size_t)b * S.NN + hn] * inv / dw - (dg / dw) * (dg / dw);
  const bool can_split = bg >= 0.0 && bf < S.F && imp > 2.220446049250313e-16;
  const int idx = b * S.NN + hn;
  if (!can_split) {
    o.feat[idx] = -2;
    o.blo[idx] = 0;
    o.thr[idx] = -2.0;
    const double den = th * inv;
    o.value[idx] = fabs(den) < 1e-150 ? 0.0 : dg / den;
    return;
  }
  // children sums at the chosen bin; the following non-empty bin gives the threshold
  const long long* hf = hb + (size_t)bf * 768;
  long long lw = 0, lg = 0, lh = 0;
  for (int bb = 0; bb <= bbin; ++bb) { lg += hf[bb * 3]; lh += hf[bb * 3 + 1]; lw += hf[bb * 3 + 2]; }
  int hi = bbin + 1;
  const int nbf = nbins[bf];
  while (hi < nbf - 1 && hf[hi * 3 + 2] == 0) ++hi;
  const double a = hi_val[bf * 256 + bbin], c = lo_val[bf * 256 + hi];
  double t = a / 2.0 + c / 2.0;
  if (t == c || isinf(t)) t = a;
  o.feat[idx] = bf;
  o.blo[idx] = bbin;
  o.thr[idx] = t;
  o.value[idx] = dg / dw;  // internal node value: weighted mean residual
  const int L = 2 * hn + 1, R = 2 * hn + 2;
  long long* sl = o.stats + ((size_t)b * S.NN + L) * 4;
  long long* sr = o.stats + ((size_t)b * S.NN + R) * 4;
  sl[0] = lw; sl[1] = lg; sl[2] = lh;
  sr[0] = tw - lw; sr[1] = tg - lg; sr[2] = th - lh;
  if (last_level) {  // children are leaves: Newton values, sklearn _update_terminal_regions
    o.feat[b * S.NN + L] = -2; o.feat[b * S.NN + R] = -2;
    o.blo[b * S.NN + L] = 0; o.blo[b * S.NN + R] = 0;
    o.thr[b * S.NN + L] = -2.0; o.thr[b * S.NN + R] = -2.0;
    const double dl = lh * inv, dr = (th - lh) * inv;
    o.value[b * S.NN + L] = fabs(dl) < 1e-150 ? 0.0 : lg * inv / dl;
    o.value[b * S.NN + R] = fabs(dr) < 1e-150 ? 0.0 : (tg - lg) * inv / dr;
  }
}

// ------------------------------------------------------------------------------------------
// D: route rows of split nodes at the current level one level down (not the last level: that
// routing is fused into the next stage's apply_prep).
__global__ __launch_bounds__(256) void gbdt_route_kernel(
    GbdtShape S, const unsigned char* __restrict__ bins, const float* __restrict__ g,
    const float* __restrict__ w, int* __restrict__ node, const int* __restrict__ feat,
    const int* __restrict__ blo, long long* __restrict__ r2, int node0, int NL, double qscale) {
  const int b = blockIdx.y;
  __shared__ long long nacc[64];
  if (threadIdx.x < 64) nacc[threadIdx.x] = 0;
  __syncthreads();
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < S.n; i += gridDim.x * blockDim.x) {
    const size_t bi = (size_t)b * S.n + i;
    const int nd = node[bi];
    if (nd < node0 || nd >= node0 + NL) continue;
    const int f = feat[b * S.NN + nd];
    if (f < 0) continue;
    const int child = 2 * nd + (bins[(size_t)f * S.n + i] <= blo[b * S.NN + nd] ? 1 : 2);
    node[bi] = child;
    const float wi = w[bi];
    if (wi > 0.f) {
      const double r = (double)g[bi] / wi;
      atomicAdd((unsigned long long*)&nacc[child], (unsigned long long)q_of(wi * r * r, qscale));
    }
  }
  __syncthreads();
  if (threadIdx.x < S.NN && nacc[threadIdx.x] != 0)
    atomicAdd((unsigned long long*)&r2[(size_t)b * S.NN + threadIdx.x], (unsigned long long)nacc[threadIdx.x]);
}

// ------------------------------------------------------------------------------------------
// host entry points
static int grid_rows(int n) {
  int g = (n + 255) / 256;
  return g > 1024 ? 1024 : (g < 1 ? 1 : g);
}

void gbdt_apply_prep(int B, int n, int F, int NN, uintptr_t bins, uintptr_t y, uintptr_t w,
                     uintptr_t raw, uintptr_t g, uintptr_t h, uintptr_t node, uintptr_t prev_feat,
                     uintptr_t prev_blo, uintptr_t prev_value, uintptr_t prev_r2,
                     uintptr_t dev_acc, uintptr_t cur_r2, double lr, double qscale, double dscale,
                     uintptr_t wt, double subsample, uintptr_t seeds, long long row_off, int stage,
                     uintptr_t stream) {
  GbdtShape S{B, n, F, NN};
  const bool active = subsample < 1.0;
  HFENS_REQUIRE(!active || (wt != 0 && seeds != 0), "gbdt_apply_prep: subsample needs wt and seeds");
  GbdtBag bag{(float*)wt, (const unsigned long long*)seeds, row_off,
              (unsigned)llround(subsample * 16777216.0), stage, active ? 1 : 0};
  hipLaunchKernelGGL(gbdt_apply_prep_kernel, dim3(grid_rows(n), B), dim3(256), 0, as_stream(stream),
                     S, (const unsigned char*)bins, (const float*)y, (const float*)w, (double*)raw,
                     (float*)g, (float*)h, (int*)node, (const int*)prev_feat, (const int*)prev_blo,
                     (const double*)prev_value, (long long*)prev_r2, (long long*)dev_acc,
                     (long long*)cur_r2, lr, qscale, dscale, bag);
  launch_check();
}

void gbdt_hist(int B, int n, int F, uintptr_t bins, uintptr_t nbins, int max_nb, uintptr_t g,
               uintptr_t h, uintptr_t w, uintptr_t node, int node0, int NL, uintptr_t hist,
               double qscale, uintptr_t stream) {
  HFENS_REQUIRE(NL >= 1 && NL <= 16, "gbdt_hist: at most 16 nodes per level on the LDS path");
  GbdtShape S{B, n, F, 0};
  const int chunk = n <= 16384 ? 1024 : 8192;
  dim3 grid((n + chunk - 1) / chunk, F, B);
  const size_t lds = (size_t)NL * max_nb * 3 * sizeof(long long);
  HFENS_REQUIRE(lds <= 160 * 1024, "gbdt_hist: histogram does not fit LDS");
  hipLaunchKernelGGL(gbdt_hist_kernel, grid, dim3(256), lds, as_stream(stream), S,
                     (const unsigned char*)bins, (const int*)nbins, (const float*)g, (const float*)h,
                     (const float*)w, (const int*)node, node0, NL, chunk, (long long*)hist, qscale);
  launch_check();
}

void gbdt_split(int B, int F, int NN, uintptr_t hist, uintptr_t nbins, uintptr_t lo_val,
                uintptr_t hi_val, int node0, int NL, int last_level, double min_leaf_q,
                double min_split_q, double qscale, uintptr_t feat, uintptr_t blo, uintptr_t thr,
                uintptr_t value, uintptr_t stats, uintptr_t r2, uintptr_t stream) {
  GbdtShape S{B, 0, F, NN};
  SplitOut o{(int*)feat, (int*)blo, (double*)thr, (double*)value, (long long*)stats,
             (const long long*)r2};
  hipLaunchKernelGGL(gbdt_split_kernel, dim3(NL, B), dim3(256), 0, as_stream(stream), S,
                     (const long long*)hist, (const int*)nbins, (const double*)lo_val,
                     (const double*)hi_val, node0, NL, last_level, min_leaf_q, min_split_q, qscale, o);
  launch_check();
}

void gbdt_route(int B, int n, int NN, uintptr_t bins, uintptr_t g, uintptr_t w, uintptr_t node,
                uintptr_t feat, uintptr_t blo, uintptr_t r2, int node0, int NL, double qscale,
                uintptr_t stream) {
  GbdtShape S{B, n, 0, NN};
  hipLaunchKernelGGL(gbdt_route_kernel, dim3(grid_rows(n), B), dim3(256), 0, as_stream(stream), S,
                     (const unsigned char*)bins, (const float*)g, (const float*)w, (int*)node,
                     (const int*)feat, (const int*)blo, (long long*)r2, node0, NL, qscale);
  launch_check();
}

// ------------------------------------------------------------------------------------------
// E: depth-1 trees on few rows — the whole boosting run in ONE launch (gbdt_stumps_fused).
//    One 1024-thread workgroup per model runs, for every stage, exactly A (apply_prep) → B (root
//    histogram) → C (root split) above: same per-row arithmetic, same fixed-point sums, same
//    split rule and tie-breaks, so trees, leaf values, impurities and train_score_ equal the
//    launch-per-step path's.  What goes away is 4 launches and the host round trips of every stage
//    (the bench's 6-model GBC: ≈18 ms of host enqueue for 100 stages).  The root histograms of all
//    features live in LDS in a compact layout (feature f's bins start at off[f]); ≤ 8-bin features
//    accumulate in registers and fold once per feature, wider ones use ds_add_u64.
constexpr int kStThreads = 1024;
constexpr int kStWaves = kStThreads / 64;
constexpr int kStMaxF = 128;

struct StumpJob {
  const unsigned char* bins;          // [F][n]
  const int* nbins;                   // [F]
  const double* lo_val;               // [F][256]
  const double* hi_val;               // [F][256]
  const float* y;                     // [n]
  const float* w;                     // [B][n]
  double* raw;                        // [B][n]
  float* g;                           // [B][n]
  float* h;                           // [B][n]
  float* wt;                          // [B][n] in-bag weights (bagging) or nullptr
  const unsigned long long* seeds;    // [B] (bagging) or nullptr
  int* feat;                          // [T][B][3]
  int* blo;                           // [T][B][3]
  double* thr;                        // [T][B][3]
  double* value;                      // [T][B][3]
  long long* stats;                   // [T][B][3][4]
  long long* r2;                      // [T][B][3]
  long long* dev;                     // [T][B]
  double* bagw;                       // [T][B] (bagging) or nullptr
  long long row_off;
  double lr, qscale, dscale, min_leaf_q, min_split_q;
  unsigned thr24;
  int active, B, n, F, T, hist_len;   // hist_len = Σ_f nbins[f]
};

// Root histogram of one ≤ C-bin feature over the workgroup: per-thread registers, one fold.
// g/h/w were written by this workgroup earlier in the launch (vector loads, no __restrict__).
template <int C>
__device__ __forceinline__ void stump_hist_regs(const unsigned char* __restrict__ col, const float* g,
                                                const float* h, const float* w, int n, int nb, double qscale,
                                                long long* out /*[nb][3] LDS*/, long long* red) {
  long long ag[C], ah[C], aw[C];
#pragma unroll
  for (int c = 0; c < C; ++c) { ag[c] = 0; ah[c] = 0; aw[c] = 0; }
  for (int i = threadIdx.x; i < n; i += kStThreads) {
    const float wi = w[i];
    if (!(wi > 0.f)) continue;
    const int bb = col[i];
    const long long qg = q_of(g[i], qscale), qh = q_of(h[i], qscale), qw = q_of(wi, qscale);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const bool m = bb == c;
      ag[c] += m ? qg : 0;
      ah[c] += m ? qh : 0;
      aw[c] += m ? qw : 0;
    }
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const long long a = wave_sum_i64(ag[c]), b2 = wave_sum_i64(ah[c]), c2 = wave_sum_i64(aw[c]);
    if (lane == 0) {
      red[wave * 24 + 3 * c] = a;
      red[wave * 24 + 3 * c + 1] = b2;
      red[wave * 24 + 3 * c + 2] = c2;
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < 3 * nb) {
    long long s = 0;
    for (int k = 0; k < kStWaves; ++k) s += red[k * 24 + threadIdx.x];
    out[threadIdx.x] = s;
  }
  __syncthreads();
}

// Workgroup sums of NV int64 values (exact): out[0..NV) in LDS, valid for every thread on return.
template <int NV>
__device__ __forceinline__ void stump_block_sum(long long (&v)[NV], long long* red, long long* out) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const long long t = wave_sum_i64(v[k]);
    if (lane == 0) red[wave * 24 + k] = t;
  }
  __syncthreads();
  if ((int)threadIdx.x < NV) {
    long long s = 0;
    for (int k = 0; k < kStWaves; ++k) s += red[k * 24 + threadIdx.x];
    out[threadIdx.x] = s;
  }
  __syncthreads();
}

__global__ __launch_bounds__(kStThreads) void gbdt_stumps_fused_kernel(StumpJob J) {
  extern __shared__ __attribute__((aligned(16))) long long hl[];   // [hist_len][3]
  __shared__ long long red[kStWaves * 24];
  __shared__ int s_nb[kStMaxF], s_off[kStMaxF];
  __shared__ long long tot[3], root_r2;
  __shared__ double wg[kStWaves];
  __shared__ int wf[kStWaves], wbin[kStWaves];
  __shared__ int tf0, tblo, bad;   // previous tree: root feature (−3 empty, −2 leaf) and split bin
  __shared__ int l_bin[kStMaxF], l_one[kStMaxF], l_mid[kStMaxF], l_wide[kStMaxF];   // features by bin count
  __shared__ int n_bin, n_one, n_mid, n_wide;
  __shared__ long long bsum[24];
  __shared__ double tval[3];       // previous tree: node values
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = J.n, F = J.F, B = J.B;
  if (tid == 0) {
    int o = 0;
    n_bin = n_one = n_mid = n_wide = 0;
    for (int f = 0; f < F; ++f) {
      const int nb = J.nbins[f];
      s_nb[f] = nb; s_off[f] = o; o += nb;
      if (nb == 2) l_bin[n_bin++] = f;
      else if (nb <= 1) l_one[n_one++] = f;
      else if (nb <= 8) l_mid[n_mid++] = f;
      else l_wide[n_wide++] = f;
    }
    bad = o != J.hist_len || s_nb[0] < 1;   // host and device bin tables disagree: write nothing
    tf0 = -3; tblo = 0; tval[0] = tval[1] = tval[2] = 0.0;
  }
  __syncthreads();
  if (bad) return;
  const size_t boff = (size_t)b * n;
  const float* wb = J.w + boff;
  double* raw = J.raw + boff;
  float* g = J.g + boff;
  float* h = J.h + boff;
  float* wt = J.active ? J.wt + boff : nullptr;
  const float* wcur = J.active ? wt : wb;
  for (int t = 0; t <= J.T; ++t) {
    // ---- A: apply the previous stump, this stage's residuals (gbdt_apply_prep_kernel)
    const bool has_prev = t > 0;
    const int pf = tf0, pblo = tblo;
    const double pv0 = tval[0], pv1 = tval[1], pv2 = tval[2];
    long long dev_q = 0, r2_q = 0, n0 = 0, n1 = 0, n2 = 0;
    double bag = 0.0;
    for (int i = tid; i < n; i += kStThreads) {
      const float w0 = wb[i];
      float wi = w0, wp = w0;
      if (J.active) {
        const unsigned long long sd = J.seeds[b];
        wi = gb_in_bag(sd, t, J.row_off + i, J.thr24) ? w0 : 0.f;
        wp = (has_prev && gb_in_bag(sd, t - 1, J.row_off + i, J.thr24)) ? w0 : 0.f;
        wt[i] = wi;
        bag += (double)wi;
      }
      double rw = raw[i];
      const double yi = J.y[i];
      if (has_prev) {
        const int nd = pf >= 0 ? (J.bins[(size_t)pf * n + i] <= pblo ? 1 : 2) : 0;
        if (wp > 0.f) {
          const double p0 = 1.0 / (1.0 + exp(-rw));
          const double r0 = yi - p0;
          const long long q = q_of(wp * r0 * r0, J.qscale);
          n0 += nd == 0 ? q : 0;
          n1 += nd == 1 ? q : 0;
          n2 += nd == 2 ? q : 0;
        }
        rw += J.lr * (nd == 0 ? pv0 : (nd == 1 ? pv1 : pv2));
        raw[i] = rw;
      }
      const double p = 1.0 / (1.0 + exp(-rw));
      const double r = yi - p;
      g[i] = (float)(wi * r);
      h[i] = (float)(wi * p * (1.0 - p));
      if (wp > 0.f) {
        const double l1p = rw > 0 ? rw + log1p(exp(-rw)) : log1p(exp(rw));
        dev_q += q_of(wp * (-2.0) * (yi * rw - l1p), J.dscale);
      }
      if (wi > 0.f) r2_q += q_of(wi * r * r, J.qscale);
    }
    dev_q = wave_sum_i64(dev_q);
    r2_q = wave_sum_i64(r2_q);
    n0 = wave_sum_i64(n0);
    n1 = wave_sum_i64(n1);
    n2 = wave_sum_i64(n2);
    bag = wave_sum(bag);   // in-bag weights are 0/1 masks: exact in any order
    if (lane == 0) {
      long long* rr = red + wave * 24;
      rr[0] = dev_q; rr[1] = r2_q; rr[2] = n0; rr[3] = n1; rr[4] = n2; rr[5] = __double_as_longlong(bag);
    }
    __syncthreads();
    if (tid == 0) {
      long long s[5] = {0, 0, 0, 0, 0};
      double bs = 0.0;
      for (int k = 0; k < kStWaves; ++k) {
        for (int j = 0; j < 5; ++j) s[j] += red[k * 24 + j];
        bs += __longlong_as_double(red[k * 24 + 5]);
      }
      if (has_prev) {
        const size_t pb = (size_t)(t - 1) * B + b;
        J.dev[pb] += s[0];
        J.r2[pb * 3] += s[2];
        J.r2[pb * 3 + 1] += s[3];
        J.r2[pb * 3 + 2] += s[4];
      }
      if (t < J.T) {
        const size_t tb = (size_t)t * B + b;
        J.r2[tb * 3] += s[1];
        root_r2 = J.r2[tb * 3];
        if (J.active) J.bagw[tb] = bs;
      }
    }
    __syncthreads();
    if (t == J.T) break;
    // ---- B: root histograms (gbdt_hist_kernel, NL = 1).  Integer sums are exact, so features
    // may be grouped freely: node totals once; binary features 8 per row pass (bin 1 summed,
    // bin 0 = total − bin 1); 3–8-bin features one per pass in registers; every wider feature
    // in ONE row pass with ds_add_u64.
    for (int k = tid; k < 3 * J.hist_len; k += kStThreads) hl[k] = 0;
    {
      long long v[3] = {0, 0, 0};
      for (int i = tid; i < n; i += kStThreads) {
        const float wi = wcur[i];
        if (!(wi > 0.f)) continue;
        v[0] += q_of(g[i], J.qscale);
        v[1] += q_of(h[i], J.qscale);
        v[2] += q_of(wi, J.qscale);
      }
      stump_block_sum<3>(v, red, tot);
    }
    for (int b0 = 0; b0 < n_bin; b0 += 8) {
      const int nf = min(8, n_bin - b0);
      long long acc[24];
#pragma unroll
      for (int k = 0; k < 24; ++k) acc[k] = 0;
      for (int i = tid; i < n; i += kStThreads) {
        const float wi = wcur[i];
        if (!(wi > 0.f)) continue;
        const long long qg = q_of(g[i], J.qscale), qh = q_of(h[i], J.qscale), qw = q_of(wi, J.qscale);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (u < nf && J.bins[(size_t)l_bin[b0 + u] * n + i]) {
            acc[3 * u] += qg;
            acc[3 * u + 1] += qh;
            acc[3 * u + 2] += qw;
          }
        }
      }
      stump_block_sum<24>(acc, red, bsum);
      if (tid < 3 * nf) {
        const int u = tid / 3, k = tid - 3 * u;
        const int off = s_off[l_bin[b0 + u]];
        hl[(off + 1) * 3 + k] = bsum[tid];
        hl[off * 3 + k] = tot[k] - bsum[tid];
      }
    }
    for (int u = tid; u < 3 * n_one; u += kStThreads) hl[s_off[l_one[u / 3]] * 3 + u % 3] = tot[u % 3];
    for (int u = 0; u < n_mid; ++u) {
      const int f = l_mid[u], nb = s_nb[f];
      const unsigned char* col = J.bins + (size_t)f * n;
      long long* out = hl + (size_t)s_off[f] * 3;
      if (nb <= 4) stump_hist_regs<4>(col, g, h, wcur, n, nb, J.qscale, out, red);
      else stump_hist_regs<8>(col, g, h, wcur, n, nb, J.qscale, out, red);
    }
    if (n_wide > 0) {
      for (int i = tid; i < n; i += kStThreads) {
        const float wi = wcur[i];
        if (!(wi > 0.f)) continue;
        const long long qg = q_of(g[i], J.qscale), qh = q_of(h[i], J.qscale), qw = q_of(wi, J.qscale);
        for (int u = 0; u < n_wide; ++u) {
          const int f = l_wide[u];
          long long* cell = hl + ((size_t)s_off[f] + J.bins[(size_t)f * n + i]) * 3;
          atomicAdd((unsigned long long*)&cell[0], (unsigned long long)qg);
          atomicAdd((unsigned long long*)&cell[1], (unsigned long long)qh);
          atomicAdd((unsigned long long*)&cell[2], (unsigned long long)qw);
        }
      }
    }
    __syncthreads();
    // ---- C: root split (gbdt_split_kernel's rule; 16 waves scan features f ≡ wave mod 16)
    if (wave == 0) {
      long long a = 0, c = 0, d = 0;
      for (int bb = lane; bb < s_nb[0]; bb += 64) { a += hl[bb * 3]; c += hl[bb * 3 + 1]; d += hl[bb * 3 + 2]; }
      a = wave_sum_i64(a);
      c = wave_sum_i64(c);
      d = wave_sum_i64(d);
      if (lane == 0) { tot[0] = a; tot[1] = c; tot[2] = d; }
    }
    __syncthreads();
    const long long tg = tot[0], th = tot[1], tw = tot[2];
    const size_t tb = (size_t)t * B + b;
    if (tw <= 0) {   // empty root (block-uniform)
      if (tid == 0) { J.feat[tb * 3] = -3; tf0 = -3; tblo = 0; tval[0] = tval[1] = tval[2] = 0.0; }
      __syncthreads();
      continue;
    }
    double bg = -1.0;
    int bf = 0x7fffffff, bbin = 0;
    if ((double)tw >= J.min_split_q) {
      for (int f = wave; f < F; f += kStWaves) {
        double gg;
        int gb;
        scan_feature(hl + (size_t)s_off[f] * 3, s_nb[f], lane, tw, tg, J.min_leaf_q, gg, gb);
        if (gg > bg) { bg = gg; bf = f; bbin = gb; }   // f ascending within a wave
      }
    }
    if (lane == 0) { wg[wave] = bg; wf[wave] = bf; wbin[wave] = bbin; }
    __syncthreads();
    if (tid == 0) {
      bg = wg[0]; bf = wf[0]; bbin = wbin[0];
      for (int k = 1; k < kStWaves; ++k)
        if (wg[k] > bg || (wg[k] == bg && wf[k] < bf)) { bg = wg[k]; bf = wf[k]; bbin = wbin[k]; }
      long long* st = J.stats + tb * 3 * 4;
      st[0] = tw; st[1] = tg; st[2] = th;
      const double inv = 1.0 / J.qscale;
      const double dw = tw * inv, dg = tg * inv;
      const double imp = root_r2 * inv / dw - (dg / dw) * (dg / dw);
      const bool can_split = bg >= 0.0 && bf < F && imp > 2.220446049250313e-16;
      tval[1] = 0.0;
      tval[2] = 0.0;
      if (!can_split) {
        J.feat[tb * 3] = -2;
        J.blo[tb * 3] = 0;
        J.thr[tb * 3] = -2.0;
        const double den = th * inv;
        const double v = fabs(den) < 1e-150 ? 0.0 : dg / den;
        J.value[tb * 3] = v;
        tf0 = -2; tblo = 0; tval[0] = v;
      } else {
        const long long* hf = hl + (size_t)s_off[bf] * 3;
        long long lw = 0, lg = 0, lh = 0;
        for (int bb = 0; bb <= bbin; ++bb) { lg += hf[bb * 3]; lh += hf[bb * 3 + 1]; lw += hf[bb * 3 + 2]; }
        int hi = bbin + 1;
        const int nbf = s_nb[bf];
        while (hi < nbf - 1 && hf[hi * 3 + 2] == 0) ++hi;
        const double a = J.hi_val[bf * 256 + bbin], c = J.lo_val[bf * 256 + hi];
        double tt = a / 2.0 + c / 2.0;
        if (tt == c || isinf(tt)) tt = a;
        J.feat[tb * 3] = bf;
        J.blo[tb * 3] = bbin;
        J.thr[tb * 3] = tt;
        J.value[tb * 3] = dg / dw;   // internal node value: weighted mean residual
        long long* sl = st + 4;
        long long* sr = st + 8;
        sl[0] = lw; sl[1] = lg; sl[2] = lh;
        sr[0] = tw - lw; sr[1] = tg - lg; sr[2] = th - lh;
        J.feat[tb * 3 + 1] = -2; J.feat[tb * 3 + 2] = -2;
        J.blo[tb * 3 + 1] = 0; J.blo[tb * 3 + 2] = 0;
        J.thr[tb * 3 + 1] = -2.0; J.thr[tb * 3 + 2] = -2.0;
        const double dl = lh * inv, dr = (th - lh) * inv;
        const double vl = fabs(dl) < 1e-150 ? 0.0 : lg * inv / dl;
        const double vr = fabs(dr) < 1e-150 ? 0.0 : (tg - lg) * inv / dr;
        J.value[tb * 3 + 1] = vl;
        J.value[tb * 3 + 2] = vr;
        tf0 = bf; tblo = bbin; tval[0] = dg / dw; tval[1] = vl; tval[2] = vr;
      }
    }
    __syncthreads();
  }
}

void gbdt_stumps_fused(int B, int n, int F, int T, uintptr_t bins, uintptr_t nbins, int hist_len,
                       uintptr_t lo_val, uintptr_t hi_val, uintptr_t y, uintptr_t w, uintptr_t raw, uintptr_t g,
                       uintptr_t h, uintptr_t wt, uintptr_t seeds, long long row_off, double subsample,
                       uintptr_t feat, uintptr_t blo, uintptr_t thr, uintptr_t value, uintptr_t stats,
                       uintptr_t r2, uintptr_t dev, uintptr_t bagw, double lr, double qscale, double dscale,
                       double min_leaf_q, double min_split_q, uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F <= kStMaxF, "gbdt_stumps_fused: 1 <= F <= 128");
  HFENS_REQUIRE(B >= 1 && n >= 1 && T >= 1, "gbdt_stumps_fused: empty problem");
  const bool active = subsample < 1.0;
  HFENS_REQUIRE(!active || (wt != 0 && seeds != 0 && bagw != 0),
                "gbdt_stumps_fused: subsample needs wt, seeds and bagw");
  const size_t lds = (size_t)hist_len * 3 * sizeof(long long);
  HFENS_REQUIRE(hist_len >= F && lds <= 120 * 1024, "gbdt_stumps_fused: root histograms do not fit LDS");
  StumpJob J{(const unsigned char*)bins, (const int*)nbins, (const double*)lo_val, (const double*)hi_val,
             (const float*)y, (const float*)w, (double*)raw, (float*)g, (float*)h, (float*)wt,
             (const unsigned long long*)seeds, (int*)feat, (int*)blo, (double*)thr, (double*)value,
             (long long*)stats, (long long*)r2, (long long*)dev, (double*)bagw, row_off, lr, qscale, dscale,
             min_leaf_q, min_split_q, (unsigned)llround(subsample * 16777216.0), active ? 1 : 0, B, n, F, T,
             hist_len};
  hipLaunchKernelGGL(gbdt_stumps_fused_kernel, dim3(B), dim3(kStThreads), lds, as_stream(stream), J);
  launch_check();
}


// ------------------------------------------------------------------------------------------
// F: depth-1 trees, ONE launch per boosting stage over MANY workgroups (gbdt_stump_stage).
//
// The fused kernel above gives each model one workgroup for the whole run (6 CUs busy on the
// bench) and cannot take a collective between stages.  Here launch t runs over a grid of
// (row tiles × models) and does, per workgroup:
//   1. the SPLIT of tree t−1 from the fully reduced stage-(t−1) histogram (every workgroup of the
//      model computes the same split redundantly from the same integers — no grid sync; workgroup
//      0 of the model writes the tree record and the previous stage's bookkeeping);
//   2. APPLY of tree t−1 to its row tile (raw += lr·leaf, leaf Σw·r², stage deviance) and stage
//      t's residual/hessian, quantised once into an LDS row cache;
//   3. the stage-t HISTOGRAM of its tile (binary features 8 per register pass, ≤ 8-bin features in
//      registers, wider ones with ds_add_u64), flushed with int64 atomics into comm slot t mod 3,
//      plus the model's extras (root Σw·r², the previous tree's leaf Σw·r², deviance, bag count).
// Slots rotate over 3 buffers: launch t reads slot t−1, accumulates slot t and zeroes slot t+1.
// Between launches the host runs ONE all-reduce of slot t under data parallelism (histogram +
// extras in one int64 SUM: exact, so every rank computes the identical split) — the whole stage
// costs one launch and one collective.  Sums, split rule, thresholds and leaf values are the
// fused kernel's (same fixed-point integers), so trees are bit-identical to it; the only
// addition is an optional per-tree feature RANK for tie-breaks (sklearn's Fisher–Yates visit
// order, computed on the host) instead of the lowest feature index.
constexpr int kSgThreads = 512;
constexpr int kSgWaves = kSgThreads / 64;
constexpr int kSgTile = 1024;       // rows per workgroup (LDS row cache: 3 × 8 B per row)
constexpr int kSgExtra = 8;         // int64 extras per model and slot
constexpr int kSgRowPad = kSgTile + kSgTile / 16;   // padded row-cache length
constexpr int kSgArrSkew = 4;                       // int64 skew between the qg / qh / qw arrays
__device__ __forceinline__ int sg_ri(int r) { return r + (r >> 4); }

struct StageJob {
  const unsigned char* bins;          // [F][n]
  const int* nbins;                   // [F]
  const double* lo_val;               // [F][256]
  const double* hi_val;               // [F][256]
  const float* y;                     // [n]
  const float* w;                     // [B][n]
  double* raw;                        // [B][n]
  float* wt;                          // [B][n] in-bag weights (bagging) or nullptr
  const unsigned long long* seeds;    // [B] (bagging) or nullptr
  long long* comm;                    // [3][B][3·hist_len + kSgExtra]
  int* feat;                          // [T][B][3]
  int* blo;                           // [T][B][3]
  double* thr;                        // [T][B][3]
  double* value;                      // [T][B][3]
  long long* stats;                   // [T][B][3][4]
  long long* r2;                      // [T][B][3]
  long long* dev;                     // [T][B]
  double* bagw;                       // [T][B] (bagging) or nullptr
  const int* frank;                   // [T][B][F] tie-break rank of each feature, or nullptr
  long long row_off;
  double lr, qscale, dscale, min_leaf_q, min_split_q;
  unsigned thr24;
  int active, B, n, F, T, hist_len, t, rows_per_wg;
  long long ldb;                      // row stride of bins (≥ n, multiple of 1024: 16-byte lane loads)
  long long* partials;                // [B][G][3·hist_len + kSgExtra] per-workgroup slots, or nullptr
  long long* prof;                    // diagnostics: [B][G][6] s_memtime phase stamps, or nullptr
  const int* t_dev;                   // stage index read from device memory (graph replay), or nullptr: t
  unsigned* bar;                      // persistent launch: [B] monotone per-model barrier counters (zeroed)
  unsigned* err;                      // persistent launch: set when a barrier wait passed its deadline
  long long deadline;                 // persistent launch: barrier wait limit in 100 MHz ticks (< 0: fail at once)
};

// Barrier of the persistent stage loop (gbdt_stump_stage with persist = 1).  Models are independent
// (stage t of model b reads only model b's stage t−1 slot), so each model's workgroups wait only for
// each other: every workgroup adds one arrival to its model's monotone counter and waits until it
// reaches k·G (barrier k, G workgroups per model);
// agent-scope fences on both sides make the stage's int64 slot atomics and stores visible to every
// XCD's next-stage reads.  Residency: the grid is at most one workgroup per CU (sg_plan) and no
// workgroup waits on anything but this counter, so workgroups that are not yet resident (CUs held
// by another stream's kernels) are dispatched as those finish.  A wait past the deadline (fixed
// 100 MHz s_memrealtime clock, HFENS_GBDT_PERSIST_DEADLINE_MS, 2 s by default) sets *err and every
// workgroup leaves the loop; the host then re-runs the fit launch per stage (models/hist_gbdt.py).
// A negative deadline injects that failure at the first barrier (tests of the fallback).
__device__ __forceinline__ bool sg_grid_barrier(unsigned* bar, unsigned* err, unsigned target, long long deadline) {
  __syncthreads();
  __shared__ int s_ok;
  if (threadIdx.x == 0) {
    __threadfence();
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    int ok = 1;
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u ||
          deadline < 0 || (long long)__builtin_amdgcn_s_memrealtime() - t0 > deadline) {
        __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    __threadfence();
    s_ok = ok;
  }
  __syncthreads();
  return s_ok != 0;
}

template <int NV, int NW = kSgWaves>
__device__ __forceinline__ void sg_block_sum(long long (&v)[NV], long long* red, long long* out) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const long long s = wave_sum_i64(v[k]);
    if (lane == 0) red[wave * 24 + k] = s;
  }
  __syncthreads();
  if ((int)threadIdx.x < NV) {
    long long s = 0;
    for (int k = 0; k < NW; ++k) s += red[k * 24 + threadIdx.x];
    out[threadIdx.x] = s;
  }
  __syncthreads();
}

// ≤ C-bin feature over the tile from the quantised row cache: registers, one fold into LDS.
template <int C>
__device__ __forceinline__ void sg_hist_regs(const unsigned char* __restrict__ col, const long long* qg,
                                             const long long* qh, const long long* qw, int m, int nb,
                                             long long* out /*[nb][3] LDS*/, long long* red) {
  long long ag[C], ah[C], aw[C];
#pragma unroll
  for (int c = 0; c < C; ++c) { ag[c] = 0; ah[c] = 0; aw[c] = 0; }
  for (int i = threadIdx.x; i < m; i += kSgThreads) {
    const long long w = qw[i];
    if (w == 0) continue;
    const int bb = col[i];
    const long long g = qg[i], h = qh[i];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const bool k = bb == c;
      ag[c] += k ? g : 0;
      ah[c] += k ? h : 0;
      aw[c] += k ? w : 0;
    }
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const long long a = wave_sum_i64(ag[c]), b2 = wave_sum_i64(ah[c]), c2 = wave_sum_i64(aw[c]);
    if (lane == 0) {
      red[wave * 24 + 3 * c] = a;
      red[wave * 24 + 3 * c + 1] = b2;
      red[wave * 24 + 3 * c + 2] = c2;
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < 3 * nb) {
    long long s = 0;
    for (int k = 0; k < kSgWaves; ++k) s += red[k * 24 + threadIdx.x];
    out[threadIdx.x] += s;
  }
  __syncthreads();
}

// MF = true: the histogram of every feature with 2–8 bins (binary features, small ordinals) is an
// integer GEMM on the matrix cores instead of int64 VALU sums.  The stage's quantised g, h, w
// (int64 fixed point, |q| < 2^49) are cut into 7 slices of 7 bits (the top slice signed), so
// B[row][slice] is an i8 matrix of 21 columns; A[indicator][row] is the 0/1 byte (bin == c) of one
// (feature, bin c ≥ 1) pair per row of A, plus an all-ones row (the node totals, whence bin 0).
// v_mfma_i32_32x32x32_i8 sums A·B over 32 rows per instruction into exact int32 slice sums
// (|slice| ≤ 127: exact up to 16.9M rows per workgroup), folded once per sub-tile into an LDS
// table and recombined as Σ_k S_k·2^{7k} in int64 — the same integers as the VALU path, so the
// histogram, the split and the trees are bit-identical to it.  Features with more bins keep the
// LDS int64 atomics.
constexpr int kSgMaxInd = 128;      // indicator rows (4 M-blocks of 32)
constexpr int kSgSlices = 7;        // 7-bit slices per value
typedef int sg_v4i __attribute__((ext_vector_type(4)));
typedef int sg_v16i __attribute__((ext_vector_type(16)));

// 0x01 in every byte of x equal to c, 0x00 elsewhere (SWAR zero-byte test; no carries across bytes)
__device__ __forceinline__ int sg_eq_bytes(unsigned x, unsigned c) {
  const unsigned t = x ^ (c * 0x01010101u);
  const unsigned nz = ((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t;
  return (int)((~nz >> 7) & 0x01010101u);
}

__device__ __forceinline__ long long sg_comb(const int* T, int ind, int v) {
  const int* r = T + ind * 32 + kSgSlices * v;
  long long s = 0;
#pragma unroll
  for (int k = 0; k < kSgSlices - 1; ++k) s += (long long)r[k] << (7 * k);
  return s + ((long long)r[kSgSlices - 1] << (7 * (kSgSlices - 1)));
}

// Persist = false: one launch per stage t (J.t or *J.t_dev).  Persist = true: ONE launch runs every
// stage t = 0 … T+1 of the boosting, separated by sg_grid_barrier — the same per-stage body, so the
// same integers, splits and trees, without a launch boundary (and its host enqueue) per stage.
template <bool MF, int NT, bool Persist = false>
__global__ __launch_bounds__(NT) void gbdt_stump_stage_kernel(StageJob J) {
  constexpr int kT = NT, kW = NT / 64;       // threads, waves
  constexpr int RPT = kSgTile / kT;           // rows per thread in the apply
  constexpr int RPW = kSgTile / kW;           // rows per wave in the MFMA histogram
  constexpr int KS = RPW / 32;                // its K-steps of 32 rows
  static_assert(RPT * kT == kSgTile && KS * 32 * kW == kSgTile, "tile shape");
  extern __shared__ __attribute__((aligned(16))) long long sg_lds[];
  long long* hl = sg_lds;                                   // [hist_len][3]
  // row cache: quantised g, h, w of 1024 rows, row r at r + r/16 (one pad word per 16 rows: lane ℓ
  // reading row 16ℓ + j then strides 17 words — conflict-free — instead of 16, a 32-way conflict)
  // (the three arrays are 4 words apart modulo the 64 banks: the MFMA B-fragment build reads row
  // k of all three in one instruction — 3-way bank conflicts with a plain kSgRowPad stride)
  long long* qg = sg_lds + 3 * (size_t)J.hist_len;
  long long* qh = qg + kSgRowPad + kSgArrSkew;
  long long* qw = qh + kSgRowPad + kSgArrSkew;
  __shared__ long long red[kW * 24];
  __shared__ int s_nb[kStMaxF], s_off[kStMaxF];
  __shared__ int l_bin[kStMaxF], l_one[kStMaxF], l_mid[kStMaxF], l_wide[kStMaxF];
  __shared__ int n_bin, n_one, n_mid, n_wide;
  __shared__ long long tot[3], bsum[24], ext[8];
  __shared__ double wg[kW];
  __shared__ int wf[kW], wbin[kW], wrk[kW];
  __shared__ int pf_s, pblo_s;
  __shared__ double pv_s[3];
  // MF: indicator rows (feature, bin; −1 = all ones, −2 = padding), MFMA features and their first row
  __shared__ int s_indf[MF ? kSgMaxInd : 1], s_indc[MF ? kSgMaxInd : 1];
  __shared__ int l_mf[MF ? kStMaxF : 1], l_mfi[MF ? kStMaxF : 1];
  __shared__ int n_mf, n_mb;
  __shared__ int s_ord[kStMaxF];   // split-scan order: features with > 4 bins first (spread over waves)
  int* Tsl = reinterpret_cast<int*>(qw + kSgRowPad + kSgArrSkew);   // MF: [n_mb·32 indicators][32 slice columns] int32
  const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = J.n, F = J.F, B = J.B, T = J.T;
  const int t_first = Persist ? 0 : (J.t_dev != nullptr ? *J.t_dev : J.t);
  const int t_last = Persist ? T + 1 : t_first;
  const size_t slot_m = 3 * (size_t)J.hist_len + kSgExtra;
  const size_t slot_sz = (size_t)B * slot_m;
  // the features' bin counts: one load per thread, in parallel (a serial loop of dependent global
  // loads in thread 0 cost several µs per launch)
  if (tid < F) s_nb[tid] = J.nbins[tid];
  __syncthreads();
  if (tid == 0) {
    int o = 0;
    n_bin = n_one = n_mid = n_wide = 0;
    for (int f = 0; f < F; ++f) {
      const int nb = s_nb[f];
      s_off[f] = o; o += nb;
      if (nb == 2) l_bin[n_bin++] = f;
      else if (nb <= 1) l_one[n_one++] = f;
      else if (nb <= 8) l_mid[n_mid++] = f;
      else l_wide[n_wide++] = f;
    }
    {
      int o2 = 0;
      for (int f = 0; f < F; ++f) if (s_nb[f] > 4) s_ord[o2++] = f;
      for (int f = 0; f < F; ++f) if (s_nb[f] <= 4) s_ord[o2++] = f;
    }
    if constexpr (MF) {
      int ni = 1;
      s_indf[0] = -1; s_indc[0] = 0;
      n_mf = 0; n_wide = 0;
      for (int f = 0; f < F; ++f) {
        const int nb = s_nb[f];
        if (nb >= 2 && nb <= 8 && ni + nb - 1 <= kSgMaxInd) {
          l_mf[n_mf] = f; l_mfi[n_mf] = ni; ++n_mf;
          for (int c = 1; c < nb; ++c) { s_indf[ni] = f; s_indc[ni] = c; ++ni; }
        } else if (nb > 1) {
          l_wide[n_wide++] = f;
        }
      }
      n_mb = (ni + 31) / 32;
      for (int i = ni; i < n_mb * 32; ++i) { s_indf[i] = -2; s_indc[i] = 0; }
    }
    pf_s = -3; pblo_s = 0; pv_s[0] = pv_s[1] = pv_s[2] = 0.0;
  }
  for (int t = t_first;; ++t) {
  if constexpr (Persist) {
    if (t > t_first && !sg_grid_barrier(J.bar + b, J.err, (unsigned)(t - t_first) * gridDim.x, J.deadline)) return;
    if (tid == 0) { pf_s = -3; pblo_s = 0; pv_s[0] = pv_s[1] = pv_s[2] = 0.0; }
  }
  long long* slot_prev = J.comm + (size_t)((t + 2) % 3) * slot_sz + (size_t)b * slot_m;
  long long* slot_cur = J.comm + (size_t)(t % 3) * slot_sz + (size_t)b * slot_m;
  long long* slot_next = J.comm + (size_t)((t + 1) % 3) * slot_sz;
  // zero this model's part of the slot that stage t+1 accumulates (nobody reads or writes it during
  // stage t; per model, because in the persistent loop another model may still be in stage t−1,
  // reading its own part of that slot)
  for (size_t k = (size_t)blockIdx.x * kT + tid; k < slot_m; k += (size_t)gridDim.x * kT) slot_next[(size_t)b * slot_m + k] = 0;
  __syncthreads();
  const bool lead = blockIdx.x == 0;
  const double inv = 1.0 / J.qscale;
  long long* pst = J.prof ? J.prof + ((size_t)b * gridDim.x + blockIdx.x) * 6 : nullptr;
  const long long t_0 = pst ? (long long)__builtin_amdgcn_s_memtime() : 0;
  // ---- bookkeeping of the reduced previous slot (launch t−1's extras), by the model's leader
  if (lead && tid == 0 && t >= 1) {
    const long long* E = slot_prev + 3 * (size_t)J.hist_len;
    if (t - 1 < T) {
      const size_t tb = (size_t)(t - 1) * B + b;
      J.r2[tb * 3] = E[0];
      if (J.active) J.bagw[tb] = (double)E[5] * inv;
    }
    if (t - 2 >= 0 && t - 2 < T) {
      const size_t pb = (size_t)(t - 2) * B + b;
      J.r2[pb * 3] += E[1];
      J.r2[pb * 3 + 1] += E[2];
      J.r2[pb * 3 + 2] += E[3];
      J.dev[pb] += E[4];
    }
  }
  if (t > T) break;   // the closing launch only books the last slot
  // a sub-tile's row inputs (this thread's two rows: kSgTile = 2 × threads) are loaded one sub-tile
  // ahead — issued before the previous sub-tile's histogram, consumed by the next apply — so their
  // global latencies overlap the histogram instead of stalling the apply.  The first sub-tile's
  // weights, raw scores and labels do not depend on tree t−1's split: they are issued before it, so
  // their latency hides under the split (a third of a small-shard stage, profiles/r3_gbdt_dp.md);
  // only the split feature's bin column waits for it.
  const int w0r = blockIdx.x * J.rows_per_wg;
  const int w1r = min(n, w0r + J.rows_per_wg);
  float w0v[RPT];
  double rwv[RPT], yv[RPT];
  int bnv[RPT];
  auto load_vals = [&](int rs) {
    const int ms = min(kSgTile, w1r - rs);
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      const int k = tid + u * kT;
      const bool ok = k < ms;
      const int i = rs + (ok ? k : 0);
      const size_t bi = (size_t)b * n + i;
      w0v[u] = ok ? J.w[bi] : 0.f;
      rwv[u] = ok ? J.raw[bi] : 0.0;
      yv[u] = ok ? (double)J.y[i] : 0.0;
    }
  };
  auto load_bins = [&](int rs, int pfeat) {
    const int ms = min(kSgTile, w1r - rs);
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      const int k = tid + u * kT;
      const bool ok = k < ms;
      const int i = rs + (ok ? k : 0);
      bnv[u] = (ok && t >= 1 && pfeat >= 0) ? (int)J.bins[(size_t)pfeat * J.ldb + i] : 0;
    }
  };
  if (w0r < w1r) load_vals(w0r);
  // ---- 1: split of tree t−1 from the reduced stage-(t−1) histogram
  if (t >= 1) {
    // stage the reduced histogram in LDS first (one bulk round of loads, 8 in flight per thread):
    // the scans below then cost LDS latency instead of a dependent global round per feature
    const long long root_r2 = slot_prev[3 * (size_t)J.hist_len];
    {
      const int len = 3 * J.hist_len;
      for (int k0 = tid; k0 < len; k0 += 8 * kT) {
        long long v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int k = k0 + u * kT;
          v[u] = k < len ? slot_prev[k] : 0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int k = k0 + u * kT;
          if (k < len) hl[k] = v[u];
        }
      }
    }
    __syncthreads();
    const long long* hp = hl;
    if (wave == 0) {
      long long a = 0, c = 0, d = 0;
      for (int bb = lane; bb < s_nb[0]; bb += 64) { a += hp[bb * 3]; c += hp[bb * 3 + 1]; d += hp[bb * 3 + 2]; }
      a = wave_sum_i64(a); c = wave_sum_i64(c); d = wave_sum_i64(d);
      if (lane == 0) { tot[0] = a; tot[1] = c; tot[2] = d; }
    }
    __syncthreads();
    const long long tg = tot[0], th = tot[1], tw = tot[2];
    const size_t tb = (size_t)(t - 1) * B + b;
    const int* rk = J.frank ? J.frank + tb * F : nullptr;
    if (tw <= 0) {
      if (tid == 0) {
        if (lead) J.feat[tb * 3] = -3;
        pf_s = -3; pblo_s = 0; pv_s[0] = pv_s[1] = pv_s[2] = 0.0;
      }
    } else {
      double bg = -1.0;
      int bf = 0x7fffffff, bbin = 0, brk = 0x7fffffff;
      if ((double)tw >= J.min_split_q) {
        for (int fo = wave; fo < F; fo += kW) {
          const int f = s_ord[fo];
          double gg;
          int gb;
          if (s_nb[f] <= 4) scan_feature_small(hp + (size_t)s_off[f] * 3, s_nb[f], tw, tg, J.min_leaf_q, gg, gb);
          else scan_feature(hp + (size_t)s_off[f] * 3, s_nb[f], lane, tw, tg, J.min_leaf_q, gg, gb);
          const int r = rk ? rk[f] : f;
          if (gg > bg || (gg == bg && gg >= 0.0 && r < brk)) { bg = gg; bf = f; bbin = gb; brk = r; }
        }
      }
      if (lane == 0) { wg[wave] = bg; wf[wave] = bf; wbin[wave] = bbin; wrk[wave] = brk; }
      __syncthreads();
      if (tid == 0) {
        bg = wg[0]; bf = wf[0]; bbin = wbin[0]; brk = wrk[0];
        for (int k = 1; k < kW; ++k)
          if (wg[k] > bg || (wg[k] == bg && wrk[k] < brk)) { bg = wg[k]; bf = wf[k]; bbin = wbin[k]; brk = wrk[k]; }
        wg[0] = bg; wf[0] = bf; wbin[0] = bbin;
      }
      __syncthreads();
      bg = wg[0]; bf = wf[0]; bbin = wbin[0];
      const double dw = tw * inv, dg = tg * inv;
      const double imp = root_r2 * inv / dw - (dg / dw) * (dg / dw);
      const bool can_split = bg >= 0.0 && bf < F && imp > 2.220446049250313e-16;
      if (can_split && wave == 0) {
        // the chosen bin's left sums: one parallel pass of wave 0 (a serial loop over up to 256
        // bins × 3 global loads by one thread cost more than the rest of the split)
        const long long* hf = hp + (size_t)s_off[bf] * 3;
        long long lw = 0, lg = 0, lh = 0;
        for (int bb = lane; bb <= bbin; bb += 64) { lg += hf[bb * 3]; lh += hf[bb * 3 + 1]; lw += hf[bb * 3 + 2]; }
        lg = wave_sum_i64(lg);
        lh = wave_sum_i64(lh);
        lw = wave_sum_i64(lw);
        if (lane == 0) { tot[0] = lg; tot[1] = lh; tot[2] = lw; }
      }
      __syncthreads();
      if (tid == 0) {
        long long* st = J.stats + tb * 3 * 4;
        if (lead) { st[0] = tw; st[1] = tg; st[2] = th; }
        if (!can_split) {
          const double den = th * inv;
          const double v = fabs(den) < 1e-150 ? 0.0 : dg / den;
          if (lead) { J.feat[tb * 3] = -2; J.blo[tb * 3] = 0; J.thr[tb * 3] = -2.0; J.value[tb * 3] = v; }
          pf_s = -2; pblo_s = 0; pv_s[0] = v; pv_s[1] = 0.0; pv_s[2] = 0.0;
        } else {
          const long long* hf = hp + (size_t)s_off[bf] * 3;
          const long long lg = tot[0], lh = tot[1], lw = tot[2];
          const double dl = lh * inv, dr = (th - lh) * inv;
          const double vl = fabs(dl) < 1e-150 ? 0.0 : lg * inv / dl;
          const double vr = fabs(dr) < 1e-150 ? 0.0 : (tg - lg) * inv / dr;
          if (lead) {
            int hi = bbin + 1;
            const int nbf = s_nb[bf];
            while (hi < nbf - 1 && hf[hi * 3 + 2] == 0) ++hi;
            const double a = J.hi_val[bf * 256 + bbin], c = J.lo_val[bf * 256 + hi];
            double tt = a / 2.0 + c / 2.0;
            if (tt == c || isinf(tt)) tt = a;
            J.feat[tb * 3] = bf; J.blo[tb * 3] = bbin; J.thr[tb * 3] = tt; J.value[tb * 3] = dg / dw;
            long long* sl = st + 4;
            long long* sr = st + 8;
            sl[0] = lw; sl[1] = lg; sl[2] = lh;
            sr[0] = tw - lw; sr[1] = tg - lg; sr[2] = th - lh;
            J.feat[tb * 3 + 1] = -2; J.feat[tb * 3 + 2] = -2;
            J.blo[tb * 3 + 1] = 0; J.blo[tb * 3 + 2] = 0;
            J.thr[tb * 3 + 1] = -2.0; J.thr[tb * 3 + 2] = -2.0;
            J.value[tb * 3 + 1] = vl; J.value[tb * 3 + 2] = vr;
          }
          pf_s = bf; pblo_s = bbin; pv_s[0] = dg / dw; pv_s[1] = vl; pv_s[2] = vr;
        }
      }
    }
    __syncthreads();
  }
  if (pst && tid == 0) pst[0] = (long long)__builtin_amdgcn_s_memtime() - t_0;
  // ---- 2+3 over this workgroup's rows, 1024 at a time: apply tree t−1, stage t's residuals into
  // the LDS row cache, the stage-t histogram accumulated in LDS across sub-tiles (flushed once)
  const bool has_prev = t >= 1, has_cur = t < T;
  const int pf = pf_s, pblo = pblo_s;
  const double pv0 = pv_s[0], pv1 = pv_s[1], pv2 = pv_s[2];
  long long acc6[6] = {0, 0, 0, 0, 0, 0};   // dev(t−1), r2 root(t), leaf r2 n0..n2 (t−1), bag(t)
  if (has_cur) {
    for (int k = tid; k < 3 * J.hist_len; k += kT) hl[k] = 0;
    if constexpr (MF)
      for (int k = tid; k < n_mb * 32 * 32; k += kT) Tsl[k] = 0;
  }
  if (w0r < w1r) load_bins(w0r, pf);   // (its weights / raw / labels were issued before the split)
  // MF: the matrix-core slice sums stay in registers across the tile's sub-tiles (exact int32: at
  // most 127 per row per slice) and are folded into the LDS table once, after the last sub-tile
  sg_v16i acc_all[MF ? 4 : 1];
#pragma unroll
  for (int mb = 0; mb < (MF ? 4 : 1); ++mb) acc_all[mb] = sg_v16i{};
  for (int r0 = w0r; r0 < w1r; r0 += kSgTile) {
    const int m = min(kSgTile, w1r - r0);
    __syncthreads();   // the previous sub-tile's histogram passes are done with the row cache
    const long long t_ap = pst ? (long long)__builtin_amdgcn_s_memtime() : 0;
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      const int k = tid + u * kT;
      if (k >= m) continue;
      const int i = r0 + k;
      const size_t bi = (size_t)b * n + i;
      const float w0 = w0v[u];
      float wi = w0, wp = w0;
      if (J.active) {
        const unsigned long long sd = J.seeds[b];
        wi = (has_cur && gb_in_bag(sd, t, J.row_off + i, J.thr24)) ? w0 : 0.f;
        wp = (has_prev && gb_in_bag(sd, t - 1, J.row_off + i, J.thr24)) ? w0 : 0.f;
        if (has_cur) J.wt[bi] = wi;
      }
      double rw = rwv[u];
      const double yi = yv[u];
      if (has_prev) {
        const int nd = pf >= 0 ? (bnv[u] <= pblo ? 1 : 2) : 0;
        if (wp > 0.f) {
          const double p0 = 1.0 / (1.0 + exp(-rw));
          const double r0d = yi - p0;
          const long long q = q_of(wp * r0d * r0d, J.qscale);
          acc6[2] += nd == 0 ? q : 0;
          acc6[3] += nd == 1 ? q : 0;
          acc6[4] += nd == 2 ? q : 0;
        }
        rw += J.lr * (nd == 0 ? pv0 : (nd == 1 ? pv1 : pv2));
        J.raw[bi] = rw;
        if (wp > 0.f) {
          const double l1p = rw > 0 ? rw + log1p(exp(-rw)) : log1p(exp(rw));
          acc6[0] += q_of(wp * (-2.0) * (yi * rw - l1p), J.dscale);
        }
      }
      if (has_cur) {
        const double p = 1.0 / (1.0 + exp(-rw));
        const double r = yi - p;
        const float gf = (float)(wi * r);
        const float hf = (float)(wi * p * (1.0 - p));
        const bool in = wi > 0.f;
        qg[sg_ri(k)] = in ? q_of(gf, J.qscale) : 0;
        qh[sg_ri(k)] = in ? q_of(hf, J.qscale) : 0;
        qw[sg_ri(k)] = in ? q_of(wi, J.qscale) : 0;
        if (in) acc6[1] += q_of(wi * r * r, J.qscale);
        if (J.active) acc6[5] += in ? q_of(wi, J.qscale) : 0;
      }
    }
    if (r0 + kSgTile < w1r) {
      load_vals(r0 + kSgTile);
      load_bins(r0 + kSgTile, pf);
    }
    if (!has_cur) continue;
    for (int k = m + tid; k < kSgTile; k += kT) { qg[sg_ri(k)] = 0; qh[sg_ri(k)] = 0; qw[sg_ri(k)] = 0; }
    if (pst && tid == 0) pst[1] += (long long)__builtin_amdgcn_s_memtime() - t_ap;   // wave 0's apply, summed
    __syncthreads();
    if constexpr (MF) {
      const long long t_a = pst ? (long long)__builtin_amdgcn_s_memtime() : 0;
      // (a) binary / ≤ 8-bin features on the matrix cores: wave w takes rows [128w, 128w + 128) of
      // the sub-tile in 4 K-steps of 32; lane (c = lane & 31, h = lane >> 5) holds, for the 16 rows
      // 16h … 16h + 15 of the step, slice c % 7 of value c / 7 (B, c < 21) and the indicator bytes
      // of A-row c of every M-block (A and B bytes j of half h are the same row: the product sums
      // the same row set whatever the hardware's k order inside a fragment)
      const int c = lane & 31, hh = lane >> 5;
      const int vsel = c / kSgSlices, ks = c - kSgSlices * vsel;
      const long long* qv = vsel == 0 ? qg : (vsel == 1 ? qh : qw);
      const int nmb = n_mb;
      sg_v16i (&acc)[4] = acc_all;
      // A bytes of every M-block, one K-step ahead (the global loads overlap the B build and MFMAs)
      const unsigned char* arow[4];
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        const int f = mb < nmb ? s_indf[mb * 32 + c] : -2;
        arow[mb] = f >= 0 ? J.bins + (size_t)f * J.ldb + r0 + RPW * wave + 16 * hh : nullptr;
      }
      uint4 araw[4];
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
        araw[mb] = arow[mb] ? *reinterpret_cast<const uint4*>(arow[mb]) : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int kst = 0; kst < KS; ++kst) {
        const int k0 = RPW * wave + 32 * kst + 16 * hh;   // 16-aligned: rows k0 … k0+15 are contiguous in the padded cache
        uint4 anext[4];
#pragma unroll
        for (int mb = 0; mb < 4; ++mb)
          anext[mb] = (kst < KS - 1 && arow[mb]) ? *reinterpret_cast<const uint4*>(arow[mb] + 32 * (kst + 1))
                                            : make_uint4(0, 0, 0, 0);
        sg_v4i bf = sg_v4i{0, 0, 0, 0};
        if (c < 3 * kSgSlices) {
          const long long* src = qv + sg_ri(k0);
          const int sh = 7 * ks;
          const unsigned msk = ks < kSgSlices - 1 ? 127u : 255u;
          int wd[4];
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            unsigned x = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) x |= ((unsigned)(src[4 * d + e] >> sh) & msk) << (8 * e);
            wd[d] = (int)x;
          }
          bf = sg_v4i{wd[0], wd[1], wd[2], wd[3]};
        }
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
          if (mb < nmb) {
            const int f = s_indf[mb * 32 + c];
            sg_v4i af;
            if (f >= 0) {
              const uint4 x = araw[mb];
              const unsigned cc = (unsigned)s_indc[mb * 32 + c];
              af = sg_v4i{sg_eq_bytes(x.x, cc), sg_eq_bytes(x.y, cc), sg_eq_bytes(x.z, cc), sg_eq_bytes(x.w, cc)};
            } else {
              const int o = f == -1 ? 0x01010101 : 0;
              af = sg_v4i{o, o, o, o};
            }
            acc[mb] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af, bf, acc[mb], 0, 0, 0);
          }
          araw[mb] = anext[mb];
        }
      }
      const long long t_b = pst ? (long long)__builtin_amdgcn_s_memtime() : 0;
      if (pst && tid == 0) pst[4] += t_b - t_a;   // (diagnostics: wave 0's MFMA part, summed over sub-tiles)
      // (b) wider features: LDS int64 atomics (integer sums: any order is exact).  Every wave takes
      // its own RPW-row slice of the sub-tile for ALL wide features (lane ℓ: RPW/64 consecutive
      // rows), so all waves share the work whatever the number of wide features
      {
        constexpr int RL = RPW / 64;            // rows per lane (2 at 512 threads)
        static_assert(RL == 1 || RL == 2 || RL == 4, "the wide-feature pass reads 1, 2 or 4 bin bytes per lane");
        const int kb = RPW * wave + RL * lane;   // first row of this lane in the sub-tile
        long long wq2[RL], gq2[RL], hq2[RL];
#pragma unroll
        for (int j = 0; j < RL; ++j) {
          const int ri = sg_ri(kb + j);
          wq2[j] = qw[ri]; gq2[j] = qg[ri]; hq2[j] = qh[ri];
        }
        const unsigned char* bt = J.bins + r0 + kb;
        for (int fi = 0; fi < n_wide; ++fi) {
          const int f = l_wide[fi], off = s_off[f];
          const unsigned char* bf_ = bt + (size_t)f * J.ldb;
          unsigned v2;
          if constexpr (RL == 4) v2 = *reinterpret_cast<const unsigned*>(bf_);
          else if constexpr (RL == 2) v2 = *reinterpret_cast<const unsigned short*>(bf_);
          else v2 = *bf_;
#pragma unroll
          for (int j = 0; j < RL; ++j) {
            if (wq2[j] == 0) continue;
            const unsigned bb = (v2 >> (8 * j)) & 0xFFu;
            long long* cell = hl + ((size_t)off + bb) * 3;
            atomicAdd((unsigned long long*)&cell[0], (unsigned long long)gq2[j]);
            atomicAdd((unsigned long long*)&cell[1], (unsigned long long)hq2[j]);
            atomicAdd((unsigned long long*)&cell[2], (unsigned long long)wq2[j]);
          }
        }
      }
      if (pst && tid == 0) pst[5] += (long long)__builtin_amdgcn_s_memtime() - t_b;   // wave 0's wide part
    } else {
      // stage-t histogram of the sub-tile.  Every wave covers ALL 1024 rows (lane ℓ owns rows
      // 16ℓ … 16ℓ+15, their quantised g/h/w in registers) and takes features f ≡ wave (mod 8): one
      // 16-byte load per lane and feature, sums in registers, wave reductions, lane 0 adds the
      // feature's bins into the LDS histogram (features are disjoint across waves: no barrier).
      long long rg[16], rh[16], rv[16];
  #pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int ri = 17 * lane + j;   // sg_ri(16·lane + j)
        rg[j] = qg[ri]; rh[j] = qh[ri]; rv[j] = qw[ri];
      }
      long long tg3 = 0, th3 = 0, tw3 = 0;
  #pragma unroll
      for (int j = 0; j < 16; ++j) { tg3 += rg[j]; th3 += rh[j]; tw3 += rv[j]; }
      tg3 = wave_sum_i64(tg3);
      th3 = wave_sum_i64(th3);
      tw3 = wave_sum_i64(tw3);
      const unsigned char* bt = J.bins + r0 + 16 * lane;
      // this wave's features in groups of 4: the group's four 16-byte tiles are loaded together
      for (int fg = wave; fg < F; fg += 4 * kW) {
        uint4 pre[4];
  #pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int f = fg + u * kW;
          pre[u] = f < F ? *reinterpret_cast<const uint4*>(bt + (size_t)f * J.ldb) : make_uint4(0, 0, 0, 0);
        }
  #pragma unroll
        for (int u = 0; u < 4; ++u) {
        const int f = fg + u * kW;
        if (f >= F) break;
        const int nb = s_nb[f], off = s_off[f];
        const uint4 v4 = pre[u];
        const unsigned wd[4] = {v4.x, v4.y, v4.z, v4.w};
        if (nb <= 1) {
          if (lane == 0) { hl[off * 3] += tg3; hl[off * 3 + 1] += th3; hl[off * 3 + 2] += tw3; }
        } else if (nb == 2) {
          long long a = 0, c = 0, d = 0;
  #pragma unroll
          for (int j = 0; j < 16; ++j) {
            const bool one = (wd[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            a += one ? rg[j] : 0;
            c += one ? rh[j] : 0;
            d += one ? rv[j] : 0;
          }
          a = wave_sum_i64(a);
          c = wave_sum_i64(c);
          d = wave_sum_i64(d);
          if (lane == 0) {
            hl[(off + 1) * 3] += a; hl[(off + 1) * 3 + 1] += c; hl[(off + 1) * 3 + 2] += d;
            hl[off * 3] += tg3 - a; hl[off * 3 + 1] += th3 - c; hl[off * 3 + 2] += tw3 - d;
          }
        } else if (nb <= 8) {
          long long acc[24];
  #pragma unroll
          for (int k = 0; k < 24; ++k) acc[k] = 0;
  #pragma unroll
          for (int j = 0; j < 16; ++j) {
            const unsigned bb = (wd[j >> 2] >> (8 * (j & 3))) & 0xFFu;
  #pragma unroll
            for (int c = 0; c < 8; ++c) {
              const bool hit = bb == (unsigned)c;
              acc[3 * c] += hit ? rg[j] : 0;
              acc[3 * c + 1] += hit ? rh[j] : 0;
              acc[3 * c + 2] += hit ? rv[j] : 0;
            }
          }
  #pragma unroll
          for (int k = 0; k < 24; ++k) {
            if (k < 3 * nb) {
              const long long sv = wave_sum_i64(acc[k]);
              if (lane == 0) hl[off * 3 + k] += sv;
            }
          }
        } else {
  #pragma unroll
          for (int j = 0; j < 16; ++j) {
            if (rv[j] == 0) continue;
            const unsigned bb = (wd[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            long long* cell = hl + ((size_t)off + bb) * 3;
            atomicAdd((unsigned long long*)&cell[0], (unsigned long long)rg[j]);
            atomicAdd((unsigned long long*)&cell[1], (unsigned long long)rh[j]);
            atomicAdd((unsigned long long*)&cell[2], (unsigned long long)rv[j]);
          }
        }
        }
      }
    }
  }
  if constexpr (MF) {
    if (has_cur) {
      // fold each wave's 32×32 slice sums into the workgroup table (D: col = lane & 31,
      // row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)) — once per stage
      const int c = lane & 31, hh = lane >> 5;
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        if (mb >= n_mb) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = (r & 3) + 8 * (r >> 2) + 4 * hh;
          const int v = acc_all[mb][r];
          if (v != 0) atomicAdd(&Tsl[(mb * 32 + row) * 32 + c], v);
        }
      }
      // slice sums → int64 bins: bin c ≥ 1 of an MFMA feature is its indicator row, bin 0 the node
      // total (all-ones row) minus the others; constant features get the total
      __syncthreads();
      for (int u = tid; u < 3 * (n_mf + n_one); u += kT) {
        const int fi = u / 3, v = u - 3 * fi;
        const long long tot_v = sg_comb(Tsl, 0, v);
        if (fi < n_mf) {
          const int f = l_mf[fi], i0 = l_mfi[fi], off = s_off[f], nb = s_nb[f];
          long long rest = 0;
          for (int cb = 1; cb < nb; ++cb) {
            const long long sv = sg_comb(Tsl, i0 + cb - 1, v);
            hl[(off + cb) * 3 + v] += sv;
            rest += sv;
          }
          hl[off * 3 + v] += tot_v - rest;
        } else {
          hl[s_off[l_one[fi - n_mf]] * 3 + v] += tot_v;
        }
      }
    }
  }
  if (pst && tid == 0) pst[2] = (long long)__builtin_amdgcn_s_memtime() - t_0;
  sg_block_sum<6, kW>(acc6, red, ext);
  // publish: int64 atomics straight into the slot (the default at every grid size: measured faster
  // than the partial slots + reduce launch up to 245 workgroups per model, sg_plan), or plain stores
  // of the whole partial slot for gbdt_stage_reduce_kernel (HFENS_SG_ATOMIC_GROUPS)
  long long* part = J.partials ? J.partials + ((size_t)b * gridDim.x + blockIdx.x) * slot_m : nullptr;
  if (tid < kSgExtra) {
    // extras layout: [0] root Σw r² (t), [1..3] leaf Σw r² (t−1), [4] deviance (t−1), [5] bag (t)
    const int src = tid == 4 ? 0 : (tid == 0 ? 1 : (tid <= 3 ? tid + 1 : (tid == 5 ? 5 : -1)));
    const long long v = src >= 0 ? ext[src] : 0;
    if (part) part[3 * (size_t)J.hist_len + tid] = v;
    else if (v != 0) atomicAdd((unsigned long long*)&slot_cur[3 * (size_t)J.hist_len + tid], (unsigned long long)v);
  }
  __syncthreads();
  for (int k = tid; k < 3 * J.hist_len; k += kT) {
    const long long v = has_cur ? hl[k] : 0;
    if (part) part[k] = v;
    else if (v != 0) atomicAdd((unsigned long long*)&slot_cur[k], (unsigned long long)v);
  }
  if (pst && tid == 0) pst[3] = (long long)__builtin_amdgcn_s_memtime() - t_0;
  if (t >= t_last) break;
  }   // stage loop
}

// Sum of the per-workgroup partial slots into the stage's comm slot: grid (slot chunks, G splits, B)
constexpr int kRdSplit = 16;
__global__ __launch_bounds__(256) void gbdt_stage_reduce_kernel(const long long* __restrict__ partials,
                                                                long long* __restrict__ slot, int G,
                                                                long long slot_m, int* __restrict__ tick) {
  // graph replay: the device stage counter advances here (nothing in this launch reads it; the
  // next stage launch does, after it) instead of in a separate gbdt_stage_tick launch
  if (tick != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x == 0) tick[0] = tick[0] + 1;
  const int b = blockIdx.z;
  const long long k = (long long)blockIdx.x * 256 + threadIdx.x;
  if (k >= slot_m) return;
  const int g0 = blockIdx.y * G / kRdSplit, g1 = (blockIdx.y + 1) * G / kRdSplit;
  const long long* p = partials + ((size_t)b * G) * slot_m + k;
  long long s = 0;
  for (int g = g0; g < g1; ++g) s += p[(size_t)g * slot_m];
  if (s != 0) atomicAdd((unsigned long long*)&slot[(size_t)b * slot_m + k], (unsigned long long)s);
}

size_t gbdt_stump_stage_lds(int hist_len, bool mf) {
  return (3 * (size_t)hist_len + 3 * (kSgRowPad + kSgArrSkew)) * sizeof(long long) +
         (mf ? kSgMaxInd * 32 * sizeof(int) : 0);
}

// Launch geometry of gbdt_stump_stage — the ONE place it is computed (the Python side sizes the
// partial-slot buffer from gbdt_stage_plan).  Rows per workgroup: 1024-row sub-tiles, as many per
// workgroup as keeps the whole grid within k workgroups per CU (HFENS_SG_WGS_PER_CU, default 1: the
// kernel holds one workgroup per CU, so a grid one workgroup over the CU count runs a second full
// round; the redundant split and the histogram flush are per workgroup, so fewer, longer
// workgroups also do less of both).  out = {rows_per_wg, groups, uses_partials, partials_len}.
static void sg_plan(long long n, int B, int hist_len, int ncu, long long* out) {
  const char* e = std::getenv("HFENS_SG_WGS_PER_CU");   // read per call: tests sweep it
  const int wgs_per_cu = e ? std::min(4, std::max(1, std::atoi(e))) : 1;
  const long long tiles = (n + kSgTile - 1) / kSgTile;
  const long long want = std::max(1LL, (long long)wgs_per_cu * ncu / B);   // workgroups per model
  const long long per = (tiles + want - 1) / want;                          // sub-tiles per workgroup
  const long long rows = per * kSgTile;
  const long long groups = (n + rows - 1) / rows;
  const long long slot_m = 3LL * hist_len + kSgExtra;
  out[0] = rows;
  out[1] = groups;
  // every workgroup adds its histogram straight into the slot with int64 atomics (integer sums:
  // the same bits in any order); HFENS_SG_ATOMIC_GROUPS = g publishes partial slots for
  // gbdt_stage_reduce_kernel above g workgroups per model instead.  Measured (gbdt_shard_probe,
  // profiles/r3_gbdt_dp.md): atomics at 123 / 245 workgroups were 2–4 % faster per stage than
  // partials + the reduce launch (43.5 vs 45.5 µs at 125k rows, 87.7 vs 89.2 µs at 1M).
  const char* ae = std::getenv("HFENS_SG_ATOMIC_GROUPS");   // read per call: tests and probes sweep it
  const long long amax = ae ? std::max(1, std::atoi(ae)) : (1LL << 40);
  out[2] = groups > amax ? 1 : 0;
  out[3] = out[2] ? (long long)B * groups * slot_m : 0;
}

void gbdt_stage_plan(long long n, int B, int hist_len, int ncu, uintptr_t out) {
  sg_plan(n, B, hist_len, ncu, reinterpret_cast<long long*>(out));
}

void gbdt_stump_stage(int t, int B, int n, int F, int T, uintptr_t bins, long long ldb, uintptr_t nbins, int hist_len,
                      uintptr_t lo_val, uintptr_t hi_val, uintptr_t y, uintptr_t w, uintptr_t raw, uintptr_t wt,
                      uintptr_t seeds, long long row_off, double subsample, uintptr_t comm, uintptr_t feat,
                      uintptr_t blo, uintptr_t thr, uintptr_t value, uintptr_t stats, uintptr_t r2, uintptr_t dev,
                      uintptr_t bagw, uintptr_t frank, uintptr_t partials, long long partials_len, double lr,
                      double qscale, double dscale, double min_leaf_q, double min_split_q, uintptr_t prof,
                      uintptr_t t_dev, int tick_in_reduce, int persist, uintptr_t bar, uintptr_t err,
                      uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F <= kStMaxF, "gbdt_stump_stage: 1 <= F <= 128");
  HFENS_REQUIRE(B >= 1 && B <= 65535 && n >= 1 && T >= 1 && t >= 0 && t <= T + 1, "gbdt_stump_stage: bad shape");
  const bool active = subsample < 1.0;
  HFENS_REQUIRE(!active || (wt != 0 && seeds != 0 && bagw != 0), "gbdt_stump_stage: subsample needs wt, seeds, bagw");
  // MF: binary / ≤ 8-bin features on the i8 matrix cores (HFENS_GBDT_MFMA=0: int64 VALU sums)
  const char* mfe = std::getenv("HFENS_GBDT_MFMA");   // read per launch: tests toggle it
  const bool mf_env = !(mfe && mfe[0] == '0');
  const char* nte = std::getenv("HFENS_SG_THREADS");   // MFMA path: 512 or 1024 threads per workgroup
  const int nt = nte && std::atoi(nte) == 1024 ? 1024 : kSgThreads;
  bool mf = mf_env && gbdt_stump_stage_lds(hist_len, true) <= 150 * 1024;
  HFENS_REQUIRE(hist_len >= F && gbdt_stump_stage_lds(hist_len, false) <= 150 * 1024,
                "gbdt_stump_stage: histogram + row cache exceed LDS");
  StageJob J{(const unsigned char*)bins, (const int*)nbins, (const double*)lo_val, (const double*)hi_val,
             (const float*)y, (const float*)w, (double*)raw, (float*)wt, (const unsigned long long*)seeds,
             (long long*)comm, (int*)feat, (int*)blo, (double*)thr, (double*)value, (long long*)stats,
             (long long*)r2, (long long*)dev, (double*)bagw, (const int*)frank, row_off, lr, qscale, dscale,
             min_leaf_q, min_split_q, (unsigned)llround(subsample * 16777216.0), active ? 1 : 0, B, n, F, T,
             hist_len, t, 0, ldb, (long long*)partials, (long long*)prof, (const int*)t_dev, (unsigned*)bar,
             (unsigned*)err, 200000000LL};
  if (const char* dl = std::getenv("HFENS_GBDT_PERSIST_DEADLINE_MS")) J.deadline = std::atoll(dl) * 100000LL;
  // t_dev (graph replay): the kernel takes the stage index from device memory; the host t still
  // selects the comm slot of the reduce launch, so a captured unit must start at t ≡ 0 (mod 3)
  HFENS_REQUIRE(ldb >= n && ldb % kSgTile == 0 && (bins & 15) == 0, "gbdt_stump_stage: bins must be [F][ldb], ldb % 1024 == 0, 16-byte aligned");
  int dev_id = 0, ncu = 256;
  HFENS_CHECK(hipGetDevice(&dev_id));
  HFENS_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev_id));
  long long plan[4];
  sg_plan(n, B, hist_len, ncu, plan);
  J.rows_per_wg = (int)plan[0];
  const int groups = (int)plan[1];
  // exact int32 slice sums: |slice| ≤ 127 per row
  if ((long long)J.rows_per_wg * 127 >= (1LL << 31)) mf = false;
  const size_t lds = gbdt_stump_stage_lds(hist_len, mf);
  const long long slot_m = 3LL * hist_len + kSgExtra;
  if (plan[2] == 0 || partials == 0) J.partials = nullptr;
  else HFENS_REQUIRE(partials_len >= plan[3], "gbdt_stump_stage: partials buffer too small (size it with gbdt_stage_plan)");
  if (persist) {
    // the whole boosting run in one launch (t = 0 … T+1); int64 slot atomics only (no partial
    // reduce launch), no stamps, no device stage counter; at most one workgroup per CU
    HFENS_REQUIRE(bar != 0 && err != 0 && t_dev == 0 && prof == 0 && t == 0,
                  "gbdt_stump_stage: persist needs bar/err, t = 0, no t_dev/prof");
    HFENS_REQUIRE((long long)groups * B <= ncu, "gbdt_stump_stage: persist grid exceeds one workgroup per CU");
    J.partials = nullptr;
    if (mf) hipLaunchKernelGGL((gbdt_stump_stage_kernel<true, kSgThreads, true>), dim3(groups, B), dim3(kSgThreads), lds, as_stream(stream), J);
    else hipLaunchKernelGGL((gbdt_stump_stage_kernel<false, kSgThreads, true>), dim3(groups, B), dim3(kSgThreads), lds, as_stream(stream), J);
    launch_check();
    return;
  }
  if (mf && nt == 1024) hipLaunchKernelGGL((gbdt_stump_stage_kernel<true, 1024>), dim3(groups, B), dim3(1024), lds, as_stream(stream), J);
  else if (mf) hipLaunchKernelGGL((gbdt_stump_stage_kernel<true, kSgThreads>), dim3(groups, B), dim3(kSgThreads), lds, as_stream(stream), J);
  else hipLaunchKernelGGL((gbdt_stump_stage_kernel<false, kSgThreads>), dim3(groups, B), dim3(kSgThreads), lds, as_stream(stream), J);
  launch_check();
  // tick_in_reduce (graph replay with a partial reduce): the caller skips gbdt_stage_tick, so the
  // reduce launch must exist — the caller derives that from gbdt_stage_plan (uses_partials) and t ≤ T
  HFENS_REQUIRE(!tick_in_reduce || (t_dev != 0 && J.partials != nullptr && t <= T),
                "gbdt_stump_stage: tick_in_reduce needs t_dev and a partial-reduce launch");
  if (J.partials != nullptr && t <= T) {
    long long* slot = (long long*)comm + (size_t)(t % 3) * B * slot_m;
    hipLaunchKernelGGL(gbdt_stage_reduce_kernel, dim3((unsigned)((slot_m + 255) / 256), kRdSplit, B), dim3(256), 0,
                       as_stream(stream), (const long long*)J.partials, slot, groups, slot_m,
                       tick_in_reduce ? (int*)t_dev : nullptr);
    launch_check();
  }
}

// Advance the device stage counter read by graph-replayed gbdt_stump_stage launches.
__global__ void gbdt_stage_tick_kernel(int* t) {
  if (threadIdx.x == 0) t[0] = t[0] + 1;
}

void gbdt_stage_tick(uintptr_t t_dev, uintptr_t stream) {
  hipLaunchKernelGGL(gbdt_stage_tick_kernel, dim3(1), dim3(64), 0, as_stream(stream), (int*)t_dev);
  launch_check();
}

}  // namespace hfens
