// Host-side runtime helpers compiled into the extension (no device code).
//
//  libsvm_perm : the Platt-CV shuffle of libsvm's svm_binary_svc_probability as built by
//                scikit-learn (std::mt19937 seeded with sklearn's random_seed, "tweaked Lemire"
//                bounded draws from sklearn/svm/src/newrand/newrand.h), so the 5 internal folds
//                match the reference fit exactly.  Native because it is an l-step sequential
//                Fisher-Yates loop executed for every SVC fit.
// Licence: the libsvm RNG draws and the splitter's rand_r order follow scikit-learn / LIBSVM
// (BSD-3-Clause; notices in THIRD_PARTY_NOTICES.md at the repository root).
#include <algorithm>
#include <cstdint>
#include <random>
#include <vector>

namespace hfens {

static inline uint32_t bounded_rand_int(std::mt19937& mt, uint32_t range) {
  uint32_t x = mt();
  uint64_t m = uint64_t(x) * uint64_t(range);
  uint32_t l = uint32_t(m);
  if (l < range) {
    uint32_t t = -range;
    if (t >= range) {
      t -= range;
      if (t >= range) t %= range;
    }
    while (l < t) {
      x = mt();
      m = uint64_t(x) * uint64_t(range);
      l = uint32_t(m);
    }
  }
  return uint32_t(m >> 32);
}

void libsvm_perm(int l, long long seed, uintptr_t out_ptr) {
  int64_t* perm = reinterpret_cast<int64_t*>(out_ptr);
  std::mt19937 mt(static_cast<uint32_t>(seed));
  for (int i = 0; i < l; ++i) perm[i] = i;
  for (int i = 0; i < l; ++i) {
    const int j = i + static_cast<int>(bounded_rand_int(mt, static_cast<uint32_t>(l - i)));
    const int64_t tmp = perm[i];
    perm[i] = perm[j];
    perm[j] = tmp;
  }
}

// sklearn_stump_ranks : the order in which scikit-learn's BestSplitter visits the features at the
//                root of each tree (sklearn/tree/_splitter.pyx node_split_best: Fisher-Yates draws
//                with rand_int(low, high) = low + our_rand_r(state) % (high − low), xorshift32
//                our_rand_r from sklearn/utils/_random.pxd, constant features moved aside and not
//                evaluated).  seeds[t] = the tree's rand_r_state (RandomState.randint(0, 2^31−1)
//                drawn by Splitter.init, one per tree from the GBC's shared RandomState).  The split
//                kernels break EXACT gain ties by this rank, as sklearn keeps the first strictly
//                better feature it visits.  ranks[t][f] = visit position, F for constant features.
static inline uint32_t sk_rand_r(uint32_t* s) {
  if (*s == 0) *s = 1;
  *s ^= *s << 13;
  *s ^= *s >> 17;
  *s ^= *s << 5;
  return *s % (uint32_t(2147483647) + 1u);
}

void sklearn_stump_ranks(int T, int F, uintptr_t seeds_ptr, uintptr_t constant_ptr, uintptr_t ranks_ptr) {
  const int64_t* seeds = reinterpret_cast<const int64_t*>(seeds_ptr);
  const uint8_t* constant = reinterpret_cast<const uint8_t*>(constant_ptr);
  int32_t* ranks = reinterpret_cast<int32_t*>(ranks_ptr);
  int feats[256];
  for (int t = 0; t < T; ++t) {
    uint32_t st = static_cast<uint32_t>(seeds[t]);
    int32_t* rk = ranks + (size_t)t * F;
    for (int f = 0; f < F; ++f) { feats[f] = f; rk[f] = F; }
    int f_i = F, n_found = 0, n_total = 0, visited = 0, pos = 0;
    // max_features = F and no constants known at the root (n_known = n_drawn = 0)
    while (f_i > n_total && (visited < F || visited <= n_found)) {
      ++visited;
      int f_j = static_cast<int>(sk_rand_r(&st) % static_cast<uint32_t>(f_i - n_found));
      f_j += n_found;
      const int cur = feats[f_j];
      if (constant[cur]) {
        feats[f_j] = feats[n_total];
        feats[n_total] = cur;
        ++n_found;
        ++n_total;
        continue;
      }
      --f_i;
      feats[f_j] = feats[f_i];
      feats[f_i] = cur;
      rk[cur] = pos++;
    }
  }
}

// stack_predict_host : the HF stack (StandardScaler → RBF-SVC + Platt + libsvm iterative coupling,
//                      GBC tree walk, L1-LR, meta-LR) in f64 for a few rows on the host — the
//                      single-patient path of predict_hf.py (BASELINE config 1: 85 µs p50 with
//                      numpy).  Same arithmetic as ops/reference.py (decision rule float32(x) ≤
//                      threshold, trees added in order, coupling eps 0.005/k), no tensor dispatch.
#include <cmath>
static inline double hf_sigmoid(double v) { return 1.0 / (1.0 + std::exp(-v)); }

static double hf_couple2(double r01) {
  const double r10 = 1.0 - r01, q00 = r10 * r10, q11 = r01 * r01, q01 = -r10 * r01;
  double p0 = 0.5, p1 = 0.5;
  const double eps = 0.005 / 2;
  for (int it = 0; it < 100; ++it) {
    const double qp0 = q00 * p0 + q01 * p1, qp1 = q01 * p0 + q11 * p1;
    const double pqp = p0 * qp0 + p1 * qp1;
    const double err = std::fmax(std::fabs(qp0 - pqp), std::fabs(qp1 - pqp));
    if (err < eps) break;
    double d = (-qp0 + pqp) / q00;
    double np0 = p0 + d;
    const double npqp = (pqp + d * (d * q00 + 2 * qp0)) / (1 + d) / (1 + d);
    const double nqp1 = (qp1 + d * q01) / (1 + d);
    np0 = np0 / (1 + d);
    double np1 = p1 / (1 + d);
    d = (-nqp1 + npqp) / q11;
    np1 = np1 + d;
    np0 = np0 / (1 + d);
    np1 = np1 / (1 + d);
    p0 = np0;
    p1 = np1;
  }
  return p1;
}

void stack_predict_host(int n, int F, uintptr_t X_, uintptr_t mean_, uintptr_t scale_, int nsv, uintptr_t sv_,
                        uintptr_t coef_, double gamma, double svc_icpt, double probA, double probB, int T, int K,
                        uintptr_t feat_, uintptr_t thr_, uintptr_t left_, uintptr_t right_, uintptr_t value_,
                        double gbc_init, double lr, uintptr_t lrc_, double lr_icpt, uintptr_t meta_,
                        double meta_icpt, uintptr_t out_) {
  const double* X = reinterpret_cast<const double*>(X_);
  const double* mean = reinterpret_cast<const double*>(mean_);
  const double* scale = reinterpret_cast<const double*>(scale_);
  const double* sv = reinterpret_cast<const double*>(sv_);
  const double* coef = reinterpret_cast<const double*>(coef_);
  const int64_t* feat = reinterpret_cast<const int64_t*>(feat_);
  const double* thr = reinterpret_cast<const double*>(thr_);
  const int64_t* left = reinterpret_cast<const int64_t*>(left_);
  const int64_t* right = reinterpret_cast<const int64_t*>(right_);
  const double* value = reinterpret_cast<const double*>(value_);
  const double* lrc = reinterpret_cast<const double*>(lrc_);
  const double* meta = reinterpret_cast<const double*>(meta_);
  double* out = reinterpret_cast<double*>(out_);
  double z[256];
  for (int r = 0; r < n; ++r) {
    const double* x = X + (size_t)r * F;
    for (int f = 0; f < F; ++f) z[f] = (x[f] - mean[f]) / scale[f];
    double dec = 0.0;
    for (int j = 0; j < nsv; ++j) {
      const double* s = sv + (size_t)j * F;
      double d2 = 0.0;
      for (int f = 0; f < F; ++f) {
        const double t = z[f] - s[f];
        d2 += t * t;
      }
      dec += std::exp(-gamma * d2) * coef[j];
    }
    dec += svc_icpt;
    const double fApB = dec * probA + probB;
    double r01 = fApB >= 0 ? std::exp(-fApB) / (1.0 + std::exp(-fApB)) : 1.0 / (1.0 + std::exp(fApB));
    r01 = std::fmin(std::fmax(r01, 1e-7), 1 - 1e-7);
    const double p_svc = hf_couple2(r01);
    double raw = gbc_init;
    for (int t = 0; t < T; ++t) {
      int64_t nd = 0;
      const int64_t* ft = feat + (size_t)t * K;
      while (ft[nd] >= 0) {
        const double xv = (double)(float)x[ft[nd]];
        nd = xv <= thr[(size_t)t * K + nd] ? left[(size_t)t * K + nd] : right[(size_t)t * K + nd];
      }
      raw += lr * value[(size_t)t * K + nd];
    }
    const double p_gbc = hf_sigmoid(raw);
    double dl = 0.0;
    for (int f = 0; f < F; ++f) dl += x[f] * lrc[f];
    const double p_lr = hf_sigmoid(dl + lr_icpt);
    out[r] = hf_sigmoid(p_svc * meta[0] + p_gbc * meta[1] + p_lr * meta[2] + meta_icpt);
  }
}

// KNN imputation work lists from the rows' missing-column bitmasks (models/imputer.py
// _impute_device; the numpy version cost ≈ 1 ms of host time at 10k rows before the donor search
// could launch).  bits [n] u64 (bit f = column f missing); out: int64 buffer of capacity `cap`
// filled as [rows (nr) | bits of those rows (nr) | slot columns (nr × nslot, −1 padded) | flat slot
// index of every missing cell (nc) | its row (nc) | its column (nc)], cells row-major with columns
// ascending (the numpy order); dims[0..3] = nr, nc, nslot (nslot = max missing per row rounded up
// to `slots`), status (0 = written; −1 = `cap` below 2·nr + nr·nslot + 3·nc: nothing written — a
// call with cap = 0 sizes the buffer).
void knn_plan_host(uintptr_t bits_, long long n, int F, int slots, uintptr_t out_, long long cap, uintptr_t dims_) {
  const uint64_t* bits = reinterpret_cast<const uint64_t*>(bits_);
  long long* out = reinterpret_cast<long long*>(out_);
  long long* dims = reinterpret_cast<long long*>(dims_);
  const uint64_t fmask = F >= 64 ? ~0ull : ((1ull << F) - 1ull);
  long long nr = 0, nc = 0;
  int mx = 0;
  for (long long i = 0; i < n; ++i) {
    const uint64_t b = bits[i] & fmask;
    if (!b) continue;
    ++nr;
    const int c = __builtin_popcountll(b);
    nc += c;
    mx = c > mx ? c : mx;
  }
  const int nslot = nr ? (mx + slots - 1) / slots * slots : 0;
  dims[0] = nr;
  dims[1] = nc;
  dims[2] = nslot;
  dims[3] = 0;
  if (2 * nr + nr * nslot + 3 * nc > cap) {
    dims[3] = -1;
    return;
  }
  long long* rows = out;
  long long* rb = rows + nr;
  long long* slot = rb + nr;
  long long* flat = slot + nr * nslot;
  long long* ri = flat + nc;
  long long* ci = ri + nc;
  long long k = 0, e = 0;
  for (long long i = 0; i < n; ++i) {
    uint64_t b = bits[i] & fmask;
    if (!b) continue;
    rows[k] = i;
    rb[k] = (long long)b;
    int s = 0;
    while (b) {
      const int f = __builtin_ctzll(b);
      b &= b - 1ull;
      slot[k * nslot + s] = f;
      flat[e] = k * nslot + s;
      ri[e] = i;
      ci[e] = f;
      ++s;
      ++e;
    }
    for (; s < nslot; ++s) slot[k * nslot + s] = -1;
    ++k;
  }
}


// svc_expand_host: the label-only libsvm problem expansion of one probability SVC fit
// (models/smo.py _expand): class-grouped positions (class 0 first), the Platt-CV permutation
// (libsvm_perm above), and for each of the 5 internal folds the training rows in permutation order,
// class 1 first — every array the 36-problem batch is built from, in ONE host call instead of ~20
// numpy calls per fold (the stacking plan sits on the headline's host critical path).
//   y[n] (0/1) → out (int64): grouped[n] | perm[n] | gp[n] = grouped[perm] | rows of folds 0..4
//   (concatenated, ≤ 4n) ; meta (int64): n0, then per fold (n1, nn0, rows offset, rows length).
//   seed < 0: no Platt folds (only grouped).
void svc_expand_host(uintptr_t y_ptr, long long n, long long seed, uintptr_t out_ptr, uintptr_t meta_ptr) {
  const double* y = reinterpret_cast<const double*>(y_ptr);
  int64_t* out = reinterpret_cast<int64_t*>(out_ptr);
  int64_t* meta = reinterpret_cast<int64_t*>(meta_ptr);
  int64_t* grouped = out;
  int64_t n0 = 0;
  for (long long i = 0; i < n; ++i)
    if (!(y[i] > 0.5)) grouped[n0++] = i;
  int64_t w = n0;
  for (long long i = 0; i < n; ++i)
    if (y[i] > 0.5) grouped[w++] = i;
  meta[0] = n0;
  if (seed < 0) return;
  const long long l = n;
  int64_t* perm = out + l;
  int64_t* gp = out + 2 * l;
  int64_t* rows = out + 3 * l;
  libsvm_perm(static_cast<int>(l), seed, reinterpret_cast<uintptr_t>(perm));
  for (long long i = 0; i < l; ++i) gp[i] = grouped[perm[i]];
  // class-1 / class-0 permutation positions and their rows (each in position order), then every
  // fold's training rows are two contiguous copies per class around the fold's position range
  std::vector<int64_t> i1, i0, g1, g0;
  i1.reserve(l - n0);
  i0.reserve(n0);
  for (long long p = 0; p < l; ++p) (perm[p] >= n0 ? i1 : i0).push_back(p);
  g1.resize(i1.size());
  g0.resize(i0.size());
  for (size_t j = 0; j < i1.size(); ++j) g1[j] = gp[i1[j]];
  for (size_t j = 0; j < i0.size(); ++j) g0[j] = gp[i0[j]];
  int64_t off = 0;
  for (int k = 0; k < 5; ++k) {
    const long long b = k * l / 5, e = (k + 1) * l / 5;
    const int64_t lo1 = std::lower_bound(i1.begin(), i1.end(), (int64_t)b) - i1.begin();
    const int64_t hi1 = std::lower_bound(i1.begin(), i1.end(), (int64_t)e) - i1.begin();
    const int64_t lo0 = std::lower_bound(i0.begin(), i0.end(), (int64_t)b) - i0.begin();
    const int64_t hi0 = std::lower_bound(i0.begin(), i0.end(), (int64_t)e) - i0.begin();
    const int64_t n1 = lo1 + (int64_t)i1.size() - hi1, nn0 = lo0 + (int64_t)i0.size() - hi0;
    meta[1 + 4 * k] = n1;
    meta[2 + 4 * k] = nn0;
    meta[3 + 4 * k] = off;
    if (n1 == 0 || nn0 == 0) {
      meta[4 + 4 * k] = 0;
      continue;
    }
    int64_t* r = rows + off;
    r = std::copy(g1.begin(), g1.begin() + lo1, r);
    r = std::copy(g1.begin() + hi1, g1.end(), r);
    r = std::copy(g0.begin(), g0.begin() + lo0, r);
    r = std::copy(g0.begin() + hi0, g0.end(), r);
    meta[4 + 4 * k] = n1 + nn0;
    off += n1 + nn0;
  }
}

// stack_plan_host: the label-only stacking plan of pipeline.develop in ONE native call, so it can run
// on a helper thread with the GIL released while the main thread launches the imputation and the
// LassoCV prelude: StratifiedKFold(n_folds) test folds of two-class labels (sklearn's assignment:
// the class seen first is class 0, each class's members dealt to folds in row order by the counts of
// the sorted encoded labels), then every fit's (the n_folds fold fits and the refit) libsvm problem
// expansion (svc_expand_host).
//   y[n] ∈ {0, 1} (checked by the caller) → folds[n]; per fit f: out[f·7n …] and meta[f·21 …] as
//   svc_expand_host writes them for that fit's labels (fit f < n_folds: rows with fold ≠ f; the
//   refit: all rows, in row order).  rows_out[(n_folds + 1)·n]: every fit's row list; lens[n_folds+1].
void stack_plan_host(uintptr_t y_ptr, long long n, int n_folds, long long seed, uintptr_t folds_ptr,
                     uintptr_t rows_ptr, uintptr_t lens_ptr, uintptr_t out_ptr, uintptr_t meta_ptr) {
  const double* y = reinterpret_cast<const double*>(y_ptr);
  int64_t* folds = reinterpret_cast<int64_t*>(folds_ptr);
  int64_t* rows = reinterpret_cast<int64_t*>(rows_ptr);
  int64_t* lens = reinterpret_cast<int64_t*>(lens_ptr);
  const double first = y[0];
  int64_t c0 = 0;
  for (long long i = 0; i < n; ++i) c0 += (y[i] == first);
  const int64_t k = n_folds;
  std::vector<int64_t> next0(k), next1(k);
  // fold i takes the positions ≡ i (mod k) of the sorted encoded labels: class 0 holds [0, c0)
  for (int64_t i = 0; i < k; ++i) {
    const int64_t tot = (n - i + k - 1) / k;
    const int64_t a0 = c0 > i ? (c0 - i + k - 1) / k : 0;
    next0[i] = a0;
    next1[i] = tot - a0;
  }
  int64_t f0 = 0, f1 = 0;
  for (long long i = 0; i < n; ++i) {
    if (y[i] == first) {
      while (f0 < k && next0[f0] == 0) ++f0;
      folds[i] = f0;
      --next0[f0];
    } else {
      while (f1 < k && next1[f1] == 0) ++f1;
      folds[i] = f1;
      --next1[f1];
    }
  }
  std::vector<double> yf(n);
  for (int64_t f = 0; f <= k; ++f) {
    int64_t* r = rows + f * n;
    int64_t m = 0;
    for (long long i = 0; i < n; ++i)
      if (f == k || folds[i] != f) { r[m] = i; yf[m] = y[i]; ++m; }
    lens[f] = m;
    svc_expand_host(reinterpret_cast<uintptr_t>(yf.data()), m, seed,
                    out_ptr + sizeof(int64_t) * (size_t)(f * 7 * n), meta_ptr + sizeof(int64_t) * (size_t)(f * 21));
  }
}

}  // namespace hfens
