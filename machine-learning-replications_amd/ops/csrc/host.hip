// Host-side runtime helpers compiled into the extension (no device code).
//
//  libsvm_perm : the Platt-CV shuffle of libsvm's svm_binary_svc_probability as built by
//                scikit-learn (std::mt19937 seeded with sklearn's random_seed, "tweaked Lemire"
//                bounded draws from sklearn/svm/src/newrand/newrand.h), so the 5 internal folds
//                match the reference fit exactly.  Native because it is an l-step sequential
//                Fisher-Yates loop executed for every SVC fit.
#include <cstdint>
#include <random>

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

}  // namespace hfens
