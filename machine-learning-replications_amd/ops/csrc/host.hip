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

}  // namespace hfens
