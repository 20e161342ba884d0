// Host-code self-test, built with AddressSanitizer + UBSan: exercises the
// native host helpers of the extension (host.hip) outside Python, where ASan can run without
// preloading into the interpreter.  Expected values come from the pure-Python libsvm RNG mirror
// (hfens.models.smo.libsvm_perm_py), which matches sklearn's libsvm Platt-CV shuffle.
#include <cstdint>
#include <cstdio>
#include <vector>

namespace hfens {
void libsvm_perm(int l, long long seed, uintptr_t out_ptr);
}

struct Case {
  int l;
  long long seed;
  long long first[8];
  long long checksum;   // Σ (i+1)·perm[i] mod 1000003
};

int main() {
  const Case cases[] = {
      {10, 1, {4, 9, 7, 1, 0, 5, 2, 3}, 247},
      {713, 1608637542, {324, 106, 594, 455, 52, 66, 231, 183}, 59855},
      {1000, 2020, {986, 149, 873, 622, 511, 223, 276, 960}, 582710},
  };
  int bad = 0;
  for (const Case& c : cases) {
    std::vector<int64_t> p(c.l, -1);
    hfens::libsvm_perm(c.l, c.seed, reinterpret_cast<uintptr_t>(p.data()));
    std::vector<int> seen(c.l, 0);
    long long cs = 0;
    for (int i = 0; i < c.l; ++i) {
      if (p[i] < 0 || p[i] >= c.l || seen[p[i]]++) { std::printf("l=%d: not a permutation\n", c.l); ++bad; break; }
      cs = (cs + (long long)(i + 1) * p[i]) % 1000003;
    }
    for (int i = 0; i < 8; ++i)
      if (p[i] != c.first[i]) { std::printf("l=%d: perm[%d]=%lld expected %lld\n", c.l, i, (long long)p[i], c.first[i]); ++bad; }
    if (cs != c.checksum) { std::printf("l=%d: checksum %lld expected %lld\n", c.l, cs, c.checksum); ++bad; }
  }
  std::printf(bad ? "host_selftest: FAILED\n" : "host_selftest: ok\n");
  return bad ? 1 : 0;
}
