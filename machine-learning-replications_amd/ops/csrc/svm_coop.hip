// Cooperative exact SMO: one libsvm C-SVC problem spread over W workgroups.
//
// The single-workgroup solver (svm.hip smo_kernel) is VALU-bound on ONE CU: every pair (i, j)
// costs ~50 f64/bitmask instructions per point in the two WSS passes and the gradient update,
// so at l = 8-10k points one CU spends most of its ~10 µs per pair issuing them.  Here each
// problem's points are cut into W contiguous slices, one per workgroup ("member"), and the two
// block arg-reductions of every iteration become two in-launch exchanges between the members:
// every member publishes its partial (arg-max key, index and the owner's payload: α_i; α_j,
// G_j, K_ij) as data-tagged 8-byte granules {epoch, value} written by agent-scope relaxed
// atomic stores (write-through: no fence, no flag), and one wave per member sweeps all W
// partials until every tag equals the exchange's epoch.  Every member then folds the same W
// partials in the same order and performs the same pair update, so all members agree on
// (i, j, α_i, α_j) with no further communication; each member updates only its own slice of G
// with its own slices of Gram rows i and j (1/W of each row read).
//
// Exactness: the reductions are exact max / arg-max (ties → larger index) — independent of
// how the points are partitioned — and the per-point arithmetic is smo_kernel's (libsvm order,
// no FMA contraction), so the pair sequence, α and ρ match smo_kernel's.
//
// Liveness: every spin is bounded; a member that times out sets *err and leaves, its peers
// then time out too and the launch drains (the host raises on err).  The launcher admits at
// most one member per CU, so every member is resident at once; the members of one problem are
// placed on one XCD (blocks b and b+8 share an XCD under round-robin dispatch — speed only,
// never correctness).
#include <cstdlib>

#include "common.h"

namespace hfens {

typedef __attribute__((address_space(1))) unsigned long long gu64_t;

struct SmoCoopProb {
  long long koff;   // K_p offset (floats)
  long long aoff;   // alpha offset (doubles)
  long long moff;   // Mapped: offset of this problem's column map in `maps` (see smo_coop_kernel)
  int l;            // problem size
  int ld;           // K_p leading dimension
  int npos;         // indices [0, npos) have y = +1, the rest y = −1
  int S;            // points per member (multiple of 4): member w owns columns [w·S, min(lphys, (w+1)·S))
  int lphys;        // columns of K_p's rows (= l unless Mapped)
  int pad;
  double Cp, Cn;
};

struct SmoCoopOut {
  double* rho;      // [P]
  int* iters;       // [P]
  double* gap;      // [P]
  unsigned* err;    // [1] set on a spin timeout
  long long* prof;  // [P][7] s_memtime phase totals of member 0 (nullptr = off): step2, red2,
                    // xchg2, pair, update, red1, xchg1
  int prefetch;     // 1: pull the member's candidate Gram row into L2 while the exchange runs
  int pad_;
  long long wait_ticks;    // one exchange waits at most this long (100 MHz real-time counter), then
                           // flags err: a member that is not resident costs a bounded delay, and the
                           // host re-solves with the one-workgroup kernel (models/smo.py)
  long long inject_ticks;  // test hook: member 1 of problem 0 starts this late (0 = off)
};

constexpr int kCoopThreads = 512;
constexpr int kCoopWaves = kCoopThreads / 64;
constexpr int kGran = 10;             // granules per member slot
constexpr int kPkBits = 15;           // Mapped: point key = libsvm index << 15 | column
constexpr int kPkMask = (1 << kPkBits) - 1;
constexpr int kMaxMembers = 16;
constexpr double kCTau = 1e-12;
constexpr double kCInf = 1.0e300;
constexpr long long kWaitMsDefault = 20;   // HFENS_SMO_WAIT_MS: per-exchange deadline

// 100 MHz constant-rate counter (independent of the shader clock)
__device__ __forceinline__ long long rt_now() { return (long long)__builtin_amdgcn_s_memrealtime(); }

// the test hook of SmoCoopOut::inject_ticks: one member arrives late (never in production runs)
__device__ __forceinline__ void coop_inject_delay(long long ticks, int p, int w) {
  if (ticks <= 0 || p != 0 || w != 1) return;
  const long long until = rt_now() + ticks;
  while (rt_now() < until) __builtin_amdgcn_s_sleep(127);
}

__device__ __forceinline__ void put_granule(unsigned long long* g, unsigned epoch, unsigned v) {
  __hip_atomic_store((gu64_t*)g, ((unsigned long long)epoch << 32) | v, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void put_u64(unsigned long long* g, unsigned epoch, unsigned long long x) {
  put_granule(g, epoch, (unsigned)x);
  put_granule(g + 1, epoch, (unsigned)(x >> 32));
}
__device__ __forceinline__ unsigned long long u64_of(const unsigned* v) {
  return (unsigned long long)v[0] | ((unsigned long long)v[1] << 32);
}
__device__ __forceinline__ double f64_of(const unsigned* v) {
  return __longlong_as_double((long long)u64_of(v));
}
__device__ __forceinline__ unsigned long long bits_of(double x) {
  return (unsigned long long)__double_as_longlong(x);
}

struct CoopPart {
  unsigned long long ka, kb;
  int idx, pad;
};

// Member-local exact reduction (a → max; (b, idx) → arg-max, ties → larger idx): DPP/permlane
// wave maxima, one barrier, fold of the wave partials.  Every thread receives the result.
// WantA = false: the caller passes a uniform `a` and ignores the max (WSS step 1), so its two
// wave-max chains are skipped (the result's ka is then f64_okey(a)).
template <bool WantA = true>
__device__ __forceinline__ CoopPart coop_block_red(double a, double b, int idx, CoopPart* sh) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned long long ka = f64_okey(a), kb = f64_okey(b);
  unsigned ah = (unsigned)(ka >> 32), al = (unsigned)ka;
  if constexpr (WantA) {
    ah = wave_max_u32((unsigned)(ka >> 32));
    al = wave_max_u32((unsigned)(ka >> 32) == ah ? (unsigned)ka : 0u);
  }
  const unsigned bh = wave_max_u32((unsigned)(kb >> 32));
  const unsigned bl = wave_max_u32((unsigned)(kb >> 32) == bh ? (unsigned)kb : 0u);
  const bool top = (unsigned)(kb >> 32) == bh && (unsigned)kb == bl;
  const unsigned bi = wave_max_u32(top ? (unsigned)(idx + 1) : 0u);
  if (lane == 0)
    sh[wave] = CoopPart{((unsigned long long)ah << 32) | al, ((unsigned long long)bh << 32) | bl, (int)bi - 1, 0};
  __syncthreads();
  CoopPart r = sh[0];
#pragma unroll
  for (int w = 1; w < kCoopWaves; ++w) {
    const CoopPart p = sh[w];
    r.ka = p.ka > r.ka ? p.ka : r.ka;
    if (p.kb > r.kb || (p.kb == r.kb && p.idx > r.idx)) { r.kb = p.kb; r.idx = p.idx; }
  }
  return r;
}

// Wave 0 sweeps the first `ng` granules of every member's slot (GS granules per slot) until all
// of them carry `epoch` and leaves the values in vals[member][granule] (LDS); one barrier.
// false = timed out.
template <int GS>
__device__ __forceinline__ bool coop_gather_t(unsigned long long* slot, int W, int ng, unsigned epoch,
                                              unsigned (*vals)[GS], const SmoCoopOut& out, int* sh_fail) {
  constexpr int R = (kMaxMembers * GS + 63) / 64;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const int tot = W * ng;
    unsigned v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = 0u;
    const long long deadline = rt_now() + out.wait_ticks;
    unsigned spins = 0;
    bool fail = false;
    for (;;) {
      bool ok = true;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int gi = lane + 64 * r;
        if (gi < tot) {
          const int m = gi / ng, k = gi - m * ng;
          const unsigned long long x =
              __hip_atomic_load((gu64_t*)(slot + m * GS + k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          v[r] = (unsigned)x;
          ok = ok && (unsigned)(x >> 32) == epoch;
        }
      }
      if (__all(ok)) break;
      // the real-time counter is read every 64th poll only (a scalar memory read of its own)
      // every 64th poll: the deadline (real-time counter) and the error flag — once any member
      // of the launch has given up, the others leave at their next check instead of waiting out
      // their own deadlines
      if ((++spins & 63u) == 0 &&
          (rt_now() > deadline || __hip_atomic_load(out.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)) {
        fail = true;
        if (lane == 0) atomicOr(out.err, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int gi = lane + 64 * r;
      if (gi < tot) {
        const int m = gi / ng, k = gi - m * ng;
        vals[m][k] = v[r];
      }
    }
    if (lane == 0) *sh_fail = fail ? 1 : 0;
  }
  __syncthreads();
  return *sh_fail == 0;
}

__device__ __forceinline__ bool coop_gather(unsigned long long* slot, int W, int ng, unsigned epoch,
                                            unsigned (*vals)[kGran], const SmoCoopOut& out, int* sh_fail) {
  return coop_gather_t<kGran>(slot, W, ng, epoch, vals, out, sh_fail);
}

// Point ownership inside member w: thread tid, group g < K4, lane-of-vector e < 4 owns column
// c = w·S + 4·(tid + g·kCoopThreads) + e  (valid while c < min(lphys, (w+1)·S)).
//
// Mapped = false: column c of the stored Gram K_p is point c of the problem.
// Mapped = true: the problem is a Platt-CV sub-problem whose Gram is a principal submatrix of its
// parent's (the fit's final problem: same scaled rows, same γ, so the same f32 entries) — no Gram
// of its own is computed or stored.  K_p is the parent's; maps[moff + c] is the sub-problem's
// (libsvm-order) index of parent column c, or −1 when that row is in the held-out fold.  Members
// own contiguous PARENT columns, so row slices stay one float4 load; every point carries the key
// pk = index << 15 | column through the reductions and exchanges: comparing keys compares libsvm
// indices (ties → larger index, as unmapped), and the column locates its Gram row and its owner.
template <int K4, bool Mapped>
__global__ __launch_bounds__(kCoopThreads) void smo_coop_kernel(const SmoCoopProb* __restrict__ probs, int P,
                                                                int W, const float* __restrict__ K,
                                                                const int* __restrict__ maps,
                                                                double* __restrict__ alpha_all,
                                                                unsigned long long* __restrict__ xchg,
                                                                double eps, long long max_iter, SmoCoopOut out) {
  // libsvm's arithmetic (x86-64, no FMA): a*b + c*d stays un-contracted, as in smo_kernel
#pragma clang fp contract(off)
  constexpr int KM = 4 * K4;
  static_assert(KM <= 64, "per-thread point masks are 64-bit");
  const int xcd = blockIdx.x & 7, q = blockIdx.x >> 3;
  const int p = xcd + 8 * (q / W), w = q % W;
  if (p >= P) return;
  coop_inject_delay(out.inject_ticks, p, w);
  const SmoCoopProb Pr = probs[p];
  const float* Kp = K + Pr.koff;
  const int tid = threadIdx.x;
  if (Mapped && (Pr.lphys > kPkMask + 1 || Pr.l > kPkMask + 1)) {   // keys would overflow: every member leaves
    if (threadIdx.x == 0) atomicOr(out.err, 2u);
    return;
  }
  const int base = w * Pr.S;
  const int send = min(Pr.lphys, base + Pr.S);   // may be ≤ base: an empty member still exchanges
  unsigned long long* slot0 = xchg + (size_t)p * 2 * kMaxMembers * kGran;
  __shared__ CoopPart shA[kCoopWaves], shB[kCoopWaves];
  __shared__ unsigned vals[2][kMaxMembers][kGran];
  __shared__ int sh_fail;
  __shared__ double ssum[2][kCoopWaves];
  unsigned epoch = 0;

  double G[KM], A[KM];
  float Qi[KM];
  int PK[Mapped ? KM : 1];   // Mapped: key of the point in each slot
  unsigned long long ypos = 0ull, upm = 0ull, lowm = 0ull, freem = 0ull, upperm = 0ull, validm = 0ull;
#pragma unroll
  for (int g = 0; g < K4; ++g)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = 4 * g + e;
      const int c = base + 4 * (tid + g * kCoopThreads) + e;
      G[k] = -1.0;   // p_i = −1 for C-SVC, α = 0
      A[k] = 0.0;
      Qi[k] = 0.f;
      int t = c;
      if constexpr (Mapped) {
        t = c >= send ? -1 : Pr.moff >= 0 ? maps[Pr.moff + c] : c;   // moff < 0: the problem's own Gram
        PK[k] = t >= 0 ? (t << kPkBits) | c : -1;
      }
      if (c < send && t >= 0) {
        validm |= 1ull << k;
        if (t < Pr.npos) { ypos |= 1ull << k; upm |= 1ull << k; }   // α = 0 is at the lower bound
        else lowm |= 1ull << k;
      }
    }
  // key of slot k (unmapped: its column), and the column and libsvm index of a key
  auto key_of = [&](int k) {
    if constexpr (Mapped) return PK[k];
    else return base + 4 * (tid + (k >> 2) * kCoopThreads) + (k & 3);
  };
  auto col_of = [&](int t) { return Mapped ? (t & kPkMask) : t; };
  auto idx_of = [&](int t) { return Mapped ? (t >> kPkBits) : t; };
  // (thread, register slot) of the point with key t of this member
  auto owner_thr = [&](int t) { return ((col_of(t) - base) >> 2) % kCoopThreads; };
  auto owner_k = [&](int t) { return 4 * (((col_of(t) - base) >> 2) / kCoopThreads) + ((col_of(t) - base) & 3); };
  auto pick = [&](const double* arr, int kk) {
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < KM; ++k)
      if (k == kk) v = arr[k];
    return v;
  };
  auto pickf = [&](const float* arr, int kk) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < KM; ++k)
      if (k == kk) v = arr[k];
    return v;
  };
  // While wave 0 polls an exchange, waves 1.. touch one dword per 128-byte line of the FULL Gram
  // row of this member's own candidate: the winning candidate's row — whichever member proposed
  // it — is then in this XCD's L2 (members of a problem share an XCD) when every member reads its
  // slice after the exchange, so the two dependent row reads of a pair cost an L2 hit instead of
  // an HBM round trip.  Issued after the owner's granule stores (a stalled owner would delay the
  // exchange itself) and consumed only after the exchange (the barrier waits on LDS traffic only,
  // so nothing waits for these loads until the data is long there).  Rows of ≤ 4·448·32 points
  // are covered entirely; longer rows only partly (a hint, never a correctness matter).
  struct Pf { float v[4]; };
  auto prefetch_issue = [&](int r) {
    Pf pf{{0.f, 0.f, 0.f, 0.f}};
    if (out.prefetch && r >= 0 && tid >= 64) {
      const float* row = Kp + (size_t)col_of(r) * Pr.ld;
      const int lines = (Pr.lphys + 31) >> 5;
      constexpr int kPf = kCoopThreads - 64;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = tid - 64 + u * kPf;
        if (c < lines) pf.v[u] = row[(size_t)c << 5];
      }
    }
    return pf;
  };
  auto prefetch_retire = [&](const Pf& pf) { asm volatile("" ::"v"(pf.v[0]), "v"(pf.v[1]), "v"(pf.v[2]), "v"(pf.v[3])); };
  // exchange 1: every member's step-1 partial (kb, idx, α_idx) → (Gmax key, i, α_i)
  auto exchange1 = [&](const CoopPart& loc, unsigned long long& kb, int& idx, double& a_i) -> bool {
    ++epoch;
    unsigned long long* s = slot0 + (size_t)(epoch & 1) * kMaxMembers * kGran;
    const bool has = loc.idx >= 0;
    if (has ? tid == owner_thr(loc.idx) : tid == 0) {
      unsigned long long* mine = s + w * kGran;
      const double av = has ? pick(A, owner_k(loc.idx)) : 0.0;
      put_u64(mine, epoch, loc.kb);
      put_granule(mine + 2, epoch, (unsigned)loc.idx);
      put_u64(mine + 3, epoch, bits_of(av));
    }
    const Pf pf = prefetch_issue(loc.idx);
    if (!coop_gather(s, W, 5, epoch, vals[epoch & 1], out, &sh_fail)) return false;
    prefetch_retire(pf);
    const unsigned(*v)[kGran] = vals[epoch & 1];
    kb = u64_of(&v[0][0]);
    idx = (int)v[0][2];
    a_i = f64_of(&v[0][3]);
    for (int m = 1; m < W; ++m) {
      const unsigned long long k2 = u64_of(&v[m][0]);
      const int i2 = (int)v[m][2];
      if (k2 > kb || (k2 == kb && i2 > idx)) { kb = k2; idx = i2; a_i = f64_of(&v[m][3]); }
    }
    return true;
  };

  // ---- WSS step 1 for the first iteration
  CoopPart loc;
  {
    double bb = -kCInf;
    int bi = -1;
#pragma unroll
    for (int k = 0; k < KM; ++k)
      if ((upm >> k) & 1ull) {
        const int t = key_of(k);
        const double v = ((ypos >> k) & 1ull) ? -G[k] : G[k];
        if (v > bb || (v == bb && t > bi)) { bb = v; bi = t; }
      }
    loc = coop_block_red<false>(-kCInf, bb, bi, shA);
  }
  unsigned long long r1kb = 0ull;
  int i = -1;
  double ai_old = 0.0;
  if (!exchange1(loc, r1kb, i, ai_old)) return;
  long long iter = 0;
  double last_gap = 0.0;
  long long ph[7] = {0, 0, 0, 0, 0, 0, 0};
  const bool prof = out.prof != nullptr && w == 0 && tid == 0;
  long long tc = prof ? __builtin_amdgcn_s_memtime() : 0;
  auto tick = [&](int k) {
    if (prof) {
      const long long now = __builtin_amdgcn_s_memtime();
      ph[k] += now - tc;
      tc = now;
    }
  };
  for (; iter < max_iter; ++iter) {
    if (i < 0) break;
    const double Gmax = f64_from_okey(r1kb);
    const int yi = idx_of(i) < Pr.npos ? 1 : -1;
    // ---- WSS step 2 over this member's slice of row i
    const float4* Ki4 = reinterpret_cast<const float4*>(Kp + (size_t)col_of(i) * Pr.ld + base);
    double gmax2 = -kCInf, bkey = -kCInf;
    int bj = -1;
    float4 qv[K4];
#pragma unroll
    for (int g = 0; g < K4; ++g)
      qv[g] = base + 4 * (tid + g * kCoopThreads) < send ? Ki4[tid + g * kCoopThreads] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int g = 0; g < K4; ++g) {
      const int t0 = base + 4 * (tid + g * kCoopThreads);
      const float4 qq = qv[g];
      Qi[4 * g] = qq.x; Qi[4 * g + 1] = qq.y; Qi[4 * g + 2] = qq.z; Qi[4 * g + 3] = qq.w;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = 4 * g + e;
        if ((lowm >> k) & 1ull) {
          const double yG = ((ypos >> k) & 1ull) ? G[k] : -G[k];
          gmax2 = fmax(gmax2, yG);
          const double gd = Gmax + yG;
          if (gd > 0) {
            double quad = 2.0 - 2.0 * (double)Qi[k];
            if (quad <= 0) quad = kCTau;
            const double key = (gd * gd) / quad;   // smo_kernel's rank: grouping-independent
            if constexpr (Mapped) {   // slots are in column order, not index order
              if (bj < 0 || key > bkey || (key == bkey && key_of(k) > bj)) { bkey = key; bj = key_of(k); }
            } else if (bj < 0 || key >= bkey) { bkey = key; bj = t0 + e; }
          }
        }
      }
    }
    tick(0);
    loc = coop_block_red(gmax2, bj >= 0 ? bkey : -kCInf, bj, shB);
    tick(1);
    // ---- exchange 2: (max yG over I_low, best objective key, j, α_j, G_j, K_ij)
    ++epoch;
    unsigned long long* s2 = slot0 + (size_t)(epoch & 1) * kMaxMembers * kGran;
    {
      const bool has = loc.idx >= 0;
      if (has ? tid == owner_thr(loc.idx) : tid == 0) {
        unsigned long long* mine = s2 + w * kGran;
        const int kk = has ? owner_k(loc.idx) : 0;
        const double aj = has ? pick(A, kk) : 0.0;
        const double gj = has ? pick(G, kk) : 0.0;
        const float kij = has ? pickf(Qi, kk) : 0.f;
        put_u64(mine, epoch, loc.ka);
        put_u64(mine + 2, epoch, loc.kb);
        put_granule(mine + 4, epoch, (unsigned)loc.idx);
        put_u64(mine + 5, epoch, bits_of(aj));
        put_u64(mine + 7, epoch, bits_of(gj));
        put_granule(mine + 9, epoch, __float_as_uint(kij));
      }
    }
    const Pf pf2 = prefetch_issue(loc.idx);
    if (!coop_gather(s2, W, 10, epoch, vals[epoch & 1], out, &sh_fail)) return;
    prefetch_retire(pf2);
    tick(2);
    unsigned long long ka2, kb2;
    int j;
    double aj_old, Gj, Kij;
    {
      const unsigned(*v)[kGran] = vals[epoch & 1];
      ka2 = u64_of(&v[0][0]);
      kb2 = u64_of(&v[0][2]);
      j = (int)v[0][4];
      aj_old = f64_of(&v[0][5]);
      Gj = f64_of(&v[0][7]);
      Kij = (double)__uint_as_float(v[0][9]);
      for (int m = 1; m < W; ++m) {
        const unsigned long long a2 = u64_of(&v[m][0]);
        ka2 = a2 > ka2 ? a2 : ka2;
        const unsigned long long k2 = u64_of(&v[m][2]);
        const int j2 = (int)v[m][4];
        if (k2 > kb2 || (k2 == kb2 && j2 > j)) {
          kb2 = k2;
          j = j2;
          aj_old = f64_of(&v[m][5]);
          Gj = f64_of(&v[m][7]);
          Kij = (double)__uint_as_float(v[m][9]);
        }
      }
    }
    const double gmax2_all = f64_from_okey(ka2);
    last_gap = Gmax + gmax2_all;
    if (Gmax + gmax2_all < eps || j < 0) break;
    // ---- pair update (identical in every member)
    const int yj = idx_of(j) < Pr.npos ? 1 : -1;
    const double Ci = yi > 0 ? Pr.Cp : Pr.Cn, Cj = yj > 0 ? Pr.Cp : Pr.Cn;
    const double Qij = (double)(yi * yj) * Kij;
    const double Gi = -(double)yi * Gmax;
    double ai = ai_old, aj = aj_old;
    if (yi != yj) {
      double quad = 2.0 + 2.0 * Qij;
      if (quad <= 0) quad = kCTau;
      const double delta = (-Gi - Gj) / quad;
      const double diff = ai - aj;
      ai += delta;
      aj += delta;
      if (diff > 0) {
        if (aj < 0) { aj = 0; ai = diff; }
      } else {
        if (ai < 0) { ai = 0; aj = -diff; }
      }
      if (diff > Ci - Cj) {
        if (ai > Ci) { ai = Ci; aj = Ci - diff; }
      } else {
        if (aj > Cj) { aj = Cj; ai = Cj + diff; }
      }
    } else {
      double quad = 2.0 - 2.0 * Qij;
      if (quad <= 0) quad = kCTau;
      const double delta = (Gi - Gj) / quad;
      const double sum = ai + aj;
      ai -= delta;
      aj += delta;
      if (sum > Ci) {
        if (ai > Ci) { ai = Ci; aj = sum - Ci; }
      } else {
        if (aj < 0) { aj = 0; ai = sum; }
      }
      if (sum > Cj) {
        if (aj > Cj) { aj = Cj; ai = sum - Cj; }
      } else {
        if (ai < 0) { ai = 0; aj = sum; }
      }
    }
    const double ci = (double)yi * (ai - ai_old), cj = (double)yj * (aj - aj_old);
    tick(3);
    // owners in this member: α and the bound masks of i and j
#pragma unroll
    for (int wv = 0; wv < 2; ++wv) {
      const int t = wv == 0 ? i : j;
      if (col_of(t) < base || col_of(t) >= send || tid != owner_thr(t)) continue;
      const int kk = owner_k(t);
      const double a = wv == 0 ? ai : aj;
      const double C = wv == 0 ? Ci : Cj;
#pragma unroll
      for (int k = 0; k < KM; ++k)
        if (k == kk) A[k] = a;
      const unsigned long long bit = 1ull << kk;
      const bool pos = (ypos & bit) != 0ull;
      const bool atU = a >= C, atL = a <= 0;
      freem = (!atU && !atL) ? (freem | bit) : (freem & ~bit);
      upperm = atU ? (upperm | bit) : (upperm & ~bit);
      const bool up = pos ? !atU : !atL;
      const bool low = pos ? !atL : !atU;
      upm = up ? (upm | bit) : (upm & ~bit);
      lowm = low ? (lowm | bit) : (lowm & ~bit);
    }
    // ---- gradient update of this member's slice (row i in registers, row j loaded now), fused
    // with the next step-1 candidates
    const float4* Kj4 = reinterpret_cast<const float4*>(Kp + (size_t)col_of(j) * Pr.ld + base);
    float4 qjv[K4];
#pragma unroll
    for (int g = 0; g < K4; ++g)
      qjv[g] = base + 4 * (tid + g * kCoopThreads) < send ? Kj4[tid + g * kCoopThreads] : make_float4(0.f, 0.f, 0.f, 0.f);
    double bb = -kCInf;
    int bi = -1;
#pragma unroll
    for (int g = 0; g < K4; ++g) {
      const int t0 = base + 4 * (tid + g * kCoopThreads);
      const float4 qq = qjv[g];
      const float qj[4] = {qq.x, qq.y, qq.z, qq.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = 4 * g + e;
        const bool pos = (ypos >> k) & 1ull;
        const double upd = (double)Qi[k] * ci + (double)qj[e] * cj;
        G[k] += pos ? upd : -upd;
        if ((upm >> k) & 1ull) {
          const double v = pos ? -G[k] : G[k];
          const int tk = Mapped ? key_of(k) : t0 + e;
          if (v > bb || (v == bb && tk > bi)) { bb = v; bi = tk; }
        }
      }
    }
    tick(4);
    loc = coop_block_red<false>(-kCInf, bb, bi, shA);
    tick(5);
    if (!exchange1(loc, r1kb, i, ai_old)) return;
    tick(6);
  }
  if (prof)
    for (int k = 0; k < 7; ++k) out.prof[(size_t)p * 7 + k] = ph[k];
  // ---- α out (owners) and calculate_rho over all members
#pragma unroll
  for (int k = 0; k < KM; ++k)
    if ((validm >> k) & 1ull) alpha_all[Pr.aoff + idx_of(key_of(k))] = A[k];
  double ru = -kCInf, rl = -kCInf, sum_free = 0.0;
  int nfree = 0;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    if (!((validm >> k) & 1ull)) continue;
    const bool pos = (ypos >> k) & 1ull;
    const double yG = pos ? G[k] : -G[k];
    if ((upperm >> k) & 1ull) {
      if (!pos) ru = fmax(ru, -yG); else rl = fmax(rl, yG);
    } else if ((freem >> k) & 1ull) {
      ++nfree;
      sum_free += yG;
    } else {
      if (pos) ru = fmax(ru, -yG); else rl = fmax(rl, yG);
    }
  }
  __syncthreads();   // the loop may leave right after a fold that still reads shA
  const CoopPart rr = coop_block_red(ru, rl, -1, shA);
  {
    const double s = wave_sum(sum_free), c = wave_sum((double)nfree);
    if ((tid & 63) == 0) { ssum[0][tid >> 6] = s; ssum[1][tid >> 6] = c; }
  }
  __syncthreads();
  double Sm = 0.0, Cm = 0.0;
  for (int wv = 0; wv < kCoopWaves; ++wv) { Sm += ssum[0][wv]; Cm += ssum[1][wv]; }
  ++epoch;
  unsigned long long* s3 = slot0 + (size_t)(epoch & 1) * kMaxMembers * kGran;
  if (tid == 0) {
    unsigned long long* mine = s3 + w * kGran;
    put_u64(mine, epoch, rr.ka);       // max(−yG) over the upper-bound candidates
    put_u64(mine + 2, epoch, rr.kb);   // max(yG) over the lower-bound candidates
    put_u64(mine + 4, epoch, bits_of(Sm));
    put_u64(mine + 6, epoch, bits_of(Cm));
  }
  if (!coop_gather(s3, W, 8, epoch, vals[epoch & 1], out, &sh_fail)) return;
  if (w == 0 && tid == 0) {
    const unsigned(*v)[kGran] = vals[epoch & 1];
    unsigned long long kru = u64_of(&v[0][0]), krl = u64_of(&v[0][2]);
    double St = 0.0, Ct = 0.0;
    for (int m = 0; m < W; ++m) {
      const unsigned long long a2 = u64_of(&v[m][0]), b2 = u64_of(&v[m][2]);
      kru = a2 > kru ? a2 : kru;
      krl = b2 > krl ? b2 : krl;
      St += f64_of(&v[m][4]);
      Ct += f64_of(&v[m][6]);
    }
    const double ub = -f64_from_okey(kru), lb = f64_from_okey(krl);
    out.rho[p] = Ct > 0 ? St / Ct : (ub + lb) / 2;
    out.iters[p] = (int)iter;
    out.gap[p] = last_gap;
  }
}

// Exchange deadline and the late-member test hook, from the environment (read per launch).
static void coop_timing(SmoCoopOut& o) {
  const char* w = std::getenv("HFENS_SMO_WAIT_MS");
  const char* d = std::getenv("HFENS_SMO_INJECT_DELAY_MS");
  const double wait_ms = (w && w[0]) ? std::atof(w) : (double)kWaitMsDefault;
  o.wait_ticks = (long long)(wait_ms * 1e5);               // 100 MHz counter
  o.inject_ticks = (d && d[0]) ? (long long)(std::atof(d) * 1e5) : 0;
}

// Members of one problem spin on each other, so all of them must be resident together: the
// launchers bound P·W by the CU count (one member per CU), and the Python side subtracts the CUs
// it leaves to concurrent kernels.  This returns what the hardware would co-schedule of the
// kernel on an idle device (occupancy per CU × CUs): the upper bound models/smo.py clamps W with.
void coop_resident_blocks(uintptr_t out) {
  int dev = 0, ncu = 256, per_cu = 0;
  HFENS_CHECK(hipGetDevice(&dev));
  HFENS_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  HFENS_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, smo_coop_kernel<8, true>, kCoopThreads, 0));
  ((long long*)out)[0] = (long long)per_cu * ncu;
  ((long long*)out)[1] = ncu;
}

void smo_coop_batch(uintptr_t probs, int P, int W, int max_S, uintptr_t K, uintptr_t maps, uintptr_t alpha,
                    uintptr_t xchg, double eps, long long max_iter, uintptr_t rho, uintptr_t iters, uintptr_t gap,
                    uintptr_t err, uintptr_t prof, uintptr_t stream) {
  HFENS_REQUIRE(W >= 1 && W <= kMaxMembers, "smo_coop_batch: 1 <= W <= 16 members per problem");
  HFENS_REQUIRE(P >= 1, "smo_coop_batch: no problems");
  HFENS_REQUIRE(max_S >= 4 && max_S % 4 == 0, "smo_coop_batch: slice must be a positive multiple of 4");
  int dev = 0, ncu = 256;
  HFENS_CHECK(hipGetDevice(&dev));
  HFENS_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  // members spin on each other, so all of them must be resident at once: at most one member per
  // CU (a 512-thread block always fits beside anything else's finished work); the padding
  // blocks of an incomplete group of 8 problems exit at once
  HFENS_REQUIRE((long long)P * W <= ncu, "smo_coop_batch: P·W exceeds the CU count (choose a smaller W)");
  const int groups = (P + 7) / 8;
  const long long blocks = 8LL * groups * W;
  const char* pfe = std::getenv("HFENS_SMO_PREFETCH");
  SmoCoopOut o{(double*)rho, (int*)iters, (double*)gap, (unsigned*)err, (long long*)prof,
               (pfe && pfe[0] == '0') ? 0 : 1};
  coop_timing(o);
  hipStream_t st = as_stream(stream);
  // every polled granule starts at epoch 0 (epochs count from 1 within the call)
  HFENS_CHECK(hipMemsetAsync((void*)xchg, 0, (size_t)P * 2 * kMaxMembers * kGran * sizeof(unsigned long long), st));
  auto pp = (const SmoCoopProb*)probs;
  auto kp = (const float*)K;
  auto ap = (double*)alpha;
  auto xp = (unsigned long long*)xchg;
  auto mp = (const int*)maps;
  // maps != 0: Platt sub-problems index their parents' Grams (columns < 2^15: checked per problem
  // in the kernel, which flags err and leaves — the host then re-solves unmapped)
#define COOP_CASE(K4)                                                                                           \
  if (max_S <= 4 * K4 * kCoopThreads) {                                                                         \
    if (mp != nullptr)                                                                                          \
      hipLaunchKernelGGL((smo_coop_kernel<K4, true>), dim3((unsigned)blocks), dim3(kCoopThreads), 0, st, pp, P, \
                         W, kp, mp, ap, xp, eps, max_iter, o);                                                  \
    else                                                                                                        \
      hipLaunchKernelGGL((smo_coop_kernel<K4, false>), dim3((unsigned)blocks), dim3(kCoopThreads), 0, st, pp,   \
                         P, W, kp, mp, ap, xp, eps, max_iter, o);                                               \
    launch_check();                                                                                             \
    return;                                                                                                     \
  }
  COOP_CASE(1) COOP_CASE(2) COOP_CASE(4) COOP_CASE(8)
#undef COOP_CASE
  throw std::invalid_argument("smo_coop_batch: slice larger than 16384 points");
}

// ------------------------------------------------------------------------------------------
// smo_coop_otf: the same cooperative solver with NO stored Gram.  Each thread keeps its points'
// rows z_t and norms ‖z_t‖² in registers and re-evaluates its entries of Gram rows i and j per
// pair with gram_rbf_kernel's exact expression — its f32-input MFMA dot product is bit-for-bit a
// k-ordered fmaf chain, then the same norm sum, clamp and exp2 — so the values, and hence the
// pair sequence, equal the stored-Gram solvers'.  z_i and z_j travel inside the two exchanges
// (the candidate's owner publishes its row as F + 1 more granules), so a pair reads nothing from
// HBM: two in-launch exchanges plus register arithmetic.  Memory is O(l·F) instead of O(l²) (the
// bench's 36 problems: 7 GB of Gram neither written nor re-read) and the Gram launch goes away.
// Points are strided over threads (t = base + tid + 512·m): no vector-load layout to keep.
// Measured: at ≤ 2 points per thread it runs with the stored-Gram kernel; at 4 points per thread
// (256 VGPRs + spills) it is slower, so the host picks it only for slices of ≤ 1024 points.
struct SmoOtfProb {
  long long zoff;   // first row of this problem in zcat ([rows][F] f32, problem order)
  long long aoff;   // alpha offset (doubles)
  int l;            // problem size
  int npos;         // indices [0, npos) have y = +1, the rest y = −1
  int S;            // points per member: member w owns [w·S, min(l, (w+1)·S))
  float ngl2e;      // −γ·log2(e)
  double Cp, Cn;
};

constexpr int kOtfGran = 32;   // granules per member slot: exchange 2 carries 11 + F
constexpr int kOtfMaxF = 20;

__device__ __forceinline__ float rbf_entry(float dot, float nr, float nc, float ngl2e) {
  float d2 = fmaf(-2.f, dot, nr + nc);   // gram_rbf_kernel's epilogue, operand for operand
  d2 = fmaxf(d2, 0.f);
  return __builtin_amdgcn_exp2f(ngl2e * d2);
}

template <int KM, int FP>
__global__ __launch_bounds__(kCoopThreads) void smo_coop_otf_kernel(const SmoOtfProb* __restrict__ probs, int P,
                                                                    int W, int F, const float* __restrict__ zcat,
                                                                    double* __restrict__ alpha_all,
                                                                    unsigned long long* __restrict__ xchg,
                                                                    double eps, long long max_iter, SmoCoopOut out) {
#pragma clang fp contract(off)
  static_assert(KM <= 64 && FP <= kOtfMaxF, "register tile");
  const int xcd = blockIdx.x & 7, q = blockIdx.x >> 3;
  const int p = xcd + 8 * (q / W), w = q % W;
  if (p >= P) return;
  coop_inject_delay(out.inject_ticks, p, w);
  const SmoOtfProb Pr = probs[p];
  const int tid = threadIdx.x;
  const int base = w * Pr.S;
  const int send = min(Pr.l, base + Pr.S);   // may be ≤ base: an empty member still exchanges
  unsigned long long* slot0 = xchg + (size_t)p * 2 * kMaxMembers * kOtfGran;
  __shared__ CoopPart shA[kCoopWaves], shB[kCoopWaves];
  __shared__ unsigned vals[2][kMaxMembers][kOtfGran];
  __shared__ int sh_fail;
  __shared__ double ssum[2][kCoopWaves];
  unsigned epoch = 0;

  float zr[KM][FP], nz[KM];   // this thread's points: rows and squared norms
  double G[KM], A[KM];
  float Qi[KM], Qj[KM];
  unsigned long long ypos = 0ull, upm = 0ull, lowm = 0ull, freem = 0ull, upperm = 0ull, validm = 0ull;
#pragma unroll
  for (int m = 0; m < KM; ++m) {
    const int t = base + tid + kCoopThreads * m;
    const bool ok = t < send;
    const float* zt = zcat + (size_t)(Pr.zoff + (ok ? t : 0)) * F;
    float sq = 0.f;
#pragma unroll
    for (int k = 0; k < FP; ++k) {
      zr[m][k] = (ok && k < F) ? zt[k] : 0.f;
      if (k < F) sq = fmaf(zr[m][k], zr[m][k], sq);
    }
    nz[m] = sq;
    G[m] = -1.0;   // p_i = −1 for C-SVC, α = 0
    A[m] = 0.0;
    Qi[m] = 0.f;
    Qj[m] = 0.f;
    if (ok) {
      validm |= 1ull << m;
      if (t < Pr.npos) { ypos |= 1ull << m; upm |= 1ull << m; }   // α = 0 is at the lower bound
      else lowm |= 1ull << m;
    }
  }
  auto owner_thr = [&](int t) { return (t - base) % kCoopThreads; };
  auto owner_m = [&](int t) { return (t - base) / kCoopThreads; };
  auto pick = [&](const double* arr, int mm) {
    double v = 0.0;
#pragma unroll
    for (int m = 0; m < KM; ++m)
      if (m == mm) v = arr[m];
    return v;
  };
  auto pickf = [&](const float* arr, int mm) {
    float v = 0.f;
#pragma unroll
    for (int m = 0; m < KM; ++m)
      if (m == mm) v = arr[m];
    return v;
  };
  // this thread's entries of Gram row r; the row's features and norm come from an exchange (LDS)
  auto gram_row = [&](int r, const unsigned* zb, float nzr, float* Qo) {
    float zrow[FP];
#pragma unroll
    for (int k = 0; k < FP; ++k) zrow[k] = k < F ? __uint_as_float(zb[k]) : 0.f;
#pragma unroll
    for (int m = 0; m < KM; ++m) {
      float dot = 0.f;
#pragma unroll
      for (int k = 0; k < FP; ++k)
        if (k < F) dot = fmaf(zrow[k], zr[m][k], dot);
      Qo[m] = base + tid + kCoopThreads * m == r ? 1.f : rbf_entry(dot, nzr, nz[m], Pr.ngl2e);
    }
  };
  // owner of point t: granule 0 = ‖z_t‖², granules 1..F = z_t
  auto publish_row = [&](unsigned long long* dst, int t) {
    const int mm = owner_m(t);
    float nn = 0.f, zz[FP];
#pragma unroll
    for (int k = 0; k < FP; ++k) zz[k] = 0.f;
#pragma unroll
    for (int m = 0; m < KM; ++m)
      if (m == mm) {
        nn = nz[m];
#pragma unroll
        for (int k = 0; k < FP; ++k) zz[k] = zr[m][k];
      }
    put_granule(dst, epoch, __float_as_uint(nn));
#pragma unroll
    for (int k = 0; k < FP; ++k)
      if (k < F) put_granule(dst + 1 + k, epoch, __float_as_uint(zz[k]));
  };
  auto publish_zero_row = [&](unsigned long long* dst) {
    for (int k = 0; k <= F; ++k) put_granule(dst + k, epoch, 0u);
  };
  // exchange 1: (kb, idx, α_idx, ‖z_idx‖², z_idx) → (Gmax key, i, α_i, member holding z_i)
  auto exchange1 = [&](const CoopPart& loc, unsigned long long& kb, int& idx, double& a_i, int& ms) -> bool {
    ++epoch;
    unsigned long long* s = slot0 + (size_t)(epoch & 1) * kMaxMembers * kOtfGran;
    const bool has = loc.idx >= 0;
    if (has ? tid == owner_thr(loc.idx) : tid == 0) {
      unsigned long long* mine = s + w * kOtfGran;
      put_u64(mine, epoch, loc.kb);
      put_granule(mine + 2, epoch, (unsigned)loc.idx);
      put_u64(mine + 3, epoch, bits_of(has ? pick(A, owner_m(loc.idx)) : 0.0));
      if (has) publish_row(mine + 5, loc.idx);
      else publish_zero_row(mine + 5);
    }
    if (!coop_gather_t<kOtfGran>(s, W, 6 + F, epoch, vals[epoch & 1], out, &sh_fail)) return false;
    const unsigned(*v)[kOtfGran] = vals[epoch & 1];
    kb = u64_of(&v[0][0]);
    idx = (int)v[0][2];
    a_i = f64_of(&v[0][3]);
    ms = 0;
    for (int m = 1; m < W; ++m) {
      const unsigned long long k2 = u64_of(&v[m][0]);
      const int i2 = (int)v[m][2];
      if (k2 > kb || (k2 == kb && i2 > idx)) { kb = k2; idx = i2; a_i = f64_of(&v[m][3]); ms = m; }
    }
    return true;
  };

  // ---- WSS step 1 for the first iteration
  CoopPart loc;
  {
    double bb = -kCInf;
    int bi = -1;
#pragma unroll
    for (int m = 0; m < KM; ++m)
      if ((upm >> m) & 1ull) {
        const int t = base + tid + kCoopThreads * m;
        const double v = ((ypos >> m) & 1ull) ? -G[m] : G[m];
        if (v > bb || (v == bb && t > bi)) { bb = v; bi = t; }
      }
    loc = coop_block_red<false>(-kCInf, bb, bi, shA);
  }
  unsigned long long r1kb = 0ull;
  int i = -1, mi = 0;
  double ai_old = 0.0;
  if (!exchange1(loc, r1kb, i, ai_old, mi)) return;
  long long iter = 0;
  double last_gap = 0.0;
  for (; iter < max_iter; ++iter) {
    if (i < 0) break;
    const double Gmax = f64_from_okey(r1kb);
    const int yi = i < Pr.npos ? 1 : -1;
    {
      const unsigned* zb = &vals[epoch & 1][mi][6];
      gram_row(i, zb, __uint_as_float(vals[epoch & 1][mi][5]), Qi);
    }
    // ---- WSS step 2 over this member's entries of row i
    double gmax2 = -kCInf, bkey = -kCInf;
    int bj = -1;
#pragma unroll
    for (int m = 0; m < KM; ++m) {
      if ((lowm >> m) & 1ull) {
        const double yG = ((ypos >> m) & 1ull) ? G[m] : -G[m];
        gmax2 = fmax(gmax2, yG);
        const double gd = Gmax + yG;
        if (gd > 0) {
          double quad = 2.0 - 2.0 * (double)Qi[m];
          if (quad <= 0) quad = kCTau;
          const double key = (gd * gd) / quad;   // smo_kernel's rank: grouping-independent
          if (bj < 0 || key >= bkey) { bkey = key; bj = base + tid + kCoopThreads * m; }
        }
      }
    }
    loc = coop_block_red(gmax2, bj >= 0 ? bkey : -kCInf, bj, shB);
    // ---- exchange 2: (max yG over I_low, best key, j, α_j, G_j, K_ij, ‖z_j‖², z_j)
    ++epoch;
    unsigned long long* s2 = slot0 + (size_t)(epoch & 1) * kMaxMembers * kOtfGran;
    {
      const bool has = loc.idx >= 0;
      if (has ? tid == owner_thr(loc.idx) : tid == 0) {
        unsigned long long* mine = s2 + w * kOtfGran;
        const int mm = has ? owner_m(loc.idx) : 0;
        put_u64(mine, epoch, loc.ka);
        put_u64(mine + 2, epoch, loc.kb);
        put_granule(mine + 4, epoch, (unsigned)loc.idx);
        put_u64(mine + 5, epoch, bits_of(has ? pick(A, mm) : 0.0));
        put_u64(mine + 7, epoch, bits_of(has ? pick(G, mm) : 0.0));
        put_granule(mine + 9, epoch, __float_as_uint(has ? pickf(Qi, mm) : 0.f));
        if (has) publish_row(mine + 10, loc.idx);
        else publish_zero_row(mine + 10);
      }
    }
    if (!coop_gather_t<kOtfGran>(s2, W, 11 + F, epoch, vals[epoch & 1], out, &sh_fail)) return;
    unsigned long long ka2, kb2;
    int j, mj;
    double aj_old, Gj, Kij;
    {
      const unsigned(*v)[kOtfGran] = vals[epoch & 1];
      ka2 = u64_of(&v[0][0]);
      kb2 = u64_of(&v[0][2]);
      j = (int)v[0][4];
      aj_old = f64_of(&v[0][5]);
      Gj = f64_of(&v[0][7]);
      Kij = (double)__uint_as_float(v[0][9]);
      mj = 0;
      for (int m = 1; m < W; ++m) {
        const unsigned long long a2 = u64_of(&v[m][0]);
        ka2 = a2 > ka2 ? a2 : ka2;
        const unsigned long long k2 = u64_of(&v[m][2]);
        const int j2 = (int)v[m][4];
        if (k2 > kb2 || (k2 == kb2 && j2 > j)) {
          kb2 = k2;
          j = j2;
          aj_old = f64_of(&v[m][5]);
          Gj = f64_of(&v[m][7]);
          Kij = (double)__uint_as_float(v[m][9]);
          mj = m;
        }
      }
    }
    const double gmax2_all = f64_from_okey(ka2);
    last_gap = Gmax + gmax2_all;
    if (Gmax + gmax2_all < eps || j < 0) break;
    // ---- pair update (identical in every member; libsvm's clipping)
    const int yj = j < Pr.npos ? 1 : -1;
    const double Ci = yi > 0 ? Pr.Cp : Pr.Cn, Cj = yj > 0 ? Pr.Cp : Pr.Cn;
    const double Qij = (double)(yi * yj) * Kij;
    const double Gi = -(double)yi * Gmax;
    double ai = ai_old, aj = aj_old;
    if (yi != yj) {
      double quad = 2.0 + 2.0 * Qij;
      if (quad <= 0) quad = kCTau;
      const double delta = (-Gi - Gj) / quad;
      const double diff = ai - aj;
      ai += delta;
      aj += delta;
      if (diff > 0) {
        if (aj < 0) { aj = 0; ai = diff; }
      } else {
        if (ai < 0) { ai = 0; aj = -diff; }
      }
      if (diff > Ci - Cj) {
        if (ai > Ci) { ai = Ci; aj = Ci - diff; }
      } else {
        if (aj > Cj) { aj = Cj; ai = Cj + diff; }
      }
    } else {
      double quad = 2.0 - 2.0 * Qij;
      if (quad <= 0) quad = kCTau;
      const double delta = (Gi - Gj) / quad;
      const double sum = ai + aj;
      ai -= delta;
      aj += delta;
      if (sum > Ci) {
        if (ai > Ci) { ai = Ci; aj = sum - Ci; }
      } else {
        if (aj < 0) { aj = 0; ai = sum; }
      }
      if (sum > Cj) {
        if (aj > Cj) { aj = Cj; ai = sum - Cj; }
      } else {
        if (ai < 0) { ai = 0; aj = sum; }
      }
    }
    const double ci = (double)yi * (ai - ai_old), cj = (double)yj * (aj - aj_old);
#pragma unroll
    for (int wv = 0; wv < 2; ++wv) {
      const int t = wv == 0 ? i : j;
      if (t < base || t >= send || tid != owner_thr(t)) continue;
      const int mm = owner_m(t);
      const double a = wv == 0 ? ai : aj;
      const double C = wv == 0 ? Ci : Cj;
#pragma unroll
      for (int m = 0; m < KM; ++m)
        if (m == mm) A[m] = a;
      const unsigned long long bit = 1ull << mm;
      const bool pos = (ypos & bit) != 0ull;
      const bool atU = a >= C, atL = a <= 0;
      freem = (!atU && !atL) ? (freem | bit) : (freem & ~bit);
      upperm = atU ? (upperm | bit) : (upperm & ~bit);
      const bool up = pos ? !atU : !atL;
      const bool low = pos ? !atL : !atU;
      upm = up ? (upm | bit) : (upm & ~bit);
      lowm = low ? (lowm | bit) : (lowm & ~bit);
    }
    // ---- gradient update with rows i (registers) and j (recomputed now), fused with the next
    // step-1 candidates
    gram_row(j, &vals[epoch & 1][mj][11], __uint_as_float(vals[epoch & 1][mj][10]), Qj);
    double bb = -kCInf;
    int bi = -1;
#pragma unroll
    for (int m = 0; m < KM; ++m) {
      const bool pos = (ypos >> m) & 1ull;
      const double upd = (double)Qi[m] * ci + (double)Qj[m] * cj;
      G[m] += pos ? upd : -upd;
      if ((upm >> m) & 1ull) {
        const int t = base + tid + kCoopThreads * m;
        const double v = pos ? -G[m] : G[m];
        if (v > bb || (v == bb && t > bi)) { bb = v; bi = t; }
      }
    }
    loc = coop_block_red<false>(-kCInf, bb, bi, shA);
    if (!exchange1(loc, r1kb, i, ai_old, mi)) return;
  }
  // ---- α out (owners) and calculate_rho over all members
#pragma unroll
  for (int m = 0; m < KM; ++m)
    if ((validm >> m) & 1ull) alpha_all[Pr.aoff + base + tid + kCoopThreads * m] = A[m];
  double ru = -kCInf, rl = -kCInf, sum_free = 0.0;
  int nfree = 0;
#pragma unroll
  for (int m = 0; m < KM; ++m) {
    if (!((validm >> m) & 1ull)) continue;
    const bool pos = (ypos >> m) & 1ull;
    const double yG = pos ? G[m] : -G[m];
    if ((upperm >> m) & 1ull) {
      if (!pos) ru = fmax(ru, -yG); else rl = fmax(rl, yG);
    } else if ((freem >> m) & 1ull) {
      ++nfree;
      sum_free += yG;
    } else {
      if (pos) ru = fmax(ru, -yG); else rl = fmax(rl, yG);
    }
  }
  __syncthreads();   // the loop may leave right after a fold that still reads shA
  const CoopPart rr = coop_block_red(ru, rl, -1, shA);
  {
    const double sm = wave_sum(sum_free), c = wave_sum((double)nfree);
    if ((tid & 63) == 0) { ssum[0][tid >> 6] = sm; ssum[1][tid >> 6] = c; }
  }
  __syncthreads();
  double Sm = 0.0, Cm = 0.0;
  for (int wv = 0; wv < kCoopWaves; ++wv) { Sm += ssum[0][wv]; Cm += ssum[1][wv]; }
  ++epoch;
  unsigned long long* s3 = slot0 + (size_t)(epoch & 1) * kMaxMembers * kOtfGran;
  if (tid == 0) {
    unsigned long long* mine = s3 + w * kOtfGran;
    put_u64(mine, epoch, rr.ka);
    put_u64(mine + 2, epoch, rr.kb);
    put_u64(mine + 4, epoch, bits_of(Sm));
    put_u64(mine + 6, epoch, bits_of(Cm));
  }
  if (!coop_gather_t<kOtfGran>(s3, W, 8, epoch, vals[epoch & 1], out, &sh_fail)) return;
  if (w == 0 && tid == 0) {
    const unsigned(*v)[kOtfGran] = vals[epoch & 1];
    unsigned long long kru = u64_of(&v[0][0]), krl = u64_of(&v[0][2]);
    double St = 0.0, Ct = 0.0;
    for (int m = 0; m < W; ++m) {
      const unsigned long long a2 = u64_of(&v[m][0]), b2 = u64_of(&v[m][2]);
      kru = a2 > kru ? a2 : kru;
      krl = b2 > krl ? b2 : krl;
      St += f64_of(&v[m][4]);
      Ct += f64_of(&v[m][6]);
    }
    const double ub = -f64_from_okey(kru), lb = f64_from_okey(krl);
    out.rho[p] = Ct > 0 ? St / Ct : (ub + lb) / 2;
    out.iters[p] = (int)iter;
    out.gap[p] = last_gap;
  }
}

void smo_coop_otf_batch(uintptr_t probs, int P, int W, int F, int max_S, uintptr_t zcat, uintptr_t alpha,
                        uintptr_t xchg, double eps, long long max_iter, uintptr_t rho, uintptr_t iters,
                        uintptr_t gap, uintptr_t err, uintptr_t stream) {
  HFENS_REQUIRE(W >= 1 && W <= kMaxMembers, "smo_coop_otf_batch: 1 <= W <= 16 members per problem");
  HFENS_REQUIRE(P >= 1, "smo_coop_otf_batch: no problems");
  HFENS_REQUIRE(F >= 1 && F <= kOtfMaxF, "smo_coop_otf_batch: 1 <= F <= 20 (rows held in registers)");
  HFENS_REQUIRE(max_S >= 1 && max_S <= 4 * kCoopThreads, "smo_coop_otf_batch: at most 2048 points per member");
  int dev = 0, ncu = 256;
  HFENS_CHECK(hipGetDevice(&dev));
  HFENS_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  HFENS_REQUIRE((long long)P * W <= ncu, "smo_coop_otf_batch: P·W exceeds the CU count (choose a smaller W)");
  const long long blocks = 8LL * ((P + 7) / 8) * W;
  SmoCoopOut o{(double*)rho, (int*)iters, (double*)gap, (unsigned*)err, nullptr};
  coop_timing(o);
  hipStream_t st = as_stream(stream);
  HFENS_CHECK(hipMemsetAsync((void*)xchg, 0, (size_t)P * 2 * kMaxMembers * kOtfGran * sizeof(unsigned long long), st));
  auto pp = (const SmoOtfProb*)probs;
  auto zp = (const float*)zcat;
  auto ap = (double*)alpha;
  auto xp = (unsigned long long*)xchg;
  const int KM = (max_S + kCoopThreads - 1) / kCoopThreads;
#define OTF_CASE(KM_, FP_)                                                                                   \
  if (KM <= KM_ && F <= FP_) {                                                                               \
    hipLaunchKernelGGL((smo_coop_otf_kernel<KM_, FP_>), dim3((unsigned)blocks), dim3(kCoopThreads), 0, st, pp, \
                       P, W, F, zp, ap, xp, eps, max_iter, o);                                              \
    launch_check();                                                                                          \
    return;                                                                                                  \
  }
  OTF_CASE(1, 8) OTF_CASE(1, 20) OTF_CASE(2, 8) OTF_CASE(2, 20) OTF_CASE(4, 8) OTF_CASE(4, 20)
#undef OTF_CASE
  throw std::invalid_argument("smo_coop_otf_batch: unsupported tile");
}

}  // namespace hfens
