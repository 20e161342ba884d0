// SVM training kernels (SURVEY.md §2.3 K4 rbf_kernel_tile, K5 smo_step, K6 platt_fit).
//
// One stacking fit of the reference SVC is 36 dual QPs (6 SVC fits × (5 Platt CV folds + the
// final solve)); they are independent, so they run as ONE batched launch with one workgroup
// per problem.
//
//  gram_rbf_batch : K_p[a][b] = exp(-γ_p‖z_a − z_b‖²) for every problem p, rows in the
//                   problem's own (libsvm class-grouped) order so SMO row reads are contiguous.
//                   f32-input MFMA (v_mfma_f32_32x32x2_f32) for the dot products, 64×64 tile
//                   per 256-thread workgroup, diagonal forced to exactly 1 (libsvm's QD).
//  smo_batch      : libsvm Solver::Solve for C-SVC with second-order working-set selection
//                   (WSS3, Fan-Chen-Lin 2005) and libsvm's tie rules (last index wins), no
//                   shrinking.  1024 threads per problem; each thread keeps the gradient G (f64)
//                   of its strided elements in registers (KMAX per thread); α lives in global
//                   memory and only its owner thread touches it; two block arg-reductions and
//                   two contiguous Gram-row reads per iteration.  Ends with calculate_rho.
//  platt_batch    : sigmoid_train (Lin-Lin-Weng 2007 Newton + backtracking), one 1024-thread
//                   workgroup per SVC fit, decision values assembled from svm_dec_batch partials.
// Licence: the pair rule, clipping, sigmoid_train and coupling follow LIBSVM (BSD-3-Clause, Chang & Lin;
// notice in THIRD_PARTY_NOTICES.md at the repository root).
#include "common.h"

namespace hfens {

// ------------------------------------------------------------------------------------------
// Gram matrices
struct GramProb {
  long long zoff;   // first row of this problem in Z (rows of F floats)
  long long koff;   // offset of K_p in the output (floats)
  int l;            // rows
  int ld;           // leading dimension of K_p
  float ngl2e;      // −γ·log2(e)
  int pad;
};

template <int KS>
__global__ __launch_bounds__(256) void gram_rbf_kernel(const float* __restrict__ Z, int F,
                                                       const GramProb* __restrict__ probs,
                                                       float* __restrict__ K) {
  const GramProb P = probs[blockIdx.z];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  if (r0 >= P.l || c0 >= P.l) return;
  __shared__ float As[64][2 * KS + 1];
  __shared__ float Bs[64][2 * KS + 1];
  __shared__ float na[64], nb[64];
  const float* Zp = Z + P.zoff * F;
  for (int e = threadIdx.x; e < 64 * 2 * KS; e += 256) {
    const int r = e / (2 * KS), k = e % (2 * KS);
    As[r][k] = (r0 + r < P.l && k < F) ? Zp[(size_t)(r0 + r) * F + k] : 0.f;
    Bs[r][k] = (c0 + r < P.l && k < F) ? Zp[(size_t)(c0 + r) * F + k] : 0.f;
  }
  __syncthreads();
  if (threadIdx.x < 128) {
    const int r = threadIdx.x & 63;
    const float(*T)[2 * KS + 1] = threadIdx.x < 64 ? As : Bs;
    float s = 0.f;
    for (int k = 0; k < 2 * KS; ++k) s = fmaf(T[r][k], T[r][k], s);
    (threadIdx.x < 64 ? na : nb)[r] = s;
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;
  const int r32 = lane & 31, hi = lane >> 5;
  f32x16 acc = {0.f};
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const float a = As[wr + r32][2 * s + hi];
    const float b = Bs[wc + r32][2 * s + hi];
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
  }
  float* Kp = K + P.koff;
  const int col = c0 + wc + r32;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int ri = wr + (r & 3) + 8 * (r >> 2) + 4 * hi;
    const int row = r0 + ri;
    if (row < P.l && col < P.l) {
      float d2 = fmaf(-2.f, acc[r], na[ri] + nb[wc + r32]);
      d2 = fmaxf(d2, 0.f);
      float v = __builtin_amdgcn_exp2f(P.ngl2e * d2);
      if (row == col) v = 1.f;
      Kp[(size_t)row * P.ld + col] = v;
    }
  }
}

void gram_rbf_batch(uintptr_t Z, int F, uintptr_t probs, int P, int max_l, uintptr_t K,
                    uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F <= 64, "gram_rbf_batch: 1 <= F <= 64");
  const int t = (max_l + 63) / 64;
  dim3 grid(t, t, P);
  const int ks = (F + 1) / 2;
  auto zp = (const float*)Z;
  auto pp = (const GramProb*)probs;
  auto kp = (float*)K;
  hipStream_t st = as_stream(stream);
#define GRAM_CASE(KS_)                                                                   \
  if (ks <= KS_) {                                                                       \
    hipLaunchKernelGGL(gram_rbf_kernel<KS_>, grid, dim3(256), 0, st, zp, F, pp, kp);      \
    launch_check();                                                                      \
    return;                                                                              \
  }
  GRAM_CASE(4) GRAM_CASE(8) GRAM_CASE(12) GRAM_CASE(16) GRAM_CASE(24) GRAM_CASE(32)
#undef GRAM_CASE
}

// ------------------------------------------------------------------------------------------
// SMO
struct SmoProb {
  long long koff;   // K_p offset (floats)
  long long aoff;   // alpha offset (doubles)
  int l;            // problem size
  int ld;           // K_p leading dimension
  int npos;         // indices [0, npos) have y = +1, the rest y = −1
  int pad;
  double Cp, Cn;    // box constraints for y = +1 / y = −1
};

struct SmoOut {
  double* rho;      // [P]
  int* iters;       // [P]
  double* gap;      // [P]  final Gmax + Gmax2
  long long* prof;  // [P][5] s_memtime phase totals (nullptr = off): step2, r2, pair, update, r1
};

constexpr int kSmoThreads = 1024;
constexpr int kSmoWaves = kSmoThreads / 64;
constexpr double kTau = 1e-12;
constexpr double kInf = 1.0e300;

// Block reduction of (a, b, idx): a → max; (b, idx) → arg-max with ties to the larger index.
// Used with a = −∞ when only the arg-max is wanted.  All threads receive the result.
struct Red3 {
  double a, b;
  int idx;
};

__device__ __forceinline__ void red3_combine(Red3& x, double a, double b, int idx) {
  x.a = fmax(x.a, a);
  if (b > x.b || (b == x.b && idx > x.idx)) { x.b = b; x.idx = idx; }
}

// Per-wave partial of a Red3 reduction: order-preserving u64 keys (exact for f64).
struct Red3Part {
  unsigned long long ka, kb;
  int idx, pad;
};

// Block reduction: wave stage on DPP/permlane (u32 max of the key halves, then of the index among
// the lanes holding the arg-max — no LDS round trips), one barrier, then every thread folds the
// kSmoWaves partials.  Callers alternate two partial buffers so consecutive reductions need no
// second barrier.
__device__ __forceinline__ Red3 block_red3(Red3 v, Red3Part* sh) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned long long ka = f64_okey(v.a), kb = f64_okey(v.b);
  const unsigned ah = wave_max_u32((unsigned)(ka >> 32));
  const unsigned al = wave_max_u32((unsigned)(ka >> 32) == ah ? (unsigned)ka : 0u);
  const unsigned bh = wave_max_u32((unsigned)(kb >> 32));
  const unsigned bl = wave_max_u32((unsigned)(kb >> 32) == bh ? (unsigned)kb : 0u);
  const bool top = (unsigned)(kb >> 32) == bh && (unsigned)kb == bl;
  const unsigned bi = wave_max_u32(top ? (unsigned)(v.idx + 1) : 0u);
  if (lane == 0) sh[wave] = Red3Part{((unsigned long long)ah << 32) | al, ((unsigned long long)bh << 32) | bl,
                                     (int)bi - 1, 0};
  __syncthreads();
  Red3Part r = sh[0];
#pragma unroll
  for (int w = 1; w < kSmoWaves; ++w) {
    const Red3Part p = sh[w];
    r.ka = p.ka > r.ka ? p.ka : r.ka;
    if (p.kb > r.kb || (p.kb == r.kb && p.idx > r.idx)) { r.kb = p.kb; r.idx = p.idx; }
  }
  return Red3{f64_from_okey(r.ka), f64_from_okey(r.kb), r.idx};
}

// Element ownership: thread `tid`, group g < K4, lane-of-vector e < 4 owns index
// t = 4·(tid + g·kSmoThreads) + e, so every Gram-row read is one float4 per (thread, group).
template <int K4>
__global__ __launch_bounds__(kSmoThreads) void smo_kernel(const SmoProb* __restrict__ probs,
                                                          const float* __restrict__ K,
                                                          double* __restrict__ alpha_all,
                                                          double eps, long long max_iter,
                                                          SmoOut out) {
  // libsvm's arithmetic (x86-64, no FMA): keep a*b + c*d un-contracted so the gradient path
  // follows the reference bit for bit given the same Gram entries
#pragma clang fp contract(off)
  constexpr int KM = 4 * K4;
  static_assert(KM <= 64, "per-thread element masks are 64-bit");
  const SmoProb P = probs[blockIdx.x];
  const float* Kp = K + P.koff;
  double* alpha = alpha_all + P.aoff;
  const int tid = threadIdx.x;
  __shared__ Red3Part shA[kSmoWaves], shB[kSmoWaves];   // r1 / r2 partials (alternating)
  __shared__ double pub[4];

  double G[KM];
  float Qi[KM];
  unsigned long long ypos = 0ull;   // y_t = +1
  unsigned long long upm = 0ull;    // t ∈ I_up   (y=+1: α<C ; y=−1: α>0)
  unsigned long long lowm = 0ull;   // t ∈ I_low  (y=+1: α>0 ; y=−1: α<C)
  unsigned long long freem = 0ull;  // 0 < α < C
  unsigned long long upperm = 0ull; // α = C
#pragma unroll
  for (int g = 0; g < K4; ++g)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = 4 * g + e;
      const int t = 4 * (tid + g * kSmoThreads) + e;
      G[k] = -1.0;  // p_i = −1 for C-SVC, α = 0
      Qi[k] = 0.f;
      if (t < P.l) {
        alpha[t] = 0.0;
        const bool pos = t < P.npos;
        if (pos) { ypos |= 1ull << k; upm |= 1ull << k; }   // α = 0 is at the lower bound
        else lowm |= 1ull << k;
      }
    }
  // ---- WSS step 1 for the first iteration
  Red3 r1{-kInf, -kInf, -1};
#pragma unroll
  for (int k = 0; k < KM; ++k)
    if ((upm >> k) & 1ull) {
      const int t = 4 * (tid + (k >> 2) * kSmoThreads) + (k & 3);
      red3_combine(r1, -kInf, ((ypos >> k) & 1ull) ? -G[k] : G[k], t);
    }
  r1 = block_red3(r1, shA);
  long long iter = 0;
  double last_gap = 0.0;
  long long ph[5] = {0, 0, 0, 0, 0};
  const bool prof = out.prof != nullptr;
  long long tc = prof ? __builtin_amdgcn_s_memtime() : 0;
  auto tick = [&](int k) {
    if (prof) {
      const long long now = __builtin_amdgcn_s_memtime();
      ph[k] += now - tc;
      tc = now;
    }
  };
  for (; iter < max_iter; ++iter) {
    const double Gmax = r1.b;
    const int i = r1.idx;
    if (i < 0) break;
    const int yi = i < P.npos ? 1 : -1;
    // ---- WSS step 2 over row i (second order, libsvm's "last index wins" on ties).  Every
    // candidate is ranked by the quotient num/quad itself (libsvm's obj_diff, negated exactly), so
    // the choice never depends on how points are grouped over threads or workgroups.
    const float4* Ki4 = reinterpret_cast<const float4*>(Kp + (size_t)i * P.ld);
    double gmax2 = -kInf, bkey = -kInf;
    int bj = -1;
    // issue every row-i load before touching any of them: one HBM latency, not K4
    float4 qv[K4];
#pragma unroll
    for (int g = 0; g < K4; ++g)
      qv[g] = 4 * (tid + g * kSmoThreads) < P.l ? Ki4[tid + g * kSmoThreads] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int g = 0; g < K4; ++g) {
      const int t0 = 4 * (tid + g * kSmoThreads);
      if (t0 < P.l) {
        const float4 q = qv[g];
        Qi[4 * g] = q.x; Qi[4 * g + 1] = q.y; Qi[4 * g + 2] = q.z; Qi[4 * g + 3] = q.w;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = 4 * g + e;
        if ((lowm >> k) & 1ull) {
          const double yG = ((ypos >> k) & 1ull) ? G[k] : -G[k];
          gmax2 = fmax(gmax2, yG);
          const double gd = Gmax + yG;
          if (gd > 0) {
            double quad = 2.0 - 2.0 * (double)Qi[k];
            if (quad <= 0) quad = kTau;
            const double key = (gd * gd) / quad;
            if (bj < 0 || key >= bkey) { bkey = key; bj = t0 + e; }   // ties → later index
          }
        }
      }
    }
    Red3 r2{gmax2, bj >= 0 ? bkey : -kInf, bj};
    tick(0);
    r2 = block_red3(r2, shB);
    tick(1);
    const int j = r2.idx;
    last_gap = Gmax + r2.a;
    if (Gmax + r2.a < eps || j < 0) break;
    // ---- publish α_i (owner of i) and α_j, K_ij, G_j (owner of j); G_i = −y_i·Gmax exactly
    const int oi = (i >> 2) % kSmoThreads, oj = (j >> 2) % kSmoThreads;
    if (tid == oi) pub[0] = alpha[i];
    if (tid == oj) {
      pub[1] = alpha[j];
      const int kk = 4 * ((j >> 2) / kSmoThreads) + (j & 3);
      float kij = 0.f;
      double gj = 0.0;
#pragma unroll
      for (int k = 0; k < KM; ++k)
        if (k == kk) { kij = Qi[k]; gj = G[k]; }
      pub[2] = kij;
      pub[3] = gj;
    }
    __syncthreads();
    const double ai_old = pub[0], aj_old = pub[1];
    const double Kij = pub[2];
    const double Gj = pub[3];
    const int yj = j < P.npos ? 1 : -1;
    const double Ci = yi > 0 ? P.Cp : P.Cn, Cj = yj > 0 ? P.Cp : P.Cn;
    const double Qij = (double)(yi * yj) * Kij;
    const double Gi = -(double)yi * Gmax;
    double ai = ai_old, aj = aj_old;
    if (yi != yj) {
      double quad = 2.0 + 2.0 * Qij;
      if (quad <= 0) quad = kTau;
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
      if (quad <= 0) quad = kTau;
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
    // owners: store α and refresh the bound masks of i and j
    if (tid == oi || tid == oj) {
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        const int t = w == 0 ? i : j;
        if ((w == 0 && tid != oi) || (w == 1 && tid != oj)) continue;
        const double a = w == 0 ? ai : aj;
        const double C = w == 0 ? Ci : Cj;
        alpha[t] = a;
        const int kk = 4 * ((t >> 2) / kSmoThreads) + (t & 3);
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
    }
    tick(2);
    // ---- fused: gradient update with rows i (registers) and j, then next step-1 candidates
    const float4* Kj4 = reinterpret_cast<const float4*>(Kp + (size_t)j * P.ld);
    r1 = Red3{-kInf, -kInf, -1};
    float4 qjv[K4];
#pragma unroll
    for (int g = 0; g < K4; ++g)
      qjv[g] = 4 * (tid + g * kSmoThreads) < P.l ? Kj4[tid + g * kSmoThreads] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int g = 0; g < K4; ++g) {
      const int t0 = 4 * (tid + g * kSmoThreads);
      const float4 q = qjv[g];
      const float qj[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = 4 * g + e;
        const bool pos = (ypos >> k) & 1ull;
        const double upd = (double)Qi[k] * ci + (double)qj[e] * cj;
        G[k] += pos ? upd : -upd;
        if ((upm >> k) & 1ull) red3_combine(r1, -kInf, pos ? -G[k] : G[k], t0 + e);
      }
    }
    tick(3);
    r1 = block_red3(r1, shA);
    tick(4);
  }
  if (prof && tid == 0)
    for (int k = 0; k < 5; ++k) out.prof[blockIdx.x * 5 + k] = ph[k];
  // ---- calculate_rho
  Red3 ru{-kInf, -kInf, -1};   // a = max(−ub)
  Red3 rl{-kInf, -kInf, -1};   // a = max(lb)
  double sum_free = 0.0;
  int nfree = 0;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int t = 4 * (tid + (k >> 2) * kSmoThreads) + (k & 3);
    if (t < P.l) {
      const bool pos = (ypos >> k) & 1ull;
      const double yG = pos ? G[k] : -G[k];
      if ((upperm >> k) & 1ull) {
        if (!pos) ru.a = fmax(ru.a, -yG); else rl.a = fmax(rl.a, yG);
      } else if ((freem >> k) & 1ull) {
        ++nfree;
        sum_free += yG;
      } else {
        if (pos) ru.a = fmax(ru.a, -yG); else rl.a = fmax(rl.a, yG);
      }
    }
  }
  __syncthreads();   // the loop may exit right after an r1 fold that still reads shA
  ru = block_red3(ru, shA);
  rl = block_red3(rl, shB);
  Red3 rs{-kInf, sum_free, nfree};
  {
    // plain sums (not arg-max): reuse the shared buffer with a sum reduction
    double s = wave_sum(sum_free);
    double c = wave_sum((double)nfree);
    const int lane = tid & 63, wave = tid >> 6;
    __shared__ double ssum[2][kSmoWaves];
    if (lane == 0) { ssum[0][wave] = s; ssum[1][wave] = c; }
    __syncthreads();
    if (tid == 0) {
      double S = 0, Cc = 0;
      for (int w = 0; w < kSmoWaves; ++w) { S += ssum[0][w]; Cc += ssum[1][w]; }
      const double ub = -ru.a, lb = rl.a;
      out.rho[blockIdx.x] = Cc > 0 ? S / Cc : (ub + lb) / 2;
      out.iters[blockIdx.x] = (int)iter;
      out.gap[blockIdx.x] = last_gap;
    }
  }
  (void)rs;
}

void smo_batch(uintptr_t probs, int P, int max_l, uintptr_t K, uintptr_t alpha, double eps,
               long long max_iter, uintptr_t rho, uintptr_t iters, uintptr_t gap, uintptr_t prof,
               uintptr_t stream) {
  SmoOut o{(double*)rho, (int*)iters, (double*)gap, (long long*)prof};
  auto pp = (const SmoProb*)probs;
  auto kp = (const float*)K;
  auto ap = (double*)alpha;
  hipStream_t st = as_stream(stream);
#define SMO_CASE(K4)                                                                        \
  if (max_l <= 4 * K4 * kSmoThreads) {                                                      \
    hipLaunchKernelGGL(smo_kernel<K4>, dim3(P), dim3(kSmoThreads), 0, st, pp, kp, ap, eps,  \
                       max_iter, o);                                                        \
    launch_check();                                                                         \
    return;                                                                                 \
  }
  SMO_CASE(1) SMO_CASE(2) SMO_CASE(3) SMO_CASE(4) SMO_CASE(6) SMO_CASE(8)
#undef SMO_CASE
  throw std::invalid_argument("smo_batch: problem larger than 32768 points on the register path");
}

// ------------------------------------------------------------------------------------------
// Batched decision values of many sub-models on their held-out rows (the Platt CV step):
//   part[row][s] = Σ_{t ∈ split s} coef_p[t]·exp(-γ_p‖h_row − z_t‖²)
// for every problem p (SVs = the problem's training rows in zcat, coef = y·α, zero for non-SVs).
// grid = (128-row held tiles, SV splits, problems); per split the SVs stream through LDS in
// k-major chunks; f32-input MFMA as in rbf_decision.  Partials are summed on the host side in a
// fixed order (deterministic).
struct DecProb {
  long long zoff;   // first SV row in zcat
  long long hoff;   // first held row in hcat
  int l;            // SVs
  int h;            // held rows
  float ngl2e;
  int per;          // SVs per split (multiple of 32)
};

// Support-vector compaction ahead of the decisions: problem p's rows with a non-zero coefficient
// (y·α ≠ 0; ≈ 45 % of the points on the bench's problems), in their original order, copied to the
// same offsets of zc / cc, their count to counts[p].  One 1024-thread workgroup per problem: a
// ballot + wave-prefix compaction per 1024-point chunk.  The decision terms of the skipped points
// are exact zeros, so only the grouping of the f32 partial sums changes.
__global__ __launch_bounds__(1024) void svm_sv_compact_kernel(const float* __restrict__ zcat,
                                                             const float* __restrict__ coef, int F,
                                                             const DecProb* __restrict__ probs,
                                                             float* __restrict__ zc, float* __restrict__ cc,
                                                             int* __restrict__ counts) {
  const DecProb P = probs[blockIdx.x];
  __shared__ int wtot[16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int base = 0;
  for (int c0 = 0; c0 < P.l; c0 += 1024) {
    const int t = c0 + threadIdx.x;
    const float cf = t < P.l ? coef[P.zoff + t] : 0.f;
    const bool sv = cf != 0.f;
    const unsigned long long bal = __ballot(sv);
    if (lane == 0) wtot[wave] = __popcll(bal);
    __syncthreads();
    int wb = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) {
      const int v = wtot[w];
      wb += w < wave ? v : 0;
      tot += v;
    }
    if (sv) {
      const long long pos = P.zoff + base + wb + __popcll(bal & ((1ull << lane) - 1ull));
      const float* src = zcat + (P.zoff + t) * F;
      float* dst = zc + pos * F;
      for (int k = 0; k < F; ++k) dst[k] = src[k];
      cc[pos] = cf;
    }
    base += tot;
    __syncthreads();   // wtot is rewritten by the next chunk
  }
  if (threadIdx.x == 0) counts[blockIdx.x] = base;
}

void svm_sv_compact(uintptr_t zcat, uintptr_t coef, int F, uintptr_t probs, int P, uintptr_t zc, uintptr_t cc,
                    uintptr_t counts, uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F <= 64 && P >= 0, "svm_sv_compact: 1 <= F <= 64");
  if (P == 0) return;
  hipLaunchKernelGGL(svm_sv_compact_kernel, dim3(P), dim3(1024), 0, as_stream(stream), (const float*)zcat,
                     (const float*)coef, F, (const DecProb*)probs, (float*)zc, (float*)cc, (int*)counts);
  launch_check();
}

template <int KS>
__global__ __launch_bounds__(256) void svm_dec_batch_kernel(const float* __restrict__ zcat,
                                                            const float* __restrict__ coef,
                                                            const float* __restrict__ hcat, int F,
                                                            const DecProb* __restrict__ probs,
                                                            int S, float* __restrict__ part,
                                                            const int* __restrict__ counts) {
  const DecProb P = probs[blockIdx.z];
  const int row0 = blockIdx.x * 128;
  const int s = blockIdx.y;
  const int t_begin = s * P.per;
  // (counts: the compacted support vectors of each problem, svm_sv_compact; splits past them write
  // nothing — the caller's partials are zero-filled)
  const int L = counts != nullptr ? min(counts[blockIdx.z], P.l) : P.l;
  if (row0 >= P.h || t_begin >= L) return;
  const int t_end = min(L, t_begin + P.per);
  constexpr int CH = 256;
  __shared__ __attribute__((aligned(16))) float sv_l[2 * KS][CH];
  __shared__ __attribute__((aligned(16))) float sn_l[CH];
  __shared__ __attribute__((aligned(16))) float cf_l[CH];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r32 = lane & 31, hi = lane >> 5;
  const int row = row0 + wave * 32 + r32;
  float z[KS];
  float znp = 0.f;
#pragma unroll
  for (int q = 0; q < KS; ++q) {
    const int k = 2 * q + hi;
    z[q] = (row < P.h && k < F) ? hcat[(size_t)(P.hoff + row) * F + k] : 0.f;
    znp = fmaf(z[q], z[q], znp);
  }
  const float zn = znp + __shfl_xor(znp, 32, kWave);
  float acc_part = 0.f;
  for (int c0 = t_begin; c0 < t_end; c0 += CH) {
    const int cl = min(CH, t_end - c0);
    const int clp = (cl + 31) / 32 * 32;
    __syncthreads();
    for (int e = threadIdx.x; e < 2 * KS * CH; e += 256) {
      const int k = e / CH, j = e % CH;
      sv_l[k][j] = (j < cl && k < F) ? zcat[(size_t)(P.zoff + c0 + j) * F + k] : 0.f;
    }
    for (int j = threadIdx.x; j < CH; j += 256) cf_l[j] = j < cl ? coef[P.zoff + c0 + j] : 0.f;
    __syncthreads();
    for (int j = threadIdx.x; j < CH; j += 256) {
      float a = 0.f;
      for (int k = 0; k < 2 * KS; ++k) a = fmaf(sv_l[k][j], sv_l[k][j], a);
      sn_l[j] = a;
    }
    __syncthreads();
    for (int t = 0; t < clp; t += 32) {
      f32x16 acc = {0.f};
#pragma unroll
      for (int q = 0; q < KS; ++q)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(sv_l[2 * q + hi][t + r32], z[q], acc, 0, 0, 0);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int b0 = t + 8 * g + 4 * hi;
        const f32x4 snv = *reinterpret_cast<const f32x4*>(&sn_l[b0]);
        const f32x4 cfv = *reinterpret_cast<const f32x4*>(&cf_l[b0]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float d2 = fmaxf(fmaf(-2.f, acc[4 * g + q], snv[q] + zn), 0.f);
          acc_part = fmaf(cfv[q], __builtin_amdgcn_exp2f(P.ngl2e * d2), acc_part);
        }
      }
    }
  }
  acc_part += __shfl_xor(acc_part, 32, kWave);
  if (hi == 0 && row < P.h) part[(size_t)(P.hoff + row) * S + s] = acc_part;
}

void svm_dec_batch(uintptr_t zcat, uintptr_t coef, uintptr_t hcat, int F, uintptr_t probs, int P,
                   int max_h, int S, uintptr_t part, uintptr_t counts, uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F <= 64, "svm_dec_batch: 1 <= F <= 64");
  dim3 grid((max_h + 127) / 128, S, P);
  const int ks = (F + 1) / 2;
  hipStream_t st = as_stream(stream);
#define DEC_CASE(KS_)                                                                            \
  if (ks <= KS_) {                                                                               \
    hipLaunchKernelGGL(svm_dec_batch_kernel<KS_>, grid, dim3(256), 0, st, (const float*)zcat,    \
                       (const float*)coef, (const float*)hcat, F, (const DecProb*)probs, S,      \
                       (float*)part, (const int*)counts);                                        \
    launch_check();                                                                              \
    return;                                                                                      \
  }
  DEC_CASE(4) DEC_CASE(8) DEC_CASE(9) DEC_CASE(12) DEC_CASE(16) DEC_CASE(20) DEC_CASE(24) DEC_CASE(32)
#undef DEC_CASE
}

// ------------------------------------------------------------------------------------------
// Platt scaling: sigmoid_train (libsvm svm.cpp sigmoid_train; reference SVC(probability=True),
// train_ensemble_public.py:44) on one fit's cross-validated decision values, one 1024-thread
// workgroup per fit.
//
// The decision values are assembled in the kernel from the batched decision launch's f32
// partials (svm_dec_batch: part[row][S]) — d = −(Σ_s part[row][s] − ρ_k), the 1024-point partials
// summed in f64 in s order — following a host-built map from the fit's grouped positions to
// partial rows (code ≥ 0) or to a per-fold constant (code < 0: −1 − code indexes consts; a
// degenerate fold's decision value).  Labels are implied by the grouped order (position < n0 ⇒
// +1).  Up to kPlattReg·1024 points the values stay in registers for the whole Newton solve;
// larger fits keep them in the global scratch `dec`.
//
// Each Newton iteration of libsvm's loop is ONE pass over the points: the line search's trial
// objective at (A + s·dA, B + s·dB) also accumulates the Hessian and gradient there (one exp and
// one log per point, shared), which the next iteration uses when the trial is accepted — the
// same accepted iterates as the two-pass loop.  Six sums per pass, one barrier (double-buffered
// reduction slots).
struct PlattProb {
  long long off;  // offset into the fit-concatenated position arrays (srcmap / dec)
  int l;          // points of the fit
  int n0;         // positions < n0 carry label +1
};

constexpr int kPlattThreads = 1024;
constexpr int kPlattWaves = kPlattThreads / 64;
constexpr int kPlattReg = 16;

struct PlattSums {
  double f, h11, h22, h21, g1, g2;
};

__device__ __forceinline__ void platt_point(double d, double t, double a, double b, PlattSums& acc) {
  const double fApB = d * a + b;
  double p, q;
  if (fApB >= 0) {
    const double e = exp(-fApB);
    acc.f += t * fApB + log(1 + e);
    p = e / (1.0 + e);
    q = 1.0 / (1.0 + e);
  } else {
    const double e = exp(fApB);
    acc.f += (t - 1) * fApB + log(1 + e);
    p = 1.0 / (1.0 + e);
    q = e / (1.0 + e);
  }
  const double d2 = p * q;
  acc.h11 += d * d * d2;
  acc.h22 += d2;
  acc.h21 += d * d2;
  const double d1 = t - p;
  acc.g1 += d * d1;
  acc.g2 += d1;
}

__device__ __forceinline__ PlattSums platt_block_sum(PlattSums v, double* red, int& parity) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double* r = red + parity * (kPlattWaves * 6);
  parity ^= 1;
  const double w[6] = {wave_sum(v.f), wave_sum(v.h11), wave_sum(v.h22), wave_sum(v.h21), wave_sum(v.g1),
                       wave_sum(v.g2)};
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 6; ++k) r[wave * 6 + k] = w[k];
  }
  __syncthreads();
  double o[6] = {0, 0, 0, 0, 0, 0};
  for (int q = 0; q < kPlattWaves; ++q) {
#pragma unroll
    for (int k = 0; k < 6; ++k) o[k] += r[q * 6 + k];
  }
  return PlattSums{o[0], o[1], o[2], o[3], o[4], o[5]};
}

template <bool Reg>
__global__ __launch_bounds__(kPlattThreads) void platt_kernel(const PlattProb* __restrict__ probs,
                                                              const float* __restrict__ part, int S,
                                                              const int* __restrict__ rowk,
                                                              const double* __restrict__ rho,
                                                              const double* __restrict__ consts,
                                                              const int* __restrict__ srcmap,
                                                              double* __restrict__ dec,
                                                              double* __restrict__ AB) {
  const PlattProb P = probs[blockIdx.x];
  if (Reg != (P.l <= kPlattReg * kPlattThreads)) return;   // the other instantiation's fit
  __shared__ double red[2 * kPlattWaves * 6];
  const int tid = threadIdx.x;
  double dr[Reg ? kPlattReg : 1];
  double* dg = dec + P.off;
#pragma unroll
  for (int k = 0; k < (Reg ? kPlattReg : 1); ++k) dr[k] = 0.0;
  auto value = [&](int i) {
    const int code = srcmap[P.off + i];
    if (code < 0) return consts[-1 - code];
    double sum = 0.0;
    for (int j = 0; j < S; ++j) sum += (double)part[(size_t)code * S + j];
    return -(sum - rho[rowk[code]]);
  };
  if constexpr (Reg) {
#pragma unroll
    for (int k = 0; k < kPlattReg; ++k) {
      const int i = tid + k * kPlattThreads;
      if (i < P.l) dr[k] = value(i);
    }
  } else {
    for (int i = tid; i < P.l; i += kPlattThreads) dg[i] = value(i);
  }
  if constexpr (!Reg) __threadfence_block();
  __syncthreads();
  const double prior1 = P.n0, prior0 = P.l - P.n0;
  const int max_iter = 100;
  const double min_step = 1e-10, sigma = 1e-12, eps = 1e-5;
  const double hiT = (prior1 + 1.0) / (prior1 + 2.0), loT = 1 / (prior0 + 2.0);
  int parity = 0;
  auto pass = [&](double a, double b) {
    PlattSums acc{0, 0, 0, 0, 0, 0};
    if constexpr (Reg) {
#pragma unroll
      for (int k = 0; k < kPlattReg; ++k) {
        const int i = tid + k * kPlattThreads;
        if (i < P.l) platt_point(dr[k], i < P.n0 ? hiT : loT, a, b, acc);
      }
    } else {
      for (int i = tid; i < P.l; i += kPlattThreads) platt_point(dg[i], i < P.n0 ? hiT : loT, a, b, acc);
    }
    return platt_block_sum(acc, red, parity);
  };
  double A = 0.0, B = log((prior0 + 1.0) / (prior1 + 1.0));
  PlattSums v = pass(A, B);
  double fval = v.f;
  for (int it = 0; it < max_iter; ++it) {
    const double h11 = v.h11 + sigma, h22 = v.h22 + sigma, h21 = v.h21, g1 = v.g1, g2 = v.g2;
    if (fabs(g1) < eps && fabs(g2) < eps) break;
    const double det = h11 * h22 - h21 * h21;
    const double dA = -(h22 * g1 - h21 * g2) / det;
    const double dB = -(-h21 * g1 + h11 * g2) / det;
    const double gd = g1 * dA + g2 * dB;
    double step = 1;
    while (step >= min_step) {
      const double nA = A + step * dA, nB = B + step * dB;
      const PlattSums w = pass(nA, nB);
      if (w.f < fval + 0.0001 * step * gd) { A = nA; B = nB; fval = w.f; v = w; break; }
      step = step / 2.0;
    }
    if (step < min_step) break;
  }
  if (tid == 0) { AB[2 * blockIdx.x] = A; AB[2 * blockIdx.x + 1] = B; }
}

// The same Newton loop with each fit's points split over NWG workgroups (the single-workgroup kernel
// runs six fits on six CUs, its passes bound by one CU's f64 exp / log throughput).  Per pass every
// workgroup reduces its own points, publishes the six sums in a parity slot and meets the fit's other
// workgroups at a counter (vector atomics, agent scope); every workgroup then adds the NWG partials in
// workgroup order — the same sums, hence the same iterates, in every workgroup; workgroup 0 writes
// (A, B).  A counter wait past kPlattCoopDeadline (10 ms: workgroups not co-resident) turns that
// workgroup into a solo one that sums all the fit's points itself from then on — slower, same result
// up to the summation order, never stuck.
constexpr int kPlattCoopWgs = 8;
constexpr long long kPlattCoopDeadline = 1000000;   // 100 MHz real-time ticks

template <int NWG>
__global__ __launch_bounds__(kPlattThreads) void platt_coop_kernel(const PlattProb* __restrict__ probs,
                                                                   const float* __restrict__ part, int S,
                                                                   const int* __restrict__ rowk,
                                                                   const double* __restrict__ rho,
                                                                   const double* __restrict__ consts,
                                                                   const int* __restrict__ srcmap,
                                                                   double* __restrict__ AB, int* __restrict__ bar,
                                                                   double* __restrict__ cpart) {
  constexpr int R = (kPlattReg + NWG - 1) / NWG;   // register slots per thread for this workgroup's chunk
  const int g = blockIdx.x, fit = blockIdx.y;
  const PlattProb P = probs[fit];
  if (P.l > R * kPlattThreads * NWG || P.l > kPlattReg * kPlattThreads) return;   // (the scratch kernel's fits)
  __shared__ double red[2 * kPlattWaves * 6];
  __shared__ int s_solo;
  const int tid = threadIdx.x;
  const int chunk = (P.l + NWG - 1) / NWG;
  const int lo = g * chunk, hi = min(P.l, lo + chunk);
  auto value = [&](int i) {
    const int code = srcmap[P.off + i];
    if (code < 0) return consts[-1 - code];
    double sum = 0.0;
    for (int j = 0; j < S; ++j) sum += (double)part[(size_t)code * S + j];
    return -(sum - rho[rowk[code]]);
  };
  double dr[R];
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int i = lo + tid + k * kPlattThreads;
    dr[k] = i < hi ? value(i) : 0.0;
  }
  if (tid == 0) s_solo = 0;
  __syncthreads();
  const double prior1 = P.n0, prior0 = P.l - P.n0;
  const int max_iter = 100;
  const double min_step = 1e-10, sigma = 1e-12, eps = 1e-5;
  const double hiT = (prior1 + 1.0) / (prior1 + 2.0), loT = 1 / (prior0 + 2.0);
  int parity = 0, npass = 0;
  bool solo = false;
  auto pass = [&](double a, double b) {
    PlattSums acc{0, 0, 0, 0, 0, 0};
    if (!solo) {
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const int i = lo + tid + k * kPlattThreads;
        if (i < hi) platt_point(dr[k], i < P.n0 ? hiT : loT, a, b, acc);
      }
      const PlattSums loc = platt_block_sum(acc, red, parity);
      double* slot = cpart + ((size_t)(fit * 2 + (npass & 1)) * NWG) * 6;
      if (tid == 0) {
        const double v[6] = {loc.f, loc.h11, loc.h22, loc.h21, loc.g1, loc.g2};
#pragma unroll
        for (int k = 0; k < 6; ++k) __hip_atomic_store(slot + g * 6 + k, v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __threadfence();
        __hip_atomic_fetch_add(bar + fit, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        const int target = (npass + 1) * NWG;
        const long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(bar + fit, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
          if (__builtin_amdgcn_s_memrealtime() - t0 > kPlattCoopDeadline) { s_solo = 1; break; }
          __builtin_amdgcn_s_sleep(1);
        }
        __threadfence();
      }
      __syncthreads();
      ++npass;
      if (!s_solo) {
        double o[6] = {0, 0, 0, 0, 0, 0};
        for (int q = 0; q < NWG; ++q) {
#pragma unroll
          for (int k = 0; k < 6; ++k) o[k] += __hip_atomic_load(slot + q * 6 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return PlattSums{o[0], o[1], o[2], o[3], o[4], o[5]};
      }
      solo = true;
      acc = PlattSums{0, 0, 0, 0, 0, 0};
    }
    // solo: every point of the fit, values re-assembled from the partials
    for (int i = tid; i < P.l; i += kPlattThreads) platt_point(value(i), i < P.n0 ? hiT : loT, a, b, acc);
    return platt_block_sum(acc, red, parity);
  };
  double A = 0.0, B = log((prior0 + 1.0) / (prior1 + 1.0));
  PlattSums v = pass(A, B);
  double fval = v.f;
  for (int it = 0; it < max_iter; ++it) {
    const double h11 = v.h11 + sigma, h22 = v.h22 + sigma, h21 = v.h21, g1 = v.g1, g2 = v.g2;
    if (fabs(g1) < eps && fabs(g2) < eps) break;
    const double det = h11 * h22 - h21 * h21;
    const double dA = -(h22 * g1 - h21 * g2) / det;
    const double dB = -(-h21 * g1 + h11 * g2) / det;
    const double gd = g1 * dA + g2 * dB;
    double step = 1;
    while (step >= min_step) {
      const double nA = A + step * dA, nB = B + step * dB;
      const PlattSums w = pass(nA, nB);
      if (w.f < fval + 0.0001 * step * gd) { A = nA; B = nB; fval = w.f; v = w; break; }
      step = step / 2.0;
    }
    if (step < min_step) break;
  }
  if (tid == 0 && g == 0) { AB[2 * fit] = A; AB[2 * fit + 1] = B; }
}

void platt_batch(uintptr_t probs, int P, uintptr_t part, int S, uintptr_t rowk, uintptr_t rho,
                 uintptr_t consts, uintptr_t srcmap, uintptr_t dec, uintptr_t AB, uintptr_t coop_bar,
                 uintptr_t coop_part, uintptr_t stream) {
  HFENS_REQUIRE(P >= 1 && S >= 0, "platt_batch: P >= 1, S >= 0");
  hipStream_t st = as_stream(stream);
  // two launches on one stream, each skipping the other's fits: register-resident values for
  // fits of ≤ 16k points (split over kPlattCoopWgs workgroups each when coop_bar is given: a zeroed
  // int[P] counter array and a double[P][2][kPlattCoopWgs][6] partial buffer), the global scratch beyond
  if (coop_bar != 0) {
    hipLaunchKernelGGL(platt_coop_kernel<kPlattCoopWgs>, dim3(kPlattCoopWgs, P), dim3(kPlattThreads), 0, st,
                       (const PlattProb*)probs, (const float*)part, S, (const int*)rowk, (const double*)rho,
                       (const double*)consts, (const int*)srcmap, (double*)AB, (int*)coop_bar, (double*)coop_part);
  } else {
    hipLaunchKernelGGL(platt_kernel<true>, dim3(P), dim3(kPlattThreads), 0, st, (const PlattProb*)probs,
                       (const float*)part, S, (const int*)rowk, (const double*)rho, (const double*)consts,
                       (const int*)srcmap, (double*)dec, (double*)AB);
  }
  launch_check();
  hipLaunchKernelGGL(platt_kernel<false>, dim3(P), dim3(kPlattThreads), 0, st, (const PlattProb*)probs,
                     (const float*)part, S, (const int*)rowk, (const double*)rho, (const double*)consts,
                     (const int*)srcmap, (double*)dec, (double*)AB);
  launch_check();
}

}  // namespace hfens
