// Fused batched logistic regression (reference train_ensemble_public.py:46
// 'lg' = LogisticRegression(penalty='l1', solver='liblinear') and :48, the L2 meta-learner).
//
// logreg_fused runs the whole outer solve of models/logreg_solver.py for B models in ONE launch,
// one 1024-thread workgroup per model.  The host loop it replaces issues ~20 small kernels and
// three blocking host reads per outer iteration (host-bound: ≈1.5 ms per iteration on the
// bench's 6-model batch); here every iteration is three in-workgroup passes:
//   A  margins → σ, Hessian weights D = s·σ(1−σ) and gradient coefficients s·(σ−1)·y; the upper
//      triangle of H = C·X̃ᵀDX̃ and g = C·X̃ᵀr from rows staged through LDS in chunks — every
//      thread owns one (pair, row-group) task and the row-group partials fold in a fixed order
//      (deterministic for any launch);
//   B  stopping rule and subproblem: L1 → cyclic coordinate descent on the prox-Newton QP on
//      wave 0 (l1_qp_cd's owner-lane steps, H in LDS, next column prefetched); L2 → Cholesky
//      solve of (H + diag(pen)) d = −(g + pen·w);
//   C  Armijo line search over the 8 steps 2^-k in one pass (X̃d kept for the margin update).
// Stopping rules, step rule and constants are logreg_solver.py's, applied per model (a model
// stops when IT has converged, not when the whole batch has).
#include "common.h"
#include "l1qp.h"

namespace hfens {

constexpr int kLrThreads = 1024;
constexpr int kLrWaves = kLrThreads / 64;
constexpr int kLrSteps = 8;

struct LrJob {
  const double* X;             // [n][F1] augmented rows (row-major)
  const double* s;             // [B][n] sample weights (0 = row not in the model)
  const double* ypm;           // [n] labels ±1
  const unsigned char* penal;  // [F1] 1 = coordinate penalised
  double* Z;                   // [B][n] margin scratch
  double* Xd;                  // [B][n] direction scratch
  double* W;                   // [B][F1] solution
  int* iters;                  // [B] outer iterations
  double C;
  int n, F1, l1, max_outer, CR;  // CR: rows per LDS chunk
  // cooperative variant (logreg_coop): M members per model, member w owns rows [w·S, (w+1)·S)
  int B, M, S, nvmax;            // M members per model; nvmax: exchange values per member slot
  unsigned long long* xchg;      // [B][2][M][nvmax][2] epoch-tagged granules
  unsigned* err;                 // [1] set on a member-exchange timeout
};

constexpr int kLrMaxMembers = 16;
constexpr unsigned kLrSpinLimit = 1u << 22;
typedef __attribute__((address_space(1))) unsigned long long lr_gu64_t;

__device__ __forceinline__ void lr_put(unsigned long long* g, unsigned epoch, unsigned v) {
  __hip_atomic_store((lr_gu64_t*)g, ((unsigned long long)epoch << 32) | v, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// Member exchange of NV doubles (LDS v[0..NV): this member's partials in, the sums over all
// members out).  Each value is published as two epoch-tagged granules (agent-scope relaxed
// atomic stores: data and tag travel together, no fence or flag); every thread then polls the W
// members' granules of its values and sums them in member order 0..W−1, so every member gets
// bit-identical totals.  Slots alternate by epoch parity: a member reaches exchange e+2 only after
// every member published e+1, i.e. finished reading e.  false = a peer never arrived (timeout).
__device__ bool lr_exchange(double* v, int NV, const LrJob& J, int b, int w, unsigned& epoch, int* fail) {
  ++epoch;
  unsigned long long* slot = J.xchg + ((size_t)b * 2 + (epoch & 1)) * J.M * J.nvmax * 2;
  for (int k = threadIdx.x; k < NV; k += kLrThreads) {
    const unsigned long long x = (unsigned long long)__double_as_longlong(v[k]);
    unsigned long long* g = slot + ((size_t)w * J.nvmax + k) * 2;
    lr_put(g, epoch, (unsigned)x);
    lr_put(g + 1, epoch, (unsigned)(x >> 32));
  }
  bool ok_all = true;
  for (int k = threadIdx.x; k < NV && ok_all; k += kLrThreads) {
    unsigned lo[kLrMaxMembers], hi[kLrMaxMembers];
    unsigned spins = 0;
    for (;;) {
      bool ok = true;
#pragma unroll
      for (int m = 0; m < kLrMaxMembers; ++m) {
        if (m >= J.M) break;
        const unsigned long long* g = slot + ((size_t)m * J.nvmax + k) * 2;
        const unsigned long long a = __hip_atomic_load((lr_gu64_t*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long c = __hip_atomic_load((lr_gu64_t*)(g + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        lo[m] = (unsigned)a;
        hi[m] = (unsigned)c;
        ok = ok && (unsigned)(a >> 32) == epoch && (unsigned)(c >> 32) == epoch;
      }
      if (ok) break;
      if (++spins > kLrSpinLimit) {
        atomicOr(J.err, 1u);
        ok_all = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (!ok_all) break;
    double tot = 0.0;
#pragma unroll
    for (int m = 0; m < kLrMaxMembers; ++m) {
      if (m >= J.M) break;
      tot += __longlong_as_double((long long)((unsigned long long)lo[m] | ((unsigned long long)hi[m] << 32)));
    }
    v[k] = tot;
  }
  if (!ok_all) *fail = 1;
  __syncthreads();
  return *fail == 0;
}

__device__ __forceinline__ double lr_softplus(double x) {  // log(1 + e^x), overflow-free
  return x > 0 ? x + log1p(exp(-x)) : log1p(exp(x));
}

// Workgroup sum of NV per-thread values into out[0..NV) (LDS), valid for every thread on return.
template <int NV>
__device__ __forceinline__ void lr_block_sum(const double (&v)[NV], double* red, double* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const double t = wave_sum(v[k]);
    if (lane == 0) red[wave * NV + k] = t;
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    double t = 0.0;
    for (int w = 0; w < kLrWaves; ++w) t += red[w * NV + threadIdx.x];
    out[threadIdx.x] = t;
  }
  __syncthreads();
}

// Coop = false: logreg_fused, one workgroup per model (blockIdx.x = model).  Coop = true:
// logreg_coop, W workgroups ("members") per model on one XCD (blocks b, b+8, … share an XCD under
// round-robin dispatch — speed only), each owning a row slab; the two row reductions of an
// iteration (A: H, g, loss; C: the 8 trial losses) become member exchanges with ordered sums, and
// every member runs the small subproblem B itself on identical data, so all members take the same
// steps.  Members spin on each other: the host admits B·W ≤ CUs and launches it only when no other
// cooperative kernel shares the device.
template <bool Coop>
__global__ __launch_bounds__(kLrThreads) void logreg_fused_kernel(LrJob J) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int b = blockIdx.x, w = 0;
  if constexpr (Coop) {
    const int xcd = blockIdx.x & 7, q = blockIdx.x >> 3;
    b = xcd + 8 * (q / J.M);
    w = q % J.M;
    if (b >= J.B) return;
  }
  const int n = J.n, F1 = J.F1, CR = J.CR;
  const int r0 = Coop ? min(n, w * J.S) : 0, r1 = Coop ? min(n, r0 + J.S) : n;
  __shared__ int xfail;
  unsigned epoch = 0;
  const int npairs = F1 * (F1 + 1) / 2, T = npairs + F1;
  double* xs = sm;                          // [CR][F1] row chunk
  double* dv = xs + (size_t)CR * F1;        // [CR] Hessian weights of the chunk's rows
  double* cv = dv + CR;                     // [CR] gradient coefficients
  double* H = cv + CR;                      // [F1][F1]
  double* gr = H + F1 * F1;                 // [F1] gradient
  double* dd = gr + F1;                     // [F1] search direction
  double* Wl = dd + F1;                     // [F1] current solution
  double* part = Wl + F1;                   // [kLrThreads] row-group partials
  double* red = part + kLrThreads;          // [kLrWaves][kLrSteps]
  double* sc = red + kLrWaves * kLrSteps;   // [16] scalars: 0 stop, 1 delta, 2 reg0, 8.. sums
  double* mv = sc + 16;                     // [T + 1] member partials of H, g and the loss
  unsigned char* pi = reinterpret_cast<unsigned char*>(mv + T + 1);
  unsigned char* pj = pi + npairs;
  const double* s = J.s + (size_t)b * n;
  double* Z = J.Z + (size_t)b * n;
  double* Xd = J.Xd + (size_t)b * n;
  const double C = J.C;
  for (int k = tid; k < npairs; k += kLrThreads) {   // upper triangle, row-major
    int i = 0, rem = k;
    while (rem >= F1 - i) { rem -= F1 - i; ++i; }
    pi[k] = (unsigned char)i;
    pj[k] = (unsigned char)(i + rem);
  }
  for (int f = tid; f < F1; f += kLrThreads) Wl[f] = 0.0;
  for (int r = r0 + tid; r < r1; r += kLrThreads) Z[r] = 0.0;
  if (tid == 0) xfail = 0;
  // moment tasks: T ≤ kLrThreads → G row groups of T tasks each; otherwise ≤ 3 tasks per thread
  const int G = T >= kLrThreads ? 1 : kLrThreads / T;
  const int grp = T >= kLrThreads ? 0 : tid / T;
  const int task0 = T >= kLrThreads ? tid : tid % T;
  const int ntask = T >= kLrThreads ? (T - tid + kLrThreads - 1) / kLrThreads : (grp < G ? 1 : 0);
  __syncthreads();
  double g0norm = -1.0;   // wave 0
  int nit = J.max_outer;
  for (int it = 0; it < J.max_outer; ++it) {
    // ---- A: H, g and the loss at the current margins
    double acc[3] = {0.0, 0.0, 0.0};
    double loss[1] = {0.0};
    for (int c0 = r0; c0 < r1; c0 += CR) {
      const int nr = min(CR, r1 - c0);
      const double* Xc = J.X + (size_t)c0 * F1;
      for (int e = tid; e < nr * F1; e += kLrThreads) xs[e] = Xc[e];
      for (int r = tid; r < nr; r += kLrThreads) {
        const double sw = s[c0 + r];
        double Dr = 0.0, Cr = 0.0;
        if (sw != 0.0) {
          const double yp = J.ypm[c0 + r];
          const double M = yp * Z[c0 + r];
          const double sig = 1.0 / (1.0 + exp(-M));
          Cr = sw * (sig - 1.0) * yp;
          Dr = sw * sig * (1.0 - sig);
          loss[0] += sw * lr_softplus(-M);
        }
        dv[r] = Dr;
        cv[r] = Cr;
      }
      __syncthreads();
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        if (q >= ntask) break;
        const int k = task0 + q * kLrThreads;
        double a = 0.0;
        if (k < npairs) {
          const int i = pi[k], j = pj[k];
          for (int r = grp; r < nr; r += G) a = fma(dv[r] * xs[r * F1 + i], xs[r * F1 + j], a);
        } else {
          const int f = k - npairs;
          for (int r = grp; r < nr; r += G) a = fma(cv[r], xs[r * F1 + f], a);
        }
        acc[q] += a;
      }
      __syncthreads();
    }
    auto store = [&](int k, double v) {
      if (k < npairs) {
        const int i = pi[k], j = pj[k];
        H[i * F1 + j] = v;
        H[j * F1 + i] = v;
      } else {
        gr[k - npairs] = v;
      }
    };
    // this workgroup's partial of every task → mv (row groups folded in a fixed order)
    if (G > 1) {
      if (grp < G) part[grp * T + task0] = acc[0];
      __syncthreads();
      if (tid < T) {
        double t = 0.0;
        for (int g = 0; g < G; ++g) t += part[g * T + tid];
        mv[tid] = t;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 3; ++q)
        if (q < ntask) mv[task0 + q * kLrThreads] = acc[q];
    }
    lr_block_sum<1>(loss, red, sc + 8);
    if (tid == 0) mv[T] = sc[8];
    __syncthreads();
    if constexpr (Coop) {
      if (!lr_exchange(mv, T + 1, J, b, w, epoch, &xfail)) return;
    }
    for (int k = tid; k < T; k += kLrThreads) store(k, C * mv[k]);
    __syncthreads();
    const double data0 = C * mv[T];
    // ---- B: stopping rule and subproblem
    if (J.l1) {
      if (wave == 0) {
        const int j = lane;
        const double gj = j < F1 ? gr[j] : 0.0, wj = j < F1 ? Wl[j] : 0.0;
        double sub = 0.0;   // min-norm subgradient of g·w + ‖w‖₁
        if (j < F1)
          sub = wj != 0.0 ? gj + (wj > 0.0 ? 1.0 : -1.0)
                          : (gj > 0.0 ? 1.0 : (gj < 0.0 ? -1.0 : 0.0)) * fmax(fabs(gj) - 1.0, 0.0);
        const double gn = wave_sum(fabs(sub));
        if (g0norm < 0.0) g0norm = fmax(gn, 1e-300);
        const bool stop = gn <= 1e-9 * g0norm;
        double dj = 0.0;
        if (!stop) {
          // min_d gᵀd + ½dᵀ(H + 1e-12·I)d + ‖w + d‖₁ by cyclic coordinate descent (owner lanes);
          // this lane's H[j][k+1] is loaded while coordinate k is being solved
          const double hjj = j < F1 ? H[j * F1 + j] + 1e-12 : 0.0;
          const double aj = hjj > 1e-300 ? hjj : 1e-300;
          const double inv_a = 1.0 / aj;
          const double thr = (j < F1 && J.penal[j]) ? inv_a : 0.0;
          double Hd = 0.0;
          for (int sweep = 0; sweep < 200; ++sweep) {
            double maxstep = 0.0;
            double hk = j < F1 ? H[j * F1] : 0.0;
            for (int k = 0; k < F1; ++k) {
              const double hnext = (j < F1 && k + 1 < F1) ? H[j * F1 + k + 1] : 0.0;
              double step_l = 0.0;
              if (j == k) {
                const double lin = gj + Hd - aj * dj;
                const double z0 = wj - lin * inv_a;
                const double z = thr > 0 ? (z0 > thr ? z0 - thr : (z0 < -thr ? z0 + thr : 0.0)) : z0;
                const double nd = z - wj;
                step_l = nd - dj;
                dj = nd;
              }
              const double step = readlane_f64(step_l, k);
              if (step != 0.0) {
                if (j < F1) Hd += (hk + (j == k ? 1e-12 : 0.0)) * step;
                maxstep = fmax(maxstep, fabs(step));
              }
              hk = hnext;
            }
            if (maxstep <= 1e-12) break;
            // every 4 sweeps: the exact minimiser on the current sign pattern (l1qp.h), if optimal;
            // the row-chunk LDS is free during this phase and holds its scratch
            if ((sweep & 3) == 3 &&
                l1qp_newton_finish(F1, H, Wl, 1e-12, gj, wj, j < F1 && J.penal[j], 1.0, dj, xs, xs + F1 * F1))
              break;
          }
        }
        const double delta = wave_sum(j < F1 ? gj * dj + fabs(wj + dj) - fabs(wj) : 0.0);
        const double reg0 = wave_sum((j < F1 && J.penal[j]) ? fabs(wj) : 0.0);
        if (j < F1) dd[j] = dj;
        if (lane == 0) { sc[0] = stop ? 1.0 : 0.0; sc[1] = delta; sc[2] = reg0; }
      }
      __syncthreads();
    } else {
      if (wave == 0) {
        const int j = lane;
        const double gf = j < F1 ? gr[j] + (J.penal[j] ? Wl[j] : 0.0) : 0.0;
        const double gn = wave_sum(fabs(gf));
        if (g0norm < 0.0) g0norm = fmax(gn, 1e-300);
        if (j < F1) dd[j] = -gf;
        if (j < F1 && J.penal[j]) H[j * F1 + j] += 1.0;
        if (lane == 0) sc[0] = gn <= 1e-10 * g0norm ? 1.0 : 0.0;
      }
      __syncthreads();
      if (sc[0] == 0.0) {
        // Cholesky of H + diag(pen) in place (lower triangle; thread j owns row j)
        for (int k = 0; k < F1; ++k) {
          __syncthreads();
          const double piv = sqrt(H[k * F1 + k]);
          __syncthreads();
          if (tid == k) H[k * F1 + k] = piv;
          else if (tid > k && tid < F1) H[tid * F1 + k] /= piv;
          __syncthreads();
          if (tid > k && tid < F1) {
            const double ljk = H[tid * F1 + k];
            for (int i = k + 1; i <= tid; ++i) H[tid * F1 + i] -= ljk * H[i * F1 + k];
          }
        }
        __syncthreads();
        if (tid == 0) {
          for (int i = 0; i < F1; ++i) {          // L y = −g
            double v = dd[i];
            for (int k = 0; k < i; ++k) v -= H[i * F1 + k] * dd[k];
            dd[i] = v / H[i * F1 + i];
          }
          for (int i = F1 - 1; i >= 0; --i) {     // Lᵀ d = y
            double v = dd[i];
            for (int k = i + 1; k < F1; ++k) v -= H[k * F1 + i] * dd[k];
            dd[i] = v / H[i * F1 + i];
          }
          double delta = 0.0, reg0 = 0.0;
          for (int i = 0; i < F1; ++i) {
            const double gf = gr[i] + (J.penal[i] ? Wl[i] : 0.0);
            delta += gf * dd[i];
            if (J.penal[i]) reg0 += 0.5 * Wl[i] * Wl[i];
          }
          sc[1] = delta;
          sc[2] = reg0;
        }
      }
      __syncthreads();
    }
    if (sc[0] != 0.0) { nit = it + 1; break; }
    // ---- C: the loss at the full step 2^0 first (X̃d kept): a Newton step is almost always
    // accepted at once, and the 7 shorter trials cost 7 of the pass's 8 softplus per row.  Only
    // when the full step fails the Armijo test does a second pass evaluate steps 2^-1 … 2^-7 (from
    // the stored X̃d).  Every trial loss is the sum the one-pass form computed — the same per-thread
    // row order, the same per-step block reduction and member exchange order — so the chosen
    // step, and the whole solve, are unchanged bit for bit.
    const double F0 = data0 + sc[2], delta = sc[1];
    auto reg_at = [&](double a) {
      double reg = 0.0;
      for (int f = 0; f < F1; ++f) {
        if (!J.penal[f]) continue;
        const double wc = Wl[f] + a * dd[f];
        reg += J.l1 ? fabs(wc) : 0.5 * wc * wc;
      }
      return reg;
    };
    {
      double t0[1] = {0.0};
      for (int r = r0 + tid; r < r1; r += kLrThreads) {
        const double* xr = J.X + (size_t)r * F1;
        double xd = 0.0;
        for (int f = 0; f < F1; ++f) xd = fma(xr[f], dd[f], xd);
        Xd[r] = xd;
        const double sw = s[r];
        if (sw != 0.0) {
          const double yp = J.ypm[r], z = Z[r];
          t0[0] += sw * lr_softplus(-yp * (z + 1.0 * xd));
        }
      }
      lr_block_sum<1>(t0, red, sc + 8);
      if constexpr (Coop) {
        if (!lr_exchange(sc + 8, 1, J, b, w, epoch, &xfail)) return;
      }
    }
    const bool full_ok = C * sc[8] + reg_at(1.0) <= F0 + 1e-2 * 1.0 * delta;
    if (!full_ok) {
      double tk[kLrSteps - 1];
#pragma unroll
      for (int k = 0; k < kLrSteps - 1; ++k) tk[k] = 0.0;
      for (int r = r0 + tid; r < r1; r += kLrThreads) {
        const double sw = s[r];
        if (sw != 0.0) {
          const double yp = J.ypm[r], z = Z[r], xd = Xd[r];
          double a = 0.5;
#pragma unroll
          for (int k = 0; k < kLrSteps - 1; ++k) {
            tk[k] += sw * lr_softplus(-yp * (z + a * xd));
            a *= 0.5;
          }
        }
      }
      lr_block_sum<kLrSteps - 1>(tk, red, sc + 9);
      if constexpr (Coop) {
        if (!lr_exchange(sc + 9, kLrSteps - 1, J, b, w, epoch, &xfail)) return;
      }
    }
    // Armijo: largest 2^-k with F(w + a d) ≤ F(w) + 0.01·a·Δ; none → the smallest step if it
    // still decreases F, else stop (every thread evaluates the same rule on LDS values)
    int first = full_ok ? 0 : -1;
    double FK7 = 0.0, a = 1.0;
    for (int k = 0; k < (full_ok ? 0 : kLrSteps); ++k) {
      double reg = 0.0;
      for (int f = 0; f < F1; ++f) {
        if (!J.penal[f]) continue;
        const double wc = Wl[f] + a * dd[f];
        reg += J.l1 ? fabs(wc) : 0.5 * wc * wc;
      }
      const double FK = C * sc[8 + k] + reg;
      if (first < 0 && FK <= F0 + 1e-2 * a * delta) first = k;
      FK7 = FK;
      a *= 0.5;
    }
    double step = 0.0;
    if (first >= 0) step = ldexp(1.0, -first);
    else if (FK7 < F0) step = ldexp(1.0, -(kLrSteps - 1));
    if (step == 0.0) { nit = it + 1; break; }
    __syncthreads();   // every thread has read Wl, dd and sc
    if (tid < F1) Wl[tid] += step * dd[tid];
    for (int r = r0 + tid; r < r1; r += kLrThreads) Z[r] += step * Xd[r];
    __syncthreads();
    double mstep = 0.0, mw = 0.0;
    for (int f = 0; f < F1; ++f) {
      mstep = fmax(mstep, fabs(step * dd[f]));
      mw = fmax(mw, fabs(Wl[f]));
    }
    if (mstep <= 1e-14 * (1.0 + mw)) { nit = it + 1; break; }
  }
  __syncthreads();
  if (w == 0) {
    if (tid < F1) J.W[(size_t)b * F1 + tid] = Wl[tid];
    if (tid == 0) J.iters[b] = nit;
  }
}

static size_t logreg_lds_plan(int F1, int* CR_out) {
  const int npairs = F1 * (F1 + 1) / 2, T = npairs + F1;
  // ≤ 32 KiB of staged rows keeps the whole plan near 48 KiB, so a workgroup still fits beside
  // the SMO members that run concurrently on the other stream
  int CR = (32 * 1024) / (F1 * (int)sizeof(double));
  CR = CR > 1024 ? 1024 : CR / 64 * 64;
  if (CR < 64) CR = 64;
  if ((long long)CR * F1 < (long long)F1 * F1 + F1) CR = (F1 + 1 + 63) / 64 * 64;   // l1qp.h scratch
  *CR_out = CR;
  const size_t lds = ((size_t)CR * F1 + 2 * CR + F1 * F1 + 3 * F1 + kLrThreads + kLrWaves * kLrSteps + 16 +
                      (T + 1)) * sizeof(double) + 2 * (size_t)npairs;
  HFENS_REQUIRE(lds <= 160 * 1024, "logreg_fused: LDS plan exceeds 160 KiB");
  return lds;
}

void logreg_fused(int B, int n, int F1, uintptr_t X, uintptr_t s, uintptr_t ypm, uintptr_t penal, double C,
                  int l1, int max_outer, uintptr_t Z, uintptr_t Xd, uintptr_t W, uintptr_t iters,
                  uintptr_t stream) {
  HFENS_REQUIRE(F1 >= 1 && F1 <= 64, "logreg_fused: 1 <= F+1 <= 64");
  HFENS_REQUIRE(B >= 1 && n >= 1 && max_outer >= 1, "logreg_fused: empty problem");
  int CR = 0;
  const size_t lds = logreg_lds_plan(F1, &CR);
  LrJob J{(const double*)X, (const double*)s, (const double*)ypm, (const unsigned char*)penal, (double*)Z,
          (double*)Xd, (double*)W, (int*)iters, C, n, F1, l1 ? 1 : 0, max_outer, CR, B, 1, n, 0, nullptr, nullptr};
  hipLaunchKernelGGL(logreg_fused_kernel<false>, dim3(B), dim3(kLrThreads), lds, as_stream(stream), J);
  launch_check();
}

// exchange slots (u64 granules); models/logreg_solver.py sizes its buffer with the same formula
static int logreg_nvmax(int F1) {   // values per member slot: H, g and the loss, or the trial losses
  const int nv = F1 * (F1 + 1) / 2 + F1 + 1;
  return nv > kLrSteps ? nv : kLrSteps;
}

static size_t logreg_coop_xchg_bytes(int B, int members, int F1) {
  const int nvmax = logreg_nvmax(F1);
  return (size_t)B * 2 * members * nvmax * 2 * sizeof(unsigned long long);
}

void logreg_coop(int B, int members, int n, int F1, uintptr_t X, uintptr_t s, uintptr_t ypm, uintptr_t penal,
                 double C, int l1, int max_outer, uintptr_t Z, uintptr_t Xd, uintptr_t W, uintptr_t iters,
                 uintptr_t xchg, uintptr_t err, uintptr_t stream) {
  HFENS_REQUIRE(F1 >= 1 && F1 <= 64, "logreg_coop: 1 <= F+1 <= 64");
  HFENS_REQUIRE(B >= 1 && n >= 1 && max_outer >= 1, "logreg_coop: empty problem");
  HFENS_REQUIRE(members >= 1 && members <= kLrMaxMembers, "logreg_coop: 1 <= members <= 16");
  int dev = 0, ncu = 256;
  HFENS_CHECK(hipGetDevice(&dev));
  HFENS_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  // members spin on each other: all of them must be resident at once (one per CU at most)
  HFENS_REQUIRE((long long)B * members <= ncu, "logreg_coop: B·members exceeds the CU count");
  int CR = 0;
  const size_t lds = logreg_lds_plan(F1, &CR);
  const int nvmax = logreg_nvmax(F1);
  const int S = (n + members - 1) / members;
  hipStream_t st = as_stream(stream);
  // every polled granule starts at epoch 0 (epochs count from 1 within the launch)
  HFENS_CHECK(hipMemsetAsync((void*)xchg, 0, logreg_coop_xchg_bytes(B, members, F1), st));
  LrJob J{(const double*)X, (const double*)s, (const double*)ypm, (const unsigned char*)penal, (double*)Z,
          (double*)Xd, (double*)W, (int*)iters, C, n, F1, l1 ? 1 : 0, max_outer, CR, B, members, S, nvmax,
          (unsigned long long*)xchg, (unsigned*)err};
  const long long blocks = 8LL * ((B + 7) / 8) * members;
  hipLaunchKernelGGL(logreg_fused_kernel<true>, dim3((unsigned)blocks), dim3(kLrThreads), lds, st, J);
  launch_check();
}

}  // namespace hfens
