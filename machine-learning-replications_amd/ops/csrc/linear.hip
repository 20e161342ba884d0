// Small dense solvers for the linear models (SURVEY.md §2.3 K3 lasso_cd_path, K13 logreg_cd).
//
//  l1_qp_cd      : batched L1-regularised quadratic subproblem of proximal Newton (the
//                  newGLMNET inner problem of liblinear's solve_l1r_lr):
//                      min_d  gᵀd + ½ dᵀHd + λ‖w + d‖₁      (per model, dense H ≤ 64×64)
//                  One 64-lane wave per model: H lives in LDS, lane j owns coordinate j's
//                  (Hd)_j, cyclic coordinate descent with soft-thresholding.
//  lasso_cd_path : batched Gram-form coordinate descent over a decreasing alpha grid
//                  (sklearn enet_coordinate_descent_gram semantics: objective
//                  ½‖y−Xw‖²/n + α‖w‖₁ with centred X, y; duality-gap stop), one wave per
//                  problem (CV fold), warm-started along the path, recording the path.
#include "common.h"
#include "l1qp.h"

namespace hfens {

__global__ __launch_bounds__(64) void l1_qp_cd_kernel(int F1, const double* __restrict__ H,
                                                      const double* __restrict__ g,
                                                      const double* __restrict__ w,
                                                      const unsigned char* __restrict__ penal,
                                                      double lam, int max_sweeps, double tol,
                                                      double* __restrict__ d_out) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int b = blockIdx.x;
  const int j = threadIdx.x;
  double* Hs = sm;                 // [F1][F1]
  double* ws = Hs + F1 * F1;       // [F1] w
  double* A = ws + F1;             // [F1][F1] Newton scratch (l1qp.h)
  double* v = A + F1 * F1;         // [F1]
  const double* Hb = H + (size_t)b * F1 * F1;
  for (int k = j; k < F1 * F1; k += 64) Hs[k] = Hb[k];
  if (j < F1) ws[j] = w[b * F1 + j];
  __syncthreads();
  const double gj = j < F1 ? g[b * F1 + j] : 0.0;
  const double wj = j < F1 ? w[b * F1 + j] : 0.0;
  const double hjj = j < F1 ? Hs[j * F1 + j] : 0.0;
  const double aj = hjj > 1e-300 ? hjj : 1e-300;
  const double inv_a = 1.0 / aj;                                   // reciprocal once, not per sweep
  const double thr = (j < F1 && penal[j]) ? lam * inv_a : 0.0;     // soft-threshold λ/a
  double Hd = 0.0;  // (H d)_j
  double dj = 0.0;
  for (int sweep = 0; sweep < max_sweeps; ++sweep) {
    double maxstep = 0.0;
    for (int k = 0; k < F1; ++k) {
      // the owner lane solves the 1-D problem in z = w_k + d_k
      //   (g_k + (Hd)_k − a·d_k)(z − w_k) + ½a(z − w_k)² + λ|z|
      // and broadcasts the step (one readlane pair on the dependent chain instead of five)
      double step_l = 0.0;
      if (j == k) {
        const double lin = gj + Hd - aj * dj;
        const double z0 = wj - lin * inv_a;  // unpenalised minimiser
        const double z = thr > 0 ? (z0 > thr ? z0 - thr : (z0 < -thr ? z0 + thr : 0.0)) : z0;
        const double nd = z - wj;
        step_l = nd - dj;
        dj = nd;
      }
      const double step = readlane_f64(step_l, k);
      if (step != 0.0) {
        if (j < F1) Hd += Hs[j * F1 + k] * step;
        maxstep = fmax(maxstep, fabs(step));
      }
    }
    if (maxstep <= tol) break;
    // every 4 sweeps: the exact minimiser on the current sign pattern, if it is optimal
    if ((sweep & 3) == 3 && l1qp_newton_finish(F1, Hs, ws, 0.0, gj, wj, j < F1 && penal[j], lam, dj, A, v)) break;
  }
  if (j < F1) d_out[b * F1 + j] = dj;
}

void l1_qp_cd(int B, int F1, uintptr_t H, uintptr_t g, uintptr_t w, uintptr_t penal, double lam,
              int max_sweeps, double tol, uintptr_t d_out, uintptr_t stream) {
  HFENS_REQUIRE(F1 >= 1 && F1 <= 64, "l1_qp_cd: 1 <= F+1 <= 64");
  const size_t lds = (2 * (size_t)F1 * F1 + 2 * (size_t)F1) * sizeof(double);
  hipLaunchKernelGGL(l1_qp_cd_kernel, dim3(B), dim3(64), lds, as_stream(stream), F1,
                     (const double*)H, (const double*)g, (const double*)w,
                     (const unsigned char*)penal, lam, max_sweeps, tol, (double*)d_out);
  launch_check();
}

// ------------------------------------------------------------------------------------------
// Lasso path, Gram form.  Per problem p: G = XᵀX (F×F), q = Xᵀy (F), n_p rows, yy = yᵀy.
// Objective  (1/(2 n_p))‖y − Xw‖² + α‖w‖₁  ⇔ sklearn's enet with l1_ratio=1 (alpha scaled by n).
// coefs out: [P][A][F]; gaps out [P][A]; iters [P][A].
__global__ __launch_bounds__(64) void lasso_cd_path_kernel(int F, int A, const double* __restrict__ G,
                                                           const double* __restrict__ q,
                                                           const double* __restrict__ yy,
                                                           const double* __restrict__ nrows,
                                                           const double* __restrict__ alphas,
                                                           int max_iter, double tol,
                                                           double* __restrict__ coefs,
                                                           double* __restrict__ gaps,
                                                           int* __restrict__ iters) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int p = blockIdx.x;
  const int j = threadIdx.x;
  double* Gs = sm;  // [F][F]
  const double* Gp = G + (size_t)p * F * F;
  for (int k = j; k < F * F; k += 64) Gs[k] = Gp[k];
  __syncthreads();
  const double n = nrows[p];
  const double qj = j < F ? q[p * F + j] : 0.0;
  const double gjj = j < F ? Gs[j * F + j] : 0.0;
  // the coordinate step divides by G_kk every sweep of every alpha: take the reciprocal once
  // (≤ 1 ulp from the division; the f64 divide sequence was half of each coordinate's latency)
  const double inv_gjj = gjj != 0.0 ? 1.0 / gjj : 0.0;
  const unsigned long long live = __ballot(j < F && gjj != 0.0);   // coordinates with G_kk ≠ 0
  const double yyp = yy[p];
  double wj = 0.0;   // coefficient owned by lane j
  double Hw = 0.0;   // (G w)_j
  // sklearn: tol *= ‖y‖² (Gram path) ; l1_reg = alpha·n
  const double tol_s = tol * yyp;
  for (int a = 0; a < A; ++a) {
    const double l1 = alphas[p * A + a] * n;
    int it = 0;
    double gap = 0.0;
    for (it = 0; it < max_iter; ++it) {
      double w_max = 0.0, d_w_max = 0.0;
      for (int k = 0; k < F; ++k) {
        // skip ahead over coordinates that provably stay at zero (w_k = 0 and |q_k − (Gw)_k| ≤ l1
        // — exactly sklearn's "no update" branch): every lane tests its own coordinate against
        // its current (Gw)_j in parallel, one ballot finds the next coordinate that can move
        {
          const bool can_move = ((live >> j) & 1ull) && j >= k && !(wj == 0.0 && !(fabs(qj - Hw) > l1));
          const unsigned long long mv = __ballot(can_move);
          if (mv == 0ull) break;
          k = __builtin_ctzll(mv);
        }
        // column k of G is known once k is: issue its LDS read now so its latency hides under
        // the owner's step and the two readlanes instead of sitting on the Hw chain after them
        const double gjk = j < F ? Gs[j * F + k] : 0.0;
        // the owner lane evaluates tmp = q_k − (Gw)_k + G_kk w_k and the soft-threshold step,
        // then (nw, dw) are broadcast: two readlanes instead of four on the dependent chain
        double nw_l = 0.0, dw_l = 0.0;
        if (j == k) {
          const double tmp = qj - Hw + gjj * wj;
          nw_l = fabs(tmp) > l1 ? copysign(fabs(tmp) - l1, tmp) * inv_gjj : 0.0;
          dw_l = nw_l - wj;
          wj = nw_l;
        }
        const double nw = readlane_f64(nw_l, k), dw = readlane_f64(dw_l, k);
        if (dw != 0.0 && j < F) Hw += gjk * dw;
        d_w_max = fmax(d_w_max, fabs(dw));
        w_max = fmax(w_max, fabs(nw));
      }
      if (w_max == 0.0 || d_w_max / w_max < tol || it == max_iter - 1) {
        // duality gap (sklearn enet_coordinate_descent_gram, l2_reg = 0)
        const double wq = wave_sum(j < F ? wj * qj : 0.0);
        const double wHw = wave_sum(j < F ? wj * Hw : 0.0);
        const double l1n = wave_sum(j < F ? fabs(wj) : 0.0);
        double dual_norm = j < F ? fabs(qj - Hw) : 0.0;  // |Xᵀ R|_∞ with R = y − Xw
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) dual_norm = fmax(dual_norm, __shfl_xor(dual_norm, o, kWave));
        const double R_norm2 = yyp - 2.0 * wq + wHw;
        double const_ = 1.0;
        double gp = R_norm2;
        if (dual_norm > l1) {
          const_ = l1 / dual_norm;
          const double A_norm2 = R_norm2 * const_ * const_;
          gp = 0.5 * (R_norm2 + A_norm2);
        }
        // q_dot_w = wq ; y_norm2 = yy
        gap = gp + l1 * l1n - const_ * (yyp - wq);  // R·y = yy − wᵀq
        if (gap < tol_s) break;
      }
    }
    if (j < F) coefs[((size_t)p * A + a) * F + j] = wj;
    if (j == 0) { gaps[p * A + a] = gap; iters[p * A + a] = it + 1; }
  }
}

void lasso_cd_path(int P, int F, int A, uintptr_t G, uintptr_t q, uintptr_t yy, uintptr_t nrows,
                   uintptr_t alphas, int max_iter, double tol, uintptr_t coefs, uintptr_t gaps,
                   uintptr_t iters, uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F <= 64, "lasso_cd_path: 1 <= F <= 64");
  const size_t lds = (size_t)F * F * sizeof(double);
  hipLaunchKernelGGL(lasso_cd_path_kernel, dim3(P), dim3(64), lds, as_stream(stream), F, A,
                     (const double*)G, (const double*)q, (const double*)yy, (const double*)nrows,
                     (const double*)alphas, max_iter, tol, (double*)coefs, (double*)gaps,
                     (int*)iters);
  launch_check();
}

// ------------------------------------------------------------------------------------------
// Weighted moments  G_p = Σ_n W[p,n]·x_n x_nᵀ (upper triangle), a_p = Σ_n W[p,n]·x_n,
// v_p = Σ_n V[p,n]·x_n  for P weight vectors over one row matrix X [n, F] (f64).
// These are the Gram / Hessian / gradient reductions of LassoCV (per-fold moments) and of the
// logistic solvers (X̃ᵀDX̃, X̃ᵀr) — tall-skinny (n ≫ F ≤ 64) so a library GEMM runs them on one
// tile; here every (row chunk, p) is a workgroup writing a partial, summed in fixed chunk order
// (deterministic).  Row chunks are staged in LDS; each thread owns a few (i ≤ j) pairs.
constexpr int kMomRows = 128;

__global__ __launch_bounds__(256) void weighted_moments_kernel(
    const double* __restrict__ X, int n, int F, const double* __restrict__ W,
    const double* __restrict__ V, int npairs, double* __restrict__ Gpart, double* __restrict__ apart,
    double* __restrict__ vpart) {
  extern __shared__ __attribute__((aligned(16))) double xs[];  // [kMomRows][F+1] + w + v
  const int ld = F + 1;
  double* ws = xs + kMomRows * ld;
  double* vs = ws + kMomRows;
  const int c = blockIdx.x, p = blockIdx.y, C = gridDim.x;
  const int r0 = c * kMomRows;
  const int nr = min(kMomRows, n - r0);
  for (int e = threadIdx.x; e < nr * F; e += blockDim.x) {
    const int r = e / F, f = e % F;
    xs[r * ld + f] = X[(size_t)(r0 + r) * F + f];
  }
  for (int r = threadIdx.x; r < nr; r += blockDim.x) {
    ws[r] = W[(size_t)p * n + r0 + r];
    vs[r] = V != nullptr ? V[(size_t)p * n + r0 + r] : 0.0;
  }
  __syncthreads();
  // pairs: k → (i, j) with i ≤ j, row-major over the upper triangle
  for (int k = threadIdx.x; k < npairs; k += blockDim.x) {
    int i = 0, rem = k;
    while (rem >= F - i) { rem -= F - i; ++i; }
    const int j = i + rem;
    double acc = 0.0;
    for (int r = 0; r < nr; ++r) acc = fma(ws[r] * xs[r * ld + i], xs[r * ld + j], acc);
    Gpart[((size_t)p * C + c) * npairs + k] = acc;
  }
  for (int f = threadIdx.x; f < F; f += blockDim.x) {
    double a = 0.0, v = 0.0;
    for (int r = 0; r < nr; ++r) {
      a = fma(ws[r], xs[r * ld + f], a);
      v = fma(vs[r], xs[r * ld + f], v);
    }
    apart[((size_t)p * C + c) * F + f] = a;
    vpart[((size_t)p * C + c) * F + f] = v;
  }
}

void weighted_moments(uintptr_t X, int n, int F, uintptr_t W, uintptr_t V, int P, uintptr_t Gpart,
                      uintptr_t apart, uintptr_t vpart, uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F <= 128, "weighted_moments: 1 <= F <= 128");
  if (n == 0) return;
  const int C = (n + kMomRows - 1) / kMomRows;
  const size_t lds = ((size_t)kMomRows * (F + 1) + 2 * kMomRows) * sizeof(double);
  hipLaunchKernelGGL(weighted_moments_kernel, dim3(C, P), dim3(256), lds, as_stream(stream),
                     (const double*)X, n, F, (const double*)W, (const double*)V, F * (F + 1) / 2,
                     (double*)Gpart, (double*)apart, (double*)vpart);
  launch_check();
}

}  // namespace hfens
