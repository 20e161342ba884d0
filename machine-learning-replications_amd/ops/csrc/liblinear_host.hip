// liblinear's L1-regularised logistic regression as scikit-learn runs it for the reference's base
// model 'lg' (train_ensemble_public.py:46: LogisticRegression(penalty='l1', solver='liblinear',
// class_weight='balanced'), random_state=None → the seed is drawn from numpy's GLOBAL MT19937,
// seeded at train_ensemble_public.py:31).  Host code, no device work: the iterate of liblinear's
// default-tolerance solve depends on its pseudo-random coordinate order, so reproducing it to the
// last bits is a sequential CPU algorithm by nature.  The device path
// (logreg.hip) solves the same objective to optimality instead; this one reproduces the
// reference's early-stopped answer.
//
// The algorithm (newGLMNET: Yuan, Ho & Lin 2011; the appendix of Fan et al. 2008), as configured
// by scikit-learn:
//   * the problem is regrouped by class (class 0 rows first, each class in input order), class 0
//     is y = −1 and class 1 y = +1; per-row C = sample_weight · C · class_weight[class];
//   * features are the input columns plus the bias column (value intercept_scaling), and only
//     NON-ZERO entries take part (scikit-learn hands liblinear a sparse copy of the dense matrix),
//     each column's entries in row order — the summation order below follows that exactly;
//   * outer Newton iterations with outer-level shrinking; the quadratic model is minimised by
//     cyclic coordinate descent over a per-sweep random permutation (std::mt19937 seeded with the
//     wrap's seed, "tweaked Lemire" bounded draws, sklearn/svm/src/newrand/newrand.h), with
//     inner-level shrinking and active-set reactivation; then a backtracking line search;
//   * tolerance eps · max(min(#pos, #neg), 1) / l on the accumulated violation.
// Every floating-point expression keeps liblinear's evaluation order and no contraction into fma
// (scikit-learn's wheel is built for the x86-64 baseline, which has none).
//
// This file re-expresses liblinear's solve_l1r_lr (the copy vendored by scikit-learn as
// sklearn/svm/src/liblinear/linear.cpp) closely enough to reproduce its iterate bit for bit, so it
// carries liblinear's licence:
//
//   Copyright (c) 2007-2023 The LIBLINEAR Project.
//   All rights reserved.
//
//   Redistribution and use in source and binary forms, with or without modification, are permitted
//   provided that the following conditions are met:
//   1. Redistributions of source code must retain the above copyright notice, this list of
//      conditions and the following disclaimer.
//   2. Redistributions in binary form must reproduce the above copyright notice, this list of
//      conditions and the following disclaimer in the documentation and/or other materials
//      provided with the distribution.
//   3. Neither name of copyright holders nor the names of its contributors may be used to endorse
//      or promote products derived from this software without specific prior written permission.
//
//   THIS SOFTWARE IS PROVIDED BY THE COPYRIGHT HOLDERS AND CONTRIBUTORS ``AS IS'' AND ANY EXPRESS
//   OR IMPLIED WARRANTIES, INCLUDING, BUT NOT LIMITED TO, THE IMPLIED WARRANTIES OF MERCHANTABILITY
//   AND FITNESS FOR A PARTICULAR PURPOSE ARE DISCLAIMED.  IN NO EVENT SHALL THE REGENTS OR
//   CONTRIBUTORS BE LIABLE FOR ANY DIRECT, INDIRECT, INCIDENTAL, SPECIAL, EXEMPLARY, OR
//   CONSEQUENTIAL DAMAGES (INCLUDING, BUT NOT LIMITED TO, PROCUREMENT OF SUBSTITUTE GOODS OR
//   SERVICES; LOSS OF USE, DATA, OR PROFITS; OR BUSINESS INTERRUPTION) HOWEVER CAUSED AND ON ANY
//   THEORY OF LIABILITY, WHETHER IN CONTRACT, STRICT LIABILITY, OR TORT (INCLUDING NEGLIGENCE OR
//   OTHERWISE) ARISING IN ANY WAY OUT OF THE USE OF THIS SOFTWARE, EVEN IF ADVISED OF THE
//   POSSIBILITY OF SUCH DAMAGE.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <random>
#include <vector>

namespace hfens {

namespace {

inline uint32_t ll_bounded(std::mt19937& mt, uint32_t range) {
  uint32_t x = mt();
  uint64_t m = uint64_t(x) * uint64_t(range);
  uint32_t lo = uint32_t(m);
  if (lo < range) {
    uint32_t t = -range;
    if (t >= range) {
      t -= range;
      if (t >= range) t %= range;
    }
    while (lo < t) {
      x = mt();
      m = uint64_t(x) * uint64_t(range);
      lo = uint32_t(m);
    }
  }
  return uint32_t(m >> 32);
}

struct Col {             // one feature's non-zero entries, rows in problem order
  std::vector<int> row;
  std::vector<double> val;
};

}  // namespace

#pragma clang fp contract(off)
// X: [l][n] row-major f64 (input order), y01: [l] labels 0/1, sw: [l] sample weights (> 0);
// C0 / C1: C · class_weight of class 0 / 1; bias: intercept_scaling (≤ 0: no bias column).
// w_out: [n + (bias > 0)] — coef in input column order, then the bias weight.  Returns the Newton
// iteration count (scikit-learn's n_iter_).
int liblinear_l1r_lr(uintptr_t X_ptr, uintptr_t y_ptr, uintptr_t sw_ptr, int l_in, int n, double bias, double C0,
                     double C1, double eps, int max_newton_iter, long long seed, uintptr_t w_ptr) {
  const double* X = reinterpret_cast<const double*>(X_ptr);
  const double* y01 = reinterpret_cast<const double*>(y_ptr);
  const double* sw = reinterpret_cast<const double*>(sw_ptr);
  double* w_out = reinterpret_cast<double*>(w_ptr);
  // problem order: rows with weight > 0, class 0 first (each class in input order)
  std::vector<int> order;
  order.reserve(l_in);
  for (int cls = 0; cls < 2; ++cls)
    for (int i = 0; i < l_in; ++i)
      if (sw[i] > 0 && (y01[i] > 0.5 ? 1 : 0) == cls) order.push_back(i);
  const int l = (int)order.size();
  const bool has_bias = bias > 0;
  const int w_size = n + (has_bias ? 1 : 0);
  std::vector<Col> cols(w_size);
  for (int r = 0; r < l; ++r) {
    const double* xr = X + (size_t)order[r] * n;
    for (int j = 0; j < n; ++j)
      if (xr[j] != 0) {
        cols[j].row.push_back(r);
        cols[j].val.push_back(xr[j]);
      }
    if (has_bias) {
      cols[n].row.push_back(r);
      cols[n].val.push_back(bias);
    }
  }
  std::vector<signed char> y(l);
  std::vector<double> C(l);
  int pos = 0;
  for (int r = 0; r < l; ++r) {
    const bool p = y01[order[r]] > 0.5;
    y[r] = p ? 1 : -1;
    C[r] = p ? sw[order[r]] * C1 : sw[order[r]] * C0;
    pos += p;
  }
  const int neg = l - pos;
  const double tol = eps * std::max(std::min(pos, neg), 1) / l;
  std::mt19937 mt(static_cast<uint32_t>(seed));

  const int max_iter = 1000, max_num_linesearch = 20;
  const double nu = 1e-12, sigma = 0.01;
  double inner_eps = 1;
  std::vector<int> index(w_size);
  std::vector<double> w(w_size, 0.0), Hdiag(w_size), Grad(w_size), wpd(w_size), xjneg_sum(w_size);
  std::vector<double> xTd(l), exp_wTx(l, 0.0), exp_wTx_new(l), tau(l), D(l);
  double w_norm = 0;
  for (int j = 0; j < w_size; ++j) {
    w_norm += std::fabs(w[j]);
    wpd[j] = w[j];
    index[j] = j;
    xjneg_sum[j] = 0;
    const Col& c = cols[j];
    for (size_t k = 0; k < c.row.size(); ++k) {
      const int ind = c.row[k];
      exp_wTx[ind] += w[j] * c.val[k];
      if (y[ind] == -1) xjneg_sum[j] += C[ind] * c.val[k];
    }
  }
  for (int i = 0; i < l; ++i) {
    exp_wTx[i] = std::exp(exp_wTx[i]);
    const double tau_tmp = 1 / (1 + exp_wTx[i]);
    tau[i] = C[i] * tau_tmp;
    D[i] = C[i] * exp_wTx[i] * tau_tmp * tau_tmp;
  }
  int newton_iter = 0, QP_no_change = 0;
  double Gnorm1_init = -1.0, Gmax_old = INFINITY;
  while (newton_iter < max_newton_iter) {
    double Gmax_new = 0, Gnorm1_new = 0;
    int active_size = w_size;
    for (int s = 0; s < active_size; ++s) {
      const int j = index[s];
      Hdiag[j] = nu;
      Grad[j] = 0;
      double tmp = 0;
      const Col& c = cols[j];
      for (size_t k = 0; k < c.row.size(); ++k) {
        const int ind = c.row[k];
        Hdiag[j] += c.val[k] * c.val[k] * D[ind];
        tmp += c.val[k] * tau[ind];
      }
      Grad[j] = -tmp + xjneg_sum[j];
      const double Gp = Grad[j] + 1, Gn = Grad[j] - 1;
      double violation = 0;
      if (w[j] == 0) {
        if (Gp < 0) violation = -Gp;
        else if (Gn > 0) violation = Gn;
        else if (Gp > Gmax_old / l && Gn < -Gmax_old / l) {   // outer-level shrinking
          --active_size;
          std::swap(index[s], index[active_size]);
          --s;
          continue;
        }
      } else if (w[j] > 0) {
        violation = std::fabs(Gp);
      } else {
        violation = std::fabs(Gn);
      }
      Gmax_new = std::max(Gmax_new, violation);
      Gnorm1_new += violation;
    }
    if (newton_iter == 0) Gnorm1_init = Gnorm1_new;
    if (Gnorm1_new <= tol * Gnorm1_init || QP_no_change >= 10) break;
    ++QP_no_change;
    int iter = 0;
    double QP_Gmax_old = INFINITY;
    int QP_active_size = active_size;
    for (int i = 0; i < l; ++i) xTd[i] = 0;
    // the quadratic model over wpd: coordinate descent, a fresh permutation every sweep
    while (iter < max_iter) {
      double QP_Gmax_new = 0, QP_Gnorm1_new = 0;
      for (int j = 0; j < QP_active_size; ++j) {
        const int i = j + (int)ll_bounded(mt, (uint32_t)(QP_active_size - j));
        std::swap(index[i], index[j]);
      }
      for (int s = 0; s < QP_active_size; ++s) {
        const int j = index[s];
        const double H = Hdiag[j];
        const Col& c = cols[j];
        double G = Grad[j] + (wpd[j] - w[j]) * nu;
        for (size_t k = 0; k < c.row.size(); ++k) {
          const int ind = c.row[k];
          G += c.val[k] * D[ind] * xTd[ind];
        }
        const double Gp = G + 1, Gn = G - 1;
        double violation = 0;
        if (wpd[j] == 0) {
          if (Gp < 0) violation = -Gp;
          else if (Gn > 0) violation = Gn;
          else if (Gp > QP_Gmax_old / l && Gn < -QP_Gmax_old / l) {   // inner-level shrinking
            --QP_active_size;
            std::swap(index[s], index[QP_active_size]);
            --s;
            continue;
          }
        } else if (wpd[j] > 0) {
          violation = std::fabs(Gp);
        } else {
          violation = std::fabs(Gn);
        }
        double z;
        if (Gp < H * wpd[j]) z = -Gp / H;
        else if (Gn > H * wpd[j]) z = -Gn / H;
        else z = -wpd[j];
        if (std::fabs(z) < 1.0e-12) continue;
        z = std::min(std::max(z, -10.0), 10.0);
        QP_no_change = 0;
        QP_Gmax_new = std::max(QP_Gmax_new, violation);
        QP_Gnorm1_new += violation;
        wpd[j] += z;
        for (size_t k = 0; k < c.row.size(); ++k) xTd[c.row[k]] += c.val[k] * z;
      }
      ++iter;
      if (QP_Gnorm1_new <= inner_eps * Gnorm1_init) {
        if (QP_active_size == active_size) break;   // inner stopping
        QP_active_size = active_size;               // active-set reactivation
        QP_Gmax_old = INFINITY;
        continue;
      }
      QP_Gmax_old = QP_Gmax_new;
    }
    // line search on the Newton direction wpd − w
    double delta = 0, w_norm_new = 0;
    for (int j = 0; j < w_size; ++j) {
      delta += Grad[j] * (wpd[j] - w[j]);
      if (wpd[j] != 0) w_norm_new += std::fabs(wpd[j]);
    }
    delta += (w_norm_new - w_norm);
    double negsum_xTd = 0;
    for (int i = 0; i < l; ++i)
      if (y[i] == -1) negsum_xTd += C[i] * xTd[i];
    int num_linesearch;
    for (num_linesearch = 0; num_linesearch < max_num_linesearch; ++num_linesearch) {
      double cond = w_norm_new - w_norm + negsum_xTd - sigma * delta;
      for (int i = 0; i < l; ++i) {
        const double exp_xTd = std::exp(xTd[i]);
        exp_wTx_new[i] = exp_wTx[i] * exp_xTd;
        cond += C[i] * std::log((1 + exp_wTx_new[i]) / (exp_xTd + exp_wTx_new[i]));
      }
      if (cond <= 0) {
        w_norm = w_norm_new;
        for (int j = 0; j < w_size; ++j) w[j] = wpd[j];
        for (int i = 0; i < l; ++i) {
          exp_wTx[i] = exp_wTx_new[i];
          const double tau_tmp = 1 / (1 + exp_wTx[i]);
          tau[i] = C[i] * tau_tmp;
          D[i] = C[i] * exp_wTx[i] * tau_tmp * tau_tmp;
        }
        break;
      }
      w_norm_new = 0;
      for (int j = 0; j < w_size; ++j) {
        wpd[j] = (w[j] + wpd[j]) * 0.5;
        if (wpd[j] != 0) w_norm_new += std::fabs(wpd[j]);
      }
      delta *= 0.5;
      negsum_xTd *= 0.5;
      for (int i = 0; i < l; ++i) xTd[i] *= 0.5;
    }
    if (num_linesearch >= max_num_linesearch) {   // too many halvings: recompute exp(wᵀx) from w
      for (int i = 0; i < l; ++i) exp_wTx[i] = 0;
      for (int j = 0; j < w_size; ++j) {
        if (w[j] == 0) continue;
        const Col& c = cols[j];
        for (size_t k = 0; k < c.row.size(); ++k) exp_wTx[c.row[k]] += w[j] * c.val[k];
      }
      for (int i = 0; i < l; ++i) exp_wTx[i] = std::exp(exp_wTx[i]);
    }
    if (iter == 1) inner_eps *= 0.25;
    ++newton_iter;
    Gmax_old = Gmax_new;
  }
  for (int j = 0; j < w_size; ++j) w_out[j] = w[j];
  return newton_iter;
}
#pragma clang fp contract(on)

}  // namespace hfens
