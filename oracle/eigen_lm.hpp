// eigen_lm.hpp -- TEST INFRASTRUCTURE (the parity checker; never linked into the product).
//
// A CPU restatement of what PCL 1.7's optimizeModelCoefficients runs for the sphere, cylinder and
// cone models (sac_model_{sphere,cylinder,cone}.hpp):
//
//     Eigen::NumericalDiff<OptimizationFunctor> num_diff (functor);
//     Eigen::LevenbergMarquardt<Eigen::NumericalDiff<OptimizationFunctor>, float> lm (num_diff);
//     int info = lm.minimize (optimized_coefficients);
//
// i.e. Eigen 3.2's unsupported NonLinearOptimization module (a port of MINPACK's lmdif): a
// forward-difference Jacobian (NumericalDiff, h = sqrt(eps) |x_j|, or sqrt(eps) when x_j = 0),
// ColPivHouseholderQR of the Jacobian, lmpar2 / qrsolv for the Levenberg-Marquardt parameter, and
// the MINPACK step-bound / ratio logic -- all in float, with Eigen's default parameters
// (factor 100, maxfev 400, ftol = xtol = sqrt(FLT_EPSILON), gtol 0, epsfcn 0).  Eigen is not in
// this image and PCL is absent: the algorithm is restated from Eigen 3.2's published
// source, and is independent of the device's refinement.
//
// Float order.  The restatement reproduces Eigen 3.2's evaluation order for an SSE2 build without
// FMA (the reference's ROS Indigo toolchain, A3): dense sums (squaredNorm, dot, sum) are Eigen's
// LinearVectorizedTraversal redux -- two 4-lane packet accumulators, predux (a0 + a2) + (a1 + a3),
// a scalar tail; the Householder GEMV (essential^T * block) is the row-major GEMV kernel -- scalar
// head up to the rhs's 16-byte boundary, one 4-lane packet accumulator, scalar tail; triangular
// products and solves follow Eigen's panel loops; blueNorm is its sequential three-range sum and
// stableNorm its 4096-element blocked scaled sum.  Allocations are taken as 16-byte aligned
// (Eigen's aligned_malloc).  These orders are restated, not observed: PCL's own binary cannot be
// run here, so this path is "parity unpinned" against a real PCL build.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <vector>

namespace elm {

enum Status {
    ImproperInputParameters = 0,
    RelativeReductionTooSmall = 1,
    RelativeErrorTooSmall = 2,
    RelativeErrorAndReductionTooSmall = 3,
    CosinusTooSmall = 4,
    TooManyFunctionEvaluation = 5,
    FtolTooSmall = 6,
    XtolTooSmall = 7,
    GtolTooSmall = 8,
    UserAsked = 9,
    NotStarted = -2,
    Running = -1
};

struct Result {
    int status = ImproperInputParameters;
    int nfev = 0, iterations = 0;
    int njac = 0, trials = 0;  // Jacobian evaluations, trial steps (MINPACK's lmdif counts 1 + njac n + trials)
};

// Everything below is instantiated for S = float (PCL's LevenbergMarquardt<..., float>) and, for the
// independent pin against MINPACK's lmdif (scipy.optimize.leastsq), for S = double.
template <class S>
struct Impl {
    static constexpr S kEps = std::numeric_limits<S>::epsilon();



// ---- Eigen 3.2 redux of a float expression (no direct access: alignedStart = 0) --------------
template <class F>
static S redux_sum(int64_t size, F f) {
    if (size <= 0) return S(0);
    const int64_t P = 4;
    const int64_t asz2 = (size / (2 * P)) * (2 * P), asz = (size / P) * P;
    S res;
    if (asz) {
        S p0[4], p1[4];
        for (int l = 0; l < 4; ++l) p0[l] = f(l);
        if (asz > P) {
            for (int l = 0; l < 4; ++l) p1[l] = f(P + l);
            for (int64_t i = 2 * P; i < asz2; i += 2 * P)
                for (int l = 0; l < 4; ++l) {
                    p0[l] = p0[l] + f(i + l);
                    p1[l] = p1[l] + f(i + P + l);
                }
            for (int l = 0; l < 4; ++l) p0[l] = p0[l] + p1[l];
            if (asz > asz2)
                for (int l = 0; l < 4; ++l) p0[l] = p0[l] + f(asz2 + l);
        }
        res = (p0[0] + p0[2]) + (p0[1] + p0[3]);
        for (int64_t i = asz; i < size; ++i) res = res + f(i);
    } else {
        res = f(0);
        for (int64_t i = 1; i < size; ++i) res = res + f(i);
    }
    return res;
}
static S sq_norm(const S* v, int64_t n) { return redux_sum(n, [&](int64_t i) { return v[i] * v[i]; }); }
static S dot(const S* a, const S* b, int64_t n) { return redux_sum(n, [&](int64_t i) { return a[i] * b[i]; }); }

// Row-major GEMV kernel's order for one row (Eigen 3.2 general_matrix_vector_product<RowMajor>):
// sum_j lhs[j] * rhs[j], rhs starting at float offset `rhs_off` of an aligned allocation.
static S gemv_dot(const S* lhs, const S* rhs, int64_t depth, int64_t rhs_off) {
    const int64_t P = 4;
    int64_t as = (P - (rhs_off % P)) % P;
    if (as > depth) as = depth;
    const int64_t asize = as + ((depth - as) & ~(P - 1));
    S tmp = 0;
    for (int64_t j = 0; j < as; ++j) tmp = tmp + lhs[j] * rhs[j];
    if (asize > as) {
        S pk[4] = {0, 0, 0, 0};
        for (int64_t j = as; j < asize; j += P)
            for (int l = 0; l < 4; ++l) pk[l] = pk[l] + lhs[j + l] * rhs[j + l];
        tmp = tmp + ((pk[0] + pk[2]) + (pk[1] + pk[3]));
    }
    for (int64_t j = asize; j < depth; ++j) tmp = tmp + lhs[j] * rhs[j];
    return tmp;
}

// ---- norms -----------------------------------------------------------------------------------
// MatrixBase::blueNorm (Eigen 3.2, Blue's algorithm; for float b1 = 2^-63, b2 = 2^52, s1m = 2^63,
// s2m = 2^-76, relerr = sqrt(2^-23)), sequential over the elements.
static S blue_norm(const S* v, int64_t n, int64_t stride = 1) {
    // Eigen's machine constants from numeric_limits (integer divisions as written there)
    const int it = std::numeric_limits<S>::digits, iemin = std::numeric_limits<S>::min_exponent,
              iemax = std::numeric_limits<S>::max_exponent;
    const S b1 = std::ldexp(S(1), -((1 - iemin) / 2)), b2 = std::ldexp(S(1), (iemax + 1 - it) / 2),
            s1m = std::ldexp(S(1), (2 - iemin) / 2), s2m = std::ldexp(S(1), -((iemax + it) / 2)),
            rbig = std::numeric_limits<S>::max();
    const S overfl = rbig * s2m;
    const S relerr = std::sqrt((S)std::pow(2.0, 1 - it));
    const S ab2 = b2 / (S)n;
    S asml = 0, amed = 0, abig = 0;
    for (int64_t i = 0; i < n; ++i) {
        const S ax = std::fabs(v[i * stride]);
        if (ax > ab2) {
            const S t = ax * s2m;
            abig = abig + t * t;
        } else if (ax < b1) {
            const S t = ax * s1m;
            asml = asml + t * t;
        } else {
            amed = amed + ax * ax;
        }
    }
    if (abig > S(0)) {
        abig = std::sqrt(abig);
        if (abig > overfl) return rbig;
        if (amed > S(0)) {
            abig = abig / s2m;
            amed = std::sqrt(amed);
        } else {
            return abig / s2m;
        }
    } else if (asml > S(0)) {
        if (amed > S(0)) {
            abig = std::sqrt(amed);
            amed = std::sqrt(asml) / s1m;
        } else {
            return std::sqrt(asml) / s1m;
        }
    } else {
        return std::sqrt(amed);
    }
    asml = std::min(abig, amed);
    abig = std::max(abig, amed);
    if (asml <= abig * relerr) return abig;
    const S q = asml / abig;
    return abig * std::sqrt(S(1) + q * q);
}

// MatrixBase::stableNorm (Eigen 3.2): 4096-element blocks, each scaled by the running max |v|.
static S stable_norm(const S* v, int64_t n) {
    const int64_t block = 4096;
    S scale = 0, inv = 1, ssq = 0;
    for (int64_t bi = 0; bi < n; bi += block) {
        const int64_t len = std::min(block, n - bi);
        S mx = std::fabs(v[bi]);
        for (int64_t i = 1; i < len; ++i) mx = std::max(mx, std::fabs(v[bi + i]));  // maxCoeff: first max
        if (mx > scale) {
            const S r = scale / mx;
            ssq = ssq * (r * r);
            scale = mx;
            inv = S(1) / scale;
        }
        ssq = ssq + redux_sum(len, [&](int64_t i) {
                  const S t = v[bi + i] * inv;
                  return t * t;
              });
    }
    return scale * std::sqrt(ssq);
}

// ---- ColPivHouseholderQR<MatrixXf> (Eigen 3.2) -------------------------------------------------
struct ColPivQR {
    int64_t m = 0, n = 0;
    std::vector<S> qr;        // column-major m x n, allocation 16-byte aligned (offsets below)
    std::vector<S> hcoeffs;   // tau_k
    std::vector<int> perm;    // colsPermutation().indices()
    int64_t nonzero_pivots = 0;
    S maxpivot = 0;

    S& at(int64_t r, int64_t c) { return qr[(size_t)(c * m + r)]; }
    S at(int64_t r, int64_t c) const { return qr[(size_t)(c * m + r)]; }

    // block B = qr(k.., k+1..) with essential = qr(k+1.., k): applyHouseholderOnTheLeft
    void apply_left(int64_t k, S tau) {
        const int64_t rows = m - k, cols = n - k - 1;
        if (cols <= 0) return;
        if (rows == 1) {
            for (int64_t c = 0; c < cols; ++c) at(k, k + 1 + c) = at(k, k + 1 + c) * (S(1) - tau);
            return;
        }
        const S* ess = &qr[(size_t)(k * m + k + 1)];
        const int64_t ess_off = k * m + k + 1;
        std::vector<S> tmp((size_t)cols);
        for (int64_t c = 0; c < cols; ++c) {
            const S* col = &qr[(size_t)((k + 1 + c) * m + k + 1)];
            tmp[(size_t)c] = gemv_dot(col, ess, rows - 1, ess_off);  // essential^T * bottom
        }
        for (int64_t c = 0; c < cols; ++c) tmp[(size_t)c] = tmp[(size_t)c] + at(k, k + 1 + c);
        for (int64_t c = 0; c < cols; ++c) at(k, k + 1 + c) = at(k, k + 1 + c) - tau * tmp[(size_t)c];
        for (int64_t c = 0; c < cols; ++c) {
            S* col = &qr[(size_t)((k + 1 + c) * m + k + 1)];
            for (int64_t i = 0; i < rows - 1; ++i) col[i] = col[i] - (tau * ess[i]) * tmp[(size_t)c];
        }
    }

    void compute(const std::vector<S>& a, int64_t rows, int64_t cols) {
        m = rows;
        n = cols;
        qr = a;
        const int64_t size = std::min(m, n);
        hcoeffs.assign((size_t)size, 0);
        std::vector<S> sq((size_t)n);
        std::vector<int64_t> transp((size_t)n, 0);
        for (int64_t k = 0; k < n; ++k) sq[(size_t)k] = sq_norm(&qr[(size_t)(k * m)], m);
        S mx = sq[0];
        for (int64_t k = 1; k < n; ++k) mx = std::max(mx, sq[(size_t)k]);
        const S threshold_helper = mx * (kEps * kEps) / (S)m;
        nonzero_pivots = size;
        maxpivot = 0;
        for (int64_t k = 0; k < size; ++k) {
            int64_t big = k;  // maxCoeff(&index): the first maximum
            for (int64_t j = k + 1; j < n; ++j)
                if (sq[(size_t)j] > sq[(size_t)big]) big = j;
            S bigsq = sq_norm(&qr[(size_t)(big * m + k)], m - k);
            sq[(size_t)big] = bigsq;
            if (nonzero_pivots == size && bigsq < threshold_helper * (S)(m - k)) nonzero_pivots = k;
            transp[(size_t)k] = big;
            if (k != big) {
                for (int64_t r = 0; r < m; ++r) std::swap(at(r, k), at(r, big));
                std::swap(sq[(size_t)k], sq[(size_t)big]);
            }
            // makeHouseholderInPlace on qr(k.., k)
            S* v = &qr[(size_t)(k * m + k)];
            const int64_t len = m - k;
            const S tail_sq = len == 1 ? S(0) : sq_norm(v + 1, len - 1);
            const S c0 = v[0];
            S tau, beta;
            if (tail_sq == S(0)) {
                tau = 0;
                beta = c0;
                for (int64_t i = 1; i < len; ++i) v[i] = 0;
            } else {
                beta = std::sqrt(c0 * c0 + tail_sq);
                if (c0 >= S(0)) beta = -beta;
                const S den = c0 - beta;
                for (int64_t i = 1; i < len; ++i) v[i] = v[i] / den;
                tau = (beta - c0) / beta;
            }
            hcoeffs[(size_t)k] = tau;
            v[0] = beta;
            if (std::fabs(beta) > maxpivot) maxpivot = std::fabs(beta);
            apply_left(k, tau);
            for (int64_t j = k + 1; j < n; ++j) {
                const S r = at(k, j);
                sq[(size_t)j] = sq[(size_t)j] - r * r;
            }
        }
        // colsPermutation: identity, then applyTranspositionOnTheRight(k, transp[k]) in order
        perm.resize((size_t)n);
        for (int64_t k = 0; k < n; ++k) perm[(size_t)k] = (int)k;
        for (int64_t k = 0; k < size; ++k) std::swap(perm[(size_t)k], perm[(size_t)transp[(size_t)k]]);
    }

    // rank(): pivots above maxpivot * eps * diagonalSize
    int64_t rank() const {
        const S th = std::fabs(maxpivot) * (kEps * (S)std::min(m, n));
        int64_t r = 0;
        for (int64_t i = 0; i < nonzero_pivots; ++i) r += std::fabs(at(i, i)) > th ? 1 : 0;
        return r;
    }

    // householderQ().adjoint() applied to a vector of m entries (HouseholderSequence, k = 0..n-1)
    void apply_qt(std::vector<S>& w) const {
        const int64_t size = std::min(m, n);
        for (int64_t k = 0; k < size; ++k) {
            const int64_t rows = m - k;
            const S tau = hcoeffs[(size_t)k];
            if (rows == 1) {
                w[(size_t)k] = w[(size_t)k] * (S(1) - tau);
                continue;
            }
            const S* ess = &qr[(size_t)(k * m + k + 1)];
            // tmp = essential^T * bottom: a (1 x K)(K x 1) inner product, Eigen's redux (dot)
            S tmp = dot(ess, &w[(size_t)(k + 1)], rows - 1);
            tmp = tmp + w[(size_t)k];
            w[(size_t)k] = w[(size_t)k] - tau * tmp;
            for (int64_t i = 0; i < rows - 1; ++i) w[(size_t)(k + 1 + i)] = w[(size_t)(k + 1 + i)] - (tau * ess[i]) * tmp;
        }
    }
};

// Upper-triangular solve R(0..r, 0..r) x = b in place (triangular_solve_vector<OnTheLeft, Upper,
// ColMajor>: one panel for r <= 8, columns from the last).
static void solve_upper_colmajor(const ColPivQR& q, int64_t r, S* b) {
    for (int64_t k = 0; k < r; ++k) {
        const int64_t i = r - k - 1;
        if (b[i] != S(0)) {
            b[i] = b[i] / q.at(i, i);
            for (int64_t s = 0; s < i; ++s) b[s] = b[s] - b[i] * q.at(s, i);
        }
    }
}

// R^T (lower, row-major view of the column-major R) x = b in place: rhs[i] -= (row . solved).sum(),
// then /= R(i, i) (triangular_solve_vector<OnTheLeft, Lower, RowMajor>, one panel).
template <class Get>
static void solve_lower_rowmajor(int64_t n, Get L, S* b) {
    for (int64_t i = 0; i < n; ++i) {
        if (i > 0) b[i] = b[i] - redux_sum(i, [&](int64_t s) { return L(i, s) * b[s]; });
        b[i] = b[i] / L(i, i);
    }
}
// Upper, row-major (a transposed column-major lower triangle): from the last row.
template <class Get>
static void solve_upper_rowmajor(int64_t n, Get U, S* b) {
    for (int64_t k = 0; k < n; ++k) {
        const int64_t i = n - k - 1;
        if (k > 0) b[i] = b[i] - redux_sum(k, [&](int64_t s) { return U(i, i + 1 + s) * b[i + 1 + s]; });
        b[i] = b[i] / U(i, i);
    }
}

// JacobiRotation::makeGivens (real)
static void make_givens(S p, S q, S* c, S* s) {
    if (q == S(0)) {
        *c = p < S(0) ? S(-1) : S(1);
        *s = 0;
    } else if (p == S(0)) {
        *c = 0;
        *s = q < S(0) ? S(1) : S(-1);
    } else if (std::fabs(p) > std::fabs(q)) {
        const S t = q / p;
        S u = std::sqrt(S(1) + t * t);
        if (p < S(0)) u = -u;
        *c = S(1) / u;
        *s = -t * *c;
    } else {
        const S t = p / q;
        S u = std::sqrt(S(1) + t * t);
        if (q < S(0)) u = -u;
        *s = -S(1) / u;
        *c = -t * *s;
    }
}

// qrsolv (Eigen 3.2 NonLinearOptimization/qrsolv.h); s: n x n column-major copy of R's top block
static void qrsolv(std::vector<S>& s, int64_t n, const std::vector<int>& ipvt, const std::vector<S>& diag,
                   const std::vector<S>& qtb, std::vector<S>& x, std::vector<S>& sdiag) {
    auto S_ = [&](int64_t r, int64_t c) -> S& { return s[(size_t)(c * n + r)]; };
    std::vector<S> wa(qtb);
    for (int64_t j = 0; j < n; ++j) x[(size_t)j] = S_(j, j);
    for (int64_t c = 0; c < n; ++c)
        for (int64_t r = c + 1; r < n; ++r) S_(r, c) = S_(c, r);  // strictly lower = upper^T
    for (int64_t j = 0; j < n; ++j) {
        const int l = ipvt[(size_t)j];
        if (diag[(size_t)l] == S(0)) break;
        for (int64_t k = j; k < n; ++k) sdiag[(size_t)k] = 0;
        sdiag[(size_t)j] = diag[(size_t)l];
        S qtbpj = 0;
        for (int64_t k = j; k < n; ++k) {
            S gc, gs;
            make_givens(-S_(k, k), sdiag[(size_t)k], &gc, &gs);
            S_(k, k) = gc * S_(k, k) + gs * sdiag[(size_t)k];
            const S temp = gc * wa[(size_t)k] + gs * qtbpj;
            qtbpj = -gs * wa[(size_t)k] + gc * qtbpj;
            wa[(size_t)k] = temp;
            for (int64_t i = k + 1; i < n; ++i) {
                const S t2 = gc * S_(i, k) + gs * sdiag[(size_t)i];
                sdiag[(size_t)i] = -gs * S_(i, k) + gc * sdiag[(size_t)i];
                S_(i, k) = t2;
            }
        }
    }
    int64_t nsing = 0;
    while (nsing < n && sdiag[(size_t)nsing] != S(0)) ++nsing;
    for (int64_t j = nsing; j < n; ++j) wa[(size_t)j] = 0;
    // s.topLeftCorner(nsing, nsing).transpose().triangularView<Upper>(): U(i, j) = s(j, i)
    solve_upper_rowmajor(nsing, [&](int64_t i, int64_t j) { return S_(j, i); }, wa.data());
    for (int64_t j = 0; j < n; ++j) {
        sdiag[(size_t)j] = S_(j, j);
        S_(j, j) = x[(size_t)j];
    }
    for (int64_t j = 0; j < n; ++j) x[(size_t)ipvt[(size_t)j]] = wa[(size_t)j];
}

// lmpar2 (Eigen 3.2 NonLinearOptimization/lmpar.h)
static void lmpar2(const ColPivQR& qr, const std::vector<S>& diag, const std::vector<S>& qtb, S delta, S& par,
                   std::vector<S>& x) {
    const S dwarf = std::numeric_limits<S>::min();
    const int64_t n = qr.n;
    std::vector<S> wa1(qtb), wa2((size_t)n);
    const int64_t rank = qr.rank();
    for (int64_t j = rank; j < n; ++j) wa1[(size_t)j] = 0;
    solve_upper_colmajor(qr, rank, wa1.data());
    for (int64_t i = 0; i < n; ++i) x[(size_t)qr.perm[(size_t)i]] = wa1[(size_t)i];  // P * wa1
    int iter = 0;
    for (int64_t j = 0; j < n; ++j) wa2[(size_t)j] = diag[(size_t)j] * x[(size_t)j];
    S dxnorm = blue_norm(wa2.data(), n);
    S fp = dxnorm - delta;
    if (fp <= S(0.1) * delta) {
        par = 0;
        return;
    }
    S parl = 0;
    if (rank == n) {
        // wa1 = P^-1 * (diag .* wa2) / dxnorm
        for (int64_t i = 0; i < n; ++i) {
            const int64_t pi = qr.perm[(size_t)i];
            wa1[(size_t)i] = (diag[(size_t)pi] * wa2[(size_t)pi]) / dxnorm;
        }
        solve_lower_rowmajor(n, [&](int64_t i, int64_t j) { return qr.at(j, i); }, wa1.data());
        const S temp = blue_norm(wa1.data(), n);
        parl = fp / delta / temp / temp;
    }
    for (int64_t j = 0; j < n; ++j)
        wa1[(size_t)j] = dot(&qr.qr[(size_t)(j * qr.m)], qtb.data(), j + 1) / diag[(size_t)qr.perm[(size_t)j]];
    const S gnorm = stable_norm(wa1.data(), n);
    S paru = gnorm / delta;
    if (paru == S(0)) paru = dwarf / std::min(delta, S(0.1));
    par = std::max(par, parl);
    par = std::min(par, paru);
    if (par == S(0)) par = gnorm / dxnorm;
    std::vector<S> s((size_t)(n * n));
    for (int64_t c = 0; c < n; ++c)
        for (int64_t r = 0; r < n; ++r) s[(size_t)(c * n + r)] = qr.at(r, c);
    std::vector<S> sdiag((size_t)n);
    while (true) {
        ++iter;
        if (par == S(0)) par = std::max(dwarf, S(.001) * paru);
        const S sp = std::sqrt(par);
        for (int64_t j = 0; j < n; ++j) wa1[(size_t)j] = sp * diag[(size_t)j];
        qrsolv(s, n, qr.perm, wa1, qtb, x, sdiag);
        for (int64_t j = 0; j < n; ++j) wa2[(size_t)j] = diag[(size_t)j] * x[(size_t)j];
        dxnorm = blue_norm(wa2.data(), n);
        S temp = fp;
        fp = dxnorm - delta;
        if (std::fabs(fp) <= S(0.1) * delta || (parl == S(0) && fp <= temp && temp < S(0)) || iter == 10) break;
        for (int64_t i = 0; i < n; ++i) {
            const int64_t pi = qr.perm[(size_t)i];
            wa1[(size_t)i] = diag[(size_t)pi] * (wa2[(size_t)pi] / dxnorm);
        }
        for (int64_t j = 0; j < n; ++j) {
            wa1[(size_t)j] = wa1[(size_t)j] / sdiag[(size_t)j];
            temp = wa1[(size_t)j];
            for (int64_t i = j + 1; i < n; ++i) wa1[(size_t)i] = wa1[(size_t)i] - s[(size_t)(j * n + i)] * temp;
        }
        temp = blue_norm(wa1.data(), n);
        const S parc = fp / delta / temp / temp;
        if (fp > S(0)) parl = std::max(parl, par);
        if (fp < S(0)) paru = std::min(paru, par);
        par = std::max(parl, par + parc);
    }
    if (iter == 0) par = 0;
}

// LevenbergMarquardt<NumericalDiff<Functor>, float>::minimize(x).  f(x, fvec): the functor's
// operator() (m residuals, float).
template <class F>
static Result minimize(F f, int64_t m, std::vector<S>& x) {
    Result res;
    const int64_t n = (int64_t)x.size();
    const S factor = 100, ftol = std::sqrt(kEps), xtol = std::sqrt(kEps), gtol = 0;
    const int maxfev = 400;
    // minimizeInit
    if (n <= 0 || m < n) return res;  // ImproperInputParameters
    std::vector<S> fvec((size_t)m), wa1((size_t)n), wa2((size_t)n), wa3((size_t)n), wa4((size_t)m), diag((size_t)n),
        qtf((size_t)n), fjac((size_t)(m * n)), v1((size_t)m), v2((size_t)m);
    int nfev = 1;
    f(x.data(), fvec.data());
    S fnorm = stable_norm(fvec.data(), m);
    S par = 0, delta = 0, xnorm = 0, temp = 0;
    int iter = 1;
    const S neps = std::sqrt(std::max(S(0), kEps));  // NumericalDiff: sqrt(max(epsfcn, eps))
    ColPivQR qr;
    while (true) {
        // ---- minimizeOneStep ----
        // NumericalDiff<Forward>::df
        {
            std::vector<S> xx(x);
            f(xx.data(), v1.data());
            for (int64_t j = 0; j < n; ++j) {
                S h = neps * std::fabs(xx[(size_t)j]);
                if (h == S(0)) h = neps;
                xx[(size_t)j] = xx[(size_t)j] + h;
                f(xx.data(), v2.data());
                xx[(size_t)j] = x[(size_t)j];
                for (int64_t i = 0; i < m; ++i) fjac[(size_t)(j * m + i)] = (v2[(size_t)i] - v1[(size_t)i]) / h;
            }
            nfev += (int)n + 1;
            ++res.njac;
        }
        for (int64_t j = 0; j < n; ++j) wa2[(size_t)j] = blue_norm(&fjac[(size_t)(j * m)], m);
        qr.compute(fjac, m, n);
        if (iter == 1) {
            for (int64_t j = 0; j < n; ++j) diag[(size_t)j] = wa2[(size_t)j] == S(0) ? S(1) : wa2[(size_t)j];
            std::vector<S> dx((size_t)n);
            for (int64_t j = 0; j < n; ++j) dx[(size_t)j] = diag[(size_t)j] * x[(size_t)j];
            xnorm = stable_norm(dx.data(), n);
            delta = factor * xnorm;
            if (delta == S(0)) delta = factor;
        }
        wa4 = fvec;
        qr.apply_qt(wa4);
        for (int64_t j = 0; j < n; ++j) qtf[(size_t)j] = wa4[(size_t)j];
        S gnorm = 0;
        if (fnorm != S(0))
            for (int64_t j = 0; j < n; ++j) {
                const S w = wa2[(size_t)qr.perm[(size_t)j]];
                if (w != S(0)) {
                    const S d = redux_sum(j + 1, [&](int64_t i) { return qr.at(i, j) * (qtf[(size_t)i] / fnorm); });
                    gnorm = std::max(gnorm, std::fabs(d / w));
                }
            }
        if (gnorm <= gtol) {
            res.status = CosinusTooSmall;
            break;
        }
        for (int64_t j = 0; j < n; ++j) diag[(size_t)j] = std::max(diag[(size_t)j], wa2[(size_t)j]);
        int status = Running;
        S ratio = 0;
        do {
            lmpar2(qr, diag, qtf, delta, par, wa1);
            for (int64_t j = 0; j < n; ++j) wa1[(size_t)j] = -wa1[(size_t)j];
            for (int64_t j = 0; j < n; ++j) wa2[(size_t)j] = x[(size_t)j] + wa1[(size_t)j];
            std::vector<S> dp((size_t)n);
            for (int64_t j = 0; j < n; ++j) dp[(size_t)j] = diag[(size_t)j] * wa1[(size_t)j];
            const S pnorm = stable_norm(dp.data(), n);
            if (iter == 1) delta = std::min(delta, pnorm);
            f(wa2.data(), wa4.data());
            ++nfev;
            ++res.trials;
            const S fnorm1 = stable_norm(wa4.data(), m);
            S actred = -1;
            if (S(.1) * fnorm1 < fnorm) {
                const S q = fnorm1 / fnorm;
                actred = S(1) - q * q;
            }
            // wa3 = R * (P^-1 * wa1): Eigen's upper TRMV, column by column
            std::vector<S> pw((size_t)n);
            for (int64_t i = 0; i < n; ++i) pw[(size_t)i] = wa1[(size_t)qr.perm[(size_t)i]];
            for (int64_t r = 0; r < n; ++r) wa3[(size_t)r] = 0;
            for (int64_t i = 0; i < n; ++i)
                for (int64_t r = 0; r <= i; ++r) wa3[(size_t)r] = wa3[(size_t)r] + pw[(size_t)i] * qr.at(r, i);
            const S t1 = stable_norm(wa3.data(), n) / fnorm;
            const S temp1 = t1 * t1;
            const S t2 = std::sqrt(par) * pnorm / fnorm;
            const S temp2 = t2 * t2;
            const S prered = temp1 + temp2 / S(.5);
            const S dirder = -(temp1 + temp2);
            ratio = 0;
            if (prered != S(0)) ratio = actred / prered;
            if (ratio <= S(.25)) {
                if (actred >= S(0)) temp = S(.5);
                if (actred < S(0)) temp = S(.5) * dirder / (dirder + S(.5) * actred);
                if (S(.1) * fnorm1 >= fnorm || temp < S(.1)) temp = S(.1);
                delta = temp * std::min(delta, pnorm / S(.1));
                par = par / temp;
            } else if (!(par != S(0) && ratio < S(.75))) {
                delta = pnorm / S(.5);
                par = S(.5) * par;
            }
            if (ratio >= S(1e-4)) {
                x = wa2;
                for (int64_t j = 0; j < n; ++j) wa2[(size_t)j] = diag[(size_t)j] * x[(size_t)j];
                fvec = wa4;
                xnorm = stable_norm(wa2.data(), n);
                fnorm = fnorm1;
                ++iter;
            }
            if (std::fabs(actred) <= ftol && prered <= ftol && S(.5) * ratio <= S(1)) {
                status = RelativeReductionTooSmall;
                break;
            }
            if (delta <= xtol * xnorm) {
                status = RelativeErrorTooSmall;
                break;
            }
            if (nfev >= maxfev) {
                status = TooManyFunctionEvaluation;
                break;
            }
            if (std::fabs(actred) <= kEps && prered <= kEps && S(.5) * ratio <= S(1)) {
                status = FtolTooSmall;
                break;
            }
            if (delta <= kEps * xnorm) {
                status = XtolTooSmall;
                break;
            }
            if (gnorm <= kEps) {
                status = GtolTooSmall;
                break;
            }
        } while (ratio < S(1e-4));
        if (status != Running) {
            res.status = status;
            break;
        }
    }
    res.nfev = nfev;
    res.iterations = iter;
    return res;
}

};

template <class S, class F>
Result minimize(F f, int64_t m, std::vector<S>& x) {
    return Impl<S>::minimize(f, m, x);
}

}  // namespace elm
