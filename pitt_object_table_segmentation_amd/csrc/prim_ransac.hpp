// prim_ransac.hpp -- the host driver shared by the sphere, cylinder and cone services
// (SampleConsensusModel{Sphere,Cylinder,Cone} under RandomSampleConsensus::computeModel, then
// optimizeModelCoefficients and selectWithinDistance), for one cloud or for a batch of clouds.
//
// A batch runs the clouds in lockstep, phase by phase, with one host synchronisation per phase for
// the whole batch instead of one per cloud (ransac_segmentation.cpp:230-258 calls the four services
// once per cluster; pitt_classify_clusters runs them for all of a frame's clusters at once):
//   1. every cloud's sampler-table hypotheses (the model kernel, one thread per attempt) and their
//      validity flags back to the host                                            1 sync
//   2. chunks of 32, 64, 128, then 256 attempts: the count kernel of every cloud still running, the
//      counts back, and PCL's serial computeModel loop replayed per cloud on the host  1 sync / chunk
//   3. the winning models back                                                    1 sync
//   4. selectWithinDistance (isModelValid first; the cone's needs device math)     1-2 syncs
//   5. optimizeModelCoefficients (lm.hpp), the refined models back, select again   2-3 syncs
// Per cloud the launches, their order and every value are those of the single-cloud service, so a
// batch of one is the service (the single-cloud entry points call this with nc = 1).
//
// The model traits M provide (sphere.hip, cylinder.hip, cone.hip):
//   Coef, Prep                   the model's coefficients, selectWithinDistance's prepared constants
//   kSample, kName               sample size (and the w exponent of computeModel), kernel-name prefix
//   kModelBytes, kCountBytes     algorithmic bytes per attempt / per (attempt, point) for profiling
//   to_out                       the coefficients as floats
//   max_iterations, probability, seed, optimize
//   launch_model / launch_count  the hypothesis and counting kernels of one cloud
//   kDevicePrep, prep_host / launch_prep, prep_valid   isModelValid (+ constants) on host or device
//   launch_select                k_pred_count / k_scan_tiles / k_pred_apply of one cloud
//   refine_kind(n_inliers)       0: none, 1: refine and select again
//   launch_refine                the refinement of one cloud into a device Coef
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <limits>
#include <string>
#include <vector>

#include "compact.hpp"
#include "ctx.hpp"

namespace pitt {

struct PrimCloud {
    const float *x, *y, *z, *nx, *ny, *nz;  // device SoA (normals unused by the sphere)
    int64_t n;
    int32_t* inliers;  // device, capacity n: the final inliers, ascending
};

struct PrimResult {
    int status;        // PITT_OK (a model), PITT_NO_MODEL, or an error code
    int hypotheses;    // computeModel iterations
    int64_t n_inliers;
    float coef[7];
};

template <class M>
int prim_ransac_batch(pitt_ctx* ctx, const M& m, const PrimCloud* cl, int nc, PrimResult* res) {
    using Coef = typename M::Coef;
    using Prep = typename M::Prep;
    hipStream_t s = ctx->stream;
    const std::string nm = M::kName;
    if (m.max_iterations < 0 || !(m.probability > 0 && m.probability < 1))
        return ctx->fail(PITT_E_INVALID, "max_iterations / probability");
    const int64_t max_skip = (int64_t)m.max_iterations * 10;
    const int64_t A = (int64_t)m.max_iterations + 1 + max_skip;
    if (A > (1 << 24)) return ctx->fail(PITT_E_INVALID, "max_iterations too large");
    for (int c = 0; c < nc; ++c) {
        res[c].status = PITT_NO_MODEL;  // getSamples: "Can not select k unique points" below kSample
        res[c].hypotheses = 0;
        res[c].n_inliers = 0;
        for (int k = 0; k < 7; ++k) res[c].coef[k] = 0.0f;
        if (cl[c].n > 0x7fffffff) return ctx->fail(PITT_E_INVALID, "more than 2^31 points");
    }
    if (nc == 0) return PITT_OK;
    // scratch: per cloud A attempts of tables, models, flags and counts; tile counts for the selection
    std::vector<int64_t> toff((size_t)nc + 1, 0);
    for (int c = 0; c < nc; ++c) toff[(size_t)c + 1] = toff[(size_t)c] + ctiles(std::max<int64_t>(cl[c].n, 1)) + 1;
    int32_t* dtab = (int32_t*)ctx->buf(nm + "_table", (size_t)nc * A * M::kSample * 4);
    Coef* dcoef = (Coef*)ctx->buf(nm + "_coef", (size_t)nc * A * sizeof(Coef));
    int32_t* dflag = (int32_t*)ctx->buf(nm + "_flag", (size_t)nc * A * 4);
    int32_t* dcnt = (int32_t*)ctx->buf(nm + "_cnt", (size_t)nc * A * 4);
    int32_t* tc = (int32_t*)ctx->buf(nm + "_tc", (size_t)toff[(size_t)nc] * 4);
    int32_t* to = (int32_t*)ctx->buf(nm + "_to", (size_t)toff[(size_t)nc] * 4);
    Coef* dref = (Coef*)ctx->buf(nm + "_ref", (size_t)nc * sizeof(Coef));
    Prep* dprep = (Prep*)ctx->buf(nm + "_prep", (size_t)nc * sizeof(Prep));
    int32_t* htab = (int32_t*)ctx->pinned(nm + "_table_h", (size_t)nc * A * M::kSample * 4);
    int32_t* hflag = (int32_t*)ctx->pinned(nm + "_flag_h", (size_t)nc * A * 4);
    int32_t* hcnt = (int32_t*)ctx->pinned(nm + "_cnt_h", (size_t)nc * 256 * 4);
    Coef* hcoef = (Coef*)ctx->pinned(nm + "_coef_h", (size_t)nc * sizeof(Coef));
    Prep* hprep = (Prep*)ctx->pinned(nm + "_prep_h", (size_t)nc * sizeof(Prep));
    int32_t* hto = (int32_t*)ctx->pinned(nm + "_to_h", (size_t)nc * 4);
    if (!dtab || !dcoef || !dflag || !dcnt || !tc || !to || !dref || !dprep || !htab || !hflag || !hcnt || !hcoef ||
        !hprep || !hto)
        return ctx->fail(PITT_E_NOMEM, nm + " scratch");
    // per-cloud replay state (RandomSampleConsensus::computeModel)
    struct St {
        bool run = false;
        int iterations = 0, n_best = -INT32_MAX, best = -1;
        double k = 1.0;
        int64_t skipped = 0, a = 0;
    };
    std::vector<St> st((size_t)nc);
    const double log_probability = std::log(1.0 - m.probability);

    // 1. hypotheses
    for (int c = 0; c < nc; ++c) {
        if (cl[c].n < M::kSample) continue;
        st[(size_t)c].run = true;
        const std::vector<int32_t>& tab = sampler_table(ctx, cl[c].n, m.seed, A, M::kSample);
        int32_t* ht = htab + (size_t)c * A * M::kSample;
        std::copy(tab.begin(), tab.end(), ht);
        int32_t* dt = dtab + (size_t)c * A * M::kSample;
        PITT_HIP_TRY(hipMemcpyAsync(dt, ht, (size_t)A * M::kSample * 4, hipMemcpyHostToDevice, s));
        const int rec = ctx->prof_begin((nm + "_model").c_str(), (double)A * M::kModelBytes);
        m.launch_model(s, cl[c], dt, (int)A, dcoef + (size_t)c * A, dflag + (size_t)c * A);
        ctx->prof_end(rec);
        PITT_HIP_TRY(hipGetLastError());
        PITT_HIP_TRY(hipMemcpyAsync(hflag + (size_t)c * A, dflag + (size_t)c * A, (size_t)A * 4,
                                    hipMemcpyDeviceToHost, s));
    }
    PITT_HIP_TRY(hipStreamSynchronize(s));

    // 2. chunks of attempts, every running cloud per chunk, the serial loop replayed on the host
    for (int chunk = 32;; chunk = std::min(chunk * 2, 256)) {
        bool any = false;
        for (int c = 0; c < nc; ++c) {
            St& q = st[(size_t)c];
            if (!q.run) continue;
            any = true;
            const int64_t a1 = std::min<int64_t>(A, q.a + chunk);
            const int nh = (int)(a1 - q.a);
            int32_t* dc = dcnt + (size_t)c * A + q.a;
            PITT_HIP_TRY(hipMemsetAsync(dc, 0, (size_t)nh * 4, s));
            const int rec = ctx->prof_begin((nm + "_count").c_str(), (double)nh * (double)cl[c].n * M::kCountBytes);
            m.launch_count(s, cl[c], dcoef + (size_t)c * A, dflag + (size_t)c * A, (int)q.a, nh, dc);
            ctx->prof_end(rec);
            PITT_HIP_TRY(hipGetLastError());
            PITT_HIP_TRY(hipMemcpyAsync(hcnt + (size_t)c * 256, dc, (size_t)nh * 4, hipMemcpyDeviceToHost, s));
        }
        if (!any) break;
        PITT_HIP_TRY(hipStreamSynchronize(s));
        for (int c = 0; c < nc; ++c) {
            St& q = st[(size_t)c];
            if (!q.run) continue;
            const int64_t a1 = std::min<int64_t>(A, q.a + chunk);
            const double one_over_indices = 1.0 / (double)cl[c].n;
            const int32_t* hf = hflag + (size_t)c * A;
            bool done = false;
            for (int64_t i = q.a; i < a1; ++i) {
                if (!(q.iterations < q.k && q.skipped < max_skip)) {
                    done = true;
                    break;
                }
                if (hf[i] == 0) {
                    ++q.skipped;
                    continue;
                }
                const int n_in = hcnt[(size_t)c * 256 + (size_t)(i - q.a)];
                if (n_in > q.n_best) {
                    q.n_best = n_in;
                    q.best = (int)i;
                    const double w = (double)q.n_best * one_over_indices;
                    double p_no = 1.0 - std::pow(w, (double)M::kSample);
                    p_no = std::max(std::numeric_limits<double>::epsilon(), p_no);
                    p_no = std::min(1.0 - std::numeric_limits<double>::epsilon(), p_no);
                    q.k = log_probability / std::log(p_no);
                }
                ++q.iterations;
                if (q.iterations > m.max_iterations) {
                    done = true;
                    break;
                }
            }
            q.a = a1;
            if (done || q.a >= A) q.run = false;
        }
    }

    // 3. the winning models
    bool any_model = false;
    for (int c = 0; c < nc; ++c) {
        res[c].hypotheses = st[(size_t)c].iterations;
        if (st[(size_t)c].best < 0) continue;
        any_model = true;
        PITT_HIP_TRY(hipMemcpyAsync(hcoef + c, dcoef + (size_t)c * A + st[(size_t)c].best, sizeof(Coef),
                                    hipMemcpyDeviceToHost, s));
    }
    if (!any_model) return PITT_OK;
    PITT_HIP_TRY(hipStreamSynchronize(s));
    std::vector<Coef> cur((size_t)nc);
    for (int c = 0; c < nc; ++c) cur[(size_t)c] = hcoef[c];

    // 4. selectWithinDistance of the clouds in `which`
    auto select = [&](const std::vector<int>& which) -> int {
        if (which.empty()) return PITT_OK;
        if constexpr (M::kDevicePrep) {
            for (int c : which) m.launch_prep(s, cur[(size_t)c], dprep + c);
            PITT_HIP_TRY(hipGetLastError());
            PITT_HIP_TRY(hipMemcpyAsync(hprep, dprep, (size_t)nc * sizeof(Prep), hipMemcpyDeviceToHost, s));
            PITT_HIP_TRY(hipStreamSynchronize(s));
        } else {
            for (int c : which) m.prep_host(cur[(size_t)c], hprep + c);
        }
        bool launched = false;
        for (int c : which) {
            res[c].n_inliers = 0;
            hto[c] = 0;
            if (!m.prep_valid(hprep[c])) continue;
            const int64_t nt = ctiles(cl[c].n);
            int32_t* ctc = tc + toff[(size_t)c];
            int32_t* cto = to + toff[(size_t)c];
            m.launch_select(s, cl[c], cur[(size_t)c], hprep[c], ctc, cto, grid_for_tiles(nt));
            PITT_HIP_TRY(hipGetLastError());
            PITT_HIP_TRY(hipMemcpyAsync(hto + c, cto + nt, 4, hipMemcpyDeviceToHost, s));
            launched = true;
        }
        if (launched) PITT_HIP_TRY(hipStreamSynchronize(s));
        for (int c : which) res[c].n_inliers = hto[c];
        return PITT_OK;
    };
    std::vector<int> with_model;
    for (int c = 0; c < nc; ++c)
        if (st[(size_t)c].best >= 0) with_model.push_back(c);
    int rc = select(with_model);
    if (rc != PITT_OK) return rc;

    // 5. optimizeModelCoefficients, then the selection with the refined model
    if (m.optimize) {
        std::vector<int> refined;
        for (int c : with_model) {
            if (!m.refine_kind(res[c].n_inliers)) continue;
            const int rec = ctx->prof_begin((nm + "_lm").c_str(), (double)res[c].n_inliers * 12.0);
            rc = m.launch_refine(ctx, s, cl[c], cur[(size_t)c], res[c].n_inliers, dref + c);
            if (rc != PITT_OK) return rc;
            ctx->prof_end(rec);
            PITT_HIP_TRY(hipGetLastError());
            PITT_HIP_TRY(hipMemcpyAsync(hcoef + c, dref + c, sizeof(Coef), hipMemcpyDeviceToHost, s));
            refined.push_back(c);
        }
        if (!refined.empty()) {
            PITT_HIP_TRY(hipStreamSynchronize(s));
            for (int c : refined) cur[(size_t)c] = hcoef[c];
            rc = select(refined);
            if (rc != PITT_OK) return rc;
        }
    }
    for (int c : with_model) {
        res[c].status = PITT_OK;
        M::to_out(cur[(size_t)c], res[c].coef);
    }
    return PITT_OK;
}

}  // namespace pitt
