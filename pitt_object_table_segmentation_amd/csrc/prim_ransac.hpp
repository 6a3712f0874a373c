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
//   5. optimizeModelCoefficients (elm.hpp), the refined models back, select again   2-3 syncs
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
//   refine_kind(n_inliers)       0: none, 1: refine (Elm: the model's OptimizationFunctor for elm.hpp's
//                                float Levenberg-Marquardt) and select again, 2: only normalise the
//                                direction (Eigen's LM refuses m < n) and select again
//   Elm, launch_normalize        the refinement's functor; the direction normalisation of kind 2
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <limits>
#include <memory>
#include <string>
#include <vector>

#include "compact.hpp"
#include "ctx.hpp"
#include "elm.hpp"

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

// The phase interface of one model's batch (PrimRun<M> below); pitt_classify_clusters drives runs of the
// three models, built in their own translation units, through it.
struct PrimRunBase {
    int nc = 0;
    bool any_model = false, launched = false;
    std::vector<int> refined;
    virtual ~PrimRunBase() = default;
    virtual void set_stream(hipStream_t st) = 0;
    virtual int setup() = 0;
    virtual int issue_hyp() = 0;
    virtual int issue_chunk(int chunk, bool* any) = 0;
    virtual void consume_chunk(int chunk) = 0;
    virtual int issue_best() = 0;
    virtual void read_best() = 0;
    virtual bool needs_prep_sync() const = 0;
    virtual int issue_prep() = 0;
    virtual int issue_select() = 0;
    virtual void read_select() = 0;
    virtual int issue_refine() = 0;
    virtual void read_refine() = 0;
    virtual void finish() = 0;
};

// One model's batch, phase by phase: every issue_* enqueues work on the stream without waiting, every
// read_* / consume_* uses what the last synchronisation brought back.  prim_ransac_batch drives one run,
// prim_ransac_lockstep several (pitt_classify_clusters: the sphere, cylinder and cone services share
// each synchronisation).
template <class M>
struct PrimRun final : PrimRunBase {
    using Coef = typename M::Coef;
    using Prep = typename M::Prep;
    struct St {  // RandomSampleConsensus::computeModel's state per cloud
        bool run = false;
        int iterations = 0, n_best = -INT32_MAX, best = -1;
        double k = 1.0;
        int64_t skipped = 0, a = 0;
    };
    pitt_ctx* ctx;
    M m;
    const PrimCloud* cl;
    PrimResult* res;
    hipStream_t s = nullptr;
    std::string nm;
    int64_t A = 0, max_skip = 0;
    double log_probability = 0;
    std::vector<int64_t> toff;
    int32_t *dtab = nullptr, *dflag = nullptr, *dcnt = nullptr, *tc = nullptr, *to = nullptr;  // dcnt: [nc][256]
    Coef *dcoef = nullptr, *dref = nullptr, *hcoef = nullptr;
    Prep *dprep = nullptr, *hprep = nullptr;
    int32_t *htab = nullptr, *hflag = nullptr, *hcnt = nullptr, *hto = nullptr;
    std::vector<St> st;
    std::vector<Coef> cur;
    std::vector<int> with_model, sel;
    int32_t* elm_info = nullptr;  // optional device [nc][2]: the refinements' LM status and evaluations

    PrimRun(pitt_ctx* c, const M& model, const PrimCloud* clouds, int n, PrimResult* r) : ctx(c), m(model), cl(clouds), res(r) {
        nc = n;
    }

    void set_stream(hipStream_t st) override { s = st; }
    int setup() override {
        if (!s) s = ctx->stream;
        nm = M::kName;
        if (m.max_iterations < 0 || !(m.probability > 0 && m.probability < 1))
            return ctx->fail(PITT_E_INVALID, "max_iterations / probability");
        max_skip = (int64_t)m.max_iterations * 10;
        A = (int64_t)m.max_iterations + 1 + max_skip;
        if (A > (1 << 24)) return ctx->fail(PITT_E_INVALID, "max_iterations too large");
        for (int c = 0; c < nc; ++c) {
            res[c].status = PITT_NO_MODEL;  // getSamples: "Can not select k unique points" below kSample
            res[c].hypotheses = 0;
            res[c].n_inliers = 0;
            for (int k = 0; k < 7; ++k) res[c].coef[k] = 0.0f;
            if (cl[c].n > 0x7fffffff) return ctx->fail(PITT_E_INVALID, "more than 2^31 points");
        }
        if (nc == 0) return PITT_OK;
        // per cloud A attempts of tables, models, flags and counts; tile counts for the selection
        toff.assign((size_t)nc + 1, 0);
        for (int c = 0; c < nc; ++c) toff[(size_t)c + 1] = toff[(size_t)c] + ctiles(std::max<int64_t>(cl[c].n, 1)) + 1;
        dtab = (int32_t*)ctx->buf(nm + "_table", (size_t)nc * A * M::kSample * 4);
        dcoef = (Coef*)ctx->buf(nm + "_coef", (size_t)nc * A * sizeof(Coef));
        dflag = (int32_t*)ctx->buf(nm + "_flag", (size_t)nc * A * 4);
        dcnt = (int32_t*)ctx->buf(nm + "_cnt", (size_t)nc * 256 * 4);  // the chunk's counts, all clouds
        tc = (int32_t*)ctx->buf(nm + "_tc", (size_t)toff[(size_t)nc] * 4);
        to = (int32_t*)ctx->buf(nm + "_to", (size_t)toff[(size_t)nc] * 4);
        dref = (Coef*)ctx->buf(nm + "_ref", (size_t)nc * sizeof(Coef));
        dprep = (Prep*)ctx->buf(nm + "_prep", (size_t)nc * sizeof(Prep));
        htab = (int32_t*)ctx->pinned(nm + "_table_h", (size_t)nc * A * M::kSample * 4);
        hflag = (int32_t*)ctx->pinned(nm + "_flag_h", (size_t)nc * A * 4);
        hcnt = (int32_t*)ctx->pinned(nm + "_cnt_h", (size_t)nc * 256 * 4);
        hcoef = (Coef*)ctx->pinned(nm + "_coef_h", (size_t)nc * sizeof(Coef));
        hprep = (Prep*)ctx->pinned(nm + "_prep_h", (size_t)nc * sizeof(Prep));
        hto = (int32_t*)ctx->pinned(nm + "_to_h", (size_t)nc * 4);
        if (!dtab || !dcoef || !dflag || !dcnt || !tc || !to || !dref || !dprep || !htab || !hflag || !hcnt ||
            !hcoef || !hprep || !hto)
            return ctx->fail(PITT_E_NOMEM, nm + " scratch");
        st.assign((size_t)nc, St{});
        cur.assign((size_t)nc, Coef{});
        log_probability = std::log(1.0 - m.probability);
        return PITT_OK;
    }

    // 1. every cloud's hypotheses and their validity flags
    int issue_hyp() override {
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
        return PITT_OK;
    }

    // 2. the next chunk of attempts of every cloud still running (*any: something was enqueued)
    int issue_chunk(int chunk, bool* any) override {
        *any = false;
        for (int c = 0; c < nc && !*any; ++c) *any = st[(size_t)c].run;
        if (!*any) return PITT_OK;
        // one zeroed [nc][256] count block per chunk, read back whole
        PITT_HIP_TRY(hipMemsetAsync(dcnt, 0, (size_t)nc * 256 * 4, s));
        for (int c = 0; c < nc; ++c) {
            St& q = st[(size_t)c];
            if (!q.run) continue;
            const int64_t a1 = std::min<int64_t>(A, q.a + chunk);
            const int nh = (int)(a1 - q.a);
            const int rec = ctx->prof_begin((nm + "_count").c_str(), (double)nh * (double)cl[c].n * M::kCountBytes);
            m.launch_count(s, cl[c], dcoef + (size_t)c * A, dflag + (size_t)c * A, (int)q.a, nh, dcnt + (size_t)c * 256);
            ctx->prof_end(rec);
            PITT_HIP_TRY(hipGetLastError());
        }
        PITT_HIP_TRY(hipMemcpyAsync(hcnt, dcnt, (size_t)nc * 256 * 4, hipMemcpyDeviceToHost, s));
        return PITT_OK;
    }
    // the serial loop replayed on the host over the chunk's counts
    void consume_chunk(int chunk) override {
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
    int issue_best() override {
        any_model = false;
        with_model.clear();
        for (int c = 0; c < nc; ++c) {
            res[c].hypotheses = st[(size_t)c].iterations;
            if (st[(size_t)c].best < 0) continue;
            any_model = true;
            with_model.push_back(c);
            PITT_HIP_TRY(hipMemcpyAsync(hcoef + c, dcoef + (size_t)c * A + st[(size_t)c].best, sizeof(Coef),
                                        hipMemcpyDeviceToHost, s));
        }
        return PITT_OK;
    }
    void read_best() override {
        for (int c : with_model) cur[(size_t)c] = hcoef[c];
        sel = with_model;
    }

    // 4. selectWithinDistance of the clouds in `sel`: isModelValid (+ the predicate's constants) first,
    //    on the device for the cone
    bool needs_prep_sync() const override { return M::kDevicePrep && !sel.empty(); }
    int issue_prep() override {
        if constexpr (M::kDevicePrep) {
            for (int c : sel) m.launch_prep(s, cur[(size_t)c], dprep + c);
            PITT_HIP_TRY(hipGetLastError());
            PITT_HIP_TRY(hipMemcpyAsync(hprep, dprep, (size_t)nc * sizeof(Prep), hipMemcpyDeviceToHost, s));
        }
        return PITT_OK;
    }
    int issue_select() override {
        launched = false;
        if constexpr (!M::kDevicePrep)
            for (int c : sel) m.prep_host(cur[(size_t)c], hprep + c);
        for (int c : sel) {
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
        return PITT_OK;
    }
    void read_select() override {
        for (int c : sel) res[c].n_inliers = hto[c];
    }

    // 5. optimizeModelCoefficients: PCL's float Levenberg-Marquardt (elm.hpp) for every cloud at once, one
    //    block each in one launch; the refined models back; then the selection again with them
    int issue_refine() override {
        refined.clear();
        if (!m.optimize) return PITT_OK;
        using E = typename M::Elm;
        std::vector<ElmJob> jobs;
        for (int c : with_model) {
            const int kind = m.refine_kind(res[c].n_inliers);
            if (!kind) continue;
            if (kind == 2) {
                m.launch_normalize(s, cur[(size_t)c], dref + c);
            } else {
                ElmJob jb = {};
                jb.x = cl[c].x;
                jb.y = cl[c].y;
                jb.z = cl[c].z;
                jb.inl = cl[c].inliers;
                jb.m = res[c].n_inliers;
                M::to_out(cur[(size_t)c], jb.start);
                jb.out = reinterpret_cast<float*>(dref + c);
                jb.info = elm_info ? elm_info + 2 * c : nullptr;
                jobs.push_back(jb);
            }
            refined.push_back(c);
        }
        const int rec = jobs.empty() ? -1 : ctx->prof_begin((nm + "_lm").c_str(), 0.0);
        const int rc = launch_elm_batch<E>(ctx, s, jobs, M::kName);
        ctx->prof_end(rec);
        if (rc != PITT_OK) return rc;
        PITT_HIP_TRY(hipGetLastError());
        for (int c : refined) PITT_HIP_TRY(hipMemcpyAsync(hcoef + c, dref + c, sizeof(Coef), hipMemcpyDeviceToHost, s));
        return PITT_OK;
    }
    void read_refine() override {
        for (int c : refined) cur[(size_t)c] = hcoef[c];
        sel = refined;
    }

    void finish() override {
        for (int c : with_model) {
            res[c].status = PITT_OK;
            M::to_out(cur[(size_t)c], res[c].coef);
        }
    }
};

// Several runs (different models, the same clouds or not) in lockstep on one stream: each phase is
// enqueued for every run, then one synchronisation serves them all.  Every run's own launches keep their
// order, so each result is that of its run alone.
// streams: one per run (nullptr / absent: the context's), so that the runs' small launches overlap on
// the device; a phase's synchronisation then waits for all of them.
inline int prim_ransac_lockstep(pitt_ctx* ctx, const std::vector<PrimRunBase*>& runs,
                                const std::vector<hipStream_t>& streams = {}) {
#ifdef PITT_SYNC_CHECK
    ctx->check_canaries("primitive lockstep entry");
    struct ExitCheck {
        pitt_ctx* c;
        ~ExitCheck() { c->check_canaries("primitive lockstep exit"); }
    } exit_check{ctx};
#endif
    std::vector<hipStream_t> used;
    for (size_t i = 0; i < runs.size(); ++i) {
        hipStream_t st = i < streams.size() && streams[i] ? streams[i] : ctx->stream;
        runs[i]->set_stream(st);
        if (std::find(used.begin(), used.end(), st) == used.end()) used.push_back(st);
    }
    auto sync = [&]() -> int {
        for (hipStream_t st : used) PITT_HIP_TRY(hipStreamSynchronize(st));
        return PITT_OK;
    };
    int rc;
    for (PrimRunBase* r : runs)
        if ((rc = r->setup()) != PITT_OK) return rc;
    bool work = false;
    for (PrimRunBase* r : runs) work = work || r->nc > 0;
    if (!work) return PITT_OK;
    for (PrimRunBase* r : runs)
        if ((rc = r->issue_hyp()) != PITT_OK) return rc;
    if ((rc = sync()) != PITT_OK) return rc;
    for (int chunk = 32;; chunk = std::min(chunk * 2, 256)) {
        bool any = false;
        for (PrimRunBase* r : runs) {
            bool a = false;
            if ((rc = r->issue_chunk(chunk, &a)) != PITT_OK) return rc;
            any = any || a;
        }
        if (!any) break;
        if ((rc = sync()) != PITT_OK) return rc;
        for (PrimRunBase* r : runs) r->consume_chunk(chunk);
    }
    bool models = false;
    for (PrimRunBase* r : runs) {
        if ((rc = r->issue_best()) != PITT_OK) return rc;
        models = models || r->any_model;
    }
    if (!models) return PITT_OK;
    if ((rc = sync()) != PITT_OK) return rc;
    for (PrimRunBase* r : runs) r->read_best();
    auto select_phase = [&]() -> int {
        bool prep = false;
        for (PrimRunBase* r : runs) prep = prep || r->needs_prep_sync();
        int e;
        if (prep) {
            for (PrimRunBase* r : runs)
                if ((e = r->issue_prep()) != PITT_OK) return e;
            if ((e = sync()) != PITT_OK) return e;
        }
        bool any = false;
        for (PrimRunBase* r : runs) {
            if ((e = r->issue_select()) != PITT_OK) return e;
            any = any || r->launched;
        }
        if (any && (e = sync()) != PITT_OK) return e;
        for (PrimRunBase* r : runs) r->read_select();
        return PITT_OK;
    };
    if ((rc = select_phase()) != PITT_OK) return rc;
    bool refine = false;
    for (PrimRunBase* r : runs) {
        if ((rc = r->issue_refine()) != PITT_OK) return rc;
        refine = refine || !r->refined.empty();
    }
    if (refine) {
        if ((rc = sync()) != PITT_OK) return rc;
        for (PrimRunBase* r : runs) r->read_refine();
        if ((rc = select_phase()) != PITT_OK) return rc;
    }
    for (PrimRunBase* r : runs) r->finish();
    return sync();  // every stream idle: the inlier lists are complete for whoever reads them next
}

template <class M>
int prim_ransac_batch(pitt_ctx* ctx, const M& m, const PrimCloud* cl, int nc, PrimResult* res) {
    PrimRun<M> run(ctx, m, cl, nc, res);
    return prim_ransac_lockstep(ctx, {&run});
}

}  // namespace pitt
