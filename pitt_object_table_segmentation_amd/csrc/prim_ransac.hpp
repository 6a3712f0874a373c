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

// One cloud's counting launch of a chunk (the multi-cloud count kernels take an array, blockIdx.z).
template <class Coef>
struct CountJob {
    PrimCloud cl;
    const Coef* coef;
    const int32_t* flag;
    int a0, nh;
    int32_t* counts;
};

struct PrimResult {
    int status;        // PITT_OK (a model), PITT_NO_MODEL, or an error code
    int hypotheses;    // computeModel iterations
    int64_t n_inliers;
    float coef[7];
};

// The winning (or refined) model of every cloud c with sel[c] >= 0: coef[c * A + sel[c]] (A = 0, sel[c] = 0:
// coef[c]) into out[c].
template <class Coef>
__global__ void k_gather_coef(const Coef* __restrict__ coef, int64_t A, const int32_t* __restrict__ sel, int nc,
                              Coef* __restrict__ out) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c < nc && sel[c] >= 0) out[c] = coef[(int64_t)c * A + sel[c]];
}

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
    int32_t *hsel = nullptr, *dsel = nullptr;  // per cloud: the best attempt (or 0 / -1) for k_gather_coef / prep
    Coef* dbest = nullptr;
    bool prep_ready = false;  // the device prep of `sel` already came back with the models
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
        hsel = (int32_t*)ctx->pinned(nm + "_sel_idx_h", (size_t)nc * 4);
        dsel = (int32_t*)ctx->buf(nm + "_sel_idx", (size_t)nc * 4);
        dbest = (Coef*)ctx->buf(nm + "_best", (size_t)nc * sizeof(Coef));
        if (!dtab || !dcoef || !dflag || !dcnt || !tc || !to || !dref || !dprep || !htab || !hflag || !hcnt ||
            !hcoef || !hprep || !hto || !hsel || !dsel || !dbest)
            return ctx->fail(PITT_E_NOMEM, nm + " scratch");
        st.assign((size_t)nc, St{});
        cur.assign((size_t)nc, Coef{});
        log_probability = std::log(1.0 - m.probability);
        return PITT_OK;
    }

    // 1. every cloud's hypotheses and their validity flags
    //    (the clouds' sampler tables go up in one copy and their flags come back in one)
    //    (a slot that already holds the cloud's table from an earlier call -- same buffer, same arena
    //    generation, same slot stride A, same (n, seed, attempts) -- is not uploaded again)
    int issue_hyp() override {
        pitt_ctx::PrimTableMemo& memo = ctx->prim_tables[nm];
        if (memo.dev != (const void*)dtab || memo.gen != ctx->arena_gen || memo.stride != A) {
            // another buffer, or another slot layout: every slot's device region may hold anything
            memo.dev = dtab;
            memo.gen = ctx->arena_gen;
            memo.stride = A;
            memo.keys.clear();
        }
        const auto kNone = std::make_tuple((int64_t)-1, 0u, (int64_t)0);
        if (memo.keys.size() < (size_t)nc) memo.keys.resize((size_t)nc, kNone);
        int c0 = nc, c1 = 0, u0 = nc, u1 = 0;  // the clouds that sample; those whose table goes up
        for (int c = 0; c < nc; ++c) {
            if (cl[c].n < M::kSample) {
                // no table for this cloud: the range copy below may overwrite its slot with whatever the
                // pinned staging holds there, so the slot no longer holds a known table
                memo.keys[(size_t)c] = kNone;
                continue;
            }
            st[(size_t)c].run = true;
            c0 = std::min(c0, c);
            c1 = c + 1;
            const auto key = std::make_tuple(cl[c].n, m.seed, A);
            if (memo.keys[(size_t)c] == key) continue;
            const std::vector<int32_t>& tab = sampler_table(ctx, cl[c].n, m.seed, A, M::kSample);
            std::copy(tab.begin(), tab.end(), htab + (size_t)c * A * M::kSample);
            memo.keys[(size_t)c] = key;
            u0 = std::min(u0, c);
            u1 = c + 1;
        }
        if (c0 >= c1) return PITT_OK;
        if (u0 < u1)
            PITT_HIP_TRY(hipMemcpyAsync(dtab + (size_t)u0 * A * M::kSample, htab + (size_t)u0 * A * M::kSample,
                                        (size_t)(u1 - u0) * A * M::kSample * 4, hipMemcpyHostToDevice, s));
        for (int c = c0; c < c1; ++c) {
            if (!st[(size_t)c].run) continue;
            const int rec = ctx->prof_begin((nm + "_model").c_str(), (double)A * M::kModelBytes);
            m.launch_model(s, cl[c], dtab + (size_t)c * A * M::kSample, (int)A, dcoef + (size_t)c * A,
                           dflag + (size_t)c * A);
            ctx->prof_end(rec);
            PITT_HIP_TRY(hipGetLastError());
        }
        PITT_HIP_TRY(hipMemcpyAsync(hflag + (size_t)c0 * A, dflag + (size_t)c0 * A, (size_t)(c1 - c0) * A * 4,
                                    hipMemcpyDeviceToHost, s));
        return PITT_OK;
    }

    // 2. the next chunk of attempts of every cloud still running (*any: something was enqueued)
    int issue_chunk(int chunk, bool* any) override {
        *any = false;
        for (int c = 0; c < nc && !*any; ++c) *any = st[(size_t)c].run;
        if (!*any) return PITT_OK;
        // one zeroed [nc][256] count block per chunk, read back whole
        PITT_HIP_TRY(hipMemsetAsync(dcnt, 0, (size_t)nc * 256 * 4, s));
        if (!ctx->prof) {  // every running cloud's counts in one launch (profiling runs keep one per cloud)
            using Job = CountJob<Coef>;
            Job* hj = (Job*)ctx->pinned(nm + "_cjobs_h", (size_t)nc * sizeof(Job));
            Job* dj = (Job*)ctx->buf(nm + "_cjobs", (size_t)nc * sizeof(Job));
            if (!hj || !dj) return ctx->fail(PITT_E_NOMEM, nm + " count jobs");
            int k = 0, nh_max = 0;
            int64_t bx_max = 0;
            for (int c = 0; c < nc; ++c) {
                St& q = st[(size_t)c];
                if (!q.run) continue;
                const int nh = (int)(std::min<int64_t>(A, q.a + chunk) - q.a);
                hj[k++] = Job{cl[c], dcoef + (size_t)c * A, dflag + (size_t)c * A, (int)q.a, nh, dcnt + (size_t)c * 256};
                nh_max = std::max(nh_max, nh);
                bx_max = std::max<int64_t>(bx_max, (cl[c].n + M::kCountSpan - 1) / M::kCountSpan);
            }
            PITT_HIP_TRY(hipMemcpyAsync(dj, hj, (size_t)k * sizeof(Job), hipMemcpyHostToDevice, s));
            m.launch_count_multi(s, dj, k, (int)std::max<int64_t>(bx_max, 1), nh_max);
            PITT_HIP_TRY(hipGetLastError());
            PITT_HIP_TRY(hipMemcpyAsync(hcnt, dcnt, (size_t)nc * 256 * 4, hipMemcpyDeviceToHost, s));
            return PITT_OK;
        }
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
    //    (gathered on the device and read back in one copy; the cone's device prep of them rides along)
    int issue_best() override {
        any_model = false;
        prep_ready = false;
        with_model.clear();
        for (int c = 0; c < nc; ++c) {
            res[c].hypotheses = st[(size_t)c].iterations;
            hsel[c] = st[(size_t)c].best;
            if (st[(size_t)c].best < 0) continue;
            any_model = true;
            with_model.push_back(c);
        }
        if (!any_model) return PITT_OK;
        PITT_HIP_TRY(hipMemcpyAsync(dsel, hsel, (size_t)nc * 4, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_gather_coef<Coef>, dim3((unsigned)((nc + 63) / 64)), dim3(64), 0, s, dcoef, A, dsel, nc, dbest);
        PITT_HIP_TRY(hipGetLastError());
        PITT_HIP_TRY(hipMemcpyAsync(hcoef, dbest, (size_t)nc * sizeof(Coef), hipMemcpyDeviceToHost, s));
        if constexpr (M::kDevicePrep) {
            if (!ctx->prof) {  // profiling runs keep the per-cloud prep launches
                m.launch_prep_multi(s, dbest, dsel, nc, dprep);
                PITT_HIP_TRY(hipGetLastError());
                PITT_HIP_TRY(hipMemcpyAsync(hprep, dprep, (size_t)nc * sizeof(Prep), hipMemcpyDeviceToHost, s));
                prep_ready = true;
            }
        }
        return PITT_OK;
    }
    void read_best() override {
        for (int c : with_model) cur[(size_t)c] = hcoef[c];
        sel = with_model;
    }

    // 4. selectWithinDistance of the clouds in `sel`: isModelValid (+ the predicate's constants) first,
    //    on the device for the cone
    bool needs_prep_sync() const override { return M::kDevicePrep && !sel.empty() && !prep_ready; }
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
        // every selected cloud small (the classification's clusters): one k_select_small launch, one block
        // per cloud, and their counts back in one copy
        bool small = !ctx->prof;  // profiling runs keep the per-cloud kernels (their names are priced)
        for (int c : sel) small = small && ctiles(cl[c].n) <= kSelectSmallTiles;
        if (small && !sel.empty()) {
            using Item = SelectItem<typename M::SelPred, typename M::SelAct>;
            Item* hi = (Item*)ctx->pinned(nm + "_sel_h", (size_t)nc * sizeof(Item));
            Item* di = (Item*)ctx->buf(nm + "_sel", (size_t)nc * sizeof(Item));
            int32_t* dn = (int32_t*)ctx->buf(nm + "_sel_n", (size_t)nc * 4);
            if (!hi || !di || !dn) return ctx->fail(PITT_E_NOMEM, nm + " selection");
            int k = 0;
            for (int c : sel) {
                res[c].n_inliers = 0;
                if (!m.prep_valid(hprep[c])) continue;
                hi[k++] = Item{m.sel_pred(cl[c], cur[(size_t)c], hprep[c]), M::sel_act(cl[c]), cl[c].n, dn + c};
            }
            PITT_HIP_TRY(hipMemsetAsync(dn, 0, (size_t)nc * 4, s));
            if (k > 0) {
                PITT_HIP_TRY(hipMemcpyAsync(di, hi, (size_t)k * sizeof(Item), hipMemcpyHostToDevice, s));
                hipLaunchKernelGGL((k_select_small<typename M::SelPred, typename M::SelAct>), dim3((unsigned)k),
                                   dim3(kBlock), 0, s, di);
                PITT_HIP_TRY(hipGetLastError());
            }
            PITT_HIP_TRY(hipMemcpyAsync(hto, dn, (size_t)nc * 4, hipMemcpyDeviceToHost, s));
            launched = true;
            return PITT_OK;
        }
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
        prep_ready = false;
        if (refined.empty()) return PITT_OK;
        PITT_HIP_TRY(hipMemcpyAsync(hcoef, dref, (size_t)nc * sizeof(Coef), hipMemcpyDeviceToHost, s));
        if constexpr (M::kDevicePrep) {
            if (!ctx->prof) {  // the refined models' device prep rides along
                for (int c = 0; c < nc; ++c) hsel[c] = -1;
                for (int c : refined) hsel[c] = 0;
                PITT_HIP_TRY(hipMemcpyAsync(dsel, hsel, (size_t)nc * 4, hipMemcpyHostToDevice, s));
                m.launch_prep_multi(s, dref, dsel, nc, dprep);
                PITT_HIP_TRY(hipGetLastError());
                PITT_HIP_TRY(hipMemcpyAsync(hprep, dprep, (size_t)nc * sizeof(Prep), hipMemcpyDeviceToHost, s));
                prep_ready = true;
            }
        }
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
