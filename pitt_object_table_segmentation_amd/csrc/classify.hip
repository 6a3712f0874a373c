// classify.hip -- primitive classification of a frame's clusters in one call: the loop of
// ransac_segmentation.cpp:230-302 (clustersAcquisition), which per cluster estimates normals (k = 50,
// :233), calls the sphere, cylinder, cone and plane services (:239-258) and arbitrates on their inlier
// counts (:265-302).  SURVEY.md s8f row 4; VERDICT r2 next #8.
//
// All clusters go through every stage together, so the host synchronises once per stage for the whole
// frame, not once per cluster and service:
//   staging      the clusters into one tile-padded device SoA (NaN padding)           no sync
//   normals      normals_batch: exhaustive k-NN inside each cluster, then k_normals   no sync
//   plane        the plane service's SACSegmentation for every cluster: one plane batch on an
//                auxiliary context's stream, overlapping the next three                 1 sync
//   sphere / cylinder / cone   one prim_ransac_lockstep of the three models' runs (sphere.hip,
//                cylinder.hip, cone.hip): each phase's synchronisation serves all three  ~6 + chunks
//   axis height  the cylinder and cone services' post-processing, axis_height_batch    1 sync
//   responses    PCManager::inlierToVectorMsg drops inlier index 0 (Q1): the first inlier of every
//                list read back in one copy                                          1 sync
//   arbitration  on the response sizes, as the reference (host, scalar)
// Each stage runs the same kernels on the same values as the per-cluster service, so the counts,
// coefficients, heights and centroids equal the services' (tests/test_classify_gpu.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "compact.hpp"
#include "ctx.hpp"
#include "prim_ransac.hpp"

namespace pitt {

int finish_batch(pitt_ctx* ctx);
int normals_batch(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n_total, const int64_t* off,
                  const int64_t* cnt, int nc, int k, const float vp[3], float* nx, float* ny, float* nz, float* curv);
std::unique_ptr<PrimRunBase> sphere_run(pitt_ctx* ctx, const pitt_sphere_params* p, const PrimCloud* cl, int nc,
                                        PrimResult* res);
std::unique_ptr<PrimRunBase> cylinder_run(pitt_ctx* ctx, const pitt_cylinder_params* p, const PrimCloud* cl, int nc,
                                          PrimResult* res);
std::unique_ptr<PrimRunBase> cone_run(pitt_ctx* ctx, const pitt_cone_params* p, const PrimCloud* cl, int nc,
                                      PrimResult* res);
int axis_height_batch(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n_total,
                      const int64_t* off, const int64_t* n, const float* coef6, const int32_t* mode, int nj,
                      float* height, int32_t* idx1, int32_t* idx2, float* centroid3);

// the first inlier of every (service, cluster) list with inliers (-1 for an empty one)
__global__ void k_first_inliers(const int32_t* __restrict__ const* lists, const int64_t* __restrict__ off,
                                const int64_t* __restrict__ n_inl, int nc, int32_t* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 4 * nc) return;
    const int srv = i / nc, c = i - srv * nc;
    out[i] = n_inl[i] > 0 ? lists[srv][off[c]] : -1;
}

// ransac_segmentation.cpp:265-302 on the response sizes (size_t); the cone's priority compares
// (float)coneInl with (float)cylinderInl * 0.9f
int arbitrate(int64_t sph, int64_t cyl, int64_t cone, int64_t plane, float cone_over_cylinder) {
    if (!plane && !sph && !cyl && !cone) return PITT_SHAPE_UNKNOWN;
    if (cone >= plane && cone >= sph && (float)cone >= (float)cyl * cone_over_cylinder) return PITT_SHAPE_CONE;
    if (cyl >= plane && cyl >= cone && cyl >= sph) return PITT_SHAPE_CYLINDER;
    if (plane >= cone && plane >= sph && plane >= cyl) return PITT_SHAPE_PLANE;
    if (sph >= plane && sph >= cone && sph >= cyl) return PITT_SHAPE_SPHERE;
    return PITT_SHAPE_UNKNOWN;
}

}  // namespace pitt

extern "C" void pitt_classify_params_default(pitt_classify_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof *p);
    p->k = 50;  // pc_manager.cpp:18
    pitt_sac_params_default(&p->plane);
    // sphere_segmentation_srv.cpp:20-23, :61
    p->sphere.threshold = 0.007;
    p->sphere.max_iterations = 1000;
    p->sphere.optimize = 1;
    p->sphere.probability = 0.99;
    p->sphere.radius_min = 0.005;
    p->sphere.radius_max = 0.5;
    p->sphere.seed = 12345u;
    // cylinder_segmentation_srv.cpp:23-27, :114
    p->cylinder.threshold = 0.008;
    p->cylinder.max_iterations = 1000;
    p->cylinder.optimize = 1;
    p->cylinder.probability = 0.99;
    p->cylinder.radius_min = 0.005;
    p->cylinder.radius_max = 0.5;
    p->cylinder.normal_distance_weight = 0.001;
    p->cylinder.seed = 12345u;
    // cone_segmentation_srv.cpp:24-31, :115-125
    p->cone.threshold = 0.0055;
    p->cone.max_iterations = 1000;
    p->cone.optimize = 1;
    p->cone.probability = 0.99;
    p->cone.normal_distance_weight = 0.0006;
    p->cone.min_angle = 10.0 / 180.0 * M_PI;
    p->cone.max_angle = 170.0 / 180.0 * M_PI;
    p->cone.eps_angle = 0.4;
    p->cone.seed = 12345u;
    p->cone_over_cylinder = 0.9f;  // DEFAULT_CONE_OVER_CYLINDER_PRIORITY, ransac_segmentation.cpp:37
}

namespace pitt {
// The clusters staged into the tile-padded SoA: cluster blockIdx.y's points [0, span) of its slot, the
// cluster's own points first, NaN after them.  meta: offsets [nc], counts [nc], slot starts [nc].
__global__ __launch_bounds__(256) void k_stage_clusters(const float* __restrict__ x, const float* __restrict__ y,
                                                        const float* __restrict__ z, const int64_t* __restrict__ meta,
                                                        int nc, int64_t total, float* __restrict__ sx,
                                                        float* __restrict__ sy, float* __restrict__ sz) {
    const int c = blockIdx.y;
    const int64_t off = meta[c], n = meta[nc + c], so = meta[2 * nc + c];
    const int64_t end = c + 1 < nc ? meta[2 * nc + c + 1] : total;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (so + i >= end) return;
    const bool in = i < n;
    sx[so + i] = in ? x[off + i] : __builtin_nanf("");
    sy[so + i] = in ? y[off + i] : __builtin_nanf("");
    sz[so + i] = in ? z[off + i] : __builtin_nanf("");
}
}  // namespace pitt

extern "C" int pitt_classify_clusters(pitt_ctx* ctx, const float* x, const float* y, const float* z,
                                      const int64_t* offsets, const int64_t* counts, int32_t n_clusters,
                                      const pitt_classify_params* prm, pitt_cluster_shape* out) {
    using namespace pitt;
    if (!ctx) return PITT_E_INVALID;
    if (n_clusters < 0 || (n_clusters > 0 && (!x || !y || !z || !offsets || !counts || !prm || !out)))
        return ctx->fail(PITT_E_INVALID, "null argument");
    if (n_clusters > 65535) return ctx->fail(PITT_E_INVALID, "more than 65535 clusters");
    if (prm && (prm->k < 1 || prm->k > 64)) return ctx->fail(PITT_E_INVALID, "k must be in [1, 64]");
    const int nc = n_clusters;
    for (int c = 0; c < nc; ++c)
        if (offsets[c] < 0 || counts[c] < 0 || counts[c] > 0x7fffffff) return ctx->fail(PITT_E_INVALID, "cluster range");
    if (nc == 0) return PITT_OK;
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    int rc = finish_batch(ctx);  // a plane batch still in flight on this context
    if (rc != PITT_OK) return rc;
    hipStream_t s = ctx->stream;

    // --- staging: cluster c at soff[c] (a whole number of tiles each), NaN between clusters ---
    std::vector<int64_t> soff((size_t)nc), cnt(counts, counts + nc);
    int64_t total = 0;
    for (int c = 0; c < nc; ++c) {
        soff[(size_t)c] = total;
        total += std::max<int64_t>(1, (cnt[(size_t)c] + PITT_TILE_POINTS - 1) / PITT_TILE_POINTS) * PITT_TILE_POINTS;
    }
    const size_t nb = (size_t)total * 4;
    float* sx = (float*)ctx->buf("cls_x", nb);
    float* sy = (float*)ctx->buf("cls_y", nb);
    float* sz = (float*)ctx->buf("cls_z", nb);
    float* nx = (float*)ctx->buf("cls_nx", nb);
    float* ny = (float*)ctx->buf("cls_ny", nb);
    float* nz = (float*)ctx->buf("cls_nz", nb);
    float* curv = (float*)ctx->buf("cls_curv", nb);
    int32_t* inl = (int32_t*)ctx->buf("cls_inl", nb * 4);  // sphere | cylinder | cone | plane lists
    int64_t* dmeta = (int64_t*)ctx->buf("cls_meta", (size_t)nc * 5 * 8 + 64);
    int32_t* dfirst = (int32_t*)ctx->buf("cls_first", (size_t)nc * 4 * 4);
    int64_t* hmeta = (int64_t*)ctx->pinned("cls_meta_h", (size_t)nc * 5 * 8 + 64);
    int32_t* hfirst = (int32_t*)ctx->pinned("cls_first_h", (size_t)nc * 4 * 4);
    if (!sx || !sy || !sz || !nx || !ny || !nz || !curv || !inl || !dmeta || !dfirst || !hmeta || !hfirst)
        return ctx->fail(PITT_E_NOMEM, "classification scratch");
    auto on_device = [](const void* p) {
        hipPointerAttribute_t a;
        return hipPointerGetAttributes(&a, p) == hipSuccess && a.type == hipMemoryTypeDevice;
    };
    if (on_device(x) && on_device(y) && on_device(z)) {  // one gather launch (its NaN padding included)
        int64_t* hst = (int64_t*)ctx->pinned("cls_stage_h", (size_t)nc * 3 * 8);
        int64_t* dst = (int64_t*)ctx->buf("cls_stage", (size_t)nc * 3 * 8);
        if (!hst || !dst) return ctx->fail(PITT_E_NOMEM, "classification staging");
        int64_t span = 1;
        for (int c = 0; c < nc; ++c) {
            hst[c] = offsets[c];
            hst[nc + c] = cnt[(size_t)c];
            hst[2 * nc + c] = soff[(size_t)c];
            span = std::max<int64_t>(span, (c + 1 < nc ? soff[(size_t)c + 1] : total) - soff[(size_t)c]);
        }
        PITT_HIP_TRY(hipMemcpyAsync(dst, hst, (size_t)nc * 3 * 8, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_stage_clusters, dim3((unsigned)((span + 255) / 256), (unsigned)nc), dim3(256), 0, s, x, y, z,
                           (const int64_t*)dst, nc, total, sx, sy, sz);
        PITT_HIP_TRY(hipGetLastError());
    } else {
        PITT_HIP_TRY(hipMemsetAsync(sx, 0xff, nb, s));  // NaN
        PITT_HIP_TRY(hipMemsetAsync(sy, 0xff, nb, s));
        PITT_HIP_TRY(hipMemsetAsync(sz, 0xff, nb, s));
        for (int c = 0; c < nc; ++c) {
            if (!cnt[(size_t)c]) continue;
            const size_t b = (size_t)cnt[(size_t)c] * 4;
            PITT_HIP_TRY(hipMemcpyAsync(sx + soff[(size_t)c], x + offsets[c], b, hipMemcpyDefault, s));
            PITT_HIP_TRY(hipMemcpyAsync(sy + soff[(size_t)c], y + offsets[c], b, hipMemcpyDefault, s));
            PITT_HIP_TRY(hipMemcpyAsync(sz + soff[(size_t)c], z + offsets[c], b, hipMemcpyDefault, s));
        }
    }

    // --- normals (PCManager::estimateNormal per cluster) ---
    rc = normals_batch(ctx, sx, sy, sz, total, soff.data(), cnt.data(), nc, prm->k, prm->viewpoint, nx, ny, nz, curv);
    if (rc != PITT_OK) return rc;

    // --- plane service: its batch on the auxiliary context's stream, overlapping the other services
    //     (the staged clusters are ready once this stream's work so far has run: an event orders it) ---
    if (!ctx->aux) {
        if (pitt_create(&ctx->aux, ctx->device) != PITT_OK || !ctx->aux) return ctx->fail(PITT_E_HIP, "auxiliary context");
    }
    {
        hipEvent_t staged = nullptr;
        PITT_HIP_TRY(hipEventCreateWithFlags(&staged, hipEventDisableTiming));
        PITT_HIP_TRY(hipEventRecord(staged, s));
        const hipError_t we = hipStreamWaitEvent(ctx->aux->stream, staged, 0);
        (void)hipEventDestroy(staged);
        PITT_HIP_TRY(we);
    }
    std::vector<pitt_plane_result> pr((size_t)nc);
    pitt_frames fr;
    fr.x = sx;
    fr.y = sy;
    fr.z = sz;
    fr.offsets = soff.data();
    fr.counts = cnt.data();
    fr.n_frames = nc;
    fr.capacity = total;
    int32_t* inl_plane = inl + 3 * total;
    rc = pitt_plane_segment_batch_async(ctx->aux, &fr, &prm->plane, pr.data(), inl_plane);
    if (rc < 0) return ctx->fail(rc, std::string("plane batch: ") + pitt_last_error(ctx->aux));
    // the batch writes into pr when it completes: never leave this function with it in flight
    struct AuxWait {
        pitt_ctx* a;
        ~AuxWait() { (void)pitt_wait(a); }
    } aux_wait{ctx->aux};

    // --- sphere, cylinder, cone services, in lockstep (each synchronisation serves all three) ---
    std::vector<PrimCloud> cls[3];
    std::vector<PrimResult> rs((size_t)nc), ry((size_t)nc), rk((size_t)nc);
    for (int srv = 0; srv < 3; ++srv) {
        cls[srv].resize((size_t)nc);
        for (int c = 0; c < nc; ++c) {
            const int64_t o = soff[(size_t)c];
            cls[srv][(size_t)c] = PrimCloud{sx + o, sy + o, sz + o, nx + o, ny + o, nz + o, cnt[(size_t)c],
                                            inl + srv * total + o};
        }
    }
    {
        // the sphere and cylinder runs on the two side streams, the cone on the context's: their small
        // per-cluster launches overlap on the device (each phase's synchronisation waits for all three)
        for (hipStream_t& sd : ctx->side)
            if (!sd) PITT_HIP_TRY(hipStreamCreateWithFlags(&sd, hipStreamNonBlocking));
        hipEvent_t ready = nullptr;  // the staged clusters and their normals
        PITT_HIP_TRY(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
        hipError_t e = hipEventRecord(ready, s);
        for (hipStream_t sd : ctx->side)
            if (e == hipSuccess) e = hipStreamWaitEvent(sd, ready, 0);
        (void)hipEventDestroy(ready);
        PITT_HIP_TRY(e);
        std::unique_ptr<PrimRunBase> runs[3] = {sphere_run(ctx, &prm->sphere, cls[0].data(), nc, rs.data()),
                                                cylinder_run(ctx, &prm->cylinder, cls[1].data(), nc, ry.data()),
                                                cone_run(ctx, &prm->cone, cls[2].data(), nc, rk.data())};
        // the cone first in every phase: its refinement is the longest, so its launches go out first
        rc = prim_ransac_lockstep(ctx, {runs[2].get(), runs[1].get(), runs[0].get()}, {s, ctx->side[1], ctx->side[0]});
        if (rc != PITT_OK) {
            for (hipStream_t sd : ctx->side) (void)hipStreamSynchronize(sd);
            return rc;
        }
    }

    rc = pitt_wait(ctx->aux);  // the plane batch (results into pr)
    if (rc < 0) return ctx->fail(rc, std::string("plane batch: ") + pitt_last_error(ctx->aux));

    // --- axis height of every cylinder / cone with inliers ---
    std::vector<int64_t> joff, jn;
    std::vector<float> jcoef;
    std::vector<int32_t> jmode, jsrc;  // jsrc: 2 c + (0 cylinder, 1 cone)
    for (int c = 0; c < nc; ++c)
        for (int q = 0; q < 2; ++q) {
            const PrimResult& r = q == 0 ? ry[(size_t)c] : rk[(size_t)c];
            if (r.status != PITT_OK || r.n_inliers <= 0) continue;
            joff.push_back(soff[(size_t)c]);
            jn.push_back(cnt[(size_t)c]);
            jcoef.insert(jcoef.end(), r.coef, r.coef + 6);
            jmode.push_back(q == 0 ? PITT_AXIS_CYLINDER : PITT_AXIS_CONE);
            jsrc.push_back(2 * c + q);
        }
    const int nj = (int)jn.size();
    std::vector<float> height((size_t)nj), cen((size_t)nj * 3);
    std::vector<int32_t> i1((size_t)nj), i2((size_t)nj);
    rc = axis_height_batch(ctx, sx, sy, sz, total, joff.data(), jn.data(), jcoef.data(), jmode.data(), nj,
                           height.data(), i1.data(), i2.data(), cen.data());
    if (rc != PITT_OK) return rc;

    // --- responses: the first inlier of each list (Q1) ---
    for (int c = 0; c < nc; ++c) {
        hmeta[c] = soff[(size_t)c];
        hmeta[nc + c] = rs[(size_t)c].status == PITT_OK ? rs[(size_t)c].n_inliers : 0;
        hmeta[2 * nc + c] = ry[(size_t)c].status == PITT_OK ? ry[(size_t)c].n_inliers : 0;
        hmeta[3 * nc + c] = rk[(size_t)c].status == PITT_OK ? rk[(size_t)c].n_inliers : 0;
        hmeta[4 * nc + c] = pr[(size_t)c].status == PITT_OK && pr[(size_t)c].n_coeff ? pr[(size_t)c].n_inliers : 0;
    }
    int32_t* hl[4] = {inl, inl + total, inl + 2 * total, inl_plane};
    std::memcpy(hmeta + 5 * nc, hl, sizeof hl);  // the 4 list pointers after the counts
    PITT_HIP_TRY(hipMemcpyAsync(dmeta, hmeta, (size_t)nc * 5 * 8 + sizeof hl, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_first_inliers, dim3((4 * nc + 255) / 256), dim3(256), 0, s,
                       (const int32_t* const*)(dmeta + 5 * nc), dmeta, dmeta + nc, nc, dfirst);
    PITT_HIP_TRY(hipGetLastError());
    PITT_HIP_TRY(hipMemcpyAsync(hfirst, dfirst, (size_t)nc * 4 * 4, hipMemcpyDeviceToHost, s));
    PITT_HIP_TRY(hipStreamSynchronize(s));

    // --- the services' responses and the arbitration ---
    for (int c = 0; c < nc; ++c) {
        pitt_cluster_shape& o = out[c];
        std::memset(&o, 0, sizeof o);
        o.n_points = cnt[(size_t)c];
        const PrimResult* r3[3] = {&rs[(size_t)c], &ry[(size_t)c], &rk[(size_t)c]};
        for (int q = 0; q < 4; ++q) {
            const int64_t n_inl = hmeta[(size_t)(q + 1) * nc + c];
            o.inliers[q] = (int32_t)(n_inl - (n_inl > 0 && hfirst[q * nc + c] == 0 ? 1 : 0));
        }
        // sphere: 4 coefficients with a model, the centre as the centroid (:79-83)
        o.status[0] = rs[(size_t)c].status;
        o.hypotheses[0] = rs[(size_t)c].hypotheses;
        if (rs[(size_t)c].status == PITT_OK) {
            o.n_coef[0] = 4;
            for (int k = 0; k < 4; ++k) o.sphere[k] = rs[(size_t)c].coef[k];
            for (int k = 0; k < 3; ++k) o.centroid[0][k] = rs[(size_t)c].coef[k];
        }
        // cylinder / cone: 7 coefficients with a model, then the height; the centroid when inliers
        for (int q = 1; q <= 2; ++q) {
            const PrimResult& r = *r3[q];
            float* cf = q == 1 ? o.cylinder : o.cone;
            o.status[q] = r.status;
            o.hypotheses[q] = r.hypotheses;
            int nco = 0;
            if (r.status == PITT_OK)
                for (int k = 0; k < 7; ++k) cf[nco++] = r.coef[k];
            float h = -1.0f;
            for (int j = 0; j < nj; ++j)
                if (jsrc[(size_t)j] == 2 * c + (q - 1)) {
                    h = height[(size_t)j];
                    for (int k = 0; k < 3; ++k) o.centroid[q][k] = cen[(size_t)j * 3 + k];
                }
            cf[nco++] = h;
            o.n_coef[q] = nco;
        }
        // plane: 4 coefficients with a model, no centroid (plane_segmentation_srv.cpp sets none)
        o.status[3] = pr[(size_t)c].n_coeff ? PITT_OK : (pr[(size_t)c].status < 0 ? pr[(size_t)c].status : PITT_NO_MODEL);
        o.hypotheses[3] = pr[(size_t)c].hypotheses;
        if (pr[(size_t)c].n_coeff) {
            o.n_coef[3] = 4;
            for (int k = 0; k < 4; ++k) o.plane[k] = pr[(size_t)c].coefficients[k];
        }
        o.tag = arbitrate(o.inliers[0], o.inliers[1], o.inliers[2], o.inliers[3], prm->cone_over_cylinder);
        const int src = o.tag == PITT_SHAPE_SPHERE ? 0 : o.tag == PITT_SHAPE_CYLINDER ? 1 : o.tag == PITT_SHAPE_CONE ? 2
                      : o.tag == PITT_SHAPE_PLANE ? 3 : -1;
        if (src >= 0)
            for (int k = 0; k < 3; ++k) o.est_centroid[k] = o.centroid[src][k];
    }
    return PITT_OK;
}
