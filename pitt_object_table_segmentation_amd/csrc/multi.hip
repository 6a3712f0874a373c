// Frame-sharded plane segmentation over several devices from one host process.
//
// The reference's C++ host (obj_segmentation.cpp:381 spinning ransac_segmentation / the services) is
// one process.  A C++ caller with frames in host memory and G gfx950 devices uses one pitt_multi:
// frames [g F / G, (g + 1) F / G) go to device g (contiguous shards, the same split as the Python
// one-process-per-GPU path, distributed.shard_range), each shard is uploaded to its device and
// segmented there by that device's own context, and the per-frame results and inlier lists are
// gathered on the host in frame order.  The only exchange is that gather: results are 56-byte
// records and the inlier lists land straight in the caller's host array, so no collective is
// involved (the in-process analogue of the RCCL all-gather of distributed.py).  One host thread per
// device drives its shard (pageable H2D / D2H copies run on the calling thread), so the shards'
// transfers and kernels overlap across devices.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "ctx.hpp"

struct pitt_multi {
    std::vector<pitt_ctx*> ctxs;  // one per listed device (a device may be listed more than once)
    std::string err;
};

namespace {

struct Shard {
    int f0 = 0, f1 = 0;          // frames [f0, f1)
    int64_t base = 0, cap = 0;   // host plane span [base, base + cap) holding them (tile spans included)
    int64_t out_end = 0;         // inliers of the shard lie in [base, out_end)
};

// Device g's part: upload its span, segment, copy the inliers back into the caller's host array.
int run_shard(pitt_ctx* ctx, const pitt_frames* hf, const Shard& sh, const pitt_sac_params* p,
              pitt_plane_result* results, int32_t* inliers_out) {
    if (sh.f1 <= sh.f0) return PITT_OK;
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    const size_t pb = (size_t)sh.cap * sizeof(float);
    const int64_t stride = (sh.cap + 3) / 4 * 4;  // 16-byte aligned planes
    float* d = (float*)ctx->buf("multi_xyz", (size_t)stride * 3 * sizeof(float));
    int32_t* di = inliers_out ? (int32_t*)ctx->buf("multi_inl", pb) : nullptr;
    if (!d || (inliers_out && !di)) return ctx->fail(PITT_E_NOMEM, "multi-device shard buffers");
    hipStream_t s = ctx->stream;
    PITT_HIP_TRY(hipMemcpyAsync(d, hf->x + sh.base, pb, hipMemcpyHostToDevice, s));
    PITT_HIP_TRY(hipMemcpyAsync(d + stride, hf->y + sh.base, pb, hipMemcpyHostToDevice, s));
    PITT_HIP_TRY(hipMemcpyAsync(d + 2 * stride, hf->z + sh.base, pb, hipMemcpyHostToDevice, s));
    const int nf = sh.f1 - sh.f0;
    std::vector<int64_t> off((size_t)nf);
    for (int f = 0; f < nf; ++f) off[(size_t)f] = hf->offsets[sh.f0 + f] - sh.base;
    pitt_frames fr;
    fr.x = d;
    fr.y = d + stride;
    fr.z = d + 2 * stride;
    fr.offsets = off.data();
    fr.counts = hf->counts + sh.f0;
    fr.n_frames = nf;
    fr.capacity = sh.cap;
    const int rc = pitt_plane_segment_batch(ctx, &fr, p, results + sh.f0, di);
    if (rc < 0) return rc;
    if (inliers_out && sh.out_end > sh.base)
        PITT_HIP_TRY(hipMemcpy(inliers_out + sh.base, di, (size_t)(sh.out_end - sh.base) * sizeof(int32_t),
                               hipMemcpyDeviceToHost));
    return PITT_OK;
}

}  // namespace

extern "C" {

int pitt_multi_create(pitt_multi** out, const int32_t* hip_devices, int32_t n_devices) {
    if (!out) return PITT_E_INVALID;
    *out = nullptr;
    if (!hip_devices || n_devices <= 0) return PITT_E_INVALID;
    pitt_multi* m = new pitt_multi;
    for (int g = 0; g < n_devices; ++g) {
        pitt_ctx* c = nullptr;
        const int rc = pitt_create(&c, hip_devices[g]);
        if (rc != PITT_OK) {
            for (pitt_ctx* x : m->ctxs) pitt_destroy(x);
            delete m;
            return rc;
        }
        m->ctxs.push_back(c);
    }
    *out = m;
    return PITT_OK;
}

void pitt_multi_destroy(pitt_multi* m) {
    if (!m) return;
    for (pitt_ctx* c : m->ctxs) pitt_destroy(c);
    delete m;
}

int32_t pitt_multi_devices(const pitt_multi* m) { return m ? (int32_t)m->ctxs.size() : 0; }

pitt_ctx* pitt_multi_context(pitt_multi* m, int32_t g) {
    return m && g >= 0 && g < (int32_t)m->ctxs.size() ? m->ctxs[(size_t)g] : nullptr;
}

const char* pitt_multi_last_error(const pitt_multi* m) { return m ? m->err.c_str() : ""; }

int pitt_plane_segment_batch_multi(pitt_multi* m, const pitt_frames* hf, const pitt_sac_params* p,
                                   pitt_plane_result* results, int32_t* inliers_out) {
    if (!m) return PITT_E_INVALID;
    m->err.clear();
    auto fail = [&](int code, const char* msg) {
        m->err = msg;
        return code;
    };
    if (!hf || !p || !results) return fail(PITT_E_INVALID, "null argument");
    const int F = hf->n_frames;
    if (F < 0) return fail(PITT_E_INVALID, "n_frames < 0");
    if (F == 0) return PITT_OK;
    if (!hf->x || !hf->y || !hf->z || !hf->offsets || !hf->counts) return fail(PITT_E_INVALID, "null frame pointer");
    // frames in ascending, non-overlapping order: each shard's host span then holds only its frames
    // (and the gaps between them), so the shards' uploads and inlier copy-backs never touch another
    // shard's frames
    for (int f = 0; f < F; ++f) {
        const int64_t o = hf->offsets[f], n = hf->counts[f];
        if (o < 0 || n < 0 || (o & 3) != 0) return fail(PITT_E_INVALID, "frame offset must be >= 0 and a multiple of 4");
        const int64_t span = (n + PITT_TILE_POINTS - 1) / PITT_TILE_POINTS * PITT_TILE_POINTS;
        if (o + span > hf->capacity) return fail(PITT_E_INVALID, "frame tile span exceeds capacity");
        if (f > 0 && o < hf->offsets[f - 1] + hf->counts[f - 1])
            return fail(PITT_E_INVALID, "multi-device frames must be ascending and non-overlapping");
    }
    const int G = (int)m->ctxs.size();
    std::vector<Shard> sh((size_t)G);
    for (int g = 0; g < G; ++g) {
        Shard& s = sh[(size_t)g];
        s.f0 = (int)((int64_t)g * F / G);
        s.f1 = (int)((int64_t)(g + 1) * F / G);
        if (s.f1 <= s.f0) continue;
        s.base = hf->offsets[s.f0];
        int64_t end = s.base;
        for (int f = s.f0; f < s.f1; ++f) {
            const int64_t span = (hf->counts[f] + PITT_TILE_POINTS - 1) / PITT_TILE_POINTS * PITT_TILE_POINTS;
            end = std::max(end, hf->offsets[f] + span);
        }
        s.cap = std::max<int64_t>(std::min(end, hf->capacity) - s.base, 0);
        s.out_end = hf->offsets[s.f1 - 1] + hf->counts[s.f1 - 1];
    }
    std::vector<int> rc((size_t)G, PITT_OK);
    std::vector<std::thread> th;
    th.reserve((size_t)G);
    for (int g = 0; g < G; ++g)
        th.emplace_back([&, g] { rc[(size_t)g] = run_shard(m->ctxs[(size_t)g], hf, sh[(size_t)g], p, results, inliers_out); });
    for (std::thread& t : th) t.join();
    for (int g = 0; g < G; ++g)
        if (rc[(size_t)g] < 0) {
            m->err = "device " + std::to_string(g) + ": " + m->ctxs[(size_t)g]->err;
            return rc[(size_t)g];
        }
    return PITT_OK;
}

}  // extern "C"
