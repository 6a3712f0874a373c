// abi_host_emu.cpp -- TEST INFRASTRUCTURE ONLY.  The C-ABI calls the two orchestrator nodes make,
// emulated on the host over the oracle (oracle/pitt_oracle.cpp), and hipMalloc / hipFree over malloc, so
// that tests/test_ros_adapters.py can run the nodes' own code (argument parsing, TF, parameter forwarding,
// the arm filter round trip, message assembly, publication) on a machine without a GPU.  The product
// library is never linked into these binaries and nothing here is shipped: the GPU tests
// (tests/test_ros_orchestrators_gpu.py) run the same nodes on libpitt_seg.so.
//
// pitt_srv_segment_objects_dev: the oracle's findSupports, then its Euclidean clusters of every support's
// on-support cloud with at least 30 points; member sums in index order (what the device returns).  Only the
// parameters the CPU test sets are honoured (max_iter, in_shape_distance_th).
// pitt_srv_classify_clusters: a deterministic stand-in (tag = points mod 5, coefficient k of cluster c =
// 10 c + k) that exercises the node's mapping from the result to TrackedShape.
#include <hip/hip_runtime_api.h>

#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "pitt_oracle.h"
#include "pitt_srv.h"

struct pitt_ctx {
    std::string err;
};

struct pitt_srv {
    pitt_ctx* ctx = nullptr;
    std::map<std::string, double> num;
    std::vector<std::vector<int32_t>> idx_maps;
    std::vector<std::vector<float>> sup_planes, on_planes;
    std::vector<pitt_support_dev> sups;
    std::vector<pitt_object> objs;
    std::vector<int32_t> members;
};

extern "C" {

hipError_t hipMalloc(void** p, size_t n) {
    *p = std::malloc(n ? n : 1);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFree(void* p) {
    std::free(p);
    return hipSuccess;
}

int pitt_create(pitt_ctx** out, int) {
    *out = new pitt_ctx;
    return PITT_OK;
}
void pitt_destroy(pitt_ctx* c) { delete c; }
const char* pitt_last_error(pitt_ctx* c) { return c ? c->err.c_str() : "null context"; }
int pitt_memcpy(pitt_ctx*, void* d, const void* s, int64_t bytes) {
    if (bytes > 0) std::memcpy(d, s, (size_t)bytes);
    return PITT_OK;
}

pitt_srv* pitt_srv_create(pitt_ctx* c) {
    pitt_srv* s = new pitt_srv;
    s->ctx = c;
    return s;
}
void pitt_srv_destroy(pitt_srv* s) { delete s; }
int pitt_srv_param_set_int(pitt_srv* s, const char* name, int32_t v) {
    s->num[name] = v;
    return PITT_OK;
}
int pitt_srv_param_set_double(pitt_srv* s, const char* name, double v) {
    s->num[name] = v;
    return PITT_OK;
}
int pitt_srv_param_set_list(pitt_srv*, const char*, const double*, int32_t) { return PITT_OK; }
int pitt_srv_param_erase(pitt_srv* s, const char* name) {
    s->num.erase(name);
    return PITT_OK;
}

int pitt_unpack_pointcloud2(pitt_ctx* ctx, const void* data, int64_t data_bytes, int32_t width, int32_t height,
                            int32_t point_step, int64_t row_step, int32_t off_x, int32_t off_y, int32_t off_z, float* x,
                            float* y, float* z) {
    const int64_t n = (int64_t)width * height;
    if (n > 0 && (height - 1) * row_step + (int64_t)width * point_step > data_bytes) {
        ctx->err = "payload shorter than its layout";
        return PITT_E_INVALID;
    }
    return orc_unpack_pointcloud2((const uint8_t*)data, width, height, point_step, row_step, off_x, off_y, off_z, x, y,
                                  z) < 0
               ? PITT_E_INVALID
               : PITT_OK;
}

int pitt_voxel_grid(pitt_ctx*, const float* x, const float* y, const float* z, int64_t n, float lx, float ly, float lz,
                    int32_t order, float* ox, float* oy, float* oz, int64_t* n_out, int32_t* flags) {
    *flags = 0;
    if (orc_voxel_grid(x, y, z, n, lx, ly, lz, order, ox, oy, oz, n_out) != 0) {  // PCL's overflow copy
        std::memcpy(ox, x, (size_t)n * 4);
        std::memcpy(oy, y, (size_t)n * 4);
        std::memcpy(oz, z, (size_t)n * 4);
        *n_out = n;
        *flags = PITT_VOXEL_OVERFLOW_COPY;
    }
    return PITT_OK;
}

int pitt_deep_filter(pitt_ctx*, const float* x, const float* y, const float* z, int64_t n, float th, float* cx,
                     float* cy, float* cz, int64_t* n_closer, float* fx, float* fy, float* fz, int64_t* n_further,
                     float* used) {
    const float t = orc_service_float_param(th, 3.0f);
    std::vector<float> c(3 * (size_t)(n > 0 ? n : 1)), f(3 * (size_t)(n > 0 ? n : 1));
    int64_t nc = 0, nf = 0;
    orc_deep_filter(x, y, z, n, t, c.data(), c.data() + n, c.data() + 2 * n, &nc, f.data(), f.data() + n,
                    f.data() + 2 * n, &nf);
    if (cx) {
        std::memcpy(cx, c.data(), (size_t)nc * 4);
        std::memcpy(cy, c.data() + n, (size_t)nc * 4);
        std::memcpy(cz, c.data() + 2 * n, (size_t)nc * 4);
    }
    if (fx) {
        std::memcpy(fx, f.data(), (size_t)nf * 4);
        std::memcpy(fy, f.data() + n, (size_t)nf * 4);
        std::memcpy(fz, f.data() + 2 * n, (size_t)nf * 4);
    }
    if (n_closer) *n_closer = nc;
    if (n_further) *n_further = nf;
    if (used) *used = t;
    return PITT_OK;
}

int pitt_transform_cloud(pitt_ctx*, const float* x, const float* y, const float* z, int64_t n, const float matrix[16],
                         int32_t dense, float* ox, float* oy, float* oz) {
    orc_transform_cloud(x, y, z, n, matrix, dense, ox, oy, oz);
    return PITT_OK;
}

int pitt_srv_segment_objects_dev(pitt_srv* s, const float* x, const float* y, const float* z, int64_t n,
                                 pitt_scene* out) {
    orc_support_params p = {0.03f, 0.03f, 0.09f, 0.02f, 10, {0.0f, 0.0f, -1.0f}, {0.02f, 0.02f, 0.005f},
                            ORC_REDUCE_SSE2, ORC_TRIG_CR, ORC_DIV_EIGEN32};
    auto it = s->num.find("/pitt/srv/supports_segmentation/max_iter");
    if (it != s->num.end() && it->second >= 0) p.ransac_max_iterations = (int32_t)it->second;
    it = s->num.find("/pitt/srv/supports_segmentation/in_shape_distance_th");
    if (it != s->num.end() && it->second >= 0) p.ransac_distance_threshold = (float)it->second;
    s->idx_maps.clear();
    s->sup_planes.clear();
    s->on_planes.clear();
    s->sups.clear();
    s->objs.clear();
    s->members.clear();
    orc_support_list* L = orc_find_supports(x, y, z, n, &p);
    const int32_t ns = orc_support_count(L);
    s->idx_maps.resize((size_t)ns);
    s->sup_planes.resize((size_t)ns);
    s->on_planes.resize((size_t)ns);
    for (int32_t k = 0; k < ns; ++k) {
        pitt_support_dev d = {};
        s->idx_maps[(size_t)k].resize((size_t)(n > 0 ? n : 1));
        int64_t a = 0, b = 0;
        orc_support_get(L, k, s->idx_maps[(size_t)k].data(), d.coefficients, &a, &b);
        std::vector<float>& sp = s->sup_planes[(size_t)k];
        std::vector<float>& on = s->on_planes[(size_t)k];
        sp.resize(3 * (size_t)(a > 0 ? a : 1));
        on.resize(3 * (size_t)(b > 0 ? b : 1));
        orc_support_cloud(L, k, 0, sp.data(), sp.data() + a, sp.data() + 2 * a);
        orc_support_cloud(L, k, 1, on.data(), on.data() + b, on.data() + 2 * b);
        d.n_points = (int32_t)n;
        d.idx_map = s->idx_maps[(size_t)k].data();
        d.n_support = a;
        d.support_xyz = sp.data();
        d.n_on_support = b;
        d.on_support_xyz = on.data();
        d.stride = b;
        s->sups.push_back(d);
        if (b < 30) continue;  // clusterize's min_input_size (cluster_segmentation_srv.cpp:54)
        orc_cluster_list* C = orc_euclidean_clusters(on.data(), on.data() + b, on.data() + 2 * b, b, 0.03, 0.01, 0.99, 30);
        for (int32_t c = 0; c < orc_cluster_count(C); ++c) {
            const int64_t m = orc_cluster_size(C, c);
            std::vector<int32_t> idx((size_t)(m > 0 ? m : 1));
            float centroid[3];
            orc_cluster_get(C, c, idx.data(), centroid);
            pitt_object o = {};
            o.support = k;
            o.size = m;
            o.offset = (int64_t)s->members.size();
            for (int64_t j = 0; j < m; ++j) {  // float sums in index order
                const int32_t i = idx[(size_t)j];
                o.sum_xyz[0] += on[(size_t)i];
                o.sum_xyz[1] += on[(size_t)(b + i)];
                o.sum_xyz[2] += on[(size_t)(2 * b + i)];
            }
            s->members.insert(s->members.end(), idx.begin(), idx.begin() + m);
            s->objs.push_back(o);
        }
        orc_cluster_free(C);
    }
    orc_support_free(L);
    out->supports.n_supports = ns;
    out->supports.supports = s->sups.data();
    out->supports.iterations = 0;
    out->n_objects = (int32_t)s->objs.size();
    out->objects = s->objs.data();
    out->indices = s->members.data();
    return PITT_OK;
}

int pitt_srv_classify_clusters(pitt_srv*, const float*, const float*, const float*, const int64_t*,
                               const int64_t* counts, int32_t n_clusters, pitt_cluster_shape* out) {
    for (int32_t c = 0; c < n_clusters; ++c) {
        pitt_cluster_shape& r = out[c];
        std::memset(&r, 0, sizeof r);
        r.n_points = counts[c];
        r.tag = (int32_t)(counts[c] % 5);
        const int ncoef[4] = {4, 8, 8, 4};  // sphere, cylinder, cone, plane
        float* arr[4] = {r.sphere, r.cylinder, r.cone, r.plane};
        for (int q = 0; q < 4; ++q) {
            r.inliers[q] = (int32_t)(counts[c] / (q + 2));
            r.n_coef[q] = ncoef[q];
            for (int k = 0; k < ncoef[q]; ++k) arr[q][k] = (float)(10 * c + k) + 0.25f * (float)q;
            for (int k = 0; k < 3; ++k) r.centroid[q][k] = (float)c + 0.5f * (float)k + 0.125f * (float)q;
        }
        for (int k = 0; k < 3; ++k) r.est_centroid[k] = (float)c + 0.5f * (float)k;
    }
    return PITT_OK;
}

}  // extern "C"
