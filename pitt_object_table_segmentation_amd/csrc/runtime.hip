// runtime.hip -- pitt_ctx lifecycle, scratch arena, sampler tables, profiler and the C ABI entry
// points of include/pitt_seg.h for the plane path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "ctx.hpp"

#if !defined(__HIP_DEVICE_COMPILE__)
#include <immintrin.h>
#endif

namespace pitt {
#if !defined(__HIP_DEVICE_COMPILE__)
// PointXYZ (x, y, z, pad) -> x[], y[], z[] for m points.  AVX-512 where the host has it (16 points per
// step: four loads, six two-source permutes, three stores), else one point at a time.
__attribute__((target("avx512f"))) static void deinterleave4_avx512(const float* src, int64_t m, float* x, float* y,
                                                                    float* z) {
    const __m512i ixy = _mm512_setr_epi32(0, 4, 8, 12, 16, 20, 24, 28, 1, 5, 9, 13, 17, 21, 25, 29);
    const __m512i iz = _mm512_setr_epi32(2, 6, 10, 14, 18, 22, 26, 30, 2, 6, 10, 14, 18, 22, 26, 30);
    const __m512i lo = _mm512_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7, 16, 17, 18, 19, 20, 21, 22, 23);
    const __m512i hi = _mm512_setr_epi32(8, 9, 10, 11, 12, 13, 14, 15, 24, 25, 26, 27, 28, 29, 30, 31);
    int64_t i = 0;
    for (; i + 16 <= m; i += 16) {
        const float* p = src + 4 * i;
        const __m512 a0 = _mm512_loadu_ps(p), a1 = _mm512_loadu_ps(p + 16), a2 = _mm512_loadu_ps(p + 32),
                     a3 = _mm512_loadu_ps(p + 48);
        const __m512 xy01 = _mm512_permutex2var_ps(a0, ixy, a1), xy23 = _mm512_permutex2var_ps(a2, ixy, a3);
        const __m512 z01 = _mm512_permutex2var_ps(a0, iz, a1), z23 = _mm512_permutex2var_ps(a2, iz, a3);
        _mm512_storeu_ps(x + i, _mm512_permutex2var_ps(xy01, lo, xy23));
        _mm512_storeu_ps(y + i, _mm512_permutex2var_ps(xy01, hi, xy23));
        _mm512_storeu_ps(z + i, _mm512_permutex2var_ps(z01, lo, z23));
    }
    for (; i < m; ++i) {
        x[i] = src[4 * i];
        y[i] = src[4 * i + 1];
        z[i] = src[4 * i + 2];
    }
}
#endif
static void deinterleave4(const float* src, int64_t m, float* x, float* y, float* z) {
#if !defined(__HIP_DEVICE_COMPILE__)
    static const bool avx512 = __builtin_cpu_supports("avx512f");
    if (avx512) {
        deinterleave4_avx512(src, m, x, y, z);
        return;
    }
#endif
    for (int64_t i = 0; i < m; ++i) {
        float q[4];
        std::memcpy(q, src + 4 * i, sizeof q);
        x[i] = q[0];
        y[i] = q[1];
        z[i] = q[2];
    }
}

int plane_segment_batch_impl(pitt_ctx* ctx, const pitt_frames* fr, const pitt_sac_params* p,
                             pitt_plane_result* results, int32_t* inliers_dev);
int finish_batch(pitt_ctx* ctx);

// A2: drawIndexSample's index triples for a cloud of n points.  The shuffled index vector of
// SampleConsensusModel is the identity except at the positions the swaps touched, so it is kept
// sparsely: O(attempts) instead of the O(n) array PCL rebuilds on every segment().
const std::vector<int32_t>& sampler_table(pitt_ctx* ctx, int64_t n, uint32_t seed, int64_t attempts, int k) {
    auto key = std::make_tuple(n, seed, attempts, k);
    auto it = ctx->tables.find(key);
    if (it != ctx->tables.end()) return it->second;
    // bounded: a tracking session sees a new cluster size almost every frame.  Callers copy a table
    // out before asking for the next one, so dropping the cache here invalidates nothing in use.
    if (ctx->tables.size() >= 512) ctx->tables.clear();
    std::vector<int32_t> t((size_t)attempts * k);
    std::mt19937 mt(seed);  // boost::mt19937 and std::mt19937 produce the same stream
    std::unordered_map<int64_t, int64_t> sh;
    sh.reserve((size_t)attempts * 4);
    auto get = [&](int64_t i) {
        auto f = sh.find(i);
        return f == sh.end() ? i : f->second;
    };
    for (int64_t a = 0; a < attempts; ++a) {
        for (int64_t i = 0; i < k; ++i) {
            const uint32_t r = (uint32_t)mt() >> 1;           // uniform_int<>(0, INT_MAX)
            const int64_t j = i + (int64_t)((uint64_t)r % (uint64_t)(n - i));
            const int64_t vi = get(i), vj = get(j);
            sh[i] = vj;
            sh[j] = vi;
        }
        for (int64_t i = 0; i < k; ++i) t[(size_t)(a * k + i)] = (int32_t)get(i);
    }
    return ctx->tables.emplace(key, std::move(t)).first->second;
}

// A4: fabs(float) < (double)th  <=>  fabs(float) < t, t = the smallest float >= th.
float float_threshold(double th) {
    if (std::isnan(th)) return std::nanf("");
    float f = (float)th;
    if ((double)f < th) f = std::nextafter(f, INFINITY);
    return f;
}

// pitt_plane_segment's staging layout -> the frame's planes: chunk c of C points arrives as
// [x(C) y(C) z(C)] (one H2D copy per chunk); point i of the cloud lands at x[i], y[i], z[i].
__global__ __launch_bounds__(256) void k_single_planes(const float* __restrict__ stage, int64_t n, int64_t C,
                                                       int64_t cap, float* __restrict__ d) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t c = i / C, j = i - c * C, b = c * 3 * C + j;
        const int64_t m = std::min(C, n - c * C);  // the last chunk is packed to its own length
        d[i] = stage[b];
        d[cap + i] = stage[b + m];
        d[2 * cap + i] = stage[b + 2 * m];
    }
}
// The caller's AoS cloud (sf floats per point, copied up as it is) -> the frame's planes.
__global__ __launch_bounds__(256) void k_single_aos(const float* __restrict__ aos, int64_t n, int sf, int64_t cap,
                                                    float* __restrict__ d) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        d[i] = aos[i * sf];
        d[cap + i] = aos[i * sf + 1];
        d[2 * cap + i] = aos[i * sf + 2];
    }
}
}  // namespace pitt

#ifdef PITT_SYNC_CHECK
static constexpr size_t kCanaryBytes = (size_t)256 << 10;
#endif

void pitt_ctx::drain() {
    if (stream) (void)hipStreamSynchronize(stream);
    for (hipStream_t sd : side)
        if (sd) (void)hipStreamSynchronize(sd);
}

void* pitt_ctx::buf(const std::string& name, size_t bytes) {
    pitt::DevBuf& b = bufs[name];
    if (b.bytes < bytes || !b.p) {
        // work queued on the context's streams may still use the old block: let it drain first
        if (b.p) {
            drain();
            (void)hipFree(b.p);
        }
        size_t nb = std::max(bytes, b.bytes + b.bytes / 2);
        nb = (nb + ((size_t)1 << 21) - 1) & ~(((size_t)1 << 21) - 1);
        if (nb == 0) nb = (size_t)1 << 21;
#ifdef PITT_SYNC_CHECK
        if (hipMalloc(&b.p, nb + kCanaryBytes) != hipSuccess) {
#else
        if (hipMalloc(&b.p, nb) != hipSuccess) {
#endif
            b.p = nullptr;
            b.bytes = 0;
            return nullptr;
        }
#ifdef PITT_SYNC_CHECK
        (void)hipMemset((char*)b.p + nb, 0xA5, kCanaryBytes);
#endif
        b.bytes = nb;
        ++arena_gen;  // memoised device contents at the old pointer are stale
        if (name == "tables") pool_keys.clear();  // device table pool lost
    }
    return b.p;
}

void pitt_ctx::check_canaries(const char* where) {
#ifdef PITT_SYNC_CHECK
    (void)hipDeviceSynchronize();
    std::vector<unsigned char> h(kCanaryBytes);
    for (auto& kv : bufs) {
        if (!kv.second.p) continue;
        (void)hipMemcpy(h.data(), (char*)kv.second.p + kv.second.bytes, kCanaryBytes, hipMemcpyDeviceToHost);
        for (size_t i = 0; i < kCanaryBytes; ++i)
            if (h[i] != 0xA5) {
                std::fprintf(stderr, "PITT_SYNC_CHECK canary of %s (%zu B) corrupted at +%zu (%s)\n", kv.first.c_str(),
                             kv.second.bytes, i, where);
                break;
            }
    }
    const size_t kSentinel = (size_t)256 << 20;
    if (!sentinel) {
        if (hipMalloc(&sentinel, kSentinel) != hipSuccess) sentinel = nullptr;
        if (sentinel) (void)hipMemset(sentinel, 0xA5, kSentinel);
        return;
    }
    std::vector<unsigned char> s(kSentinel);
    (void)hipMemcpy(s.data(), sentinel, kSentinel, hipMemcpyDeviceToHost);
    for (size_t i = 0; i < kSentinel; ++i)
        if (s[i] != 0xA5) {
            std::fprintf(stderr, "PITT_SYNC_CHECK sentinel corrupted at +%zu (%s)\n", i, where);
            (void)hipMemset(sentinel, 0xA5, kSentinel);
            break;
        }
#else
    (void)where;
#endif
}

void* pitt_ctx::pinned(const std::string& name, size_t bytes) {
    auto& e = host_pinned[name];
    if (e.second < bytes || !e.first) {
        // an async copy queued on the stream may still read or write the old block
        if (e.first) {
            drain();
            (void)hipHostFree(e.first);
        }
        ++arena_gen;
        size_t nb = std::max<size_t>(bytes, 4096);
        if (hipHostMalloc(&e.first, nb, hipHostMallocDefault) != hipSuccess) {
            e.first = nullptr;
            e.second = 0;
            return nullptr;
        }
        e.second = nb;
    }
    return e.first;
}

int pitt_ctx::prof_begin(const char* name, double bytes) {
    if (!prof) return -1;
    pitt::ProfRec r;
    r.name = name;
    r.alias.clear();
    r.bytes = bytes;
    for (hipEvent_t* e : {&r.a, &r.b}) {
        if (!event_pool.empty()) {
            *e = event_pool.back();
            event_pool.pop_back();
        } else {
            (void)hipEventCreate(e);
        }
    }
    (void)hipEventRecord(r.a, stream);
    pending.push_back(r);
    return (int)pending.size() - 1;
}

void pitt_ctx::prof_end(int rec) {
    if (rec < 0) return;
    (void)hipEventRecord(pending[(size_t)rec].b, stream);
}

int pitt_ctx::prof_collect() {
    if (pending.empty()) return PITT_OK;
    if (hipStreamSynchronize(stream) != hipSuccess) return PITT_E_HIP;
    for (pitt::ProfRec& r : pending) {
        float ms = 0.0f;
        (void)hipEventElapsedTime(&ms, r.a, r.b);
        // a scoring chunk with no active frame (its k_score/k_replay launches only retire empty
        // blocks) is accounted apart: the roofline covers the launches that score tiles
        const bool empty = r.name == "k_score" && r.bytes == 0.0;
        pitt::ProfTotal& t = totals[empty ? std::string("k_score:empty") : r.name];
        t.launches += 1;
        t.ms += ms;
        t.bytes += r.bytes;
        if (!r.alias.empty() && !empty) {
            pitt::ProfTotal& u = totals[r.alias];
            u.launches += 1;
            u.ms += ms;
            u.bytes += r.bytes;
        }
        event_pool.push_back(r.a);
        event_pool.push_back(r.b);
    }
    pending.clear();
    return PITT_OK;
}

extern "C" {

int pitt_abi_version(void) { return PITT_ABI_VERSION; }

int pitt_build_flags(void) { return pitt_ctx::kVariants ? PITT_BUILD_AB_VARIANTS : 0; }

void pitt_sac_params_default(pitt_sac_params* p) {
    if (!p) return;
    p->threshold = 0.007;        // plane_segmentation_srv.cpp:20
    p->max_iterations = 1000;    // :21
    p->probability = 0.99;       // RandomSampleConsensus default
    p->seed = 12345u;            // SampleConsensusModel, random_ == false
    p->optimize = 1;             // :55
    p->reduce_order = PITT_REDUCE_SSE2;
    p->div_mode = PITT_DIV_EIGEN32;
    p->sampler_slack = 1000;     // >= getSamples' 1000-draw limit (sac_model.hpp)
    p->cov_mode = PITT_COV_EXACT;
    p->pad = 0;
}

int pitt_create(pitt_ctx** out, int hip_device) {
    if (!out) return PITT_E_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return PITT_E_NODEVICE;
    if (hip_device < 0 || hip_device >= n) return PITT_E_INVALID;
    if (hipSetDevice(hip_device) != hipSuccess) return PITT_E_HIP;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, hip_device) != hipSuccess) return PITT_E_HIP;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return PITT_E_NODEVICE;
    pitt_ctx* c = new pitt_ctx;
    c->device = hip_device;
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return PITT_E_HIP;
    }
    c->stream = c->own_stream;
    *out = c;
    return PITT_OK;
}

void pitt_destroy(pitt_ctx* ctx) {
    if (!ctx) return;
    if (ctx->aux) pitt_destroy(ctx->aux);
    ctx->aux = nullptr;
    (void)pitt::finish_batch(ctx);
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (auto& kv : ctx->bufs)
        if (kv.second.p) (void)hipFree(kv.second.p);
    if (ctx->sentinel) (void)hipFree(ctx->sentinel);
    for (auto& kv : ctx->host_pinned)
        if (kv.second.first) (void)hipHostFree(kv.second.first);
    for (auto& r : ctx->pending) {
        (void)hipEventDestroy(r.a);
        (void)hipEventDestroy(r.b);
    }
    for (hipEvent_t e : ctx->event_pool) (void)hipEventDestroy(e);
    for (hipEvent_t e : ctx->er_ev)
        if (e) (void)hipEventDestroy(e);
    for (hipStream_t& sd : ctx->side)
        if (sd) {
            (void)hipStreamSynchronize(sd);
            (void)hipStreamDestroy(sd);
            sd = nullptr;
        }
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
    delete ctx;
}

int pitt_set_stream(pitt_ctx* ctx, void* s) {
    if (!ctx) return PITT_E_INVALID;
    // a batch in flight was queued on the old stream: finish it there before switching, so that
    // its results are copied out and its scratch is not reused under it by the next batch
    const int rc = pitt::finish_batch(ctx);
    if (rc) return rc;
    ctx->stream = s ? (hipStream_t)s : ctx->own_stream;
    return PITT_OK;
}

void* pitt_get_stream(pitt_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int pitt_schedule_stats(pitt_ctx* ctx, int64_t* continuations, int32_t* last_chunks) {
    if (!ctx) return PITT_E_INVALID;
    if (continuations) *continuations = ctx->continuations;
    if (last_chunks) *last_chunks = ctx->inflight_k;
    return PITT_OK;
}

int pitt_refine_stats(pitt_ctx* ctx, int64_t* batches, int64_t* fallback_frames) {
    if (!ctx) return PITT_E_INVALID;
    if (batches) *batches = ctx->xrefine_batches;
    if (fallback_frames) *fallback_frames = ctx->xrefine_fallbacks;
    return PITT_OK;
}

int pitt_memcpy(pitt_ctx* ctx, void* dst, const void* src, int64_t bytes) {
    if (!ctx) return PITT_E_INVALID;
    if (bytes < 0 || (bytes > 0 && (!dst || !src))) return ctx->fail(PITT_E_INVALID, "null argument");
    if (bytes == 0) return PITT_OK;
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    // a batch in flight may still have chunks to run (the adaptive schedule's continuation): complete
    // it first, so that a copy of its inliers_dev sees the whole batch
    if (int rc = pitt::finish_batch(ctx)) return rc;
    PITT_HIP_TRY(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDefault, ctx->stream));
    PITT_HIP_TRY(hipStreamSynchronize(ctx->stream));
    return PITT_OK;
}

const char* pitt_last_error(pitt_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int pitt_plane_segment_batch(pitt_ctx* ctx, const pitt_frames* fr, const pitt_sac_params* p,
                             pitt_plane_result* results, int32_t* inliers_dev) {
    int rc = pitt_plane_segment_batch_async(ctx, fr, p, results, inliers_dev);
    if (rc < 0) return rc;
    return pitt_wait(ctx);
}

int pitt_wait(pitt_ctx* ctx) {
    if (!ctx) return PITT_E_INVALID;
    return pitt::finish_batch(ctx);
}

int pitt_plane_segment_batch_async(pitt_ctx* ctx, const pitt_frames* fr, const pitt_sac_params* p,
                                   pitt_plane_result* results, int32_t* inliers_dev) {
    if (!ctx) return PITT_E_INVALID;
    if (!fr || !p || !results) return ctx->fail(PITT_E_INVALID, "null argument");
    if (fr->n_frames < 0) return ctx->fail(PITT_E_INVALID, "n_frames < 0");
    if (fr->n_frames == 0) return PITT_OK;
    if (!fr->x || !fr->y || !fr->z || !fr->offsets || !fr->counts)
        return ctx->fail(PITT_E_INVALID, "null frame pointer");
    if (((uintptr_t)fr->x | (uintptr_t)fr->y | (uintptr_t)fr->z) & 15u)
        return ctx->fail(PITT_E_INVALID, "x/y/z planes must be 16-byte aligned");
    if (inliers_dev && ((uintptr_t)inliers_dev & 3u))
        return ctx->fail(PITT_E_INVALID, "inliers_dev must be 4-byte aligned");
    if (p->reduce_order < 0 || p->reduce_order > 2 || p->div_mode < 0 || p->div_mode > 1)
        return ctx->fail(PITT_E_INVALID, "reduce_order / div_mode out of range");
    // cov_mode is an ABI-3 field: callers check pitt_abi_version() == PITT_ABI_VERSION at load
    // (pitt_seg.h), so the struct passed here is always the ABI-3 layout
    if (p->cov_mode != PITT_COV_EXACT && p->cov_mode != PITT_COV_FAST)
        return ctx->fail(PITT_E_INVALID, "cov_mode out of range");
    for (int f = 0; f < fr->n_frames; ++f) {
        const int64_t o = fr->offsets[f], n = fr->counts[f];
        if (o < 0 || n < 0 || (o & 3) != 0) return ctx->fail(PITT_E_INVALID, "frame offset must be >= 0 and a multiple of 4");
        if (n > 0x7fffffff) return ctx->fail(PITT_E_INVALID, "frame larger than 2^31 points");
        const int64_t span = (n + PITT_TILE_POINTS - 1) / PITT_TILE_POINTS * PITT_TILE_POINTS;
        if (o + span > fr->capacity) return ctx->fail(PITT_E_INVALID, "frame tile span exceeds capacity");
    }
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    return pitt::plane_segment_batch_impl(ctx, fr, p, results, inliers_dev);
}

int pitt_plane_segment(pitt_ctx* ctx, const float* xyz, int64_t n, int32_t stride_bytes,
                       const pitt_sac_params* p, int32_t* inliers_out, int64_t* n_inliers,
                       float coeff_out[4], int32_t* n_coeff) {
    if (!ctx) return PITT_E_INVALID;
    if ((!xyz && n > 0) || !p || !n_inliers || !n_coeff || n < 0)
        return ctx->fail(PITT_E_INVALID, "null argument");
    if (stride_bytes != 12 && stride_bytes != 16) return ctx->fail(PITT_E_INVALID, "stride must be 12 or 16");
    *n_inliers = 0;
    *n_coeff = 0;
    const int64_t cap = std::max<int64_t>(PITT_TILE_POINTS,
                                          (n + PITT_TILE_POINTS - 1) / PITT_TILE_POINTS * PITT_TILE_POINTS);
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    if (int rc = pitt::finish_batch(ctx)) return rc;  // a batch in flight completes first
    const int64_t C = ctx->single_chunk > 0 ? std::min<int64_t>(ctx->single_chunk, std::max<int64_t>(n, 1))
                                            : std::max<int64_t>(n, 1);
    // bit 0: the caller's AoS bytes go up as they are (no host staging); bit 1: the inliers come down
    // straight into the caller's memory (no pinned staging).  The default (3) sets both, and only the
    // buffers a mode uses are allocated: growing a pinned block drains the context and bumps arena_gen.
    const int mode = ctx->single_mode;
    const bool in_staged = !(mode & 1), out_staged = !(mode & 2);
    float* h = in_staged ? (float*)ctx->pinned("single_h", (size_t)cap * 3 * sizeof(float)) : nullptr;
    int32_t* hi = out_staged ? (int32_t*)ctx->pinned("single_hinl", (size_t)cap * sizeof(int32_t)) : nullptr;
    if ((in_staged && !h) || (out_staged && !hi)) return ctx->fail(PITT_E_NOMEM, "pinned allocation failed");
    float* d = (float*)ctx->buf("single_xyz", (size_t)cap * 3 * sizeof(float));
    float* ds = in_staged ? (float*)ctx->buf("single_stage", (size_t)cap * 3 * sizeof(float)) : nullptr;
    int32_t* di = (int32_t*)ctx->buf("single_inl", (size_t)cap * sizeof(int32_t));
    if (!d || (in_staged && !ds) || !di) return ctx->fail(PITT_E_NOMEM, "device allocation failed");
    // Staged input: the cloud goes up in chunks of C points, each deinterleaved on the host into [x y z]
    // runs of the pinned staging buffer and sent by ONE copy as soon as it is ready, so the DMA of chunk k
    // runs under the deinterleave of chunk k+1; k_single_planes then lays the chunks out as the planes.
    const bool timing = ctx->host_timing;
    const double t0 = timing ? pitt::wall_ms() : 0.0;
    const int sf = stride_bytes / 4;
    if (!in_staged && n > 0) {
        float* da = (float*)ctx->buf("single_aos", (size_t)n * stride_bytes);
        if (!da) return ctx->fail(PITT_E_NOMEM, "device allocation failed");
        PITT_HIP_TRY(hipMemcpyAsync(da, xyz, (size_t)n * stride_bytes, hipMemcpyHostToDevice, ctx->stream));
        hipLaunchKernelGGL(pitt::k_single_aos, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 2048)), dim3(256), 0,
                           ctx->stream, da, n, sf, cap, d);
        PITT_HIP_TRY(hipGetLastError());
    }
    for (int64_t b = 0; in_staged && b < n; b += C) {
        const int64_t m = std::min(C, n - b);
        float* hx = h + 3 * b;  // chunk b / C starts at 3 b (every earlier chunk is full)
        float *hy = hx + m, *hz = hx + 2 * m;
        const float* src = xyz + b * sf;
        if (sf == 4) {
            pitt::deinterleave4(src, m, hx, hy, hz);
        } else {
            for (int64_t i = 0; i < m; ++i) {
                hx[i] = src[3 * i];
                hy[i] = src[3 * i + 1];
                hz[i] = src[3 * i + 2];
            }
        }
        PITT_HIP_TRY(hipMemcpyAsync(ds + 3 * b, hx, (size_t)(3 * m) * sizeof(float), hipMemcpyHostToDevice,
                                    ctx->stream));
    }
    if (in_staged && n > 0) {
        hipLaunchKernelGGL(pitt::k_single_planes, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 2048)), dim3(256),
                           0, ctx->stream, ds, n, C, cap, d);
        PITT_HIP_TRY(hipGetLastError());
    }
    const double t1 = timing ? pitt::wall_ms() : 0.0;
    int64_t off = 0;
    pitt_frames fr;
    fr.x = d;
    fr.y = d + cap;
    fr.z = d + 2 * cap;
    fr.offsets = &off;
    fr.counts = &n;
    fr.n_frames = 1;
    fr.capacity = cap;
    pitt_plane_result r;
    int rc = pitt_plane_segment_batch_async(ctx, &fr, p, &r, di);
    if (rc < 0) return rc;
    // the inlier list comes back with the batch: a copy of the whole list buffer into pinned memory
    // enqueued behind it (a continuation would enqueue more work after this copy: then copy again)
    const int64_t cont0 = ctx->continuations;
    if (out_staged && inliers_out && n > 0) {
        const hipError_t ce = hipMemcpyAsync(hi, di, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream);
        if (ce != hipSuccess) {
            // the batch is in flight with its results bound for r (this frame): complete it first
            (void)pitt::finish_batch(ctx);
            return ctx->fail(PITT_E_HIP, std::string("hipMemcpyAsync (inliers): ") + hipGetErrorString(ce));
        }
    }
    rc = pitt_wait(ctx);
    if (rc < 0) return rc;
    const double t2 = timing ? pitt::wall_ms() : 0.0;
    if (r.status < 0) return ctx->fail(r.status, "plane segmentation failed");
    if (r.n_coeff == 0) return PITT_NO_MODEL;
    if (inliers_out && r.n_inliers > 0) {
        if (!out_staged) {
            PITT_HIP_TRY(hipMemcpy(inliers_out, di, (size_t)r.n_inliers * sizeof(int32_t), hipMemcpyDeviceToHost));
        } else {
            if (ctx->continuations != cont0)
                PITT_HIP_TRY(hipMemcpy(hi, di, (size_t)r.n_inliers * sizeof(int32_t), hipMemcpyDeviceToHost));
            std::memcpy(inliers_out, hi, (size_t)r.n_inliers * sizeof(int32_t));
        }
    }
    if (timing)
        std::fprintf(stderr, "pitt_plane_segment n=%lld: convert+enqueue %.3f ms, batch+inliers D2H %.3f ms, copy out %.3f ms\n",
                     (long long)n, t1 - t0, t2 - t1, pitt::wall_ms() - t2);
    *n_inliers = r.n_inliers;
    *n_coeff = 4;
    if (coeff_out) std::memcpy(coeff_out, r.coefficients, 4 * sizeof(float));
    return PITT_OK;
}

int pitt_last_hypothesis_counts(pitt_ctx* ctx, int32_t frame, int32_t* counts, int32_t cap) {
    if (!ctx || !counts) return PITT_E_INVALID;
    if (int rc = pitt::finish_batch(ctx)) return rc;
    if (frame < 0 || frame >= ctx->last_frames) return ctx->fail(PITT_E_INVALID, "frame out of range");
    auto it = ctx->bufs.find("hyp_total");
    if (it == ctx->bufs.end()) return ctx->fail(PITT_E_INVALID, "no batch run yet");
    const int32_t m = std::min(cap, ctx->last_hcap);
    PITT_HIP_TRY(hipStreamSynchronize(ctx->stream));
    PITT_HIP_TRY(hipMemcpy(counts, (int32_t*)it->second.p + (size_t)frame * ctx->last_hcap,
                           (size_t)m * sizeof(int32_t), hipMemcpyDeviceToHost));
    return PITT_OK;
}

int pitt_sampler_table(int64_t n, uint32_t seed, int64_t attempts, int32_t* out) {
    if (n < 3 || attempts < 0 || (attempts > 0 && !out)) return PITT_E_INVALID;
    pitt_ctx tmp;  // host-only: table cache lives in a throwaway context
    const std::vector<int32_t>& t = pitt::sampler_table(&tmp, n, seed, attempts);
    std::memcpy(out, t.data(), t.size() * sizeof(int32_t));
    return PITT_OK;
}

float pitt_float_threshold(double threshold) { return pitt::float_threshold(threshold); }

int pitt_profile_enable(pitt_ctx* ctx, int32_t on) {
    if (!ctx) return PITT_E_INVALID;
    if (!on) (void)ctx->prof_collect();
    ctx->prof = on != 0;
    return PITT_OK;
}

int pitt_profile_get(pitt_ctx* ctx, const char* kernel, int64_t* launches, double* total_ms,
                     double* algorithmic_bytes) {
    if (!ctx || !kernel) return PITT_E_INVALID;
    if (int rc = pitt::finish_batch(ctx)) return rc;
    int rc = ctx->prof_collect();
    if (rc) return rc;
    auto it = ctx->totals.find(kernel);
    const pitt::ProfTotal t = it == ctx->totals.end() ? pitt::ProfTotal() : it->second;
    if (launches) *launches = t.launches;
    if (total_ms) *total_ms = t.ms;
    if (algorithmic_bytes) *algorithmic_bytes = t.bytes;
    return PITT_OK;
}

int pitt_profile_reset(pitt_ctx* ctx) {
    if (!ctx) return PITT_E_INVALID;
    (void)ctx->prof_collect();
    ctx->totals.clear();
    return PITT_OK;
}

}  // extern "C"
