// supports.hip -- ExtractIndices and the support (table) segmentation loop on gfx950.
//
// Replaces, in src/segmentation_services/supports_segmentation_srv.cpp (reference paths):
//   removePlaneInliner  :114-127  -> k_gather (positive) + ordered compaction (negative)
//   createNewIdxMap     :139-157  -> membership bitmask + ordered rank (O(N), not O(N*|inl|))
//   getPointOnPlane     :187-238  -> prefix-max scan for the `if / else if` bbox (Q5), exact
//                                    double z sum (Q10), ordered compaction of the originals
//   findSupports        :241-361  -> host loop driving the device (stop tests in float, Q9)
// The RANSAC inside the loop is pitt_plane_segment_batch with one frame.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

#include "compact.hpp"
#include "ctx.hpp"

#pragma clang fp contract(off)

namespace pitt {

__global__ __launch_bounds__(kBlock) void k_scan_tiles(const int32_t* __restrict__ counts, int64_t nt,
                                                       int32_t* __restrict__ offsets) {
    __shared__ int32_t lds4[kBlock / 64];
    int carry = 0;
    for (int64_t base = 0; base < nt; base += kBlock) {
        const int64_t t = base + threadIdx.x;
        const int v = t < nt ? counts[t] : 0;
        int total;
        const int ex = block_exscan(v, lds4, &total);
        if (t < nt) offsets[t] = carry + ex;
        carry += total;
    }
    if (threadIdx.x == 0) offsets[nt] = carry;
}

// ---- predicates / actions --------------------------------------------------------------------
struct NotMember {  // negative ExtractIndices: keep points whose index is not in the bitmask
    const uint32_t* bits;
    __device__ bool operator()(int64_t i) const { return !((bits[i >> 5] >> (i & 31)) & 1u); }
};
struct CopyXYZ {
    const float *x, *y, *z;
    float *ox, *oy, *oz;
    __device__ void operator()(int64_t i, int64_t p) const {
        ox[p] = x[i];
        oy[p] = y[i];
        oz[p] = z[i];
    }
};

__global__ void k_mark(const int32_t* __restrict__ idx, int64_t m, int64_t n, uint32_t* __restrict__ bits,
                       int32_t* __restrict__ bad) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        const int32_t i = idx[k];
        if (i < 0 || i >= n) { atomicOr(bad, 1); continue; }
        atomicOr(&bits[i >> 5], 1u << (i & 31));
    }
}

__global__ void k_gather(const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ z,
                         const int32_t* __restrict__ idx, int64_t m, float* __restrict__ ox, float* __restrict__ oy,
                         float* __restrict__ oz) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        const int32_t i = idx[k];
        ox[k] = x[i];
        oy[k] = y[i];
        oz[k] = z[i];
    }
}

__global__ void k_iota(int32_t* __restrict__ v, int64_t n) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
        v[k] = (int32_t)k;
}

// createNewIdxMap: propagate (level < v < 0), tag members with `level`; the rest get a running
// counter assigned by the ordered compaction below (MapRest / MapRank).
__global__ void k_map_tags(const int32_t* __restrict__ prev, int64_t n, const uint32_t* __restrict__ bits,
                           int64_t nbits, int level, int32_t* __restrict__ out) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const int v = prev[p];
        if (v > level && v < 0) out[p] = v;
        else if (v >= 0 && v < nbits && ((bits[v >> 5] >> (v & 31)) & 1u)) out[p] = level;
    }
}
struct MapRest {
    const int32_t* prev;
    const uint32_t* bits;
    int64_t nbits;
    int level;
    __device__ bool operator()(int64_t p) const {
        const int v = prev[p];
        if (v > level && v < 0) return false;
        if (v >= 0 && v < nbits && ((bits[v >> 5] >> (v & 31)) & 1u)) return false;
        return true;
    }
};
struct MapRank {
    int32_t* out;
    __device__ void operator()(int64_t p, int64_t pos) const { out[p] = (int32_t)pos; }
};

// ---- getPointOnPlane bbox (Q5) -----------------------------------------------------------------
// xMax = max x; xMin = min { x_i : i >= 1, x_i <= max(x_0..x_{i-1}) } (the `else if` branch);
// same for y.  zsum in double: computed in parallel and proven equal to the sequential sum when
// every partial sum is exactly representable (all |z| multiples of 2^q and sum|z| <= 2^(52+q)).
struct BBoxTile {
    float mx, my;        // inclusive tile max
    float cx, cy;        // candidate minima (else-if branch)
    double zs, za;       // sum z, sum |z|
    int32_t q;           // min ulp exponent of nonzero |z|
    int32_t pad;
};

__device__ __forceinline__ float fmax_nan_free(float a, float b) { return (a < b) ? b : a; }

__global__ __launch_bounds__(kBlock) void k_bbox_tilemax(const float* __restrict__ x, const float* __restrict__ y,
                                                         int64_t n, BBoxTile* __restrict__ tiles) {
    __shared__ float sx[kBlock / 64], sy[kBlock / 64];
    const int64_t nt = ctiles(n);
    for (int64_t t = blockIdx.x; t < nt; t += gridDim.x) {
        const int64_t b = t * kCTile + threadIdx.x * 8;
        float mx = -INFINITY, my = -INFINITY;
        for (int k = 0; k < 8; ++k)
            if (b + k < n) { mx = fmax_nan_free(mx, x[b + k]); my = fmax_nan_free(my, y[b + k]); }
        for (int d = 32; d >= 1; d >>= 1) {
            mx = fmax_nan_free(mx, __shfl_xor(mx, d, 64));
            my = fmax_nan_free(my, __shfl_xor(my, d, 64));
        }
        if ((threadIdx.x & 63) == 0) { sx[threadIdx.x >> 6] = mx; sy[threadIdx.x >> 6] = my; }
        __syncthreads();
        if (threadIdx.x == 0) {
            float ax = sx[0], ay = sy[0];
            for (int w = 1; w < kBlock / 64; ++w) { ax = fmax_nan_free(ax, sx[w]); ay = fmax_nan_free(ay, sy[w]); }
            tiles[t].mx = ax;
            tiles[t].my = ay;
        }
        __syncthreads();
    }
}

// exclusive prefix max over tiles (single block, serial: tiles are few)
__global__ void k_bbox_tilescan(BBoxTile* __restrict__ tiles, int64_t nt, float* __restrict__ pre /*2*nt*/) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    float ax = -INFINITY, ay = -INFINITY;
    for (int64_t t = 0; t < nt; ++t) {
        pre[2 * t] = ax;
        pre[2 * t + 1] = ay;
        ax = fmax_nan_free(ax, tiles[t].mx);
        ay = fmax_nan_free(ay, tiles[t].my);
    }
}

__device__ __forceinline__ void excl_max_scan(float v, float* lds, float& ex) {
    // block-wide exclusive max scan (kBlock threads)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float inc = v;
    for (int d = 1; d < 64; d <<= 1) {
        float t = __shfl_up(inc, d, 64);
        if (lane >= d) inc = fmax_nan_free(inc, t);
    }
    float exw = __shfl_up(inc, 1, 64);
    if (lane == 0) exw = -INFINITY;
    if (lane == 63) lds[w] = inc;
    __syncthreads();
    float pre = -INFINITY;
    for (int i = 0; i < w; ++i) pre = fmax_nan_free(pre, lds[i]);
    __syncthreads();
    ex = fmax_nan_free(pre, exw);
}

__global__ __launch_bounds__(kBlock) void k_bbox_tilemin(const float* __restrict__ x, const float* __restrict__ y,
                                                         const float* __restrict__ z, int64_t n,
                                                         const float* __restrict__ pre, BBoxTile* __restrict__ tiles) {
    __shared__ float lx[kBlock / 64], ly[kBlock / 64];
    __shared__ float rcx[kBlock / 64], rcy[kBlock / 64];
    __shared__ double rzs[kBlock / 64], rza[kBlock / 64];
    __shared__ int32_t rq[kBlock / 64];
    const int64_t nt = ctiles(n);
    for (int64_t t = blockIdx.x; t < nt; t += gridDim.x) {
        const int64_t b = t * kCTile + threadIdx.x * 8;
        float vx[8], vy[8];
        float tmx = -INFINITY, tmy = -INFINITY;
        for (int k = 0; k < 8; ++k) {
            vx[k] = b + k < n ? x[b + k] : -INFINITY;
            vy[k] = b + k < n ? y[b + k] : -INFINITY;
            tmx = fmax_nan_free(tmx, vx[k]);
            tmy = fmax_nan_free(tmy, vy[k]);
        }
        float ex, ey;
        excl_max_scan(tmx, lx, ex);
        excl_max_scan(tmy, ly, ey);
        float runx = fmax_nan_free(pre[2 * t], ex), runy = fmax_nan_free(pre[2 * t + 1], ey);
        float cx = INFINITY, cy = INFINITY;
        double zs = 0.0, za = 0.0;
        int q = 1 << 30;
        for (int k = 0; k < 8; ++k) {
            if (b + k >= n) break;
            if (vx[k] > runx) runx = vx[k];
            else if (vx[k] < cx) cx = vx[k];
            if (vy[k] > runy) runy = vy[k];
            else if (vy[k] < cy) cy = vy[k];
            const float zz = z[b + k];
            zs += (double)zz;
            za += fabs((double)zz);
            if (zz != 0.0f) {
                int e;
                (void)frexpf(zz, &e);
                q = min(q, max(e - 24, -149));
            }
        }
        for (int d = 32; d >= 1; d >>= 1) {
            cx = fminf(cx, __shfl_xor(cx, d, 64));
            cy = fminf(cy, __shfl_xor(cy, d, 64));
            zs += __shfl_xor(zs, d, 64);
            za += __shfl_xor(za, d, 64);
            q = min(q, __shfl_xor(q, d, 64));
        }
        const int w = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) { rcx[w] = cx; rcy[w] = cy; rzs[w] = zs; rza[w] = za; rq[w] = q; }
        __syncthreads();
        if (threadIdx.x == 0) {
            BBoxTile bt = tiles[t];
            bt.cx = rcx[0]; bt.cy = rcy[0]; bt.zs = rzs[0]; bt.za = rza[0]; bt.q = rq[0];
            for (int i = 1; i < kBlock / 64; ++i) {
                bt.cx = fminf(bt.cx, rcx[i]);
                bt.cy = fminf(bt.cy, rcy[i]);
                bt.zs += rzs[i];
                bt.za += rza[i];
                bt.q = min(bt.q, rq[i]);
            }
            tiles[t] = bt;
        }
        __syncthreads();
    }
}

// out[0..7]: xMax, xMin, yMax, yMin, zsum (tile partials in tile order), zabs, q, exact(1/0).
// k_bbox_final reduces the tiles; k_onsupport_bounds (below) turns them into the on-support filter's
// bounds on the device, so the support loop needs no host round trip for them.
__global__ void k_bbox_final(const BBoxTile* __restrict__ tiles, int64_t nt, double* __restrict__ out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    float mx = -INFINITY, my = -INFINITY, cx = INFINITY, cy = INFINITY;
    double zs = 0.0, za = 0.0;
    int q = 1 << 30;
    for (int64_t t = 0; t < nt; ++t) {
        mx = fmax_nan_free(mx, tiles[t].mx);
        my = fmax_nan_free(my, tiles[t].my);
        cx = fminf(cx, tiles[t].cx);
        cy = fminf(cy, tiles[t].cy);
        zs += tiles[t].zs;
        za += tiles[t].za;
        q = min(q, tiles[t].q);
    }
    const bool exact = (q == (1 << 30)) || (za <= ldexp(1.0, 52 + q));
    out[0] = mx; out[1] = cx; out[2] = my; out[3] = cy;
    out[4] = zs; out[5] = za; out[6] = q; out[7] = exact ? 1.0 : 0.0;
}

// supports_segmentation_srv.cpp:207,217: the reference's sequential double sum of z -- only when
// the parallel sum could not be certified (flag out[8] == 0 after k_onsupport_bounds), else a no-op.
__global__ void k_zsum_seq(const float* __restrict__ z, int64_t n, double* __restrict__ out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    if (out[8] != 0.0) return;
    double zs = 0.0;
    for (int64_t i = 0; i < n; ++i) zs += (double)z[i];
    out[4] = zs;
    out[8] = 2.0;  // sequential
}

// zMed = zsum / n + off computed from a sum in another association: the sequential sum differs by
// at most 2 (n - 1) u sum|z| (u = 2^-53, both sums' error bounds), the division and the addition
// add a few ulps.  If no float lies within that bound of zMed, every `(double)z > zMed` test of
// the on-support filter decides the same way for the sequential value: returns true and zMed.
__host__ __device__ inline bool zmed_certified(double zsum, double zabs, int64_t n, double off, double* zmed) {
    const double u = 1.1102230246251565e-16;  // 2^-53
    const double m = zsum / (double)n + off;
    const double b = 2.0000001 * (double)(n - 1) * u * zabs / (double)n * (1.0 + 4.0 * u) +
                     8.0 * u * (fabs(zsum) / (double)n + fabs(off) + fabs(m)) + 1e-300;
    const double lo = m - b, hi = m + b;
    if (!isfinite(lo) || !isfinite(hi)) return false;
    float f = (float)hi;                    // the largest float <= hi
    if ((double)f > hi) f = nextafterf(f, -INFINITY);
    if ((double)f >= lo) return false;      // a float inside [lo, hi]: the sums' rounding could matter
    *zmed = m;
    return true;
}

// getPointOnPlane's bounds (supports_segmentation_srv.cpp:184-217) from k_bbox_final's reduction:
// bb[0..3] -> x/y max and min shrunk by the edge offsets, bb[9] = zMed.  bb[8]: 1 when the parallel
// z sum was exact or certified, 0 when the sequential sum must decide (k_zsum_seq, then
// k_onsupport_zmed).
__global__ void k_onsupport_bounds(double* __restrict__ bb, int64_t n, float ox, float oy, float oz) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double zmed = 0.0;
    bool ok = true;
    if (bb[7] != 0.0) zmed = bb[4] / (double)n + (double)oz;  // every partial sum exact
    else ok = zmed_certified(bb[4], bb[5], n, (double)oz, &zmed);
    bb[0] -= (double)ox;  // xMax
    bb[1] += (double)ox;  // xMin
    bb[2] -= (double)oy;  // yMax
    bb[3] += (double)oy;  // yMin
    bb[8] = ok ? 1.0 : 0.0;
    bb[9] = zmed;
}
__global__ void k_onsupport_zmed(double* __restrict__ bb, int64_t n, float oz) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    if (bb[8] == 2.0) bb[9] = bb[4] / (double)n + (double)oz;
}

struct OnSupport {  // bounds read from the device (k_onsupport_bounds): bb[0] xMax, [1] xMin, [2] yMax, [3] yMin, [9] zMed
    const float *x, *y, *z;
    const int32_t* map;
    int level;
    const double* bb;
    __device__ bool operator()(int64_t i) const {
        if (map[i] == level) return false;
        const double px = x[i], py = y[i], pz = z[i];
        return px > bb[1] && px < bb[0] && pz > bb[9] && py > bb[3] && py < bb[2];
    }
};

// ---- host helpers -------------------------------------------------------------------------------
template <class Pred, class Act>
static int run_compact(pitt_ctx* ctx, int64_t n, Pred pred, Act act, int64_t* total, int32_t* total_dev = nullptr) {
    const int64_t nt = ctiles(n);
    int32_t* counts = (int32_t*)ctx->buf("cmp_counts", (size_t)std::max<int64_t>(nt, 1) * 4);
    int32_t* offs = (int32_t*)ctx->buf("cmp_offs", (size_t)(nt + 1) * 4);
    if (!counts || !offs) return ctx->fail(PITT_E_NOMEM, "compaction scratch");
    hipStream_t s = ctx->stream;
    if (n > 0) {
        hipLaunchKernelGGL((k_pred_count<Pred>), dim3(grid_for_tiles(nt)), dim3(kBlock), 0, s, pred, n, counts);
    }
    hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(kBlock), 0, s, counts, nt, offs);
    if (n > 0) {
        hipLaunchKernelGGL((k_pred_apply<Pred, Act>), dim3(grid_for_tiles(nt)), dim3(kBlock), 0, s, pred, act, n,
                           offs);
    }
    PITT_HIP_TRY(hipGetLastError());
    if (total_dev) PITT_HIP_TRY(hipMemcpyAsync(total_dev, offs + nt, 4, hipMemcpyDeviceToDevice, s));
    if (total) {
        int32_t* h = (int32_t*)ctx->pinned("cmp_total", 16);
        PITT_HIP_TRY(hipMemcpyAsync(h, offs + nt, 4, hipMemcpyDeviceToHost, s));
        PITT_HIP_TRY(hipStreamSynchronize(s));
        *total = h[0];
    }
    return PITT_OK;
}

static inline int ew_grid(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4096)); }

int extract_indices_impl(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                         const int32_t* idx, int64_t m, int negative, float* ox, float* oy, float* oz,
                         int64_t* n_out) {
    hipStream_t s = ctx->stream;
    if (!negative) {
        if (m > 0) hipLaunchKernelGGL(k_gather, dim3(ew_grid(m)), dim3(256), 0, s, x, y, z, idx, m, ox, oy, oz);
        PITT_HIP_TRY(hipGetLastError());
        PITT_HIP_TRY(hipStreamSynchronize(s));
        *n_out = m;
        return PITT_OK;
    }
    const int64_t words = (n + 31) / 32;
    uint32_t* bits = (uint32_t*)ctx->buf("ext_bits", (size_t)std::max<int64_t>(words, 1) * 4 + 16);
    if (!bits) return ctx->fail(PITT_E_NOMEM, "bitmask");
    int32_t* bad = (int32_t*)(bits + words);
    PITT_HIP_TRY(hipMemsetAsync(bits, 0, (size_t)words * 4 + 16, s));
    if (m > 0) hipLaunchKernelGGL(k_mark, dim3(ew_grid(m)), dim3(256), 0, s, idx, m, n, bits, bad);
    return run_compact(ctx, n, NotMember{bits}, CopyXYZ{x, y, z, ox, oy, oz}, n_out);
}

// isHorizontalPlane :161-179, float.
static bool is_horizontal(const float c[4], const float axis[3], float var_th) {
    float div = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
    float nx = c[0] / div, ny = c[1] / div, nz = c[2] / div;
    float cx = ny * axis[2] - nz * axis[1];
    float cy = nz * axis[0] - nx * axis[2];
    float cz = nx * axis[1] - ny * axis[0];
    float lo = -1 * var_th, hi = var_th;
    return (cx > lo && cx < hi) && (cy > lo && cy < hi) && (cz > lo && cz < hi);
}

// The support loop (findSupports, :241-361).  x/y/z: host SoA, or device SoA when dev_in.  Results:
// host copies into `out` (pitt_find_supports), or device buffers of the context into `dout`
// (pitt_find_supports_dev: nothing leaves HBM).  Host round trips per iteration: one -- the RANSAC
// results the stop tests and the horizontality test read (:270-300); the removal, the index map,
// the on-support bounds (k_onsupport_bounds) and the on-support compaction are stream-ordered.
int find_supports_impl(pitt_ctx* ctx, const float* hx, const float* hy, const float* hz, int64_t N,
                       const pitt_support_params* sp, pitt_support_list* out, pitt_support_list_dev* dout,
                       bool dev_in, int aos_stride) {
    hipStream_t s = ctx->stream;
    const bool timing = ctx->host_timing;  // $PITT_HOST_TIMING=1: host phases on stderr
    const double tm0 = timing ? wall_ms() : 0.0;
    double tm_ransac = 0.0;
    ctx->keep_supports.clear();
    ctx->keep_supports_dev.clear();
    if (out) {
        out->n_supports = 0;
        out->supports = nullptr;
        out->iterations = 0;
    }
    if (dout) {
        dout->n_supports = 0;
        dout->supports = nullptr;
        dout->iterations = 0;
    }
    const int64_t cap = std::max<int64_t>(kCTile, (N + kCTile - 1) / kCTile * kCTile);
    auto plane3 = [&](const std::string& name) { return (float*)ctx->buf(name, (size_t)cap * 3 * sizeof(float)); };
    float* O = plane3("sup_orig");
    float* IT[2] = {plane3("sup_it0"), plane3("sup_it1")};
    int32_t* INL = (int32_t*)ctx->buf("sup_inl", (size_t)cap * 4);
    int32_t* MAP[2] = {(int32_t*)ctx->buf("sup_map0", (size_t)cap * 4), (int32_t*)ctx->buf("sup_map1", (size_t)cap * 4)};
    const int64_t words = (cap + 31) / 32;
    uint32_t* MEM = (uint32_t*)ctx->buf("sup_mem", (size_t)words * 4 + 16);
    const int64_t ntmax = ctiles(cap);
    BBoxTile* BT = (BBoxTile*)ctx->buf("sup_bbox", (size_t)ntmax * sizeof(BBoxTile));
    float* PRE = (float*)ctx->buf("sup_pre", (size_t)ntmax * 2 * sizeof(float));
    // per support (at most one per iteration; an iteration removes >= min_iterative_plane_percentage of N):
    // bounds, on-support count
    const int kMaxSup = 256;
    double* BB = (double*)ctx->buf("sup_bbout", (size_t)kMaxSup * 16 * sizeof(double));
    int32_t* NON = (int32_t*)ctx->buf("sup_non", (size_t)kMaxSup * 4);
    if (!O || !IT[0] || !IT[1] || !INL || !MAP[0] || !MAP[1] || !MEM || !BT || !PRE || !BB || !NON)
        return ctx->fail(PITT_E_NOMEM, "support scratch");
    // the original cloud -- iterativeCloud starts as its copy
    if (aos_stride) {  // the caller's host AoS cloud as it lies: one upload, deinterleaved on the device
        void* scr = ctx->buf("sup_aos", (size_t)std::max<int64_t>(N, 1) * aos_stride);
        if (!scr) return ctx->fail(PITT_E_NOMEM, "support scratch");
        PITT_HIP_TRY(upload_aos(s, scr, hx, N, aos_stride, O, O + cap, O + 2 * cap));
    } else {
        const hipMemcpyKind kin = dev_in ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
        PITT_HIP_TRY(hipMemcpyAsync(O, hx, (size_t)N * 4, kin, s));
        PITT_HIP_TRY(hipMemcpyAsync(O + cap, hy, (size_t)N * 4, kin, s));
        PITT_HIP_TRY(hipMemcpyAsync(O + 2 * cap, hz, (size_t)N * 4, kin, s));
    }
    PITT_HIP_TRY(hipMemcpyAsync(IT[0], O, (size_t)cap * 3 * 4, hipMemcpyDeviceToDevice, s));
    const double tm1 = timing ? wall_ms() : 0.0;

    pitt_sac_params p;
    pitt_sac_params_default(&p);
    p.threshold = (double)sp->ransac_distance_threshold;
    p.max_iterations = sp->ransac_max_iterations;
    p.reduce_order = sp->reduce_order;
    p.div_mode = sp->div_mode;

    struct Found {
        int32_t* map;
        float *sup, *on;
        int64_t n_sup;
        float coef[4];
    };
    std::vector<Found> found;
    int cur = 0, mcur = 0;
    int64_t Nk = N;
    int level = -2, cnt = 0, iterations = 0;
    const float Nf = (float)N;
    while (true) {
        pitt_frames fr;
        int64_t off = 0;
        fr.x = IT[cur];
        fr.y = IT[cur] + cap;
        fr.z = IT[cur] + 2 * cap;
        fr.offsets = &off;
        fr.counts = &Nk;
        fr.n_frames = 1;
        fr.capacity = cap;
        pitt_plane_result r;
        const double tr0 = timing ? wall_ms() : 0.0;
        int rc = pitt_plane_segment_batch(ctx, &fr, &p, &r, INL);  // the loop's one host round trip
        if (timing) tm_ransac += wall_ms() - tr0;
        if (rc < 0) return rc;
        if (r.status < 0) return ctx->fail(r.status, "RANSAC inside the support loop failed");
        ++iterations;
        const int64_t n_inl = r.n_coeff ? r.n_inliers : 0;
        if (n_inl == 0) break;                                                   // :270
        if ((float)Nk < Nf * sp->min_iterative_cloud_percentage) break;          // :274 (Q9)
        if ((float)n_inl < Nf * sp->min_iterative_plane_percentage) break;       // :278
        const bool horizontal = is_horizontal(r.coefficients, sp->horizontal_axis, sp->horizontal_variance_threshold);
        if (horizontal && (int)found.size() >= kMaxSup) return ctx->fail(PITT_E_INVALID, "more than 256 supports");
        const int k = (int)found.size();
        // the support cloud goes straight into its own buffer when the plane is a support
        float* S = horizontal ? plane3("sup_s" + std::to_string(k)) : plane3("sup_s");
        if (!S) return ctx->fail(PITT_E_NOMEM, "support scratch");
        // membership bitmask of the inliers (indices into the current iterative cloud)
        PITT_HIP_TRY(hipMemsetAsync(MEM, 0, (size_t)words * 4 + 16, s));
        hipLaunchKernelGGL(k_mark, dim3(ew_grid(n_inl)), dim3(256), 0, s, INL, n_inl, Nk, MEM,
                           (int32_t*)(MEM + words));
        // removePlaneInliner: support = it[inl] ; it <- it \ inl (inliers unique: |it \ inl| = Nk - n_inl)
        hipLaunchKernelGGL(k_gather, dim3(ew_grid(n_inl)), dim3(256), 0, s, IT[cur], IT[cur] + cap, IT[cur] + 2 * cap,
                           INL, n_inl, S, S + cap, S + 2 * cap);
        rc = run_compact(ctx, Nk, NotMember{MEM},
                         CopyXYZ{IT[cur], IT[cur] + cap, IT[cur] + 2 * cap, IT[cur ^ 1], IT[cur ^ 1] + cap,
                                 IT[cur ^ 1] + 2 * cap},
                         nullptr);
        if (rc) return rc;
        const int64_t Nn = Nk - n_inl;
        // index map w.r.t. the original cloud
        if (!cnt) hipLaunchKernelGGL(k_iota, dim3(ew_grid(N)), dim3(256), 0, s, MAP[mcur], N);
        const int lv = horizontal ? level : -1;
        hipLaunchKernelGGL(k_map_tags, dim3(ew_grid(N)), dim3(256), 0, s, MAP[mcur], N, MEM, Nk, lv, MAP[mcur ^ 1]);
        rc = run_compact(ctx, N, MapRest{MAP[mcur], MEM, Nk, lv}, MapRank{MAP[mcur ^ 1]}, nullptr);
        if (rc) return rc;
        if (horizontal) {
            Found fd;
            fd.map = (int32_t*)ctx->buf("sup_m" + std::to_string(k), (size_t)cap * 4);
            fd.on = plane3("sup_on" + std::to_string(k));
            if (!fd.map || !fd.on) return ctx->fail(PITT_E_NOMEM, "support outputs");
            fd.sup = S;
            fd.n_sup = n_inl;
            std::memcpy(fd.coef, r.coefficients, sizeof fd.coef);
            PITT_HIP_TRY(hipMemcpyAsync(fd.map, MAP[mcur ^ 1], (size_t)N * 4, hipMemcpyDeviceToDevice, s));
            double* bb = BB + 16 * k;
            const int64_t nt = ctiles(n_inl);
            hipLaunchKernelGGL(k_bbox_tilemax, dim3(grid_for_tiles(nt)), dim3(kBlock), 0, s, S, S + cap, n_inl, BT);
            hipLaunchKernelGGL(k_bbox_tilescan, dim3(1), dim3(64), 0, s, BT, nt, PRE);
            hipLaunchKernelGGL(k_bbox_tilemin, dim3(grid_for_tiles(nt)), dim3(kBlock), 0, s, S, S + cap, S + 2 * cap,
                               n_inl, PRE, BT);
            hipLaunchKernelGGL(k_bbox_final, dim3(1), dim3(64), 0, s, BT, nt, bb);
            hipLaunchKernelGGL(k_onsupport_bounds, dim3(1), dim3(64), 0, s, bb, n_inl, sp->edge_remove_offset[0],
                               sp->edge_remove_offset[1], sp->edge_remove_offset[2]);
            // only an uncertifiable parallel z sum pays the reference's sequential loop (a no-op otherwise)
            hipLaunchKernelGGL(k_zsum_seq, dim3(1), dim3(64), 0, s, S + 2 * cap, n_inl, bb);
            hipLaunchKernelGGL(k_onsupport_zmed, dim3(1), dim3(64), 0, s, bb, n_inl, sp->edge_remove_offset[2]);
            rc = run_compact(ctx, N, OnSupport{O, O + cap, O + 2 * cap, MAP[mcur ^ 1], lv, bb},
                             CopyXYZ{O, O + cap, O + 2 * cap, fd.on, fd.on + cap, fd.on + 2 * cap}, nullptr, NON + k);
            if (rc) return rc;
            found.push_back(fd);
        }
        mcur ^= 1;
        cur ^= 1;
        Nk = Nn;
        ++cnt;
        --level;
    }
    // sizes of the on-support clouds and the z-sum path taken, in one round trip
    const double tm2 = timing ? wall_ms() : 0.0;
    const int nsup = (int)found.size();
    std::vector<int64_t> n_on((size_t)nsup, 0);
    if (nsup > 0) {
        int32_t* h = (int32_t*)ctx->pinned("sup_non_h", (size_t)kMaxSup * 4);
        double* hb = (double*)ctx->pinned("sup_bb_h", (size_t)kMaxSup * 16 * sizeof(double));
        PITT_HIP_TRY(hipMemcpyAsync(h, NON, (size_t)nsup * 4, hipMemcpyDeviceToHost, s));
        PITT_HIP_TRY(hipMemcpyAsync(hb, BB, (size_t)nsup * 16 * sizeof(double), hipMemcpyDeviceToHost, s));
        PITT_HIP_TRY(hipStreamSynchronize(s));
        for (int k = 0; k < nsup; ++k) {
            n_on[(size_t)k] = h[k];
            if (hb[16 * k + 8] == 2.0) ++ctx->zsum_sequential;
        }
    }
    if (dout) {
        for (int k = 0; k < nsup; ++k) {
            const Found& fd = found[(size_t)k];
            pitt_support_dev su;
            su.n_points = (int32_t)N;
            su.idx_map = fd.map;
            std::memcpy(su.coefficients, fd.coef, sizeof su.coefficients);
            su.n_support = fd.n_sup;
            su.support_xyz = fd.sup;
            su.n_on_support = n_on[(size_t)k];
            su.on_support_xyz = fd.on;
            su.stride = cap;
            ctx->keep_supports_dev.push_back(su);
        }
        dout->n_supports = nsup;
        dout->supports = ctx->keep_supports_dev.data();
        dout->iterations = iterations;
        return PITT_OK;
    }
    // host results: one copy per output at the end, into the context's pinned output block (reused
    // across calls, so no page faults and full-rate DMA; valid until the next support call)
    auto al16 = [](size_t b) { return (b + 15) / 16 * 16; };
    size_t out_bytes = 16;
    for (int k = 0; k < nsup; ++k)
        out_bytes += al16((size_t)N * 4) + al16((size_t)found[(size_t)k].n_sup * 12) + al16((size_t)n_on[(size_t)k] * 12);
    char* hout = (char*)ctx->pinned("sup_out_h", out_bytes);
    if (!hout) return ctx->fail(PITT_E_NOMEM, "support outputs (pinned)");
    std::vector<char*> hmap((size_t)nsup), hsup((size_t)nsup), hon((size_t)nsup);
    size_t o = 0;
    for (int k = 0; k < nsup; ++k) {
        const Found& fd = found[(size_t)k];
        const int64_t ns = fd.n_sup, no = n_on[(size_t)k];
        hmap[(size_t)k] = hout + o;
        o += al16((size_t)N * 4);
        hsup[(size_t)k] = hout + o;
        o += al16((size_t)ns * 12);
        hon[(size_t)k] = hout + o;
        o += al16((size_t)no * 12);
        PITT_HIP_TRY(hipMemcpyAsync(hmap[(size_t)k], fd.map, (size_t)N * 4, hipMemcpyDeviceToHost, s));
        // the support / on-support planes are cap apart on the device, packed (ns / no apart) on the host
        if (ns) PITT_HIP_TRY(hipMemcpy2DAsync(hsup[(size_t)k], (size_t)ns * 4, fd.sup, (size_t)cap * 4, (size_t)ns * 4, 3,
                                              hipMemcpyDeviceToHost, s));
        if (no) PITT_HIP_TRY(hipMemcpy2DAsync(hon[(size_t)k], (size_t)no * 4, fd.on, (size_t)cap * 4, (size_t)no * 4, 3,
                                              hipMemcpyDeviceToHost, s));
    }
    PITT_HIP_TRY(hipStreamSynchronize(s));
    if (timing)
        std::fprintf(stderr, "pitt_find_supports N=%lld: input %.3f ms, loop %.3f ms (%d iterations, RANSAC batches "
                     "%.3f ms), sizes + outputs D2H %.3f ms\n", (long long)N, tm1 - tm0, tm2 - tm1, iterations,
                     tm_ransac, wall_ms() - tm2);
    for (int k = 0; k < nsup; ++k) {
        const Found& fd = found[(size_t)k];
        pitt_support su;
        su.n_points = (int32_t)N;
        su.idx_map = (int32_t*)hmap[(size_t)k];
        std::memcpy(su.coefficients, fd.coef, sizeof su.coefficients);
        su.support_xyz = (float*)hsup[(size_t)k];
        su.n_support = fd.n_sup;
        su.on_support_xyz = (float*)hon[(size_t)k];
        su.n_on_support = n_on[(size_t)k];
        ctx->keep_supports.push_back(su);
    }
    out->n_supports = nsup;
    out->supports = ctx->keep_supports.data();
    out->iterations = iterations;
    return PITT_OK;
}

}  // namespace pitt

extern "C" {

void pitt_support_params_default(pitt_support_params* p) {
    if (!p) return;
    p->min_iterative_cloud_percentage = 0.030f;   // supports_segmentation_srv.cpp:30
    p->min_iterative_plane_percentage = 0.030f;   // :31
    p->horizontal_variance_threshold = 0.09f;     // :33
    p->ransac_distance_threshold = 0.02f;         // :35
    p->ransac_max_iterations = 10;                // :37
    p->horizontal_axis[0] = 0.0f;                 // :38
    p->horizontal_axis[1] = 0.0f;
    p->horizontal_axis[2] = -1.0f;
    p->edge_remove_offset[0] = 0.02f;             // :39
    p->edge_remove_offset[1] = 0.02f;
    p->edge_remove_offset[2] = 0.005f;
    p->reduce_order = PITT_REDUCE_SSE2;
    p->div_mode = PITT_DIV_EIGEN32;
}

int pitt_extract_indices(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                         const int32_t* indices_dev, int64_t n_indices, int32_t negative, float* ox, float* oy,
                         float* oz, int64_t* n_out) {
    if (!ctx) return PITT_E_INVALID;
    if (!n_out || n < 0 || n_indices < 0 || (n > 0 && (!x || !y || !z)) || (n_indices > 0 && !indices_dev))
        return ctx->fail(PITT_E_INVALID, "null argument");
    if ((n_indices > 0 || n > 0) && (!ox || !oy || !oz)) return ctx->fail(PITT_E_INVALID, "null output");
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    return pitt::extract_indices_impl(ctx, x, y, z, n, indices_dev, n_indices, negative, ox, oy, oz, n_out);
}

int pitt_find_supports(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                       const pitt_support_params* p, pitt_support_list* out) {
    if (!ctx) return PITT_E_INVALID;
    if (!p || !out || n < 0 || (n > 0 && (!x || !y || !z))) return ctx->fail(PITT_E_INVALID, "null argument");
    if (n > 0x7fffffff) return ctx->fail(PITT_E_INVALID, "cloud larger than 2^31 points");
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    return pitt::find_supports_impl(ctx, x, y, z, n, p, out, nullptr, false, 0);
}

int pitt_find_supports_aos(pitt_ctx* ctx, const float* xyz, int64_t n, int32_t stride_bytes,
                           const pitt_support_params* p, pitt_support_list* out) {
    if (!ctx) return PITT_E_INVALID;
    if (!p || !out || n < 0 || (n > 0 && !xyz)) return ctx->fail(PITT_E_INVALID, "null argument");
    if (stride_bytes != 12 && stride_bytes != 16) return ctx->fail(PITT_E_INVALID, "stride must be 12 or 16");
    if (n > 0x7fffffff) return ctx->fail(PITT_E_INVALID, "cloud larger than 2^31 points");
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    return pitt::find_supports_impl(ctx, xyz, nullptr, nullptr, n, p, out, nullptr, false, stride_bytes);
}

int pitt_find_supports_dev(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                           const pitt_support_params* p, pitt_support_list_dev* out) {
    if (!ctx) return PITT_E_INVALID;
    if (!p || !out || n < 0 || (n > 0 && (!x || !y || !z))) return ctx->fail(PITT_E_INVALID, "null argument");
    if (n > 0x7fffffff) return ctx->fail(PITT_E_INVALID, "cloud larger than 2^31 points");
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    return pitt::find_supports_impl(ctx, x, y, z, n, p, nullptr, out, true, 0);
}

}  // extern "C"
