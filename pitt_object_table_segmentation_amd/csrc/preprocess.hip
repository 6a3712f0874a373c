// preprocess.hip -- the device steps in front of findSupports, so a frame
// never leaves HBM between the camera cloud and the support loop:
//
//   pitt_deep_filter      deepFiltering (src/segmentation_services/deep_filter_srv.cpp:27-44):
//                         drop points whose z is NaN, split the rest at z > threshold into the
//                         "further" and "closer" clouds, both in input order.
//   pitt_transform_cloud  pcl::transformPointCloud(cloud, out, Eigen::Matrix4f) as called at
//                         src/obj_segmentation.cpp:248 (PCL 1.7 common/impl/transforms.hpp).
//   pitt_unpack_pointcloud2  fromROSMsg of the XYZ fields as called by
//                         PCManager::cloudForRosMsg (src/point_cloud_library/pc_manager.cpp:94-104),
//                         on a device-resident PointCloud2 payload.
//
// Both are HBM-bound byte streams: 12 B read per point, 12 B written per kept / transformed point.
//
// Deep filter: k_deep_count stores each 16,384-point super-tile's closer and further totals;
// k_scan_pair turns both lists into output offsets; k_deep_write re-evaluates the split and
// writes both outputs in input order, one super-tile per block iteration.  The z compare is PCL's float
// compare against the float threshold.
//
// Transform: one elementwise launch; out.k = m(k,0) x + m(k,1) y + m(k,2) z + m(k,3) evaluated
// left to right in float without FMA (the reference's x86 build), so results equal PCL's bit for
// bit.  A non-dense cloud keeps its non-finite points unchanged (PCL copies the cloud first and
// skips them).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "compact.hpp"
#include "ctx.hpp"
#include "device_common.hpp"

#pragma clang fp contract(off)

namespace pitt {

// per point: 0 = dropped (NaN z), 1 = closer, 2 = further
__device__ __forceinline__ int deep_class(float z, float th) { return !(z == z) ? 0 : (z > th ? 2 : 1); }

// A block walks a "super-tile" of kDSuper 2048-point tiles (16,384 points: the offset scan then
// runs over ~4,800 entries for a 256-frame batch, not 38,400).  Inside a tile, wave w owns points
// [512 w, 512 w + 512) as 8 slices of 64 (lane l: point 64 j + l of slice j), so every load and
// every run of output stores is coalesced; ranks come from ballots (mbcnt inside a slice,
// popcounts across slices, LDS across the 4 waves).
constexpr int kDSlices = kCTile / kBlock;  // 8
constexpr int kDSuper = 8;                 // tiles per super-tile
constexpr int64_t kDSuperPts = (int64_t)kCTile * kDSuper;

__host__ __device__ inline int64_t dsupers(int64_t n) { return (n + kDSuperPts - 1) / kDSuperPts; }

__device__ __forceinline__ int lane_rank(uint64_t b) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
}

// One 512-thread block per super-tile: wave w counts tile w of it (8 chunks of 256 points, lane l:
// points 256 j + 4 l .. +3 with one dwordx4; the count needs no order), the block adds the eight
// wave totals.  z is 16-byte aligned in every full chunk when the plane is (the tail goes point by
// point).
__global__ __launch_bounds__(64 * kDSuper) void k_deep_count(const float* __restrict__ z, int64_t n, float th,
                                                             int32_t* __restrict__ cnt_closer,
                                                             int32_t* __restrict__ cnt_further) {
    __shared__ int32_t part[2][kDSuper];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t ns = dsupers(n);
    const bool al16 = ((uintptr_t)z & 15u) == 0;
    for (int64_t t = blockIdx.x; t < ns; t += gridDim.x) {
        int nc = 0, nf = 0;
        const int64_t b = t * kDSuperPts + (int64_t)w * kCTile + 4 * lane;
#pragma unroll
        for (int j = 0; j < kCTile / 256; ++j) {
            const int64_t i = b + 256 * j;
            float v[4];
            if (al16 && i + 4 <= n) {
                const float4 q = *(const float4*)(z + i);
                v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) v[k] = i + k < n ? z[i + k] : __builtin_nanf("");
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int c = deep_class(v[k], th);
                nc += c == 1 ? 1 : 0;  // per lane; summed across the wave once per tile
                nf += c == 2 ? 1 : 0;
            }
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            nc += __shfl_xor(nc, d, 64);
            nf += __shfl_xor(nf, d, 64);
        }
        if (lane == 0) {
            part[0][w] = nc;
            part[1][w] = nf;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int a = 0, f = 0;
#pragma unroll
            for (int k = 0; k < kDSuper; ++k) {
                a += part[0][k];
                f += part[1][k];
            }
            cnt_closer[t] = a;
            cnt_further[t] = f;
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(kBlock) void k_deep_write(const float* __restrict__ x, const float* __restrict__ y,
                                                       const float* __restrict__ z, int64_t n, float th,
                                                       const int32_t* __restrict__ off_closer,
                                                       const int32_t* __restrict__ off_further,
                                                       float* __restrict__ cx, float* __restrict__ cy,
                                                       float* __restrict__ cz, float* __restrict__ fx,
                                                       float* __restrict__ fy, float* __restrict__ fz) {
    __shared__ int32_t part[2][kBlock / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t ns = dsupers(n);
    for (int64_t t = blockIdx.x; t < ns; t += gridDim.x) {
        int base_c = off_closer[t], base_f = off_further[t];  // the tile's first output positions
        // the next tile's points load while this one is ranked and written (two register sets)
        float qx[kDSlices], qy[kDSlices], qz[kDSlices];
        auto load = [&](int u) __attribute__((always_inline)) {
            const int64_t b = t * kDSuperPts + (int64_t)u * kCTile + w * (kDSlices * 64) + lane;
#pragma unroll
            for (int j = 0; j < kDSlices; ++j) {
                const int64_t i = b + 64 * j;
                const bool in = i < n;
                qz[j] = in ? z[i] : __builtin_nanf("");
                qx[j] = in ? x[i] : 0.0f;
                qy[j] = in ? y[i] : 0.0f;
            }
        };
        load(0);
#pragma unroll
        for (int u = 0; u < kDSuper; ++u) {
            float px[kDSlices], py[kDSlices], pz[kDSlices];
#pragma unroll
            for (int j = 0; j < kDSlices; ++j) {
                px[j] = qx[j];
                py[j] = qy[j];
                pz[j] = qz[j];
            }
            if (u + 1 < kDSuper) load(u + 1);
            uint64_t bc[kDSlices], bf[kDSlices];
            int nc = 0, nf = 0;
#pragma unroll
            for (int j = 0; j < kDSlices; ++j) {
                const int c = deep_class(pz[j], th);
                bc[j] = __builtin_amdgcn_ballot_w64(c == 1);
                bf[j] = __builtin_amdgcn_ballot_w64(c == 2);
                nc += __builtin_popcountll(bc[j]);
                nf += __builtin_popcountll(bf[j]);
            }
            if (lane == 0) {
                part[0][w] = nc;
                part[1][w] = nf;
            }
            __syncthreads();
            int pc = base_c, pf = base_f;
#pragma unroll
            for (int k = 0; k < kBlock / 64; ++k) {
                pc += k < w ? part[0][k] : 0;
                pf += k < w ? part[1][k] : 0;
                base_c += part[0][k];
                base_f += part[1][k];
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < kDSlices; ++j) {
                if (cx && ((bc[j] >> lane) & 1)) {
                    const int o = pc + lane_rank(bc[j]);
                    cx[o] = px[j];
                    cy[o] = py[j];
                    cz[o] = pz[j];
                }
                if (fx && ((bf[j] >> lane) & 1)) {
                    const int o = pf + lane_rank(bf[j]);
                    fx[o] = px[j];
                    fy[o] = py[j];
                    fz[o] = pz[j];
                }
                pc += __builtin_popcountll(bc[j]);
                pf += __builtin_popcountll(bf[j]);
            }
        }
    }
}

// Exclusive scans of the two super-tile count lists in one 1024-thread block (oa[ns], ob[ns] =
// totals): thread t sums a contiguous run of ceil(ns / 1024) entries, the block scans the run
// totals, and each thread writes its run's offsets.
__global__ __launch_bounds__(1024) void k_scan_pair(const int32_t* __restrict__ a, const int32_t* __restrict__ b,
                                                    int64_t ns, int32_t* __restrict__ oa,
                                                    int32_t* __restrict__ ob) {
    __shared__ int32_t wa[16], wb[16];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t per = (ns + 1023) / 1024;
    const int64_t lo = min((int64_t)tid * per, ns), hi = min(lo + per, ns);
    int ta = 0, tb = 0;
    for (int64_t i = lo; i < hi; ++i) {
        ta += a[i];
        tb += b[i];
    }
    int ia = ta, ib = tb;  // inclusive wave scans
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int ua = __shfl_up(ia, d, 64), ub = __shfl_up(ib, d, 64);
        if (lane >= d) {
            ia += ua;
            ib += ub;
        }
    }
    if (lane == 63) {
        wa[w] = ia;
        wb[w] = ib;
    }
    __syncthreads();
    int pa = ia - ta, pb = ib - tb;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        pa += k < w ? wa[k] : 0;
        pb += k < w ? wb[k] : 0;
    }
    for (int64_t i = lo; i < hi; ++i) {
        oa[i] = pa;
        ob[i] = pb;
        pa += a[i];
        pb += b[i];
    }
    if (tid == 1023) {  // runs past ns are empty: the last thread ends on the totals
        oa[ns] = pa;
        ob[ns] = pb;
    }
}

struct Affine {
    float m[12];  // rows 0..2 of the row-major 4x4
};

__global__ __launch_bounds__(256) void k_transform(const float* __restrict__ x, const float* __restrict__ y,
                                                   const float* __restrict__ z, int64_t n, Affine a, int dense,
                                                   float* __restrict__ ox, float* __restrict__ oy,
                                                   float* __restrict__ oz) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float px = x[i], py = y[i], pz = z[i];
        if (!dense && !(__builtin_isfinite(px) && __builtin_isfinite(py) && __builtin_isfinite(pz))) {
            ox[i] = px;
            oy[i] = py;
            oz[i] = pz;
            continue;
        }
        ox[i] = ((a.m[0] * px + a.m[1] * py) + a.m[2] * pz) + a.m[3];
        oy[i] = ((a.m[4] * px + a.m[5] * py) + a.m[6] * pz) + a.m[7];
        oz[i] = ((a.m[8] * px + a.m[9] * py) + a.m[10] * pz) + a.m[11];
    }
}

// The same on four points per thread (dwordx4 loads and stores) when every plane is 16-byte
// aligned; points [4 * n4, n) go through k_transform.
__device__ __forceinline__ void transform_one(const Affine& a, int dense, float px, float py, float pz, float& ox,
                                              float& oy, float& oz) {
    if (!dense && !(__builtin_isfinite(px) && __builtin_isfinite(py) && __builtin_isfinite(pz))) {
        ox = px;
        oy = py;
        oz = pz;
        return;
    }
    ox = ((a.m[0] * px + a.m[1] * py) + a.m[2] * pz) + a.m[3];
    oy = ((a.m[4] * px + a.m[5] * py) + a.m[6] * pz) + a.m[7];
    oz = ((a.m[8] * px + a.m[9] * py) + a.m[10] * pz) + a.m[11];
}

__global__ __launch_bounds__(256) void k_transform4(const float4* __restrict__ x, const float4* __restrict__ y,
                                                    const float4* __restrict__ z, int64_t n4, Affine a, int dense,
                                                    float4* __restrict__ ox, float4* __restrict__ oy,
                                                    float4* __restrict__ oz) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 px = x[i], py = y[i], pz = z[i];
        float4 rx, ry, rz;
        transform_one(a, dense, px.x, py.x, pz.x, rx.x, ry.x, rz.x);
        transform_one(a, dense, px.y, py.y, pz.y, rx.y, ry.y, rz.y);
        transform_one(a, dense, px.z, py.z, pz.z, rx.z, ry.z, rz.z);
        transform_one(a, dense, px.w, py.w, pz.w, rx.w, ry.w, rz.w);
        ox[i] = rx;
        oy[i] = ry;
        oz[i] = rz;
    }
}

// fromROSMsg for the XYZ fields of a sensor_msgs/PointCloud2 payload: point (r, c) at byte
// r * row_step + c * point_step, x / y / z little-endian float32 at byte offsets ox / oy / oz.
// Point-major (one thread per point); with point_step 16 and x, y, z at 0, 4, 8 (PointXYZ), one
// dwordx4 per point.
__global__ __launch_bounds__(256) void k_unpack_pc2(const uint8_t* __restrict__ data, int32_t width, int64_t n,
                                                    int32_t point_step, int64_t row_step, int32_t ox, int32_t oy,
                                                    int32_t oz, int xyz16, float* __restrict__ x,
                                                    float* __restrict__ y, float* __restrict__ z) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / width, c = i - r * width;
        const uint8_t* p = data + r * row_step + c * point_step;
        if (xyz16) {
            const float4 v = *(const float4*)p;
            x[i] = v.x;
            y[i] = v.y;
            z[i] = v.z;
        } else {
            x[i] = *(const float*)(p + ox);
            y[i] = *(const float*)(p + oy);
            z[i] = *(const float*)(p + oz);
        }
    }
}

static inline int stream_grid(int64_t n) {
    return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192));
}

static int deep_filter_impl(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, float th,
                            float* cx, float* cy, float* cz, int64_t* n_closer, float* fx, float* fy, float* fz,
                            int64_t* n_further) {
    hipStream_t s = ctx->stream;
    const int64_t ns = dsupers(n);
    int32_t* cnt = (int32_t*)ctx->buf("deep_cnt", (size_t)std::max<int64_t>(ns, 1) * 2 * 4);
    int32_t* off = (int32_t*)ctx->buf("deep_off", (size_t)(ns + 1) * 2 * 4);
    if (!cnt || !off) return ctx->fail(PITT_E_NOMEM, "deep filter scratch");
    int32_t *cc = cnt, *cf = cnt + std::max<int64_t>(ns, 1);
    int32_t *oc = off, *of = off + ns + 1;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(ns, 16384));
    int rec = ctx->prof_begin("k_deep_count", (double)n * 4.0);
    if (n > 0) hipLaunchKernelGGL(k_deep_count, dim3(grid), dim3(64 * kDSuper), 0, s, z, n, th, cc, cf);
    ctx->prof_end(rec);
    rec = ctx->prof_begin("k_scan_pair", (double)ns * 16.0);
    hipLaunchKernelGGL(k_scan_pair, dim3(1), dim3(1024), 0, s, cc, cf, ns, oc, of);
    ctx->prof_end(rec);
    const int grid_w = grid_for_tiles(ns);
    // algorithmic bytes of the write pass: 12 B read per point here; the 12 B written per kept
    // point are added by the caller's accounting (the kept count is known only afterwards)
    rec = ctx->prof_begin("k_deep_write", (double)n * 12.0);
    if (n > 0 && (cx || fx))
        hipLaunchKernelGGL(k_deep_write, dim3(grid_w), dim3(kBlock), 0, s, x, y, z, n, th, oc, of, cx, cy, cz, fx,
                           fy, fz);
    ctx->prof_end(rec);
    PITT_HIP_TRY(hipGetLastError());
    int32_t* h = (int32_t*)ctx->pinned("deep_total", 16);
    PITT_HIP_TRY(hipMemcpyAsync(h, oc + ns, 4, hipMemcpyDeviceToHost, s));
    PITT_HIP_TRY(hipMemcpyAsync(h + 1, of + ns, 4, hipMemcpyDeviceToHost, s));
    PITT_HIP_TRY(hipStreamSynchronize(s));
    if (n_closer) *n_closer = h[0];
    if (n_further) *n_further = h[1];
    return PITT_OK;
}

}  // namespace pitt

extern "C" {

int pitt_deep_filter(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                     float deep_threshold, float* cx, float* cy, float* cz, int64_t* n_closer, float* fx, float* fy,
                     float* fz, int64_t* n_further, float* used_threshold) {
    if (!ctx) return PITT_E_INVALID;
    if (n < 0 || (n > 0 && (!x || !y || !z))) return ctx->fail(PITT_E_INVALID, "null argument");
    if (n > 0x7fffffff) return ctx->fail(PITT_E_INVALID, "cloud larger than 2^31 points");
    if ((cx && (!cy || !cz)) || (fx && (!fy || !fz))) return ctx->fail(PITT_E_INVALID, "partial output planes");
    // srv_manager.h:163-167: a request value >= 0 is used, anything else selects the default
    // (deep_filter_srv.cpp:19, 3.0 m)
    const float th = deep_threshold >= 0.0f ? deep_threshold : 3.0f;
    if (used_threshold) *used_threshold = th;
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    return pitt::deep_filter_impl(ctx, x, y, z, n, th, cx, cy, cz, n_closer, fx, fy, fz, n_further);
}

int pitt_unpack_pointcloud2(pitt_ctx* ctx, const void* data, int64_t data_bytes, int32_t width, int32_t height,
                            int32_t point_step, int64_t row_step, int32_t off_x, int32_t off_y, int32_t off_z,
                            float* x, float* y, float* z) {
    if (!ctx) return PITT_E_INVALID;
    const int64_t n = (int64_t)width * height;
    if (width < 0 || height < 0 || (n > 0 && (!data || !x || !y || !z))) return ctx->fail(PITT_E_INVALID, "null argument");
    const int32_t offs[3] = {off_x, off_y, off_z};
    for (int32_t o : offs)
        if (o < 0 || o % 4 != 0 || o + 4 > point_step) return ctx->fail(PITT_E_INVALID, "field offset");
    if (point_step % 4 != 0 || row_step % 4 != 0 || ((uintptr_t)data & 3u) != 0 ||
        (height > 1 && row_step < (int64_t)width * point_step))
        return ctx->fail(PITT_E_INVALID, "point_step / row_step / alignment");
    int64_t need = 0;
    if (n > 0) {  // the last point's last field must lie inside the payload
        const int32_t omax = std::max(off_x, std::max(off_y, off_z));
        need = (int64_t)(height - 1) * row_step + (int64_t)(width - 1) * point_step + omax + 4;
        if (data_bytes < need) return ctx->fail(PITT_E_INVALID, "PointCloud2 payload shorter than its layout");
    }
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    // The fast path reads a whole 16-byte point: only when the last point's 16 bytes are inside the
    // payload too (a payload may end right after the last z: 4 bytes short of a float4).
    const int xyz16 = point_step == 16 && off_x == 0 && off_y == 4 && off_z == 8 && row_step % 16 == 0 &&
                      ((uintptr_t)data & 15u) == 0 && data_bytes >= need + 4;
    hipStream_t s = ctx->stream;
    const int rec = ctx->prof_begin("k_unpack_pc2", (double)n * (12.0 + (xyz16 ? 16.0 : 12.0)));
    if (n > 0)
        hipLaunchKernelGGL(pitt::k_unpack_pc2, dim3(pitt::stream_grid(n)), dim3(256), 0, s, (const uint8_t*)data,
                           width, n, point_step, row_step, off_x, off_y, off_z, xyz16, x, y, z);
    ctx->prof_end(rec);
    PITT_HIP_TRY(hipGetLastError());
    PITT_HIP_TRY(hipStreamSynchronize(s));
    return PITT_OK;
}

int pitt_transform_cloud(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                         const float matrix[16], int32_t dense, float* ox, float* oy, float* oz) {
    if (!ctx) return PITT_E_INVALID;
    if (!matrix || n < 0 || (n > 0 && (!x || !y || !z || !ox || !oy || !oz)))
        return ctx->fail(PITT_E_INVALID, "null argument");
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    pitt::Affine a;
    for (int k = 0; k < 12; ++k) a.m[k] = matrix[k];
    hipStream_t s = ctx->stream;
    const int rec = ctx->prof_begin("k_transform", (double)n * 24.0);
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
    const int64_t n4 = al16(x) && al16(y) && al16(z) && al16(ox) && al16(oy) && al16(oz) ? n / 4 : 0;
    if (n4 > 0)
        hipLaunchKernelGGL(pitt::k_transform4, dim3(pitt::stream_grid(n4)), dim3(256), 0, s, (const float4*)x,
                           (const float4*)y, (const float4*)z, n4, a, dense ? 1 : 0, (float4*)ox, (float4*)oy,
                           (float4*)oz);
    if (n > 4 * n4)
        hipLaunchKernelGGL(pitt::k_transform, dim3(pitt::stream_grid(n - 4 * n4)), dim3(256), 0, s, x + 4 * n4,
                           y + 4 * n4, z + 4 * n4, n - 4 * n4, a, dense ? 1 : 0, ox + 4 * n4, oy + 4 * n4,
                           oz + 4 * n4);
    ctx->prof_end(rec);
    PITT_HIP_TRY(hipGetLastError());
    PITT_HIP_TRY(hipStreamSynchronize(s));
    return PITT_OK;
}

}  // extern "C"
