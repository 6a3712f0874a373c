// k_score's memory skeleton in isolation (gfx950): 256 frames x 150 tiles of 2048 points in three
// SoA float planes (943.7 MB), each tile read in 8 sub-steps of 256 points (4 groups of 64, lane l
// holding point 64 g + l of group g, as k_score's box and list code needs it), with W fake VALU ops
// per sub-step standing in for the box / cull / pair work.  Occupancy is held at k_score's 5 waves
// per SIMD (20 per CU) by LDS.  Variants:
//   MODE 0: global_load_dword into registers, DEPTH register sets (DEPTH - 1 sub-steps in flight)
//   MODE 1: global_load_lds_dwordx4 ring of DEPTH slots (LDS-DMA, 3 KB per slot), ds_read_b32 to registers
// PERSIST 0: one wave per tile (k_score's first-chunk grid); 1: a resident grid, each wave striding over
// tiles with the ring running on across its tiles (no per-tile start-up latency).
//   hipcc --offload-arch=gfx950 -O3 tile_stream.hip -o build/tile_stream && ./build/tile_stream
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

constexpr int kTile = 2048, kSub = 256, kSubs = kTile / kSub;
constexpr int64_t kFrames = 256, kPts = 307200, kTilesPer = kPts / kTile;  // 150 tiles per frame
constexpr int64_t kN = kFrames * kPts;
constexpr int kItems = (int)(kFrames * kTilesPer);
constexpr int kLdsPerBlock = 16 * 1024;  // 10 two-wave blocks per CU = 20 waves = 5 per SIMD

typedef __attribute__((address_space(3))) void* lds_ptr;

template <int W>
__device__ __forceinline__ float work(float a, const float (&p)[12]) {
    float acc = a;
#pragma unroll
    for (int i = 0; i < 12; ++i) acc += p[i];
    if constexpr (W > 0) {
        float u = acc, v = acc + 1.0f;
#pragma unroll
        for (int i = 0; i < W / 2; ++i) asm volatile("v_fma_f32 %0, %0, %2, %1\n v_fma_f32 %1, %1, %2, %0" : "+v"(u), "+v"(v) : "v"(p[i % 12]));
        acc = u + v;
    }
    return acc;
}

// k_score's box pieces (the same instructions as plane_ransac.hip's coord_box / row_reduce)
__device__ __forceinline__ float vmin(float a, float b) { float r; asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
__device__ __forceinline__ float vmax(float a, float b) { float r; asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
__device__ __forceinline__ void swap32(float& a, float& b) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]); b = __uint_as_float(r[1]);
}
__device__ __forceinline__ void swap16(float& a, float& b) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]); b = __uint_as_float(r[1]);
}
__device__ __forceinline__ void coord_box(float& v0, float& v1, float& v2, float& v3, float& lo, float& hi) {
    swap32(v0, v2); float mn02 = vmin(v0, v2), mx02 = vmax(v0, v2); swap32(v0, v2);
    swap32(v1, v3); float mn13 = vmin(v1, v3), mx13 = vmax(v1, v3); swap32(v1, v3);
    swap16(mn02, mn13); lo = vmin(mn02, mn13);
    swap16(mx02, mx13); hi = vmax(mx02, mx13);
}
__device__ __forceinline__ float box_work(float (&p)[12], float& tb, int lane, uint32_t lds) {
    float lo[3], hi[3];
    coord_box(p[0], p[1], p[2], p[3], lo[0], hi[0]);
    coord_box(p[4], p[5], p[6], p[7], lo[1], hi[1]);
    coord_box(p[8], p[9], p[10], p[11], lo[2], hi[2]);
    asm("s_nop 4\n"
#define RR(K) "v_min_f32_dpp %0, %0, %0 row_ror:" #K " row_mask:0xf bank_mask:0xf\n" \
              "v_min_f32_dpp %1, %1, %1 row_ror:" #K " row_mask:0xf bank_mask:0xf\n" \
              "v_min_f32_dpp %2, %2, %2 row_ror:" #K " row_mask:0xf bank_mask:0xf\n" \
              "v_max_f32_dpp %3, %3, %3 row_ror:" #K " row_mask:0xf bank_mask:0xf\n" \
              "v_max_f32_dpp %4, %4, %4 row_ror:" #K " row_mask:0xf bank_mask:0xf\n" \
              "v_max_f32_dpp %5, %5, %5 row_ror:" #K " row_mask:0xf bank_mask:0xf\n"
        RR(8) RR(4) RR(2) RR(1)
#undef RR
        : "+v"(lo[0]), "+v"(lo[1]), "+v"(lo[2]), "+v"(hi[0]), "+v"(hi[1]), "+v"(hi[2]));
    const int i = lane & 15;
    float v = lo[0];
    v = i == 1 ? lo[1] : v; v = i == 2 ? lo[2] : v; v = i == 3 ? hi[0] : v; v = i == 4 ? hi[1] : v; v = i == 5 ? hi[2] : v;
    if (i < 6) *(__attribute__((address_space(3))) float*)(uintptr_t)(lds + 32u * (uint32_t)(lane >> 4) + 4u * (uint32_t)i) = v;
    tb = i < 3 ? vmin(tb, v) : vmax(tb, v);
    return lo[0] + hi[2];
}

// The same boxes through LDS: the sub-step's 12 registers written in their natural order, lane j < 48
// reducing 16 values of slice (coord, group) j / 4 with min3 / max3, a quad DPP combine, and the six
// values of each group exchanged through the item's box staging rows (the HBM group-box layout).
__device__ __forceinline__ float box_work_lds(float (&p)[12], int lane, uint32_t scratch, uint32_t stage) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    typedef float f2v __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int k = 0; k < 12; ++k)  // slice k = coord k / 4, group k % 4: float k * 64 + lane
        *(__attribute__((address_space(3))) float*)(uintptr_t)(scratch + 256u * k + 4u * lane) = p[k];
    const int j = lane < 48 ? lane : 47, sl = j >> 2, q = j & 3;
    const uint32_t a = scratch + 256u * sl + 64u * q;
    f4v v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = *(const __attribute__((address_space(3))) f4v*)(uintptr_t)(a + 16u * k);
    float lo = __builtin_fminf(__builtin_fminf(v[0].x, v[0].y), v[0].z), hi = __builtin_fmaxf(__builtin_fmaxf(v[0].x, v[0].y), v[0].z);
    asm("v_min3_f32 %0, %0, %2, %3\n v_max3_f32 %1, %1, %2, %3" : "+v"(lo), "+v"(hi) : "v"(v[0].w), "v"(v[1].x));
    asm("v_min3_f32 %0, %0, %2, %3\n v_max3_f32 %1, %1, %2, %3" : "+v"(lo), "+v"(hi) : "v"(v[1].y), "v"(v[1].z));
    asm("v_min3_f32 %0, %0, %2, %3\n v_max3_f32 %1, %1, %2, %3" : "+v"(lo), "+v"(hi) : "v"(v[1].w), "v"(v[2].x));
    asm("v_min3_f32 %0, %0, %2, %3\n v_max3_f32 %1, %1, %2, %3" : "+v"(lo), "+v"(hi) : "v"(v[2].y), "v"(v[2].z));
    asm("v_min3_f32 %0, %0, %2, %3\n v_max3_f32 %1, %1, %2, %3" : "+v"(lo), "+v"(hi) : "v"(v[2].w), "v"(v[3].x));
    asm("v_min3_f32 %0, %0, %2, %3\n v_max3_f32 %1, %1, %2, %3" : "+v"(lo), "+v"(hi) : "v"(v[3].y), "v"(v[3].z));
    asm("v_min_f32 %0, %0, %2\n v_max_f32 %1, %1, %2" : "+v"(lo), "+v"(hi) : "v"(v[3].w));
    asm("s_nop 1\n v_min_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
        "v_max_f32_dpp %1, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 1\n"
        "v_min_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"
        "v_max_f32_dpp %1, %1, %1 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf" : "+v"(lo), "+v"(hi));
    // slice sl = coord c * 4 + group g: lo to value c, hi to value 3 + c of group g's 8-float row
    const int c = sl >> 2, g = sl & 3;
    if (q == 0 && lane < 48) {
        *(__attribute__((address_space(3))) float*)(uintptr_t)(stage + 32u * g + 4u * c) = lo;
        *(__attribute__((address_space(3))) float*)(uintptr_t)(stage + 32u * g + 12u + 4u * c) = hi;
    }
    // row g gets its group's six values (broadcast reads)
    const uint32_t r = stage + 32u * (uint32_t)(lane >> 4);
    const f4v b0 = *(const __attribute__((address_space(3))) f4v*)(uintptr_t)r;
    const f2v b1 = *(const __attribute__((address_space(3))) f2v*)(uintptr_t)(r + 16u);
    return b0.x + b0.y + b0.z + b0.w + b1.x + b1.y;
}

struct Meta { int64_t off; int32_t n, tiles; };

// MODE 0, register ring.  BOX: k_score's box work per sub-step (and the boxes stored once per tile);
// META: the tile's frame from a list and a metadata array by dependent scalar loads (as resolve_item)
// STORE (BOX 1): 0 group boxes + tile box at the tile's end; 1 the same, then s_waitcnt vmcnt(0);
// 2 only the tile box; 3 nontemporal stores; 4 half the group boxes after sub-step 3, the rest at the end
template <int DEPTH, int W, int PERSIST, int BOX = 0, bool META = false, int STORE = 0>
__global__ __launch_bounds__(128) void k_regs(const float* X, const float* Y, const float* Z, float* out,
                                              const int32_t* list, const Meta* meta, float* gbox) {
    __shared__ float pad[kLdsPerBlock / 4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) pad[w] = 0.0f;
    const int gw = blockIdx.x * 2 + w, nw = gridDim.x * 2;
    float acc = 0.0f;
    for (int it = gw; it < kItems; it += (PERSIST ? nw : kItems)) {
        int64_t base;
        if constexpr (META) {
            const int li = it / (int)kTilesPer, t = it - li * (int)kTilesPer;
            const int f = __builtin_amdgcn_readfirstlane(list[li]);
            const Meta m = meta[f];
            base = m.off + (t < m.tiles ? (int64_t)t * kTile : 0);
        } else {
            base = (int64_t)(it / kTilesPer) * kPts + (int64_t)(it % kTilesPer) * kTile;
        }
        float tb = 0.0f;
        const uint32_t lds = (uint32_t)(uintptr_t)(pad + 1024 * w);  // [0, 1 KB): the item's boxes; then 3 KB scratch
        float P[DEPTH][12];
        auto load = [&](int s, float (&q)[12]) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int64_t i = base + s * kSub + g * 64 + lane;
                q[g] = X[i];
                q[4 + g] = Y[i];
                q[8 + g] = Z[i];
            }
        };
#pragma unroll
        for (int k = 0; k < DEPTH - 1; ++k) load(k, P[k]);
#pragma unroll
        for (int s = 0; s < kSubs; ++s) {
            load(s + DEPTH - 1 < kSubs ? s + DEPTH - 1 : kSubs - 1, P[(s + DEPTH - 1) % DEPTH]);
            if constexpr (BOX == 1) acc += box_work(P[s % DEPTH], tb, lane, lds + 128u * s);
            if constexpr (BOX == 1 && STORE == 4)
                if (s == 3 && lane < 32)
                    reinterpret_cast<float4*>(gbox)[(int64_t)it * 64 + lane] = reinterpret_cast<const float4*>(pad + 1024 * w)[lane];
            if constexpr (BOX == 2 || BOX == 4) acc += box_work_lds(P[s % DEPTH], lane, lds + 1024u + 3072u * 0, lds + 128u * s);
            if constexpr (BOX == 3) acc += box_work(P[s % DEPTH], tb, lane, lds + 128u * s);
            acc = work<W>(acc, P[s % DEPTH]);
        }
        if constexpr (BOX == 3 || BOX == 4) {  // the boxes computed, not stored
            const float4 q = reinterpret_cast<const float4*>(pad + 1024 * w)[lane];
            acc += q.x + q.y + q.z + q.w + tb;
        }
        if constexpr (BOX == 1 || BOX == 2) {
            const float4 q = reinterpret_cast<const float4*>(pad + 1024 * w)[lane];
            float4* dst = reinterpret_cast<float4*>(gbox) + (int64_t)it * 64 + lane;
            if constexpr (STORE == 0 || STORE == 1) *dst = q;
            if constexpr (STORE == 3) {
                typedef float f4v __attribute__((ext_vector_type(4)));
                __builtin_nontemporal_store(f4v{q.x, q.y, q.z, q.w}, reinterpret_cast<f4v*>(dst));
            }
            if constexpr (STORE == 4) if (lane >= 32) *dst = q;
            if constexpr (STORE == 5) if (lane < 32) *dst = q;   // 512 B per tile
            if constexpr (STORE == 6) if (lane < 16) *dst = q;   // 256 B per tile
            if constexpr (STORE == 7) if (lane < 24) {           // 384 B per tile, packed (f16-sized boxes)
                reinterpret_cast<float4*>(gbox)[(int64_t)it * 24 + lane] = q;
            }
            if (lane < 6) {
                if constexpr (STORE == 3) __builtin_nontemporal_store(tb, gbox + (int64_t)kItems * 256 + it * 8 + lane);
                else gbox[(int64_t)kItems * 256 + it * 8 + lane] = tb;
            }
            if constexpr (STORE == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    if (acc == 1.2345f) out[threadIdx.x] = acc + pad[0];
}

// MODE 1, LDS-DMA ring of DEPTH slots per wave (3 x 1 KB each), counted vmcnt waits
template <int DEPTH, int W, int PERSIST>
__global__ __launch_bounds__(128) void k_glds(const float* X, const float* Y, const float* Z, float* out,
                                              const int32_t*, const Meta*, float*) {
    // the ring, or k_score's 16 KB per block when that is more (occupancy: 5 waves per SIMD at most)
    constexpr int kRing = 2 * DEPTH * 3 * kSub * 4;
    __shared__ __attribute__((aligned(16))) float raw[(kRing > kLdsPerBlock ? kRing : kLdsPerBlock) / 4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float* ring = raw + w * DEPTH * 3 * kSub;
    const int gw = blockIdx.x * 2 + w, nw = gridDim.x * 2;
    const int n_it = PERSIST ? (kItems - gw + nw - 1) / nw : (gw < kItems ? 1 : 0);
    const int total = n_it * kSubs;  // sub-steps this wave streams
    auto src = [&](int q) -> int64_t {  // global point index of lane 0's float4 in sub-step q
        const int it = gw + (q / kSubs) * nw;
        return (int64_t)(it / kTilesPer) * kPts + (int64_t)(it % kTilesPer) * kTile + (q % kSubs) * kSub;
    };
    auto issue = [&](int q) {
        const int qq = q < total ? q : total - 1;
        float* b = ring + (q % DEPTH) * 3 * kSub;
        const int64_t o = src(qq) + lane * 4;
        __builtin_amdgcn_global_load_lds(X + o, (lds_ptr)(b), 16, 0, 0);
        __builtin_amdgcn_global_load_lds(Y + o, (lds_ptr)(b + kSub), 16, 0, 0);
        __builtin_amdgcn_global_load_lds(Z + o, (lds_ptr)(b + 2 * kSub), 16, 0, 0);
    };
    float acc = 0.0f;
    if (total > 0) {
#pragma unroll
        for (int k = 0; k < DEPTH - 1; ++k) issue(k);
        for (int q = 0; q < total; ++q) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot refilled below has been read
            issue(q + DEPTH - 1);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * (DEPTH - 1)) : "memory");
            __builtin_amdgcn_sched_barrier(0);
            const float* b = ring + (q % DEPTH) * 3 * kSub;
            float p[12];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                p[g] = b[g * 64 + lane];
                p[4 + g] = b[kSub + g * 64 + lane];
                p[8 + g] = b[2 * kSub + g * 64 + lane];
            }
            acc = work<W>(acc, p);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (acc == 1.2345f) out[threadIdx.x] = acc;
}

static const int32_t* g_list = nullptr;
static const Meta* g_meta = nullptr;
static float* g_box = nullptr;
template <typename K>
static float time_kernel(K kern, int blocks, const float* X, const float* Y, const float* Z, float* out) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(128), 0, 0, X, Y, Z, out, g_list, g_meta, g_box);  // warm-up
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        (void)hipEventRecord(a, 0);
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(128), 0, 0, X, Y, Z, out, g_list, g_meta, g_box);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0.0f;
        (void)hipEventElapsedTime(&ms, a, b);
        best = ms < best ? ms : best;
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return best * 1e3f;  // us
}

#define RUN(NAME, KERN, BLOCKS)                                                                          \
    do {                                                                                                 \
        const float us = time_kernel(KERN, BLOCKS, X, Y, Z, out);                                        \
        std::printf("%-34s %8.1f us  %6.2f TB/s  %.3f of 8 TB/s\n", NAME, us, bytes / us * 1e-6,          \
                    bytes / us * 1e-6 / 8.0);                                                            \
    } while (0)

int main() {
    float *X, *Y, *Z, *out;
    if (hipMalloc(&X, kN * 4) || hipMalloc(&Y, kN * 4) || hipMalloc(&Z, kN * 4) || hipMalloc(&out, 4096)) return 1;
    (void)hipMemset(X, 0, kN * 4);
    (void)hipMemset(Y, 0, kN * 4);
    (void)hipMemset(Z, 0, kN * 4);
    const double bytes = 12.0 * kN;
    {
        std::vector<int32_t> hl(kFrames);
        std::vector<Meta> hm(kFrames);
        for (int f = 0; f < kFrames; ++f) {
            hl[f] = (int)((f * 37) % kFrames);  // a permutation, as k_hypothesize's atomic order
            hm[f] = Meta{(int64_t)f * kPts, (int32_t)kPts, (int32_t)kTilesPer};
        }
        int32_t* dl; Meta* dm; float* db;
        if (hipMalloc(&dl, kFrames * 4) || hipMalloc(&dm, kFrames * sizeof(Meta)) || hipMalloc(&db, (size_t)kItems * 264 * 4)) return 1;
        (void)hipMemcpy(dl, hl.data(), kFrames * 4, hipMemcpyHostToDevice);
        (void)hipMemcpy(dm, hm.data(), kFrames * sizeof(Meta), hipMemcpyHostToDevice);
        g_list = dl; g_meta = dm; g_box = db;
    }
    const int per_item = (kItems + 1) / 2, resident = 256 * 10;
    RUN("regs d2 w0 per-tile", (k_regs<2, 0, 0>), per_item);
    RUN("BOX store 1 KB", (k_regs<2, 0, 0, 1, false, 0>), per_item);
    RUN("BOX store 512 B", (k_regs<2, 0, 0, 1, false, 5>), per_item);
    RUN("BOX store 384 B packed", (k_regs<2, 0, 0, 1, false, 7>), per_item);
    RUN("BOX store 256 B", (k_regs<2, 0, 0, 1, false, 6>), per_item);
    RUN("BOX tile box only", (k_regs<2, 0, 0, 1, false, 2>), per_item);
    RUN("BOX no store", (k_regs<2, 0, 0, 3, false>), per_item);
    RUN("regs d2 META", (k_regs<2, 0, 0, 0, true>), per_item);
    RUN("BOX no store META", (k_regs<2, 0, 0, 3, true>), per_item);
    RUN("BOX no store W=100", (k_regs<2, 100, 0, 3, false>), per_item);
    RUN("BOX no store W=200", (k_regs<2, 200, 0, 3, false>), per_item);
    RUN("BOX no store W=300", (k_regs<2, 300, 0, 3, false>), per_item);
    RUN("BOX store 1 KB W=300", (k_regs<2, 300, 0, 1, false, 0>), per_item);
    return 0;
}
