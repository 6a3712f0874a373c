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

// MODE 0, register ring
template <int DEPTH, int W, int PERSIST>
__global__ __launch_bounds__(128) void k_regs(const float* X, const float* Y, const float* Z, float* out) {
    __shared__ float pad[kLdsPerBlock / 4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) pad[w] = 0.0f;
    const int gw = blockIdx.x * 2 + w, nw = gridDim.x * 2;
    float acc = 0.0f;
    for (int it = gw; it < kItems; it += (PERSIST ? nw : kItems)) {
        const int64_t base = (int64_t)(it / kTilesPer) * kPts + (int64_t)(it % kTilesPer) * kTile;
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
            acc = work<W>(acc, P[s % DEPTH]);
        }
    }
    if (acc == 1.2345f) out[threadIdx.x] = acc + pad[0];
}

// MODE 1, LDS-DMA ring of DEPTH slots per wave (3 x 1 KB each), counted vmcnt waits
template <int DEPTH, int W, int PERSIST>
__global__ __launch_bounds__(128) void k_glds(const float* X, const float* Y, const float* Z, float* out) {
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

template <typename K>
static float time_kernel(K kern, int blocks, const float* X, const float* Y, const float* Z, float* out) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(128), 0, 0, X, Y, Z, out);  // warm-up
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        (void)hipEventRecord(a, 0);
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(128), 0, 0, X, Y, Z, out);
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
    const int per_item = (kItems + 1) / 2, resident = 256 * 10;
    RUN("regs d2 w0 per-tile", (k_regs<2, 0, 0>), per_item);
    RUN("regs d3 w0 per-tile", (k_regs<3, 0, 0>), per_item);
    RUN("regs d4 w0 per-tile", (k_regs<4, 0, 0>), per_item);
    RUN("regs d2 w0 persistent", (k_regs<2, 0, 1>), resident);
    RUN("regs d3 w0 persistent", (k_regs<3, 0, 1>), resident);
    RUN("glds d2 w0 per-tile", (k_glds<2, 0, 0>), per_item);
    RUN("glds d4 w0 per-tile", (k_glds<4, 0, 0>), per_item);
    RUN("glds d2 w0 persistent", (k_glds<2, 0, 1>), resident);
    RUN("glds d3 w0 persistent", (k_glds<3, 0, 1>), resident);
    RUN("glds d4 w0 persistent", (k_glds<4, 0, 1>), resident);
    RUN("regs d2 w200 per-tile", (k_regs<2, 200, 0>), per_item);
    RUN("regs d3 w200 per-tile", (k_regs<3, 200, 0>), per_item);
    RUN("regs d2 w200 persistent", (k_regs<2, 200, 1>), resident);
    RUN("glds d3 w200 persistent", (k_glds<3, 200, 1>), resident);
    RUN("glds d4 w200 persistent", (k_glds<4, 200, 1>), resident);
    RUN("regs d2 w400 per-tile", (k_regs<2, 400, 0>), per_item);
    RUN("regs d2 w400 persistent", (k_regs<2, 400, 1>), resident);
    RUN("glds d4 w400 persistent", (k_glds<4, 400, 1>), resident);
    return 0;
}
