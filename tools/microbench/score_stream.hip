// Read-rate ceiling of k_score's access pattern on gfx950: 256 frames x 307,200 points, SoA x/y/z
// planes, one item = (frame, 2048-point tile) = 8 sub-steps of 256 points per coordinate.  Variants
// differ only in how a wave brings the sub-steps in; the "work" per sub-step is a cheap sum so
// nothing is dropped.  Prints GB/s of algorithmic bytes (12 B per point) per variant.
//   hipcc --offload-arch=gfx950 -O3 score_stream.hip -o /tmp/score_stream && /tmp/score_stream
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

constexpr int kTile = 2048, kSub = 256, kSubs = kTile / kSub;

struct Pts { float v[12]; };

// A: k_score's scheme: dword loads, lane l <- point 64 g + l of each group, two sub-steps in registers.
template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_a(const float* X, const float* Y, const float* Z, int items, int tiles,
                                                  int64_t fstride, float* out) {
    const int lane = threadIdx.x & 63;
    const int it = blockIdx.x * WAVES + (threadIdx.x >> 6);
    if (it >= items) return;
    const int f = it / tiles, t = it % tiles;
    const int64_t base = f * fstride + (int64_t)t * kTile;
    Pts P[2];
    auto load = [&](int s, Pts& p) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int64_t i = base + s * kSub + g * 64 + lane;
            p.v[g] = X[i]; p.v[4 + g] = Y[i]; p.v[8 + g] = Z[i];
        }
    };
    float acc = 0.f;
    load(0, P[0]);
    for (int s = 0; s < kSubs; s += 2) {
        load(s + 1, P[1]);
#pragma unroll
        for (int k = 0; k < 12; ++k) acc += P[0].v[k];
        if (s + 2 < kSubs) load(s + 2, P[0]);
#pragma unroll
        for (int k = 0; k < 12; ++k) acc += P[1].v[k];
    }
    if (acc == 1.2345f) out[lane] = acc;
}

// B: dwordx4 loads (lane l <- points 4 l .. 4 l + 3 of the sub-step), two sub-steps in registers.
template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_b(const float4* X, const float4* Y, const float4* Z, int items, int tiles,
                                                  int64_t fstride4, float* out) {
    const int lane = threadIdx.x & 63;
    const int it = blockIdx.x * WAVES + (threadIdx.x >> 6);
    if (it >= items) return;
    const int f = it / tiles, t = it % tiles;
    const int64_t base = f * fstride4 + (int64_t)t * (kTile / 4);
    float acc = 0.f;
    float4 a[3], b[3];
    a[0] = X[base + lane]; a[1] = Y[base + lane]; a[2] = Z[base + lane];
    for (int s = 0; s < kSubs; s += 2) {
        const int64_t o1 = base + (s + 1) * (kSub / 4) + lane;
        b[0] = X[o1]; b[1] = Y[o1]; b[2] = Z[o1];
        for (int k = 0; k < 3; ++k) acc += a[k].x + a[k].y + a[k].z + a[k].w;
        if (s + 2 < kSubs) {
            const int64_t o2 = base + (s + 2) * (kSub / 4) + lane;
            a[0] = X[o2]; a[1] = Y[o2]; a[2] = Z[o2];
        }
        for (int k = 0; k < 3; ++k) acc += b[k].x + b[k].y + b[k].z + b[k].w;
    }
    if (acc == 1.2345f) out[lane] = acc;
}

// C: global_load_lds dwordx4 ring of DEPTH sub-steps per wave, read back as k_score's group layout
// (12 ds_read_b32 per sub-step).
template <int WAVES, int DEPTH>
__global__ __launch_bounds__(64 * WAVES) void k_c(const float* X, const float* Y, const float* Z, int items, int tiles,
                                                  int64_t fstride, float* out) {
    __shared__ __attribute__((aligned(16))) float ring[WAVES][DEPTH][3 * kSub];
    typedef __attribute__((address_space(3))) void* lds_ptr;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int it = blockIdx.x * WAVES + w;
    if (it >= items) return;
    const int f = it / tiles, t = it % tiles;
    const int64_t base = f * fstride + (int64_t)t * kTile;
    auto issue = [&](int s) {
        const int ss = s < kSubs ? s : kSubs - 1;
        float* b = ring[w][s % DEPTH];
        const int64_t o = base + ss * kSub + lane * 4;
        __builtin_amdgcn_global_load_lds(X + o, (lds_ptr)(b), 16, 0, 0);
        __builtin_amdgcn_global_load_lds(Y + o, (lds_ptr)(b + kSub), 16, 0, 0);
        __builtin_amdgcn_global_load_lds(Z + o, (lds_ptr)(b + 2 * kSub), 16, 0, 0);
    };
#pragma unroll
    for (int k = 0; k < DEPTH - 1; ++k) issue(k);
    float acc = 0.f;
    for (int s = 0; s < kSubs; ++s) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        issue(s + DEPTH - 1);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * (DEPTH - 1)) : "memory");
        __builtin_amdgcn_sched_barrier(0);
        const float* b = ring[w][s % DEPTH];
        float v[12];
        const uint32_t a = (uint32_t)(uintptr_t)(b + lane);
        asm volatile("ds_read_b32 %0, %12\n ds_read_b32 %1, %12 offset:256\n ds_read_b32 %2, %12 offset:512\n"
                     "ds_read_b32 %3, %12 offset:768\n ds_read_b32 %4, %12 offset:1024\n ds_read_b32 %5, %12 offset:1280\n"
                     "ds_read_b32 %6, %12 offset:1536\n ds_read_b32 %7, %12 offset:1792\n ds_read_b32 %8, %12 offset:2048\n"
                     "ds_read_b32 %9, %12 offset:2304\n ds_read_b32 %10, %12 offset:2560\n ds_read_b32 %11, %12 offset:2816\n"
                     "s_waitcnt lgkmcnt(0)"
                     : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]),
                       "=&v"(v[7]), "=&v"(v[8]), "=&v"(v[9]), "=&v"(v[10]), "=&v"(v[11])
                     : "v"(a) : "memory");
#pragma unroll
        for (int k = 0; k < 12; ++k) acc += v[k];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (acc == 1.2345f) out[lane] = acc;
}

// D: as A, but each wave runs ITEMS consecutive items with the next item's first sub-step loaded
// during the last one (no per-wave pipeline restart).
template <int WAVES, int ITEMS>
__global__ __launch_bounds__(64 * WAVES) void k_d(const float* X, const float* Y, const float* Z, int items, int tiles,
                                                  int64_t fstride, float* out) {
    const int lane = threadIdx.x & 63;
    const int it0 = (blockIdx.x * WAVES + (threadIdx.x >> 6)) * ITEMS;
    if (it0 >= items) return;
    const int nsub = min(ITEMS, items - it0) * kSubs;
    auto addr = [&](int q) {
        const int it = it0 + q / kSubs, s = q % kSubs;
        const int f = it / tiles, t = it % tiles;
        return f * fstride + (int64_t)t * kTile + s * kSub;
    };
    Pts P[2];
    auto load = [&](int q, Pts& p) {
        const int64_t b = addr(q < nsub ? q : nsub - 1);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int64_t i = b + g * 64 + lane;
            p.v[g] = X[i]; p.v[4 + g] = Y[i]; p.v[8 + g] = Z[i];
        }
    };
    float acc = 0.f;
    load(0, P[0]);
    for (int q = 0; q < nsub; q += 2) {
        load(q + 1, P[1]);
#pragma unroll
        for (int k = 0; k < 12; ++k) acc += P[0].v[k];
        load(q + 2, P[0]);
#pragma unroll
        for (int k = 0; k < 12; ++k) acc += P[1].v[k];
    }
    if (acc == 1.2345f) out[lane] = acc;
}

int main() {
    const int frames = 256, n = 307200, tiles = (n + kTile - 1) / kTile;
    const int64_t fstride = (int64_t)tiles * kTile;
    const int64_t total = frames * fstride;
    float *X, *Y, *Z, *out;
    hipMalloc(&X, total * 4); hipMalloc(&Y, total * 4); hipMalloc(&Z, total * 4); hipMalloc(&out, 4096);
    hipMemset(X, 0, total * 4); hipMemset(Y, 0, total * 4); hipMemset(Z, 0, total * 4);
    const int items = frames * tiles;
    const double bytes = (double)frames * n * 12.0;
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    auto run = [&](const char* name, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        hipEventRecord(a);
        const int reps = 20;
        for (int r = 0; r < reps; ++r) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0; hipEventElapsedTime(&ms, a, b);
        const double us = ms * 1e3 / reps;
        printf("%-34s %8.1f us  %7.1f GB/s\n", name, us, bytes / (us * 1e-6) / 1e9);
    };
#define RUN(NAME, K, W, ...) run(NAME, [&] { hipLaunchKernelGGL((K), dim3((items + (W) - 1) / (W)), dim3(64 * (W)), 0, 0, __VA_ARGS__); })
    RUN("A dword, 2-wave blocks", (k_a<2>), 2, X, Y, Z, items, tiles, fstride, out);
    RUN("A dword, 4-wave blocks", (k_a<4>), 4, X, Y, Z, items, tiles, fstride, out);
    RUN("B dwordx4, 2-wave blocks", (k_b<2>), 2, (const float4*)X, (const float4*)Y, (const float4*)Z, items, tiles, fstride / 4, out);
    RUN("B dwordx4, 4-wave blocks", (k_b<4>), 4, (const float4*)X, (const float4*)Y, (const float4*)Z, items, tiles, fstride / 4, out);
    RUN("C lds ring d2, 2-wave", (k_c<2, 2>), 2, X, Y, Z, items, tiles, fstride, out);
    RUN("C lds ring d3, 2-wave", (k_c<2, 3>), 2, X, Y, Z, items, tiles, fstride, out);
    RUN("C lds ring d4, 2-wave", (k_c<2, 4>), 2, X, Y, Z, items, tiles, fstride, out);
    RUN("C lds ring d4, 4-wave", (k_c<4, 4>), 4, X, Y, Z, items, tiles, fstride, out);
#define RUND(NAME, W, IT) run(NAME, [&] { hipLaunchKernelGGL((k_d<W, IT>), dim3((items + (W) * (IT) - 1) / ((W) * (IT))), dim3(64 * (W)), 0, 0, X, Y, Z, items, tiles, fstride, out); })
    RUND("D dword, 2 items/wave", 2, 2);
    RUND("D dword, 4 items/wave", 2, 4);
    RUND("D dword, 8 items/wave", 2, 8);
    return 0;
}
