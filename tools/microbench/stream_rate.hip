// Streaming-rate microbenchmark for k_refine's producer loop: one wave per block, one block per
// "frame" (256 blocks), each streaming NPTS points of x, y, z (12 B per point) in 256-point steps.
//   mode 0: global_load_lds ring, DEPTH steps in flight, counted vmcnt waits (k_refine's scheme)
//   mode 1: mode 0 plus an s_waitcnt lgkmcnt(0) before every issue (as k_refine's loop top)
//   mode 2: global_load_dwordx4 into VGPRs, DEPTH steps in flight (register ring, unrolled)
// The per-step "work" is a sum of the 12 floats per lane (kept so loads cannot be dropped).
//   hipcc --offload-arch=gfx950 -O3 stream_rate.hip -o build/stream_rate && ./build/stream_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kStep = 256;
constexpr int kSlot = 3 * kStep;

template <int DEPTH, bool LGKM>
__global__ __launch_bounds__(64) void k_glds(const float* X, const float* Y, const float* Z, int64_t npts, float* out) {
    __shared__ __attribute__((aligned(16))) float raw[DEPTH * kSlot];
    typedef __attribute__((address_space(3))) void* lds_ptr;
    const int lane = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x * npts;
    const int nsteps = (int)(npts / kStep);
    auto issue = [&](int c) {
        const int cc = c < nsteps ? c : nsteps - 1;
        float* b = raw + (c % DEPTH) * kSlot;
        const int64_t o = base + (int64_t)cc * kStep + lane * 4;
        __builtin_amdgcn_global_load_lds(X + o, (lds_ptr)(b), 16, 0, 0);
        __builtin_amdgcn_global_load_lds(Y + o, (lds_ptr)(b + kStep), 16, 0, 0);
        __builtin_amdgcn_global_load_lds(Z + o, (lds_ptr)(b + 2 * kStep), 16, 0, 0);
    };
#pragma unroll
    for (int k = 0; k < DEPTH - 1; ++k) issue(k);
    float acc = 0.0f;
    for (int st = 0; st < nsteps; ++st) {
        if (LGKM) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        issue(st + DEPTH - 1);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * (DEPTH - 1)) : "memory");
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t b = (uint32_t)(uintptr_t)(raw + (st % DEPTH) * kSlot + lane * 4);
        float4 x4, y4, z4;
        asm volatile("ds_read_b128 %0, %3\n ds_read_b128 %1, %3 offset:1024\n ds_read_b128 %2, %3 offset:2048\n s_waitcnt lgkmcnt(0)"
                     : "=&v"(x4), "=&v"(y4), "=&v"(z4) : "v"(b) : "memory");
        acc += x4.x + x4.y + x4.z + x4.w + y4.x + y4.y + y4.z + y4.w + z4.x + z4.y + z4.z + z4.w;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (acc == 1.2345f) out[lane] = acc;
}

template <int DEPTH>
__global__ __launch_bounds__(64) void k_vgpr(const float* X, const float* Y, const float* Z, int64_t npts, float* out) {
    const int lane = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x * npts;
    const int nsteps = (int)(npts / kStep);
    float4 rx[DEPTH], ry[DEPTH], rz[DEPTH];
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < DEPTH - 1; ++k) {
        const int64_t o = base + (int64_t)k * kStep + lane * 4;
        rx[k] = *reinterpret_cast<const float4*>(X + o);
        ry[k] = *reinterpret_cast<const float4*>(Y + o);
        rz[k] = *reinterpret_cast<const float4*>(Z + o);
    }
    for (int st0 = 0; st0 < nsteps; st0 += DEPTH) {
#pragma unroll
        for (int k = 0; k < DEPTH; ++k) {
            const int st = st0 + k;
            const int c = st + DEPTH - 1;
            const int cc = c < nsteps ? c : nsteps - 1;
            const int64_t o = base + (int64_t)cc * kStep + lane * 4;
            const int slot = (k + DEPTH - 1) % DEPTH;
            rx[slot] = *reinterpret_cast<const float4*>(X + o);
            ry[slot] = *reinterpret_cast<const float4*>(Y + o);
            rz[slot] = *reinterpret_cast<const float4*>(Z + o);
            const float4 x4 = rx[k], y4 = ry[k], z4 = rz[k];
            acc += x4.x + x4.y + x4.z + x4.w + y4.x + y4.y + y4.z + y4.w + z4.x + z4.y + z4.z + z4.w;
        }
    }
    if (acc == 1.2345f) out[lane] = acc;
}

int main() {
    setvbuf(stdout, nullptr, _IOLBF, 0);
    const int nblk = 256;
    const int64_t npts = 307200;
    float *X, *Y, *Z, *out;
    const size_t bytes = (size_t)nblk * npts * 4;
    (void)hipMalloc(&X, bytes);
    (void)hipMalloc(&Y, bytes);
    (void)hipMalloc(&Z, bytes);
    (void)hipMalloc(&out, 4096);
    (void)hipMemset(X, 0, bytes);
    (void)hipMemset(Y, 0, bytes);
    (void)hipMemset(Z, 0, bytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto run = [&](const char* name, auto kern) {
        float ms = 0, best = 1e9f;
        for (int rep = 0; rep < 4; ++rep) {
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(nblk), dim3(64), 0, 0, X, Y, Z, npts, out);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
        }
        const double gb = 3.0 * bytes / 1e9;
        printf("%-28s %8.3f ms  %7.1f GB/s total  %6.2f GB/s per block  %.3f us/step\n", name, best, gb / (best * 1e-3),
               gb / nblk / (best * 1e-3), best * 1e3 / (npts / kStep));
    };
    run("glds D=6", k_glds<6, false>);
    run("glds D=10", k_glds<10, false>);
    run("glds D=16", k_glds<16, false>);
    run("glds D=10 + lgkmcnt(0)", k_glds<10, true>);
    run("vgpr D=4", k_vgpr<4>);
    run("vgpr D=8", k_vgpr<8>);
    return 0;
}
