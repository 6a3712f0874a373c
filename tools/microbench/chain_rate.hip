// The k_refine chain loop in isolation (gfx950): cycles per element of one wave running nine
// dependent float chains over LDS blocks (double-buffered ds_read_b128 + 32-add asm chains, as
// refine_chain), with the other waves of its block idle, VALU-busy or LDS-polling.
//   hipcc --offload-arch=gfx950 -O3 chain_rate.hip -o build/chain_rate && ./build/chain_rate
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void chain16(float& s, const f4v& a, const f4v& b, const f4v& c, const f4v& d) {
    asm volatile(
        "v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %2\n v_add_f32 %0, %0, %3\n v_add_f32 %0, %0, %4\n"
        "v_add_f32 %0, %0, %5\n v_add_f32 %0, %0, %6\n v_add_f32 %0, %0, %7\n v_add_f32 %0, %0, %8\n"
        "v_add_f32 %0, %0, %9\n v_add_f32 %0, %0, %10\n v_add_f32 %0, %0, %11\n v_add_f32 %0, %0, %12\n"
        "v_add_f32 %0, %0, %13\n v_add_f32 %0, %0, %14\n v_add_f32 %0, %0, %15\n v_add_f32 %0, %0, %16"
        : "+v"(s)
        : "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w), "v"(c.x), "v"(c.y),
          "v"(c.z), "v"(c.w), "v"(d.x), "v"(d.y), "v"(d.z), "v"(d.w));
}
__device__ __forceinline__ void lds_read32(f4v (&v)[8], uint32_t a) {
    asm volatile(
        "ds_read_b128 %0, %8\n ds_read_b128 %1, %8 offset:16\n ds_read_b128 %2, %8 offset:32\n"
        "ds_read_b128 %3, %8 offset:48\n ds_read_b128 %4, %8 offset:64\n ds_read_b128 %5, %8 offset:80\n"
        "ds_read_b128 %6, %8 offset:96\n ds_read_b128 %7, %8 offset:112"
        : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7])
        : "v"(a)
        : "memory");
}
__device__ __forceinline__ void chain32(float& s, const f4v (&v)[8]) {
    chain16(s, v[0], v[1], v[2], v[3]);
    chain16(s, v[4], v[5], v[6], v[7]);
}

constexpr int kBlk = 256, kStride = kBlk + 4;

// MODE bits: 1 = chain on lanes 0..8 only; 2 = no LDS reads (registers only); 4 = others VALU-busy;
// 8 = others poll LDS with s_sleep(1); 16 = setprio(3) on the chain; 32 = others generate the
// producer's LDS traffic (global_load_lds 3 KB + 3 ds_read_b128 + 12 scattered ds_write_b32 per
// step); 64 = 16-element groups, 3 in flight (<= 12 LDS reads outstanding)
template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, long long* clk, int blocks, int nwaves, const float* gsrc) {
    __shared__ float buf[9 * kStride];
    __shared__ float pbuf[3 * 4 * 768 + 3 * 1028];
    __shared__ int flag;
    for (int i = threadIdx.x; i < 9 * kStride; i += blockDim.x) buf[i] = 1.0f + i * 1e-7f;
    if (threadIdx.x == 0) flag = 0;
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (wave == 0) {
        if (MODE & 16) __builtin_amdgcn_s_setprio(3);
        float s = 0.0f;
        const long long t0 = clock64();
        if (!(MODE & 1) || lane < 9) {
            const int k = lane < 9 ? lane : 0;
            const uint32_t pa = (uint32_t)(uintptr_t)(buf + k * kStride);
            f4v A[8], B[8];
            if (MODE & 2) {
                lds_read32(A, pa);
                lds_read32(B, pa + 128);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
            for (int b = 0; b < blocks; ++b) {
                if (MODE & 64) {
                    f4v X[4][4];
                    auto rd4 = [&](f4v (&v)[4], uint32_t a) {
                        asm volatile("ds_read_b128 %0, %4\n ds_read_b128 %1, %4 offset:16\n ds_read_b128 %2, %4 offset:32\n ds_read_b128 %3, %4 offset:48"
                                     : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]) : "v"(a) : "memory");
                    };
                    rd4(X[0], pa); rd4(X[1], pa + 64); rd4(X[2], pa + 128);
#pragma unroll
                    for (int g = 0; g < kBlk / 16; ++g) {
                        if (g + 2 < kBlk / 16) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
                        else if (g + 1 < kBlk / 16) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
                        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        chain16(s, X[g % 4][0], X[g % 4][1], X[g % 4][2], X[g % 4][3]);
                        if (g + 3 < kBlk / 16) rd4(X[(g + 3) % 4], pa + 64u * (g + 3));
                    }
                } else if (MODE & 2) {
#pragma unroll
                    for (int i = 0; i < kBlk / 32; i += 2) {
                        chain32(s, A);
                        chain32(s, B);
                    }
                } else {
                    lds_read32(A, pa);
#pragma unroll
                    for (int i = 0; i < kBlk / 32; i += 2) {
                        lds_read32(B, pa + 128u * (i + 1));
                        asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
                        chain32(s, A);
                        if (i + 2 < kBlk / 32) {
                            lds_read32(A, pa + 128u * (i + 2));
                            asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
                        } else {
                            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        }
                        chain32(s, B);
                    }
                }
            }
        }
        const long long t1 = clock64();
        if (lane == 0) {
            clk[blockIdx.x] = t1 - t0;
            *(volatile int*)&flag = 1;
        }
        if (s == 1.2345f) out[threadIdx.x] = s;
    } else if (wave < nwaves) {
        if (MODE & 4) {
            float v0 = lane, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3;
            while (!*(volatile int*)&flag) {
                for (int i = 0; i < 64; ++i)
                    asm volatile("v_mul_f32 %0, %0, %1\n v_mul_f32 %1, %1, %2\n v_mul_f32 %2, %2, %3\n v_mul_f32 %3, %3, %0"
                                 : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));
            }
            if (v0 + v1 + v2 + v3 == 1.2345f) out[threadIdx.x] = v0;
        } else if (MODE & 8) {
            while (!*(volatile int*)&flag) __builtin_amdgcn_s_sleep(1);
        } else if (MODE & 32) {
            typedef __attribute__((address_space(3))) void* lds_ptr;
            float* raw = pbuf + (wave - 1) * 4 * 768;
            float* ring = pbuf + 3 * 4 * 768;
            int st = 0, pos = 0;
            float acc = 0.0f;
            while (!*(volatile int*)&flag) {
                const float* g = gsrc + (int64_t)((st * 256) & ((1 << 22) - 1)) + lane * 4;
                float* b = raw + (st & 3) * 768;
                __builtin_amdgcn_global_load_lds(g, (lds_ptr)b, 16, 0, 0);
                __builtin_amdgcn_global_load_lds(g + (1 << 22), (lds_ptr)(b + 256), 16, 0, 0);
                __builtin_amdgcn_global_load_lds(g + (2 << 22), (lds_ptr)(b + 512), 16, 0, 0);
                asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
                const float* rb = raw + ((st + 1) & 3) * 768 + lane * 4;
                float x[4], y[4], z[4];
                asm volatile("ds_read_b128 %0, %3\n ds_read_b128 %1, %3 offset:1024\n ds_read_b128 %2, %3 offset:2048\n s_waitcnt lgkmcnt(0)"
                             : "=&v"(*(f4v*)x), "=&v"(*(f4v*)y), "=&v"(*(f4v*)z) : "v"((uint32_t)(uintptr_t)rb) : "memory");
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const bool in = ((lane + e + st) & 3) != 0;
                    const int r = in ? ((pos + lane * 3 + e) & 1023) : 1024;
                    ring[r] = x[e];
                    ring[1028 + r] = y[e];
                    ring[2056 + r] = z[e];
                    acc += x[e] * y[e] - z[e];
                }
                pos += 190;
                ++st;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (acc == 1.2345f) out[threadIdx.x] = acc;
        }
    }
}

int main() {
    float* out;
    long long* clk;
    (void)hipMalloc(&out, 4096 * 4);
    (void)hipMalloc(&clk, 4096 * 8);
    float* gsrc;
    (void)hipMalloc(&gsrc, (size_t)3 << 24);
    (void)hipMemset(gsrc, 0, (size_t)3 << 24);
    setvbuf(stdout, nullptr, _IOLBF, 0);
    const int blocks = 2000;
    struct V { int mode; int nw; const char* name; };
    const V vs[] = {{32, 2, "reads, 64 lanes, 1 producer-traffic wave"},
                    {32, 3, "reads, 64 lanes, 2 producer-traffic waves"},
                    {64, 1, "16-elem groups x3, alone"},
                    {64 | 32, 2, "16-elem groups x3, 1 producer wave"},
                    {64 | 32, 3, "16-elem groups x3, 2 producer waves"},{0, 1, "reads, 64 lanes, alone"},        {1, 1, "reads, 9 lanes, alone"},
                    {2, 1, "no reads (registers), alone"},   {4, 3, "reads, 64 lanes, 2 VALU-busy waves"},
                    {5, 3, "reads, 9 lanes, 2 VALU-busy"},   {4 | 16, 3, "reads, 64 lanes, 2 VALU-busy, prio"},
                    {8, 3, "reads, 64 lanes, 2 polling"},    {4, 4, "reads, 64 lanes, 3 VALU-busy"},
                    {4 | 16, 5, "reads, 64, 4 VALU-busy, prio"}, {2 | 4, 5, "no reads, 4 VALU-busy"},
                    {2 | 4 | 16, 5, "no reads, 4 VALU-busy, prio"}};
    long long h[256];
    for (const V& v : vs) {
        for (int grid : {1, 256}) {
            switch (v.mode) {
#define L(M) case M: hipLaunchKernelGGL(k<M>, dim3(grid), dim3(64 * v.nw), 0, 0, out, clk, blocks, v.nw, gsrc); break;
                L(0) L(1) L(2) L(4) L(5) L(20) L(8) L(6) L(22) L(32) L(64) L(96)
#undef L
            }
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(h, clk, grid * 8, hipMemcpyDeviceToHost);
            double mean = 0, mx = 0;
            for (int i = 0; i < grid; ++i) { mean += h[i]; mx = h[i] > mx ? h[i] : mx; }
            mean /= grid;
            printf("%-40s waves %d grid %3d: %.2f cycles/element (max %.2f)\n", v.name, v.nw, grid,
                   mean / (blocks * (double)kBlk), mx / (blocks * (double)kBlk));
        }
    }
    return 0;
}
