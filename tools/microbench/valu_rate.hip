// VALU issue-rate microbenchmark for k_score's instruction mix (wave64, gfx950).
// Each wave runs ITER iterations of a block of independent v_mul/v_add/v_cmp chains; the kernel
// time gives cycles per wave-instruction per SIMD at the given waves/SIMD.
//   hipcc --offload-arch=gfx950 -O3 valu_rate.hip -o valu_rate && ./valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, float a, float b, float c, float w, float t, int iters) {
    float x[8], y[8], z[8];
    for (int p = 0; p < 8; ++p) { x[p] = threadIdx.x * 0.001f + p; y[p] = x[p] * 0.5f; z[p] = x[p] * 0.25f; }
    int cnt = 0;
    float acc = 0.0f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            if constexpr (MODE == 0) {  // 3 mul + 3 add + cmp(abs) -> SGPR mask -> s_bcnt
                float d = (a * x[p] + c * z[p]) + (b * y[p] + w);
                cnt += __builtin_popcountll(__builtin_amdgcn_ballot_w64(fabsf(d) < t));
            } else if constexpr (MODE == 1) {  // 6 arithmetic ops only, accumulated
                float d = (a * x[p] + c * z[p]) + (b * y[p] + w);
                acc += d;
            } else if constexpr (MODE == 2) {  // plain independent v_add chains (8 per point)
                x[p] = x[p] + a; y[p] = y[p] + b; z[p] = z[p] + c;
            }
        }
        a = __builtin_amdgcn_readfirstlane(__float_as_int(a)) == 7 ? w : a;  // keep loop-variant
    }
    if (cnt == 12345 || acc == 1.2345f) out[threadIdx.x] = acc + cnt;
    if (MODE == 2 && x[0] + y[1] + z[2] == 1.2345f) out[0] = 1.0f;
}

int main() {
    float* out;
    hipMalloc(&out, 4096);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 4000;
    for (int mode = 0; mode < 3; ++mode) {
        for (int wpe : {1, 2, 4, 6, 8}) {
            const int blocks = 256 * wpe;  // 4 waves per block -> wpe waves per SIMD
            float ms = 0;
            for (int rep = 0; rep < 3; ++rep) {
                hipEventRecord(e0);
                if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, 0.5f, 0.25f, 0.125f, 0.1f, 0.007f, iters);
                if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, 0.5f, 0.25f, 0.125f, 0.1f, 0.007f, iters);
                if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, 0.5f, 0.25f, 0.125f, 0.1f, 0.007f, iters);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                hipEventElapsedTime(&ms, e0, e1);
            }
            const double per_mode = mode == 0 ? 7.0 : mode == 1 ? 7.0 : 3.0;  // VALU per point
            const double wave_instr = (double)blocks * 4 * iters * 8 * per_mode;
            const double per_simd = wave_instr / 1024.0;
            printf("mode %d waves/SIMD %d: %.3f ms  -> %.2f ns per VALU wave-instr per SIMD (%.2f cyc @2.4GHz)\n", mode, wpe,
                   ms, ms * 1e6 / per_simd, ms * 1e6 / per_simd * 2.4);
        }
    }
    return 0;
}
