// Per-instruction VALU issue rates on gfx950 (wave64), measured with inline asm the compiler cannot
// restructure.  Each wave runs ITER x 32 copies of one instruction on 8 independent registers.
// Reports ns per wave-instruction per SIMD and, from s_memtime, the shader clock.
//   hipcc --offload-arch=gfx950 -O3 valu_asm.hip -o build/valu_asm && ./build/valu_asm
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define R8(X) X X X X X X X X
#define R32(X) R8(X) R8(X) R8(X) R8(X)

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, long long* clk, float s0, int iters) {
    (void)s0;
    float v0 = threadIdx.x, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6, v7 = v0 + 7;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if constexpr (MODE == 0)  // v_add_f32 VGPR,VGPR
            asm volatile(R32("v_add_f32 %0, %0, %1\n v_add_f32 %1, %1, %2\n v_add_f32 %2, %2, %3\n v_add_f32 %3, %3, %4\n"
                             "v_add_f32 %4, %4, %5\n v_add_f32 %5, %5, %6\n v_add_f32 %6, %6, %7\n v_add_f32 %7, %7, %0\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7));
        else if constexpr (MODE == 1)  // v_mul_f32 SGPR,VGPR (independent)
            asm volatile(R32("v_mul_f32 %0, %8, %0\n v_mul_f32 %1, %8, %1\n v_mul_f32 %2, %8, %2\n v_mul_f32 %3, %8, %3\n"
                             "v_mul_f32 %4, %8, %4\n v_mul_f32 %5, %8, %5\n v_mul_f32 %6, %8, %6\n v_mul_f32 %7, %8, %7\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7)
                         : "s"(s0));
        else if constexpr (MODE == 2)  // v_cmp_lt_f32_e64 -> distinct SGPR pairs
            asm volatile(R32("v_cmp_lt_f32_e64 s[40:41], |%0|, %8\n v_cmp_lt_f32_e64 s[42:43], |%1|, %8\n"
                             "v_cmp_lt_f32_e64 s[44:45], |%2|, %8\n v_cmp_lt_f32_e64 s[46:47], |%3|, %8\n"
                             "v_cmp_lt_f32_e64 s[48:49], |%4|, %8\n v_cmp_lt_f32_e64 s[50:51], |%5|, %8\n"
                             "v_cmp_lt_f32_e64 s[52:53], |%6|, %8\n v_cmp_lt_f32_e64 s[54:55], |%7|, %8\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7)
                         : "s"(s0)
                         : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52",
                           "s53", "s54", "s55");
        else if constexpr (MODE == 3)  // v_mul_f32 v,v
            asm volatile(R32("v_mul_f32 %0, %8, %0\n v_mul_f32 %1, %8, %1\n v_mul_f32 %2, %8, %2\n v_mul_f32 %3, %8, %3\n"
                             "v_mul_f32 %4, %8, %4\n v_mul_f32 %5, %8, %5\n v_mul_f32 %6, %8, %6\n v_mul_f32 %7, %8, %7\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7)
                         : "v"(s0));
        else if constexpr (MODE == 4)  // v_cmp_lt_f32_e64 s, |v|, v
            asm volatile(R32("v_cmp_lt_f32_e64 s[40:41], |%0|, %8\n v_cmp_lt_f32_e64 s[42:43], |%1|, %8\n"
                             "v_cmp_lt_f32_e64 s[44:45], |%2|, %8\n v_cmp_lt_f32_e64 s[46:47], |%3|, %8\n"
                             "v_cmp_lt_f32_e64 s[48:49], |%4|, %8\n v_cmp_lt_f32_e64 s[50:51], |%5|, %8\n"
                             "v_cmp_lt_f32_e64 s[52:53], |%6|, %8\n v_cmp_lt_f32_e64 s[54:55], |%7|, %8\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7)
                         : "v"(s0)
                         : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52",
                           "s53", "s54", "s55");
        else if constexpr (MODE == 6)  // v_mov_b32 v, s
            asm volatile(R32("v_mov_b32 %0, %8\n v_mov_b32 %1, %8\n v_mov_b32 %2, %8\n v_mov_b32 %3, %8\n"
                             "v_mov_b32 %4, %8\n v_mov_b32 %5, %8\n v_mov_b32 %6, %8\n v_mov_b32 %7, %8\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7)
                         : "s"(s0));
        else if constexpr (MODE == 7)  // v_cmp_gt_f32_e32 vcc, v, v + s_bcnt1 + s_add
            asm volatile(R32("v_cmp_gt_f32_e32 vcc, %8, %0\n s_bcnt1_i32_b64 s40, vcc\n v_cmp_gt_f32_e32 vcc, %8, %1\n s_bcnt1_i32_b64 s41, vcc\n"
                             "v_cmp_gt_f32_e32 vcc, %8, %2\n s_bcnt1_i32_b64 s42, vcc\n v_cmp_gt_f32_e32 vcc, %8, %3\n s_bcnt1_i32_b64 s43, vcc\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7)
                         : "v"(s0)
                         : "s40", "s41", "s42", "s43", "vcc", "scc");
        else if constexpr (MODE == 8)  // all-VGPR k_score mix: 3 mul + 3 add + cmp(e64 |v|, v) -> s + bcnt + add
            asm volatile(R8("v_mul_f32 %0, %8, %1\n v_mul_f32 %2, %8, %3\n v_mul_f32 %4, %8, %5\n v_add_f32 %6, %0, %2\n"
                            "v_add_f32 %7, %8, %4\n v_add_f32 %6, %6, %7\n v_cmp_lt_f32_e64 s[40:41], |%6|, %8\n"
                            "v_mul_f32 %1, %8, %0\n v_mul_f32 %3, %8, %2\n v_mul_f32 %5, %8, %4\n v_add_f32 %7, %1, %3\n"
                            "v_add_f32 %6, %8, %5\n v_add_f32 %7, %7, %6\n v_cmp_lt_f32_e64 s[42:43], |%7|, %8\n"
                            "s_bcnt1_i32_b64 s44, s[40:41]\n s_bcnt1_i32_b64 s45, s[42:43]\n s_add_u32 s46, s44, s45\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7)
                         : "v"(s0)
                         : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "scc");
        else if constexpr (MODE == 9)  // one fully dependent chain (latency)
            asm volatile(R32("v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %2\n v_add_f32 %0, %0, %3\n v_add_f32 %0, %0, %4\n"
                             "v_add_f32 %0, %0, %5\n v_add_f32 %0, %0, %6\n v_add_f32 %0, %0, %7\n v_add_f32 %0, %0, %1\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7));
        else if constexpr (MODE == 10)  // two interleaved dependent chains
            asm volatile(R32("v_add_f32 %0, %0, %2\n v_add_f32 %1, %1, %3\n v_add_f32 %0, %0, %4\n v_add_f32 %1, %1, %5\n"
                             "v_add_f32 %0, %0, %6\n v_add_f32 %1, %1, %7\n v_add_f32 %0, %0, %2\n v_add_f32 %1, %1, %3\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7));
        else if constexpr (MODE == 11)  // v_mul_f32_dpp row_newbcast (src0 broadcast), independent
            asm volatile(R32("v_mul_f32_dpp %0, %8, %0 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                             "v_mul_f32_dpp %1, %8, %1 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
                             "v_mul_f32_dpp %2, %8, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                             "v_mul_f32_dpp %3, %8, %3 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
                             "v_mul_f32_dpp %4, %8, %4 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
                             "v_mul_f32_dpp %5, %8, %5 row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
                             "v_mul_f32_dpp %6, %8, %6 row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
                             "v_mul_f32_dpp %7, %8, %7 row_newbcast:8 row_mask:0xf bank_mask:0xf\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7)
                         : "v"(s0));
        else if constexpr (MODE == 12)  // dpp k_score mix: 3 mul_dpp + add + add_dpp + add + cmp(e64, v)
            asm volatile(R8("v_mul_f32_dpp %0, %8, %1 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                            "v_mul_f32_dpp %2, %8, %3 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
                            "v_mul_f32_dpp %4, %8, %5 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                            "v_add_f32 %6, %0, %4\n"
                            "v_add_f32_dpp %7, %8, %2 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
                            "v_add_f32 %6, %6, %7\n v_cmp_lt_f32_e64 s[40:41], |%6|, %8\n"
                            "v_mul_f32_dpp %1, %8, %0 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
                            "v_mul_f32_dpp %3, %8, %2 row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
                            "v_mul_f32_dpp %5, %8, %4 row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
                            "v_add_f32 %7, %1, %5\n"
                            "v_add_f32_dpp %6, %8, %3 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
                            "v_add_f32 %7, %7, %6\n v_cmp_lt_f32_e64 s[42:43], |%7|, %8\n"
                            "s_bcnt1_i32_b64 s44, s[40:41]\n s_bcnt1_i32_b64 s45, s[42:43]\n s_add_u32 s46, s44, s45\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7)
                         : "v"(s0)
                         : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "scc");
        else if constexpr (MODE == 5)  // mixed: 3 mul(s,v) + 3 add + cmp, like k_score, 8-way independent
            asm volatile(R8("v_mul_f32 %0, %8, %1\n v_mul_f32 %2, %8, %3\n v_mul_f32 %4, %8, %5\n v_add_f32 %6, %0, %2\n"
                            "v_add_f32 %7, %8, %4\n v_add_f32 %6, %6, %7\n v_cmp_lt_f32_e64 s[40:41], |%6|, %8\n"
                            "v_mul_f32 %1, %8, %0\n v_mul_f32 %3, %8, %2\n v_mul_f32 %5, %8, %4\n v_add_f32 %7, %1, %3\n"
                            "v_add_f32 %6, %8, %5\n v_add_f32 %7, %7, %6\n v_cmp_lt_f32_e64 s[42:43], |%7|, %8\n"
                            "v_nop\n v_nop\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7)
                         : "s"(s0)
                         : "s40", "s41", "s42", "s43");
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) clk[MODE] = t1 - t0;
    if (v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7 == 1.2345f) out[threadIdx.x] = 1.0f;
}

int main() {
    float* out;
    long long* clk;
    (void)hipMalloc(&out, 4096);
    (void)hipMalloc(&clk, 64);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    setvbuf(stdout, nullptr, _IOLBF, 0);
    const int iters = 2000;
    const char* names[] = {"v_add_f32 v,v", "v_mul_f32 s,v", "v_cmp_lt_f32_e64 |v|,s", "v_mul_f32 v,v",
                           "v_cmp_lt_f32_e64 |v|,v", "k_score mix (16 incl 2 v_nop)", "v_mov_b32 v,s",
                           "v_cmp_gt_e32 vcc,v,v + s_bcnt (per cmp)", "all-VGPR mix (14 VALU + 3 SALU)",
                           "dependent v_add chain", "2 interleaved dependent chains", "v_mul_f32_dpp row_newbcast",
                           "dpp k_score mix (14 VALU + 3 SALU)"};
    for (int mode = 0; mode < 13; ++mode) {
        if (mode != 3 && mode != 8 && mode < 11) continue;
        for (int wpe : {1, 4, 8}) {
            const int blocks = 256 * wpe;
            float ms = 0;
            long long c = 0;
            for (int rep = 0; rep < 3; ++rep) {
                (void)hipEventRecord(e0);
                switch (mode) {
                    case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, clk, 0.999f, iters); break;
                    case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, clk, 0.999f, iters); break;
                    case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, clk, 0.999f, iters); break;
                    case 3: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, clk, 0.999f, iters); break;
                    case 4: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, out, clk, 0.999f, iters); break;
                    case 5: hipLaunchKernelGGL(k<5>, dim3(blocks), dim3(256), 0, 0, out, clk, 0.999f, iters); break;
                    case 6: hipLaunchKernelGGL(k<6>, dim3(blocks), dim3(256), 0, 0, out, clk, 0.999f, iters); break;
                    case 7: hipLaunchKernelGGL(k<7>, dim3(blocks), dim3(256), 0, 0, out, clk, 0.999f, iters); break;
                    case 8: hipLaunchKernelGGL(k<8>, dim3(blocks), dim3(256), 0, 0, out, clk, 0.999f, iters); break;
                    case 9: hipLaunchKernelGGL(k<9>, dim3(blocks), dim3(256), 0, 0, out, clk, 0.999f, iters); break;
                    case 10: hipLaunchKernelGGL(k<10>, dim3(blocks), dim3(256), 0, 0, out, clk, 0.999f, iters); break;
                    case 11: hipLaunchKernelGGL(k<11>, dim3(blocks), dim3(256), 0, 0, out, clk, 0.999f, iters); break;
                    case 12: hipLaunchKernelGGL(k<12>, dim3(blocks), dim3(256), 0, 0, out, clk, 0.999f, iters); break;
                }
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                (void)hipEventElapsedTime(&ms, e0, e1);
                (void)hipMemcpy(&c, clk + mode, 8, hipMemcpyDeviceToHost);
            }
            const double per_wave = (mode == 5) ? iters * 8.0 * 16 : (mode == 8 || mode == 12) ? iters * 8.0 * 14 : (mode == 7) ? iters * 32.0 * 4 : iters * 32.0 * 8;
            const double per_simd = per_wave * blocks * 4 / 1024.0;
            printf("%-30s waves/SIMD %d: %8.3f ms  %.3f ns/instr/SIMD  memtime %lld ticks/wave (%.1f ticks/instr/wave)\n",
                   names[mode], wpe, ms, ms * 1e6 / per_simd, c, c / per_wave);
        }
    }
    return 0;
}
