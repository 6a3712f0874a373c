// Issue cost of candidate k_score instructions on gfx950 (wave64): each wave runs ITER x 8 copies of
// a block on independent registers; reports ns per block per SIMD at 4 and 8 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 op_rates.hip -o op_rates && ./op_rates
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(X) X X X X X X X X

#define OUTS "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7)

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, float s0, int iters) {
    float v0 = threadIdx.x * 1e-3f, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6,
          v7 = v0 + 7;
    int c0 = 0, c1 = 0;
    for (int it = 0; it < iters; ++it) {
        if constexpr (MODE == 0)  // 8 x v_fma_f32 (independent)
            asm volatile(R8("v_fma_f32 %0, %1, %8, %0\n v_fma_f32 %1, %2, %8, %1\n v_fma_f32 %2, %3, %8, %2\n"
                            "v_fma_f32 %3, %4, %8, %3\n v_fma_f32 %4, %5, %8, %4\n v_fma_f32 %5, %6, %8, %5\n"
                            "v_fma_f32 %6, %7, %8, %6\n v_fma_f32 %7, %0, %8, %7\n")
                         : OUTS : "v"(s0));
        else if constexpr (MODE == 1)  // 8 x v_cmp_lt_f32_e32 vcc (independent sources)
            asm volatile(R8("v_cmp_lt_f32_e32 vcc, %0, %8\n v_cmp_lt_f32_e32 vcc, %1, %8\n v_cmp_lt_f32_e32 vcc, %2, %8\n"
                            "v_cmp_lt_f32_e32 vcc, %3, %8\n v_cmp_lt_f32_e32 vcc, %4, %8\n v_cmp_lt_f32_e32 vcc, %5, %8\n"
                            "v_cmp_lt_f32_e32 vcc, %6, %8\n v_cmp_lt_f32_e32 vcc, %7, %8\n")
                         : OUTS : "v"(s0) : "vcc");
        else if constexpr (MODE == 2)  // 8 x v_writelane_b32 (SGPR value, immediate lane)
            asm volatile(R8("v_writelane_b32 %0, %8, 1\n v_writelane_b32 %1, %8, 2\n v_writelane_b32 %2, %8, 3\n"
                            "v_writelane_b32 %3, %8, 4\n v_writelane_b32 %4, %8, 5\n v_writelane_b32 %5, %8, 6\n"
                            "v_writelane_b32 %6, %8, 7\n v_writelane_b32 %7, %8, 8\n")
                         : OUTS : "s"(s0));
        else if constexpr (MODE == 3)  // 8 x v_sub_f32_e64 |v|, v (VOP3 abs modifier, VGPR only)
            asm volatile(R8("v_sub_f32_e64 %0, |%1|, %8\n v_sub_f32_e64 %1, |%2|, %8\n v_sub_f32_e64 %2, |%3|, %8\n"
                            "v_sub_f32_e64 %3, |%4|, %8\n v_sub_f32_e64 %4, |%5|, %8\n v_sub_f32_e64 %5, |%6|, %8\n"
                            "v_sub_f32_e64 %6, |%7|, %8\n v_sub_f32_e64 %7, |%0|, %8\n")
                         : OUTS : "v"(s0));
        else if constexpr (MODE == 4)  // 8 x v_pk_fma_f32 (two lanes' worth each)
            asm volatile(R8("v_pk_fma_f32 v[40:41], v[42:43], v[44:45], v[40:41]\n"
                            "v_pk_fma_f32 v[46:47], v[42:43], v[44:45], v[46:47]\n"
                            "v_pk_fma_f32 v[48:49], v[42:43], v[44:45], v[48:49]\n"
                            "v_pk_fma_f32 v[50:51], v[42:43], v[44:45], v[50:51]\n"
                            "v_pk_fma_f32 v[52:53], v[42:43], v[44:45], v[52:53]\n"
                            "v_pk_fma_f32 v[54:55], v[42:43], v[44:45], v[54:55]\n"
                            "v_pk_fma_f32 v[56:57], v[42:43], v[44:45], v[56:57]\n"
                            "v_pk_fma_f32 v[58:59], v[42:43], v[44:45], v[58:59]\n")
                         : OUTS : "v"(s0) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49",
                           "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59");
        else if constexpr (MODE == 5)  // 8 x v_addc_co_u32 (VCC carry-in)
            asm volatile(R8("v_addc_co_u32 %0, vcc, 0, %0, vcc\n v_addc_co_u32 %1, vcc, 0, %1, vcc\n"
                            "v_addc_co_u32 %2, vcc, 0, %2, vcc\n v_addc_co_u32 %3, vcc, 0, %3, vcc\n"
                            "v_addc_co_u32 %4, vcc, 0, %4, vcc\n v_addc_co_u32 %5, vcc, 0, %5, vcc\n"
                            "v_addc_co_u32 %6, vcc, 0, %6, vcc\n v_addc_co_u32 %7, vcc, 0, %7, vcc\n")
                         : OUTS : "v"(s0) : "vcc");
        else if constexpr (MODE == 6)  // current entry: 3 mul + 3 add + cmp_e64 -> s + bcnt + writelane, x2 chains
            asm volatile(R8("v_mul_f32 %0, %8, %4\n v_mul_f32 %1, %8, %5\n v_mul_f32 %2, %8, %6\n v_mul_f32 %3, %8, %7\n"
                            "v_add_f32 %0, %0, %2\n v_add_f32 %1, %1, %3\n v_mul_f32 %2, %8, %6\n v_mul_f32 %3, %8, %7\n"
                            "v_add_f32 %2, %2, %8\n v_add_f32 %3, %3, %8\n v_add_f32 %0, %0, %2\n v_add_f32 %1, %1, %3\n"
                            "v_cmp_lt_f32_e64 s[40:41], |%0|, %8\n v_cmp_lt_f32_e64 s[42:43], |%1|, %8\n"
                            "s_bcnt1_i32_b64 s44, s[40:41]\n s_bcnt1_i32_b64 s45, s[42:43]\n"
                            "v_writelane_b32 %9, s44, 3\n v_writelane_b32 %10, s45, 4\n")
                         : OUTS, "+v"(c0), "+v"(c1) : "v"(s0) : "s40", "s41", "s42", "s43", "s44", "s45", "scc");
        else if constexpr (MODE == 7)  // fma entry: 3 fma + cmp_e64 + sub|.| + min|.| + bcnt + writelane, x2
            asm volatile(R8("v_fma_f32 %0, %8, %4, %8\n v_fma_f32 %1, %8, %5, %8\n v_fma_f32 %0, %8, %6, %0\n"
                            "v_fma_f32 %1, %8, %7, %1\n v_fma_f32 %0, %8, %7, %0\n v_fma_f32 %1, %8, %6, %1\n"
                            "v_cmp_lt_f32_e64 s[40:41], |%0|, %8\n v_cmp_lt_f32_e64 s[42:43], |%1|, %8\n"
                            "v_sub_f32_e64 %2, |%0|, %8\n v_sub_f32_e64 %3, |%1|, %8\n"
                            "v_min_f32_e64 %2, |%2|, %3\n v_min3_f32 %4, %4, %2, %3\n"
                            "s_bcnt1_i32_b64 s44, s[40:41]\n s_bcnt1_i32_b64 s45, s[42:43]\n"
                            "v_writelane_b32 %9, s44, 3\n v_writelane_b32 %10, s45, 4\n")
                         : OUTS, "+v"(c0), "+v"(c1) : "v"(s0) : "s40", "s41", "s42", "s43", "s44", "s45", "scc");
        else if constexpr (MODE == 8)  // fma entry, VCC compare on d^2: 3 fma + mul + cmp_e32 + bcnt + packed writelane
            asm volatile(R8("v_fma_f32 %0, %8, %4, %8\n v_fma_f32 %1, %8, %5, %8\n v_fma_f32 %0, %8, %6, %0\n"
                            "v_fma_f32 %1, %8, %7, %1\n v_fma_f32 %0, %8, %7, %0\n v_fma_f32 %1, %8, %6, %1\n"
                            "v_mul_f32 %2, %0, %0\n v_mul_f32 %3, %1, %1\n"
                            "v_cmp_gt_f32_e32 vcc, %8, %2\n s_bcnt1_i32_b64 s44, vcc\n"
                            "v_cmp_gt_f32_e32 vcc, %8, %3\n s_bcnt1_i32_b64 s45, vcc\n"
                            "s_pack_ll_b32_b16 s44, s44, s45\n v_writelane_b32 %9, s44, 3\n")
                         : OUTS, "+v"(c0), "+v"(c1) : "v"(s0) : "s44", "s45", "vcc", "scc");
        else if constexpr (MODE == 9)  // 8 x v_bcnt_u32_b32
            asm volatile(R8("v_bcnt_u32_b32 %0, %0, %8\n v_bcnt_u32_b32 %1, %1, %8\n v_bcnt_u32_b32 %2, %2, %8\n"
                            "v_bcnt_u32_b32 %3, %3, %8\n v_bcnt_u32_b32 %4, %4, %8\n v_bcnt_u32_b32 %5, %5, %8\n"
                            "v_bcnt_u32_b32 %6, %6, %8\n v_bcnt_u32_b32 %7, %7, %8\n")
                         : OUTS : "v"(s0));
        else if constexpr (MODE == 10)  // 8 x v_cmp_lt_f32_e64 -> distinct SGPR pairs, VGPR operands
            asm volatile(R8("v_cmp_lt_f32_e64 s[40:41], |%0|, %8\n v_cmp_lt_f32_e64 s[42:43], |%1|, %8\n"
                            "v_cmp_lt_f32_e64 s[44:45], |%2|, %8\n v_cmp_lt_f32_e64 s[46:47], |%3|, %8\n"
                            "v_cmp_lt_f32_e64 s[48:49], |%4|, %8\n v_cmp_lt_f32_e64 s[50:51], |%5|, %8\n"
                            "v_cmp_lt_f32_e64 s[52:53], |%6|, %8\n v_cmp_lt_f32_e64 s[54:55], |%7|, %8\n")
                         : OUTS : "v"(s0) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49",
                           "s50", "s51", "s52", "s53", "s54", "s55");
        else if constexpr (MODE == 11)  // 8 x v_mul_f32 v,v (reference)
            asm volatile(R8("v_mul_f32 %0, %8, %0\n v_mul_f32 %1, %8, %1\n v_mul_f32 %2, %8, %2\n v_mul_f32 %3, %8, %3\n"
                            "v_mul_f32 %4, %8, %4\n v_mul_f32 %5, %8, %5\n v_mul_f32 %6, %8, %6\n v_mul_f32 %7, %8, %7\n")
                         : OUTS : "v"(s0));
        else if constexpr (MODE == 12)  // 8 x v_pk_mul_f32
            asm volatile(R8("v_pk_mul_f32 v[40:41], v[42:43], v[40:41]\n v_pk_mul_f32 v[46:47], v[42:43], v[46:47]\n"
                            "v_pk_mul_f32 v[48:49], v[42:43], v[48:49]\n v_pk_mul_f32 v[50:51], v[42:43], v[50:51]\n"
                            "v_pk_mul_f32 v[52:53], v[42:43], v[52:53]\n v_pk_mul_f32 v[54:55], v[42:43], v[54:55]\n"
                            "v_pk_mul_f32 v[56:57], v[42:43], v[56:57]\n v_pk_mul_f32 v[58:59], v[42:43], v[58:59]\n")
                         : OUTS : "v"(s0) : "v40", "v41", "v42", "v43", "v46", "v47", "v48", "v49",
                           "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59");
        else if constexpr (MODE == 13)  // 8 x v_cndmask_b32 (VCC select)
            asm volatile(R8("v_cndmask_b32 %0, %0, %8, vcc\n v_cndmask_b32 %1, %1, %8, vcc\n v_cndmask_b32 %2, %2, %8, vcc\n"
                            "v_cndmask_b32 %3, %3, %8, vcc\n v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n"
                            "v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc\n")
                         : OUTS : "v"(s0) : "vcc");
        else if constexpr (MODE == 14)  // 8 x v_permlane32_swap (4 independent pairs, twice)
            asm volatile(R8("v_permlane32_swap_b32_e32 %0, %1\n v_permlane32_swap_b32_e32 %2, %3\n"
                            "v_permlane32_swap_b32_e32 %4, %5\n v_permlane32_swap_b32_e32 %6, %7\n"
                            "v_permlane32_swap_b32_e32 %0, %2\n v_permlane32_swap_b32_e32 %1, %3\n"
                            "v_permlane32_swap_b32_e32 %4, %6\n v_permlane32_swap_b32_e32 %5, %7\n")
                         : OUTS);
        else if constexpr (MODE == 15)  // 8 x v_permlane16_swap
            asm volatile(R8("v_permlane16_swap_b32_e32 %0, %1\n v_permlane16_swap_b32_e32 %2, %3\n"
                            "v_permlane16_swap_b32_e32 %4, %5\n v_permlane16_swap_b32_e32 %6, %7\n"
                            "v_permlane16_swap_b32_e32 %0, %2\n v_permlane16_swap_b32_e32 %1, %3\n"
                            "v_permlane16_swap_b32_e32 %4, %6\n v_permlane16_swap_b32_e32 %5, %7\n")
                         : OUTS);
        else if constexpr (MODE == 16)  // 8 x v_min_f32_dpp row_ror (independent registers)
            asm volatile(R8("v_min_f32_dpp %0, %0, %0 row_ror:8 row_mask:0xf bank_mask:0xf\n"
                            "v_min_f32_dpp %1, %1, %1 row_ror:8 row_mask:0xf bank_mask:0xf\n"
                            "v_min_f32_dpp %2, %2, %2 row_ror:8 row_mask:0xf bank_mask:0xf\n"
                            "v_min_f32_dpp %3, %3, %3 row_ror:8 row_mask:0xf bank_mask:0xf\n"
                            "v_min_f32_dpp %4, %4, %4 row_ror:8 row_mask:0xf bank_mask:0xf\n"
                            "v_min_f32_dpp %5, %5, %5 row_ror:8 row_mask:0xf bank_mask:0xf\n"
                            "v_min_f32_dpp %6, %6, %6 row_ror:8 row_mask:0xf bank_mask:0xf\n"
                            "v_min_f32_dpp %7, %7, %7 row_ror:8 row_mask:0xf bank_mask:0xf\n")
                         : OUTS);
        else if constexpr (MODE == 17)  // 8 x v_min_f32 v,v (VOP2, reference for 16)
            asm volatile(R8("v_min_f32 %0, %0, %1\n v_min_f32 %1, %1, %2\n v_min_f32 %2, %2, %3\n v_min_f32 %3, %3, %4\n"
                            "v_min_f32 %4, %4, %5\n v_min_f32 %5, %5, %6\n v_min_f32 %6, %6, %7\n v_min_f32 %7, %7, %0\n")
                         : OUTS);
        else if constexpr (MODE == 19)  // 8 x v_cndmask_b32_e64 with an SGPR-pair mask (set once per iteration)
            asm volatile("s_mov_b32 s40, 0xffff\n s_mov_b32 s41, 0xffff\n" R8("v_cndmask_b32_e64 %0, %0, %8, s[40:41]\n v_cndmask_b32_e64 %1, %1, %8, s[40:41]\n"
                            "v_cndmask_b32_e64 %2, %2, %8, s[40:41]\n v_cndmask_b32_e64 %3, %3, %8, s[40:41]\n"
                            "v_cndmask_b32_e64 %4, %4, %8, s[40:41]\n v_cndmask_b32_e64 %5, %5, %8, s[40:41]\n"
                            "v_cndmask_b32_e64 %6, %6, %8, s[40:41]\n v_cndmask_b32_e64 %7, %7, %8, s[40:41]\n")
                         : OUTS : "v"(s0) : "s40", "s41");
        else if constexpr (MODE == 20)  // 8 x v_bfi_b32 with a VGPR mask
            asm volatile(R8("v_bfi_b32 %0, %9, %0, %8\n v_bfi_b32 %1, %9, %1, %8\n v_bfi_b32 %2, %9, %2, %8\n"
                            "v_bfi_b32 %3, %9, %3, %8\n v_bfi_b32 %4, %9, %4, %8\n v_bfi_b32 %5, %9, %5, %8\n"
                            "v_bfi_b32 %6, %9, %6, %8\n v_bfi_b32 %7, %9, %7, %8\n")
                         : OUTS : "v"(s0), "v"(c0));
        else if constexpr (MODE == 21)  // 8 x v_min3_f32
            asm volatile(R8("v_min3_f32 %0, %0, %1, %8\n v_min3_f32 %1, %1, %2, %8\n v_min3_f32 %2, %2, %3, %8\n"
                            "v_min3_f32 %3, %3, %4, %8\n v_min3_f32 %4, %4, %5, %8\n v_min3_f32 %5, %5, %6, %8\n"
                            "v_min3_f32 %6, %6, %7, %8\n v_min3_f32 %7, %7, %0, %8\n")
                         : OUTS : "v"(s0));
        else if constexpr (MODE == 22)  // 8 x v_mov_b32
            asm volatile(R8("v_mov_b32 %0, %1\n v_mov_b32 %1, %2\n v_mov_b32 %2, %3\n v_mov_b32 %3, %4\n"
                            "v_mov_b32 %4, %5\n v_mov_b32 %5, %6\n v_mov_b32 %6, %7\n v_mov_b32 %7, %0\n")
                         : OUTS);
        else if constexpr (MODE == 23)  // 8 x v_cndmask_b32_e32 vcc, VCC written by a v_cmp once per iteration
            asm volatile("v_cmp_lt_f32_e32 vcc, %0, %8\n" R8("v_cndmask_b32 %0, %0, %8, vcc\n v_cndmask_b32 %1, %1, %8, vcc\n v_cndmask_b32 %2, %2, %8, vcc\n"
                            "v_cndmask_b32 %3, %3, %8, vcc\n v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n"
                            "v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc\n")
                         : OUTS : "v"(s0) : "vcc");
        else if constexpr (MODE == 24)  // 8 x v_max_f32_e64 |a|, |b|
            asm volatile(R8("v_max_f32_e64 %0, |%0|, |%1|\n v_max_f32_e64 %1, |%1|, |%2|\n v_max_f32_e64 %2, |%2|, |%3|\n"
                            "v_max_f32_e64 %3, |%3|, |%4|\n v_max_f32_e64 %4, |%4|, |%5|\n v_max_f32_e64 %5, |%5|, |%6|\n"
                            "v_max_f32_e64 %6, |%6|, |%7|\n v_max_f32_e64 %7, |%7|, |%0|\n")
                         : OUTS);
        else if constexpr (MODE == 25)  // 8 x v_add_f32 (dependency pattern of mode 17)
            asm volatile(R8("v_add_f32 %0, %0, %1\n v_add_f32 %1, %1, %2\n v_add_f32 %2, %2, %3\n v_add_f32 %3, %3, %4\n"
                            "v_add_f32 %4, %4, %5\n v_add_f32 %5, %5, %6\n v_add_f32 %6, %6, %7\n v_add_f32 %7, %7, %0\n")
                         : OUTS);
        else if constexpr (MODE == 18)  // 8 x ds_swizzle_b32 (row rotate), then one wait
            asm volatile(R8("ds_swizzle_b32 %0, %0 offset:swizzle(SWAP,8)\n ds_swizzle_b32 %1, %1 offset:swizzle(SWAP,8)\n"
                            "ds_swizzle_b32 %2, %2 offset:swizzle(SWAP,8)\n ds_swizzle_b32 %3, %3 offset:swizzle(SWAP,8)\n"
                            "ds_swizzle_b32 %4, %4 offset:swizzle(SWAP,8)\n ds_swizzle_b32 %5, %5 offset:swizzle(SWAP,8)\n"
                            "ds_swizzle_b32 %6, %6 offset:swizzle(SWAP,8)\n ds_swizzle_b32 %7, %7 offset:swizzle(SWAP,8)\n"
                            "s_waitcnt lgkmcnt(0)\n")
                         : OUTS);
    }
    if (v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7 + c0 + c1 == 1.2345f) out[threadIdx.x] = 1.0f;
}

template <int M>
float run(float* out, int blocks, int iters) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float ms = 0;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k<M>, dim3(blocks), dim3(256), 0, 0, out, 0.999f, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
    }
    return ms;
}

int main() {
    float* out;
    (void)hipMalloc(&out, 4096);
    setvbuf(stdout, nullptr, _IOLBF, 0);
    const int iters = 1000;
    const char* names[] = {"v_fma_f32 x8", "v_cmp_e32 vcc x8", "v_writelane x8", "v_sub_e64 |v| x8",
                           "v_pk_fma_f32 x8", "v_addc vcc x8", "entry: current x2 (18 ops)",
                           "entry: fma+cmp+amb x2 (16 ops)", "entry: fma+sq+vcc+pack x2 (14 ops)", "v_bcnt x8",
                           "v_cmp_e64 sgpr x8", "v_mul_f32 x8", "v_pk_mul_f32 x8", "v_cndmask vcc x8",
                           "v_permlane32_swap x8", "v_permlane16_swap x8", "v_min_f32_dpp row_ror x8",
                           "v_min_f32 x8", "ds_swizzle x8 + wait", "v_cndmask_e64 sgpr x8", "v_bfi_b32 x8",
                           "v_min3_f32 x8", "v_mov_b32 x8", "v_cndmask_e32 vcc(cmp) x8", "v_max_f32 |.| x8",
                           "v_add_f32 (chain 17) x8"};
    float (*fns[26])(float*, int, int) = {run<0>, run<1>, run<2>, run<3>, run<4>, run<5>, run<6>,
                                           run<7>, run<8>, run<9>, run<10>, run<11>, run<12>, run<13>,
                                           run<14>, run<15>, run<16>, run<17>, run<18>, run<19>, run<20>,
                                           run<21>, run<22>, run<23>, run<24>, run<25>};
    for (int wpe : {5}) {
        const int blocks = 256 * wpe;
        for (int m : {11, 25, 17, 21, 24, 22, 13, 19, 23, 20, 14, 16}) {
            printf("%-36s waves/SIMD %d: ", names[m], wpe);
            fflush(stdout);
            const float ms = fns[m](out, blocks, iters);
            // each wave runs iters x 8 blocks; blocks * 4 waves spread over 1024 SIMDs
            const double per_simd = (double)iters * 8 * blocks * 4 / 1024.0;
            printf("%8.3f ms  %6.3f ns per block per SIMD\n", ms, ms * 1e6 / per_simd);
        }
    }
    return 0;
}
