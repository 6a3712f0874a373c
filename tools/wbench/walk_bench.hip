// walk_bench.hip -- the exact walk (csrc/xsum.hpp) alone on the nine covariance streams of one 640x480
// table frame (tools/wbench/walk_streams.bin: n, the 9 x n products in inlier order, the 9 sequential
// float sums).  Times k_xs_est / k_xs_scan / k_xs_summ / k_xs_walk with HIP events, and the walk in its
// measurement modes (1: staging only, 3: cycles per phase), and checks the sums bit for bit.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../../pitt_object_table_segmentation_amd/csrc \
//         walk_bench.hip -o walk_bench && ./walk_bench walk_streams.bin
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "xsum.hpp"

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
            return 1;                                                          \
        }                                                                      \
    } while (0)

using namespace pitt;

int main(int argc, char** argv) {
    const char* path = argc > 1 ? argv[1] : "walk_streams.bin";
    FILE* f = std::fopen(path, "rb");
    if (!f) return 2;
    int64_t n = 0;
    if (std::fread(&n, 8, 1, f) != 1) return 2;
    const int S = 9;
    std::vector<float> h((size_t)S * n), ref(S);
    if (std::fread(h.data(), 4, h.size(), f) != h.size() || std::fread(ref.data(), 4, S, f) != (size_t)S) return 2;
    std::fclose(f);
    const int64_t nblk = (n + kXsBlk - 1) / kXsBlk, T = nblk * kXsBlk;
    std::vector<float> hv((size_t)S * T, 0.0f);
    for (int s = 0; s < S; ++s) std::memcpy(&hv[(size_t)s * T], &h[(size_t)s * n], n * 4);
    float *v, *out;
    XsSeg* seg;
    int32_t* bseg;
    XsScratch x;
    CK(hipMalloc(&v, hv.size() * 4));
    CK(hipMalloc(&out, S * 4 * 8));
    CK(hipMalloc(&seg, sizeof(XsSeg)));
    CK(hipMalloc(&bseg, nblk * 4));
    CK(hipMalloc(&x.dsub, S * nblk * kXsSubs * 8));
    CK(hipMalloc(&x.dblk, S * nblk * 8));
    CK(hipMalloc(&x.eblk, S * nblk * 8));
    CK(hipMalloc(&x.sblk, S * nblk * sizeof(XsSum)));
    CK(hipMalloc(&x.ssub, S * nblk * kXsSubs * sizeof(XsSum)));
    CK(hipMemcpy(v, hv.data(), hv.size() * 4, hipMemcpyHostToDevice));
    const XsSeg sg{0, n};
    CK(hipMemcpy(seg, &sg, sizeof sg, hipMemcpyHostToDevice));
    CK(hipMemset(bseg, 0, nblk * 4));
    hipEvent_t e[6];
    for (auto& ev : e) CK(hipEventCreate(&ev));
    const unsigned waves = (unsigned)((nblk * S + 3) / 4);
    float ms[5] = {0, 0, 0, 0, 0};
    const int reps = 20;
    for (int r = 0; r <= reps; ++r) {
        CK(hipEventRecord(e[0], 0));
        hipLaunchKernelGGL(k_xs_est<>, dim3(waves), dim3(256), 0, 0, v, T, S, nblk, seg, bseg, x.dsub, x.dblk);
        CK(hipEventRecord(e[1], 0));
        hipLaunchKernelGGL(k_xs_scan<>, dim3(S), dim3(256), 0, 0, 1, S, nblk, seg, x.dblk, x.eblk);
        CK(hipEventRecord(e[2], 0));
        hipLaunchKernelGGL(k_xs_summ<>, dim3(waves), dim3(256), 0, 0, v, T, S, nblk, seg, bseg, x.dsub, x.eblk, x.sblk,
                           x.ssub);
        CK(hipEventRecord(e[3], 0));
        hipLaunchKernelGGL(k_xs_walk<0>, dim3(S), dim3(256), 0, 0, v, T, S, nblk, 1, seg, x.sblk, x.ssub, out);
        CK(hipEventRecord(e[4], 0));
        CK(hipEventSynchronize(e[4]));
        if (r == 0) continue;
        for (int k = 0; k < 4; ++k) {
            float t = 0;
            CK(hipEventElapsedTime(&t, e[k], e[k + 1]));
            ms[k] += t / reps;
        }
    }
    std::vector<float> got(S);
    CK(hipMemcpy(got.data(), out, S * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int s = 0; s < S; ++s) bad += std::memcmp(&got[s], &ref[s], 4) != 0;
    std::printf("n %lld blocks %lld: est %.1f us, scan %.1f us, summ %.1f us, walk %.1f us; sums %s\n", (long long)n,
                (long long)nblk, ms[0] * 1e3, ms[1] * 1e3, ms[2] * 1e3, ms[3] * 1e3, bad ? "DIFFER" : "bit-exact");
    // the walk's measurement modes, and each stream alone
    for (int mode = 1; mode <= 1; ++mode) {
        float t = 0;
        for (int r = 0; r <= reps; ++r) {
            CK(hipEventRecord(e[0], 0));
            if (mode == 1) hipLaunchKernelGGL(k_xs_walk<1>, dim3(S), dim3(256), 0, 0, v, T, S, nblk, 1, seg, x.sblk, x.ssub, out);
            CK(hipEventRecord(e[1], 0));
            CK(hipEventSynchronize(e[1]));
            float q = 0;
            CK(hipEventElapsedTime(&q, e[0], e[1]));
            if (r) t += q / reps;
        }
        std::printf("walk mode %d (%s): %.1f us\n", mode, mode == 1 ? "staging only" : "every block taken", t * 1e3);
    }
    {  // wave 0's cycles per phase (MODE 3)
        hipLaunchKernelGGL(k_xs_walk<3>, dim3(S), dim3(256), 0, 0, v, T, S, nblk, 1, seg, x.sblk, x.ssub, out);
        CK(hipDeviceSynchronize());
        std::vector<float> c((size_t)S * 5);
        CK(hipMemcpy(c.data(), out, c.size() * 4, hipMemcpyDeviceToHost));
        for (int s = 0; s < S; ++s)
            std::printf("stream %d cycles: runs %.0f, failing blocks %.0f, staging+barriers %.0f\n", s,
                        c[S + 4 * s], c[S + 4 * s + 1], c[S + 4 * s + 2]);
    }
    for (int s = 0; s < S; ++s) {
        float t = 0;
        for (int r = 0; r <= reps; ++r) {
            CK(hipEventRecord(e[0], 0));
            hipLaunchKernelGGL(k_xs_walk<0>, dim3(1), dim3(256), 0, 0, v + (size_t)s * T, T, 1, nblk, 1, seg,
                               x.sblk + (size_t)s * nblk, x.ssub + (size_t)s * nblk * kXsSubs, out);
            CK(hipEventRecord(e[1], 0));
            CK(hipEventSynchronize(e[1]));
            float q = 0;
            CK(hipEventElapsedTime(&q, e[0], e[1]));
            if (r) t += q / reps;
        }
        std::printf("stream %d alone: %.1f us\n", s, t * 1e3);
    }
    return bad ? 1 : 0;
}
