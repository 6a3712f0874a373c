// xsum.hpp -- sequential float sums s_{i+1} = fl(s_i + v_i), s_0 = +0, reproduced bit for bit by a
// block-parallel walk (PCL's accumulators: computeMeanAndCovarianceMatrix's nine sums, the cluster
// centroids' three).  The serial chain costs one dependent add per element (~1.9 ns); this costs one
// dependent step per 256 elements where the sum's rounding is predictable, and falls back to the
// elements only where it is not.
//
// While |s| stays inside one binade [2^e, 2^(e+1)) its float spacing u = 2^(e-23) is fixed, s = K u with
// K in [2^23, 2^24), and fl(s + v) = (K + q) u with q = round-to-nearest(v / u) -- unless v / u is a tie
// (its fraction exactly 1/2: the rounding then depends on K's parity) or K + q leaves the binade.  So a
// block of elements whose quotients q_j (for an assumed e and sign) have no tie advances s by R u,
// R = sum q_j, whenever every partial K + P_m (P_0 = 0) stays in [2^23 + 1, 2^24 - 1]: an interval of
// entry values [L, H] that the block's prefix minimum and maximum of P give exactly.
//
//   xs_est    per 256-element block: double sums of its 16-element sub-blocks and of the block;
//   xs_scan   per (segment, stream): exclusive prefix of the block sums in double -- an estimate of
//             every block's entry s, used only to choose the binade a summary assumes;
//   xs_summ   per block: the summary (L, H, R u) for the binade of the block's estimated entry, and one
//             per 16-element sub-block for the binade of its own estimated entry;
//   xs_walk   per (segment, stream), lane 0 of a wave: s += R u for a block whose [L, H] holds s,
//             else the same per sub-block, else the sub-block's 16 adds.  The estimate only decides
//             how often the walk falls back, never the result: every accepted step is exact.
//
// Layout: S streams of T floats each (stream s at v + s T), segments on 256-element block boundaries
// (XsSeg: first block, length -- the length may be written on the device); elements past a segment's
// length are never added (the summaries treat them as +0, which leaves any sum unchanged: s is never
// -0 in round-to-nearest starting from +0).
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>
#include <string>

#include "ctx.hpp"

#pragma clang fp contract(off)

namespace pitt {

constexpr int kXsBlk = 256;   // elements per block
constexpr int kXsSub = 16;    // elements per sub-block
constexpr int kXsSubs = kXsBlk / kXsSub;

struct XsSeg {
    int64_t blk0;  // first block
    int64_t len;   // elements
};

struct XsSum {  // one summary: s in [lo, hi] -> s + ru exactly (lo > hi: never)
    float lo, hi, ru, pad;
};

// floor(log2 |a|) of a normal double, or a flag outside float's normal range
__device__ __forceinline__ int xs_binade(double a, bool* ok) {
    const double m = fabs(a);
    *ok = m >= (double)FLT_MIN && m < (double)FLT_MAX;
    int e = 0;
    (void)frexp(m, &e);
    return e - 1;
}

// One element's step for binade e and sign neg: q = rint(v / u) in magnitude, or bad (a tie, or |q| too
// large for the block to stay in the binade).
__device__ __forceinline__ int xs_step(float v, double scale, bool neg, bool* bad) {
    double x = (double)v * scale;
    if (neg) x = -x;
    if (!(fabs(x) < 8388608.0)) {  // |q| >= 2^23 leaves the binade (NaN and infinities too)
        *bad = true;
        return 0;
    }
    const double fl = floor(x);
    if (x - fl == 0.5) *bad = true;
    return (int)rint(x);
}

__device__ __forceinline__ XsSum xs_never() { return XsSum{1.0f, -1.0f, 0.0f, 0.0f}; }

// The summary of a run with quotient prefix sum R and prefix extremes mn <= 0 <= mx, for binade e.
__device__ __forceinline__ XsSum xs_make(int e, bool neg, int R, int mn, int mx) {
    const int64_t klo = (int64_t)(1 << 23) + 1 - mn, khi = (int64_t)(1 << 24) - 1 - mx;
    if (klo > khi) return xs_never();  // (a valid block has |R|, -mn, mx < 2^23: every float below is exact)
    const float u = ldexpf(1.0f, e - 23);
    const float lo = (float)klo * u, hi = (float)khi * u, ru = (float)R * u;
    return neg ? XsSum{-hi, -lo, -ru, 0.0f} : XsSum{lo, hi, ru, 0.0f};
}

// xs_est: one wave per (block, stream); lane l holds elements 4 l .. 4 l + 3 of the block.
template <int = 0>  // a template: the header is included by several translation units
__global__ __launch_bounds__(256) void k_xs_est(const float* __restrict__ v, int64_t T, int S, int64_t nblk,
                                                const XsSeg* __restrict__ seg, const int32_t* __restrict__ blk_seg,
                                                double* __restrict__ dsub, double* __restrict__ dblk) {
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nblk * S) return;
    const int lane = threadIdx.x & 63;
    const int s = (int)(w / nblk);
    const int64_t b = w - (int64_t)s * nblk;
    const XsSeg g = seg[blk_seg[b]];
    const int64_t i0 = (b - g.blk0) * kXsBlk + 4 * lane;  // element index inside the segment
    const float4 q = *reinterpret_cast<const float4*>(v + (int64_t)s * T + b * kXsBlk + 4 * lane);
    double d = 0.0;
    d += i0 + 0 < g.len ? (double)q.x : 0.0;
    d += i0 + 1 < g.len ? (double)q.y : 0.0;
    d += i0 + 2 < g.len ? (double)q.z : 0.0;
    d += i0 + 3 < g.len ? (double)q.w : 0.0;
    // 4 lanes per sub-block
    d += __shfl_xor(d, 1, 64);
    d += __shfl_xor(d, 2, 64);
    if ((lane & 3) == 0) dsub[((int64_t)s * nblk + b) * kXsSubs + (lane >> 2)] = d;
    double t = d;
    for (int off = 4; off < 64; off <<= 1) t += __shfl_xor(t, off, 64);
    if (lane == 0) dblk[(int64_t)s * nblk + b] = t;
}

// xs_scan: one block per (segment, stream): the exclusive prefix of the segment's block sums.
template <int = 0>  // a template: the header is included by several translation units
__global__ __launch_bounds__(256) void k_xs_scan(int nseg, int S, int64_t nblk, const XsSeg* __restrict__ seg,
                                                 const double* __restrict__ dblk, double* __restrict__ eblk) {
    const int k = blockIdx.x % nseg, s = blockIdx.x / nseg;
    const XsSeg g = seg[k];
    const int64_t nb = (g.len + kXsBlk - 1) / kXsBlk;
    const double* in = dblk + (int64_t)s * nblk + g.blk0;
    double* out = eblk + (int64_t)s * nblk + g.blk0;
    __shared__ double part[256];
    const int64_t per = (nb + 255) / 256;
    const int64_t a = (int64_t)threadIdx.x * per, e = a + per < nb ? a + per : nb;
    double acc = 0.0;
    for (int64_t i = a; i < e; ++i) acc += in[i];
    part[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double run = 0.0;
        for (int i = 0; i < 256; ++i) {
            const double t = part[i];
            part[i] = run;
            run += t;
        }
    }
    __syncthreads();
    acc = part[threadIdx.x];
    for (int64_t i = a; i < e; ++i) {
        out[i] = acc;
        acc += in[i];
    }
}

// xs_summ: one wave per (block, stream): the block's summary and its 16 sub-blocks'.
template <int = 0>  // a template: the header is included by several translation units
__global__ __launch_bounds__(256) void k_xs_summ(const float* __restrict__ v, int64_t T, int S, int64_t nblk,
                                                 const XsSeg* __restrict__ seg, const int32_t* __restrict__ blk_seg,
                                                 const double* __restrict__ dsub, const double* __restrict__ eblk,
                                                 XsSum* __restrict__ sblk, XsSum* __restrict__ ssub) {
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nblk * S) return;
    const int lane = threadIdx.x & 63;
    const int s = (int)(w / nblk);
    const int64_t b = w - (int64_t)s * nblk;
    const XsSeg g = seg[blk_seg[b]];
    const int64_t i0 = (b - g.blk0) * kXsBlk + 4 * lane;
    if ((b - g.blk0) * kXsBlk >= g.len) return;  // past the segment: never walked
    const float4 q4 = *reinterpret_cast<const float4*>(v + (int64_t)s * T + b * kXsBlk + 4 * lane);
    float e4[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (i0 + k >= g.len) e4[k] = 0.0f;
    const int64_t sb = (int64_t)s * nblk + b;
    // the block's estimated entry and its sub-blocks' (lane 4 j + r belongs to sub-block j)
    const double E = eblk[sb];
    const int j = lane >> 2;
    double Ej = E;
    for (int t = 0; t < j; ++t) Ej += dsub[sb * kXsSubs + t];  // the same in every lane of the sub-block
    // --- the block, for the binade of E ---
    {
        bool ok;
        const int e = xs_binade(E, &ok);
        const bool neg = E < 0.0;
        const double scale = ldexp(1.0, 23 - e);
        bool bad = !ok;
        int q[4], p = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            q[k] = ok ? xs_step(e4[k], scale, neg, &bad) : 0;
            p += q[k];
        }
        // inclusive prefix of the lanes' sums, then the per-element prefix extremes
        int incl = p;
        for (int off = 1; off < 64; off <<= 1) {
            const int o = __shfl_up(incl, off, 64);
            if (lane >= off) incl += o;
        }
        int run = incl - p, mn = 0, mx = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            run += q[k];
            mn = run < mn ? run : mn;
            mx = run > mx ? run : mx;
        }
        for (int off = 32; off > 0; off >>= 1) {
            const int a = __shfl_xor(mn, off, 64), c = __shfl_xor(mx, off, 64);
            mn = a < mn ? a : mn;
            mx = c > mx ? c : mx;
        }
        const bool anybad = __builtin_amdgcn_ballot_w64(bad) != 0;
        const int R = __shfl(incl, 63, 64);
        if (lane == 0) sblk[sb] = anybad ? xs_never() : xs_make(e, neg, R, mn, mx);
    }
    // --- each sub-block, for the binade of its own estimate ---
    {
        bool ok;
        const int e = xs_binade(Ej, &ok);
        const bool neg = Ej < 0.0;
        const double scale = ldexp(1.0, 23 - e);
        bool bad = !ok;
        int q[4], p = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            q[k] = ok ? xs_step(e4[k], scale, neg, &bad) : 0;
            p += q[k];
        }
        // prefix over the 4 lanes of the sub-block
        int incl = p;
        for (int off = 1; off < 4; off <<= 1) {
            const int o = __shfl_up(incl, off, 64);
            if ((lane & 3) >= off) incl += o;
        }
        int run = incl - p, mn = 0, mx = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            run += q[k];
            mn = run < mn ? run : mn;
            mx = run > mx ? run : mx;
        }
        for (int off = 1; off < 4; off <<= 1) {
            const int a = __shfl_xor(mn, off, 64), c = __shfl_xor(mx, off, 64);
            mn = a < mn ? a : mn;
            mx = c > mx ? c : mx;
        }
        const uint64_t bb = __builtin_amdgcn_ballot_w64(bad);
        const bool subbad = ((bb >> (4 * j)) & 0xFull) != 0;
        const int R = __shfl(incl, 4 * j + 3, 64);
        if ((lane & 3) == 0) ssub[sb * kXsSubs + j] = subbad ? xs_never() : xs_make(e, neg, R, mn, mx);
    }
}

// xs_walk: one 256-thread block per (segment, stream).  The walk itself is serial (the sum s is one
// value; wave 0 carries it), but nothing it reads comes from memory at its own latency: the segment is
// staged in windows of kXsWin blocks -- the block summaries, their sub-block summaries and the elements
// -- into a double-buffered LDS area by all four waves, the next window's loads in flight while wave 0
// walks the current one.  Per block the walk reads its summary by v_readlane; a block whose summary
// fails reads its 16 sub-block summaries (lanes 0-15, one LDS read), a sub-block that fails its 16
// elements.  The adds and their order are exactly those of a lane walking element by element.
// out[k * S + s] = the segment's float sum.
constexpr int kXsWin = 32;  // blocks per staged window
struct XsWalkLds {
    float4 el[2][kXsWin * kXsBlk / 4];   // elements (32 KB per window)
    XsSum sub[2][kXsWin * kXsSubs];      // sub-block summaries
    XsSum blk[2][kXsWin];                // block summaries
};

__device__ __forceinline__ float xs_lane(float v, int i) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), i));
}

template <int = 0>  // a template: the header is included by several translation units
__global__ __launch_bounds__(256) void k_xs_walk(const float* __restrict__ v, int64_t T, int S, int64_t nblk,
                                                 int nseg, const XsSeg* __restrict__ seg,
                                                 const XsSum* __restrict__ sblk, const XsSum* __restrict__ ssub,
                                                 float* __restrict__ out) {
    __shared__ XsWalkLds L;
    const int k = blockIdx.x % nseg, s = blockIdx.x / nseg;
    const int tid = threadIdx.x, lane = tid & 63;
    const XsSeg g = seg[k];
    const float4* vs4 = reinterpret_cast<const float4*>(v + (int64_t)s * T + g.blk0 * kXsBlk);
    const XsSum* sb = sblk + (int64_t)s * nblk + g.blk0;
    const XsSum* ss = ssub + ((int64_t)s * nblk + g.blk0) * kXsSubs;
    const int64_t nb = (g.len + kXsBlk - 1) / kXsBlk;
    constexpr int kEl = kXsWin * kXsBlk / 4 / 256, kSub = kXsWin * kXsSubs / 256;  // per thread
    float4 re[kEl];
    XsSum rs[kSub], rb;
    auto load = [&](int64_t w0) {  // window w0 .. w0 + kXsWin into registers (blocks past nb: never read)
        const int64_t nbw = nb - w0 < kXsWin ? nb - w0 : kXsWin;
#pragma unroll
        for (int q = 0; q < kEl; ++q) {
            const int i = tid + 256 * q;  // float4 index in the window
            re[q] = i < nbw * (kXsBlk / 4) ? vs4[w0 * (kXsBlk / 4) + i] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int q = 0; q < kSub; ++q) {
            const int i = tid + 256 * q;
            rs[q] = i < nbw * kXsSubs ? ss[w0 * kXsSubs + i] : xs_never();
        }
        rb = tid < nbw ? sb[w0 + tid] : xs_never();
    };
    auto store = [&](int slot) {
#pragma unroll
        for (int q = 0; q < kEl; ++q) L.el[slot][tid + 256 * q] = re[q];
#pragma unroll
        for (int q = 0; q < kSub; ++q) L.sub[slot][tid + 256 * q] = rs[q];
        if (tid < kXsWin) L.blk[slot][tid] = rb;
    };
    const float* el0 = reinterpret_cast<const float*>(&L.el[0][0]);
    const float* el1 = reinterpret_cast<const float*>(&L.el[1][0]);
    float acc = 0.0f;  // wave 0: the same value in every lane
    if (nb > 0) {
        load(0);
        store(0);
    }
    __syncthreads();
    for (int64_t w0 = 0, w = 0; w0 < nb; w0 += kXsWin, ++w) {
        const int slot = (int)(w & 1);
        if (w0 + kXsWin < nb) load(w0 + kXsWin);  // in flight while wave 0 walks this window
        if (tid < 64) {
            const int cnt = (int)(nb - w0 < kXsWin ? nb - w0 : kXsWin);
            const XsSum cur = lane < kXsWin ? L.blk[slot][lane] : xs_never();
            const float* el = slot ? el1 : el0;
            for (int i = 0; i < cnt; ++i) {
                const float lo = xs_lane(cur.lo, i), hi = xs_lane(cur.hi, i);
                if (acc >= lo && acc <= hi) {
                    acc = acc + xs_lane(cur.ru, i);  // exactly (K + R) u
                    continue;
                }
                const int64_t base = (w0 + i) * kXsBlk;  // the block's first element in the segment
                const XsSum sub = lane < kXsSubs ? L.sub[slot][i * kXsSubs + lane] : xs_never();
                for (int j = 0; j < kXsSubs; ++j) {
                    const int64_t e0 = base + j * kXsSub;
                    if (e0 >= g.len) break;
                    const float clo = xs_lane(sub.lo, j), chi = xs_lane(sub.hi, j);
                    if (acc >= clo && acc <= chi) {
                        acc = acc + xs_lane(sub.ru, j);
                        continue;
                    }
                    const int n_e = (int)(g.len - e0 < kXsSub ? g.len - e0 : kXsSub);
                    const float ev = lane < n_e ? el[i * kXsBlk + j * kXsSub + lane] : 0.0f;
                    for (int t = 0; t < n_e; ++t) acc = acc + xs_lane(ev, t);
                }
            }
        }
        if (w0 + kXsWin < nb) store(slot ^ 1);  // the other slot was last read in the previous window
        __syncthreads();
    }
    if (tid == 0) out[(int64_t)k * S + s] = acc;
}

// Scratch of the four launches over S streams of nblk blocks, allocated before any enqueue (a captured
// graph must not allocate).
struct XsScratch {
    double *dsub = nullptr, *dblk = nullptr, *eblk = nullptr;
    XsSum *sblk = nullptr, *ssub = nullptr;
};
inline int xs_scratch(pitt_ctx* ctx, int64_t nblk, int S, const std::string& name, XsScratch* x) {
    x->dsub = (double*)ctx->buf(name + "_xs_dsub", (size_t)S * nblk * kXsSubs * 8);
    x->dblk = (double*)ctx->buf(name + "_xs_dblk", (size_t)S * nblk * 8);
    x->eblk = (double*)ctx->buf(name + "_xs_eblk", (size_t)S * nblk * 8);
    x->sblk = (XsSum*)ctx->buf(name + "_xs_sblk", (size_t)S * nblk * sizeof(XsSum));
    x->ssub = (XsSum*)ctx->buf(name + "_xs_ssub", (size_t)S * nblk * kXsSubs * sizeof(XsSum));
    if (!x->dsub || !x->dblk || !x->eblk || !x->sblk || !x->ssub) return ctx->fail(PITT_E_NOMEM, "exact-sum scratch");
    return PITT_OK;
}

// The four launches over S streams of T floats (T a multiple of kXsBlk; nblk = T / kXsBlk blocks),
// nseg segments (device XsSeg, the block -> segment map blk_seg on the device), sums into out[k S + s].
inline void xs_enqueue(hipStream_t st, const float* v, int64_t T, int S, int nseg, const XsSeg* seg,
                       const int32_t* blk_seg, float* out, const XsScratch& x) {
    const int64_t nblk = T / kXsBlk;
    if (nblk == 0 || nseg == 0) return;
    const unsigned waves = (unsigned)((nblk * S + 3) / 4);
    hipLaunchKernelGGL(k_xs_est<>, dim3(waves), dim3(256), 0, st, v, T, S, nblk, seg, blk_seg, x.dsub, x.dblk);
    hipLaunchKernelGGL(k_xs_scan<>, dim3((unsigned)(nseg * S)), dim3(256), 0, st, nseg, S, nblk, seg, x.dblk, x.eblk);
    hipLaunchKernelGGL(k_xs_summ<>, dim3(waves), dim3(256), 0, st, v, T, S, nblk, seg, blk_seg, x.dsub, x.eblk, x.sblk,
                       x.ssub);
    hipLaunchKernelGGL(k_xs_walk<>, dim3((unsigned)(nseg * S)), dim3(256), 0, st, v, T, S, nblk, nseg, seg, x.sblk,
                       x.ssub, out);
}

}  // namespace pitt
