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
#include <climits>
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

// xs_walk: one 256-thread block per (segment, stream).  The sum s is one value (wave 0 carries it), but
// the walk does not take one summary at a time.  While s stays in one binade e (s = +-K u, u = 2^(e-23),
// K the 24-bit significand), a summary (L, H, R u) holds exactly when its binade and sign are s's and K
// lies in its integer range [klo, khi]; after it K becomes K + R.  So a run of summaries is tested at
// once: lane j holds summary j, an integer prefix scan of the R's gives every lane the K it would enter
// with if all before it held, and the first lane whose test fails ends the run (every lane before it
// held, so s after them is exact: K plus the scan, rebuilt as a float).  Only the failing summary's
// range is walked below it: a failing block runs the same test over its 16 sub-block summaries, a
// failing sub-block adds its elements one by one.  Every step is an exact float add of the sequential
// chain, so the result is the chain's bit for bit.
// The segment is staged in windows of kXsWin blocks (block summaries, sub-block summaries, elements)
// into a double-buffered LDS area by all four waves, the next window's loads in flight while wave 0
// walks the current one.  out[k * S + s] = the segment's float sum.
constexpr int kXsWin = 32;  // blocks per staged window
struct XsWalkLds {
    float4 el[2][kXsWin * kXsBlk / 4];   // elements (32 KB per window)
    XsSum sub[2][kXsWin * kXsSubs];      // sub-block summaries
    XsSum blk[2][kXsWin];                // block summaries
};

// a normal float as sign, binade and 24-bit significand (ok: a normal float)
struct XsK {
    int e, s, K;
    bool ok;
};
__device__ __forceinline__ XsK xs_k(float a) {
    const uint32_t b = __float_as_uint(a);
    const int ef = (int)((b >> 23) & 0xffu);
    return XsK{ef - 127, (int)(b >> 31), (int)((b & 0x7fffffu) | 0x800000u), ef != 0 && ef != 255};
}

// inclusive prefix sum over the wave's lanes (DPP row shifts, then the row broadcasts)
__device__ __forceinline__ int xs_scan64(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}

// One lane's summary in significand units: its binade and sign (es = 2 e + s, or INT_MIN for a summary
// that never holds), the significand range it holds for, its step R, and the inclusive prefix of the
// steps over the lanes below n (decoded and scanned once per window or per failing block).
struct XsLane {
    int es, kmin, kmax, dk, incl;
};
__device__ __forceinline__ XsLane xs_decode(const XsSum& c, int n, int lane) {
    const XsK l = xs_k(c.lo), h = xs_k(c.hi);
    const bool valid = lane < n && c.lo <= c.hi && l.ok && h.ok;  // xs_never: lo > hi
    XsLane d;
    d.es = valid ? 2 * l.e + l.s : INT_MIN;
    d.kmin = l.K < h.K ? l.K : h.K;
    d.kmax = l.K < h.K ? h.K : l.K;
    d.dk = 0;
    if (valid) {
        const int r = (int)ldexpf(c.ru, 23 - l.e);  // R u / u, exact
        d.dk = l.s ? -r : r;
    }
    d.incl = xs_scan64(lane < n ? d.dk : 0);
    return d;
}

// The summaries of lanes [i0, n) applied to acc in order, as far as they hold: returns the first lane
// whose summary does not hold for the value acc has when it is reached (n if all hold), with acc advanced
// over the lanes before it.  All lanes of the wave call it with the same acc, i0 and n.
__device__ __forceinline__ int xs_run(float& acc, const XsLane& d, int i0, int n, int lane) {
    const XsK a = xs_k(acc);
    const int base = i0 > 0 ? __builtin_amdgcn_readlane(d.incl, i0 - 1) : 0;
    const int kj = a.K + (d.incl - d.dk - base);  // the significand this lane's summary would see
    const bool holds = a.ok && d.es == 2 * a.e + a.s && kj >= d.kmin && kj <= d.kmax;
    const uint64_t fail = __builtin_amdgcn_ballot_w64(lane >= i0 && lane < n && !holds);
    const int f = fail ? (int)__builtin_ctzll(fail) : n;
    if (f > i0) {  // lanes [i0, f) held: s = +-(K + their R's) u, inside binade e
        const int kf = a.K + (__builtin_amdgcn_readlane(d.incl, f - 1) - base);
        acc = __uint_as_float(((uint32_t)a.s << 31) | ((uint32_t)(a.e + 127) << 23) | ((uint32_t)kf & 0x7fffffu));
    }
    return f;
}

// MODE (tools/wbench only, a measurement): 1 = the staging without the walk, 3 = the exact walk with
// wave 0's cycles per phase written after the sums (out[nseg S + 4 s + k]: runs, failing blocks, staging
// and barriers); the library uses 0.
template <int MODE = 0>  // a template: the header is included by several translation units
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
    float acc = 0.0f;  // wave 0: the same value in every lane
    long long cyc_run = 0, cyc_fail = 0, cyc_stage = 0, t_mark = MODE == 3 ? clock64() : 0;
    if (nb > 0) {
        load(0);
        store(0);
    }
    __syncthreads();
    for (int64_t w0 = 0, w = 0; w0 < nb; w0 += kXsWin, ++w) {
        const int slot = (int)(w & 1);
        if (w0 + kXsWin < nb) load(w0 + kXsWin);  // in flight while wave 0 walks this window
        if (MODE == 3) {
            const long long t = clock64();
            cyc_stage += t - t_mark;
            t_mark = t;
        }
        if (tid < 64 && MODE != 1) {
            // every loop bound and index below is wave-uniform (a ballot's first bit, a readlane): scalar
            // control flow; indices are window-local 32-bit
            const int cnt = (int)(nb - w0 < kXsWin ? nb - w0 : kXsWin);
            const int rem = (int)(g.len - w0 * kXsBlk < (int64_t)kXsWin * kXsBlk ? g.len - w0 * kXsBlk
                                                                                 : (int64_t)kXsWin * kXsBlk);
            const XsLane cur = xs_decode(lane < kXsWin ? L.blk[slot][lane] : xs_never(), cnt, lane);
            const float* el = reinterpret_cast<const float*>(&L.el[slot][0]);
            int i = 0;
            while (i < cnt) {
                const int f = xs_run(acc, cur, i, cnt, lane);
                if (f >= cnt) break;
                long long tf = 0;
                if (MODE == 3) {
                    tf = clock64();
                    cyc_run += tf - t_mark;
                }
                // block f does not hold: its sub-blocks (those that hold elements of the segment)
                const int nsub = rem - f * kXsBlk >= kXsBlk ? kXsSubs : (rem - f * kXsBlk + kXsSub - 1) / kXsSub;
                const XsLane sub = xs_decode(lane < kXsSubs ? L.sub[slot][f * kXsSubs + lane] : xs_never(), nsub, lane);
                int j = 0;
                while (j < nsub) {
                    const int q = xs_run(acc, sub, j, nsub, lane);
                    if (q >= nsub) break;
                    // sub-block q does not hold: its elements, in order (one broadcast read of all 16)
                    const int e0 = f * kXsBlk + q * kXsSub;
                    const int n_e = rem - e0 < kXsSub ? rem - e0 : kXsSub;
                    const float4* p = reinterpret_cast<const float4*>(el + e0);
                    const float4 a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
                    const float ev[16] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w,
                                          a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
#pragma unroll
                    for (int t = 0; t < kXsSub; ++t)
                        if (t < n_e) acc = acc + ev[t];
                    j = q + 1;
                }
                if (MODE == 3) {
                    t_mark = clock64();
                    cyc_fail += t_mark - tf;
                }
                i = f + 1;
            }
            if (MODE == 3) {
                const long long t = clock64();
                cyc_run += t - t_mark;
                t_mark = t;
            }
        }
        if (w0 + kXsWin < nb) store(slot ^ 1);  // the other slot was last read in the previous window
        __syncthreads();
    }
    if (tid == 0) out[(int64_t)k * S + s] = acc;
    if (MODE == 3 && tid == 0) {
        cyc_stage += clock64() - t_mark;
        out[(int64_t)nseg * S + 4 * s] = (float)cyc_run;
        out[(int64_t)nseg * S + 4 * s + 1] = (float)cyc_fail;
        out[(int64_t)nseg * S + 4 * s + 2] = (float)cyc_stage;
    }
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
