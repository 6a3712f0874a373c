// plane_ransac.hip -- SACSegmentation::segment (SACMODEL_PLANE, SAC_RANSAC) for batches of frames
// on gfx950.  Replaces the PCL call at src/segmentation_services/plane_segmentation_srv.cpp:67 and
// supports_segmentation_srv.cpp:110 (reference paths).  Pipeline per batch:
//
//   k_hypothesize   sampler-table attempts -> isSampleGood -> compacted plane hypotheses (A2)
//   k_score  x C    inlier counts of H hypotheses per (frame, 2048-point tile), points held in
//                   VGPRs and reused across the H hypotheses, wave ballot + s_bcnt1 counting
//   k_replay x C    PCL's serial best / adaptive-k logic over the chunk's counts (A5); builds
//                   the next chunk's active-frame list on the device (no host round trip)
//   k_decide        model / refinement decision per frame
//   k_refine        per frame: winning model's inliers streamed in order into the nine exact-order
//                   float accumulators + eigen33 (A6, A7), then the refined model's ascending
//                   inlier list (one 2-wave block per frame)
//   k_finalize      per-frame pitt_plane_result
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "ctx.hpp"
#include "device_common.hpp"
#include "score_list_asm.inc"
#include "xsum.hpp"

#pragma clang fp contract(off)

namespace pitt {

// Sampler attempts per frame (table triples).  Only memory bounds it: the table is 12 B per attempt
// and per distinct point count, generated on the host once per (n, seed, attempts).
constexpr int kMaxAttempts = 1 << 24;

struct FrameMeta {
    int64_t off;    // first point (multiple of 4)
    int64_t n;      // points
    int64_t tab;    // sampler table offset (int32 units)
    int32_t tiles;  // ceil(n / kTile)
    int32_t pad;
};

struct FrameState {
    double k;
    int32_t it, best_count, best_h, done;
    int32_t n_avail, exhausted, flags, status;
    int32_t has_model, need_refine, pad0, pad1;
    // hypothesis generation so far (hyp_extend): attempts examined, good samples before the
    // 1000-rejection cut-off, the current run of rejections, and whether generation has ended
    int32_t gen_att, gen_good, gen_run, gen_done;
};

struct ChunkStat {
    int32_t frames;
    int32_t tiles;
    int64_t points;
};

// Bytes a data-dependent kernel actually moved, counted on the device only while profiling (acct
// non-null): kAcShards slots per kernel so that concurrent waves rarely hit the same address.
enum { kAcHyp = 0, kAcReplay = 1, kAcRefine = 2, kAcSelMark = 3, kAcSelWrite = 4, kAcKernels = 5 };
constexpr int kAcShards = 64;
__device__ __forceinline__ void acct_add(unsigned long long* acct, int k, unsigned long long bytes) {
    if (acct && bytes) atomicAdd(&acct[k * kAcShards + (blockIdx.x & (kAcShards - 1))], bytes);
}

// Debug builds (-DPITT_SYNC_CHECK): every batch stamps its frame metadata with a call sequence number,
// and k_hypothesize compares the stamp it reads with the one the host wrote into a pinned (host-
// coherent) word just before the launch.  A mismatch means the batch's kernels started before the
// metadata copy enqueued ahead of them had landed: k_hypothesize records it and every later kernel of
// the path returns at entry, so stale metadata is reported instead of being indexed with.
#ifdef PITT_SYNC_CHECK
__device__ unsigned int g_dbg_stale;
__device__ unsigned int g_dbg_seen[4];
#define PITT_DBG_GUARD()                                                  \
    do {                                                                  \
        if (*(volatile unsigned int*)&g_dbg_stale) return;                \
    } while (0)
#else
#define PITT_DBG_GUARD() \
    do {                 \
    } while (0)
#endif

// ------------------------------------------------------------------------------------------
// Hypotheses, generated lazily in windows of kBlock sampler-table attempts.  Attempt a uses table
// triple a (the sampler's draws depend only on (n, seed) until a sample is rejected; rejected
// attempts are simply skipped and hypothesis h is the h-th good attempt).  getSamples gives up
// after 1000 consecutive rejects: good attempts past such a run are never used.  A frame's
// hypotheses are generated only as far as the chunks that score it need them (k_hypothesize for
// the first chunk, k_replay for the next), so a table frame that stops after ~30 hypotheses
// examines ~256 attempts instead of max_iterations + slack.
struct GenLds {
    uint32_t bits[kBlock / 32];
    int32_t wpre[kBlock / 32];
    FrameState s;
};

// One block: extend frame f's hypotheses until n_avail >= target or generation ends.  G.s holds
// the frame's state (read and written by thread 0 only, between barriers).
template <int ORDER, int DIV>
__device__ void hyp_extend(GenLds& G, int f, const FrameMeta& m, const float* __restrict__ X,
                           const float* __restrict__ Y, const float* __restrict__ Z,
                           const int32_t* __restrict__ tab, int A, int hcap, int target,
                           float4* __restrict__ hyp_coef, int32_t* __restrict__ hyp_attempt) {
    const float* x = X + m.off;
    const float* y = Y + m.off;
    const float* z = Z + m.off;
    __syncthreads();
    while (G.s.n_avail < target && !G.s.gen_done) {
        const int a0 = G.s.gen_att;  // multiple of kBlock
        const int a = a0 + (int)threadIdx.x;
        bool good = false;
        float4 cf = make_float4(0.f, 0.f, 0.f, 0.f);
        if (a < A) {
            const int i0 = tab[3 * a], i1 = tab[3 * a + 1], i2 = tab[3 * a + 2];
            const float3 p0 = make_float3(x[i0], y[i0], z[i0]);
            const float3 p1 = make_float3(x[i1], y[i1], z[i1]);
            const float3 p2 = make_float3(x[i2], y[i2], z[i2]);
            good = sample_good(p0, p1, p2);
            if (good) cf = plane_from3<ORDER, DIV>(p0, p1, p2);
        }
        const uint64_t bw = __builtin_amdgcn_ballot_w64(good);
        if ((threadIdx.x & 63) == 0) {
            G.bits[2 * (threadIdx.x >> 6)] = (uint32_t)bw;
            G.bits[2 * (threadIdx.x >> 6) + 1] = (uint32_t)(bw >> 32);
        }
        __syncthreads();
        if (threadIdx.x == 0) {  // the serial getSamples scan over the window's 32-attempt words
            FrameState& st = G.s;
            int good_n = st.gen_good, run = st.gen_run, cut = 0;
            for (int w = 0; w < kBlock / 32; ++w) {
                const int nbits = min(32, A - (a0 + 32 * w));
                G.wpre[w] = good_n;
                if (cut || nbits <= 0) continue;
                const uint32_t word = G.bits[w];
                if (word == 0u) {
                    run += nbits;
                    if (run >= 1000) cut = 1;
                    continue;
                }
                const int tz = __builtin_ctz(word);
                if (run + tz >= 1000) { cut = 1; continue; }
                good_n += __builtin_popcount(word);
                run = nbits - 1 - (31 - __builtin_clz(word));
            }
            st.gen_att = min(A, a0 + kBlock);
            st.gen_good = good_n;
            st.gen_run = run;
            st.n_avail = min(good_n, hcap);
            if (cut) {  // "No samples could be selected!": RANSAC stops at hypothesis good_n
                st.gen_done = 1;
            } else if (st.gen_att >= A) {  // the table ran out first (documented limit)
                st.gen_done = 1;
                st.exhausted = good_n < hcap ? 1 : 0;
            } else if (good_n >= hcap) {
                st.gen_done = 1;
            }
        }
        __syncthreads();
        if (good) {
            const int w = (int)threadIdx.x >> 5;
            const int h = G.wpre[w] + __builtin_popcount(G.bits[w] & ((1u << (threadIdx.x & 31)) - 1u));
            if (h < G.s.n_avail && h < G.s.gen_good) {
                hyp_coef[(int64_t)f * hcap + h] = cf;
                hyp_attempt[(int64_t)f * hcap + h] = a;
            }
        }
        __syncthreads();
    }
}

// k_hypothesize: one block per frame -- initial state and the first chunk's hypotheses.
template <int ORDER, int DIV>
__global__ __launch_bounds__(kBlock) void k_hypothesize(
    const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
    const FrameMeta* __restrict__ meta, const int32_t* __restrict__ tables, int A, int hcap, int target,
    int runnable_all, float4* __restrict__ hyp_coef, int32_t* __restrict__ hyp_attempt,
    FrameState* __restrict__ st, int32_t* __restrict__ list0, int32_t* __restrict__ cnt0,
    ChunkStat* __restrict__ stat0, unsigned long long* __restrict__ acct, const unsigned int* dbg_seq) {
    __shared__ GenLds G;
    const int f = blockIdx.x;
    const FrameMeta m = meta[f];
#ifdef PITT_SYNC_CHECK
    {
        __shared__ int stale;
        if (threadIdx.x == 0) {
            const unsigned int want = dbg_seq ? *(const volatile unsigned int*)dbg_seq : (unsigned int)m.pad;
            stale = (unsigned int)m.pad != want;
            if (stale) {
                g_dbg_seen[0] = (unsigned int)m.pad;
                g_dbg_seen[1] = want;
                g_dbg_seen[2] = (unsigned int)m.n;
                g_dbg_seen[3] = (unsigned int)f;
                __threadfence();
                atomicExch(&g_dbg_stale, 1u);
            }
        }
        __syncthreads();
        if (stale || *(volatile unsigned int*)&g_dbg_stale) return;
    }
#else
    (void)dbg_seq;
#endif
    const bool runnable = runnable_all && m.n >= 3;
    if (threadIdx.x == 0) {
        FrameState& s = G.s;
        s.k = 1.0;
        s.it = 0;
        s.best_count = -INT_MAX;
        s.best_h = -1;
        s.done = 0;
        s.n_avail = 0;
        s.exhausted = 0;
        s.flags = 0;
        s.status = PITT_OK;
        s.has_model = 0;
        s.need_refine = 0;
        s.pad0 = s.pad1 = 0;
        s.gen_att = s.gen_good = s.gen_run = 0;
        s.gen_done = runnable ? 0 : 1;
    }
    if (runnable) hyp_extend<ORDER, DIV>(G, f, m, X, Y, Z, tables + m.tab, A, hcap, target, hyp_coef, hyp_attempt);
    __syncthreads();
    if (threadIdx.x == 0) {
        FrameState s = G.s;
        if (!runnable) {
            s.done = 1;
            s.status = PITT_NO_MODEL;
        } else if (s.n_avail == 0) {  // generation ended without a single sample
            s.done = 1;
            s.status = s.exhausted ? PITT_E_SAMPLER : PITT_NO_MODEL;
            s.pad0 = s.exhausted ? 0 : 1;
        }
        st[f] = s;
        if (!s.done) {
            const int idx = atomicAdd(cnt0, 1);
            list0[idx] = f;
            atomicAdd(&stat0->tiles, m.tiles);
            atomicAdd((unsigned long long*)&stat0->points, (unsigned long long)m.n);
        }
        // attempts examined: 3 table indices + 3 gathered points; hypotheses written: 16 + 4 B
        acct_add(acct, kAcHyp, (unsigned long long)s.gen_att * 48ull + (unsigned long long)s.n_avail * 20ull);
    }
}

// ------------------------------------------------------------------------------------------
// k_score: inlier counts of the chunk's hypotheses per (active frame, 2048-point tile), one wave
// per item, 4 waves per block, one block per 4 items (the grid covers every frame's tiles; waves
// past the active items exit at once).  The wave walks its tile in kSubs sub-steps of kGPS groups
// of 64 points; lane l holds point 64 g + l of group g, so one VALU instruction covers exactly one
// group and a (group, hypothesis) pair can be skipped as a whole.  Per sub-step:
//
//   1. box: the groups' bounding boxes (permlane32/16 swaps, then a DPP all-reduce inside each
//      16-lane row: row g of the six box registers = group g's box);
//   2. cull: 16 hypotheses per round, lane 16 g + h' tests hypothesis 16 r + h' against group g's
//      box; a miss is certified only when every point of the box clears the threshold by a margin
//      far above any rounding (box_clear below), so a culled pair counts 0 exactly;
//   3. score: every surviving pair in PCL's float order -- 3 mul + 3 add (no FMA) + |d| < t --
//      ballot -> s_bcnt1, the count written to lane 16 g + h' and accumulated in the wave's LDS row.
//
// On the table scenes ~27 % of the (64-point group, hypothesis) pairs survive (~21 % hold an
// inlier), so a 32-hypothesis chunk costs less VALU than 16 unculled hypotheses.  Coefficients and
// the threshold are VGPR operands (a wave64 VALU op reading an SGPR issues at half rate on gfx950,
// tools/microbench/valu_asm.hip): the item's coefficients are staged into the wave's LDS row and
// read back by broadcast ds_read_b128.
constexpr int kGrp = 64;                   // points per culling group (one per lane)
constexpr int kGPS = 4;                    // groups per sub-step (permlane32 + permlane16 swaps)
constexpr int kSub = kGrp * kGPS;          // points per sub-step
constexpr int kSubs = kTile / kSub;        // sub-steps per item
constexpr int kRnd = 16;                   // hypotheses tested per round (16-lane rows)
constexpr int kWaves = kBlock / 64;
#ifndef PITT_SCORE_WAVES
#define PITT_SCORE_WAVES 2
#endif
constexpr int kScoreWaves = PITT_SCORE_WAVES;  // waves (items) per k_score block
#ifndef PITT_SCORE_DEPTH
#define PITT_SCORE_DEPTH 2  // register sets of points in flight in k_score (3: an A/B variant)
#endif
#ifndef PITT_LIST_PIPE
#define PITT_LIST_PIPE 1  // software-pipelined 32-entry list walks (0: a pair's counts before the next pair)
#endif
#ifndef PITT_SCORE_MERGE
#define PITT_SCORE_MERGE 1  // two 16-hypothesis rounds per pass, 32-entry survivor lists (0: one round per pass)
#endif
constexpr bool kScoreMerge = PITT_SCORE_MERGE != 0;
constexpr int kListRows = kScoreMerge ? 32 : 16;  // LDS rows of one group's survivor list
constexpr int kMaxScoreChunk = 256;        // hypotheses per k_score launch (NST <= 4)
#ifndef PITT_SCORE_GRID_CAP
#define PITT_SCORE_GRID_CAP (256 * 32)
#endif
constexpr int kScoreGridCap = PITT_SCORE_GRID_CAP;  // blocks of a later chunk's launch (~ resident capacity)
// PITT_SCORE_EXPERIMENT (undefined in every library build): measurement-only variants that drop parts
// of k_score to time the rest, with wrong counts by design: 1 no list walks,
// 2 the group boxes only, 3 no stores, 4 no count stores.
#if defined(PITT_SCORE_EXPERIMENT) && (defined(PITT_AB_VARIANTS) || !defined(PITT_MEASUREMENT_ONLY))
#error "PITT_SCORE_EXPERIMENT builds give wrong counts: build them only with -DPITT_MEASUREMENT_ONLY, outside the product and A/B libraries"
#endif

struct SubPts {
    float x[kGPS], y[kGPS], z[kGPS];
};

// One entry of a later chunk's work list, written by the k_replay that lists the frame: everything
// k_score needs to resolve the frame's items in one load (instead of the list entry, then the frame's
// metadata and state behind it).
struct ScoreSlot {
    int64_t off, n;  // the frame's first point and points
    int32_t f;       // the frame
    int32_t tiles;
    int32_t h;       // hypotheses of the chunk the frame can still need (resolve_item's limit)
    int32_t pad;
};

struct ScoreItem {
    int64_t base;  // first point of the tile (global)
    int32_t rem;   // points of the frame from the tile start, clamped to kTile
    int32_t f, t;
    int32_t h;     // hypotheses of this chunk the frame can still need
};

__device__ __forceinline__ void load_sub(const float* __restrict__ X, const float* __restrict__ Y,
                                         const float* __restrict__ Z, int64_t p0, int lane, SubPts& P) {
#pragma unroll
    for (int g = 0; g < kGPS; ++g) {
        const int64_t i = p0 + g * kGrp + lane;
        P.x[g] = X[i];
        P.y[g] = Y[i];
        P.z[g] = Z[i];
    }
}

// Box arithmetic in asm: clang's fminf/fmaxf canonicalise every operand first (an extra v_max
// per input), and IEEE v_min/v_max already skip quiet-NaN operands.
__device__ __forceinline__ float vmin(float a, float b) {
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float vmax(float a, float b) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float vmaxabs(float a, float b) {
    float r;
    asm("v_max_f32_e64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// v_permlane32_swap: a's lanes 32..63 <-> b's lanes 0..31.  v_permlane16_swap: a's odd rows <->
// b's even rows (rows of 16 lanes).
__device__ __forceinline__ void swap32(float& a, float& b) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}
__device__ __forceinline__ void swap16(float& a, float& b) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}

// Row g of lo/hi = the 16-lane partial of group g (v0..v3 = groups 0..3, one point per lane).  The
// first swaps are undone afterwards (one swap instead of two register copies): the groups' points
// stay in place for the scoring.
__device__ __forceinline__ void coord_box(float& v0, float& v1, float& v2, float& v3, float& lo, float& hi) {
    swap32(v0, v2);  // v0 = [g0 lanes 0-31 | g2 lanes 0-31], v2 = [g0 32-63 | g2 32-63]
    float mn02 = vmin(v0, v2), mx02 = vmax(v0, v2);
    swap32(v0, v2);
    swap32(v1, v3);
    float mn13 = vmin(v1, v3), mx13 = vmax(v1, v3);
    swap32(v1, v3);
    swap16(mn02, mn13);  // rows of mn02 = [g0, g1, g2, g3] halves, mn13 the other halves
    lo = vmin(mn02, mn13);
    swap16(mx02, mx13);
    hi = vmax(mx02, mx13);
}

struct RowBox {
    float lo[3], hi[3];
};

// All-reduce inside each 16-lane row (row_ror 8, 4, 2, 1), the six registers interleaved so that
// every DPP read is 5 VALU ops behind the write of its source (gfx9 needs 2 wait states).
__device__ __forceinline__ void row_reduce(RowBox& B) {
    asm("s_nop 4\n"
#define PITT_RR(K)                                                                 \
        "v_min_f32_dpp %0, %0, %0 row_ror:" #K " row_mask:0xf bank_mask:0xf\n"      \
        "v_min_f32_dpp %1, %1, %1 row_ror:" #K " row_mask:0xf bank_mask:0xf\n"      \
        "v_min_f32_dpp %2, %2, %2 row_ror:" #K " row_mask:0xf bank_mask:0xf\n"      \
        "v_max_f32_dpp %3, %3, %3 row_ror:" #K " row_mask:0xf bank_mask:0xf\n"      \
        "v_max_f32_dpp %4, %4, %4 row_ror:" #K " row_mask:0xf bank_mask:0xf\n"      \
        "v_max_f32_dpp %5, %5, %5 row_ror:" #K " row_mask:0xf bank_mask:0xf\n"
        PITT_RR(8) PITT_RR(4) PITT_RR(2) PITT_RR(1)
#undef PITT_RR
        : "+v"(B.lo[0]), "+v"(B.lo[1]), "+v"(B.lo[2]), "+v"(B.hi[0]), "+v"(B.hi[1]), "+v"(B.hi[2]));
}

// Culling geometry of one box (row layout): centre, half extent and the magnitude bound M.
struct RowGeo {
    float c[3], h[3], m;
};

__device__ __forceinline__ RowGeo row_geo(const RowBox& B) {
    RowGeo G;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        G.c[k] = 0.5f * (B.lo[k] + B.hi[k]);
        G.h[k] = 0.5f * (B.hi[k] - B.lo[k]);
    }
    G.m = vmax(vmaxabs(B.lo[0], B.hi[0]), vmax(vmaxabs(B.lo[1], B.hi[1]), vmaxabs(B.lo[2], B.hi[2])));
    return G;
}

// True when every point p of the box certainly fails PCL's |c . (p, 1)| < t.  Exact bound over the
// box: |d(p)| >= |d(centre)| - sum |c_k| h_k.  Every rounding here and in PCL's own float evaluation
// is below 1e-6 of S = |w| + (|a| + |b| + |c|) M (M bounds every |coordinate| of the box), so a
// margin of 1e-5 S (+1e-30 for denormal-scale scenes) certifies the miss.  NaN or infinite boxes
// (an all-NaN group, infinite coordinates) never compare true, so they are never culled.
__device__ __forceinline__ bool box_clear(const RowGeo& G, float4 c, float tv) {
    const float n1 = fabsf(c.x) + fabsf(c.y) + fabsf(c.z);
    const float s = __builtin_fmaf(n1, G.m, fabsf(c.w) + 1e-25f);
    const float lim = __builtin_fmaf(1e-5f, s, tv);
    const float dc = __builtin_fmaf(c.x, G.c[0], __builtin_fmaf(c.y, G.c[1], __builtin_fmaf(c.z, G.c[2], c.w)));
    const float rr = __builtin_fmaf(fabsf(c.x), G.h[0], __builtin_fmaf(fabsf(c.y), G.h[1], fabsf(c.z) * G.h[2]));
    return fabsf(dc) - rr > lim;
}

// True when every point p of the box certainly passes PCL's |c . (p, 1)| < t: |d(p)| <= |d(centre)| +
// sum |c_k| h_k, with box_clear's margin on the other side (1e-5 S below t).  A point with a NaN
// coordinate never widens the box and never counts (its distance is NaN), so such a pair counts the
// group's all-non-NaN points exactly.  NaN or infinite boxes never compare true.
__device__ __forceinline__ bool box_inside(const RowGeo& G, float4 c, float tv) {
    const float n1 = fabsf(c.x) + fabsf(c.y) + fabsf(c.z);
    const float s = __builtin_fmaf(n1, G.m, fabsf(c.w) + 1e-25f);
    const float lim = __builtin_fmaf(-1e-5f, s, tv);
    const float dc = __builtin_fmaf(c.x, G.c[0], __builtin_fmaf(c.y, G.c[1], __builtin_fmaf(c.z, G.c[2], c.w)));
    const float rr = __builtin_fmaf(fabsf(c.x), G.h[0], __builtin_fmaf(fabsf(c.y), G.h[1], fabsf(c.z) * G.h[2]));
    return fabsf(dc) + rr < lim;
}

// v_writelane_b32 (the compiler routes an SGPR lane select through m0: gfx9's constant bus takes
// one SGPR operand)
__device__ int writelane(int val, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

// One float4 of LDS at a byte address held in a VGPR (ds_read_b128).
__device__ __forceinline__ float4 lds_row(uint32_t addr) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v v = *(const __attribute__((address_space(3))) f4v*)(uintptr_t)addr;
    return make_float4(v.x, v.y, v.z, v.w);
}

// The same through a volatile read: it is issued where it stands (not sunk past a branch).
__device__ __forceinline__ float4 lds_row_v(uint32_t addr) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v v = *(const volatile __attribute__((address_space(3))) f4v*)(uintptr_t)addr;
    return make_float4(v.x, v.y, v.z, v.w);
}

// PCL's count of one group for one hypothesis (A3 order, no FMA).
template <int ORDER>
__device__ __forceinline__ int count_group(float4 c, float x, float y, float z, float tv) {
    return __builtin_popcountll(__builtin_amdgcn_ballot_w64(fabsf(plane_dot<ORDER>(c, x, y, z)) < tv));
}

// Item it -> (frame, tile).  Tiles past a shorter frame's end (ragged batches) are empty items.
//
// Hypotheses per frame: RandomSampleConsensus evaluates hypothesis it only while it < k, and k
// never grows once a hypothesis has been scored (a larger best count means a smaller k), so past
// the first chunk the frame needs at most ceil(k) - h0 of this chunk's hypotheses (and no more
// than it has samples for).  The first chunk is scored whole: k is still the initial 1.0 there.
// ident: the list holds every frame of the batch (the first chunk of a batch without degenerate
// frames), so list slot li is scored as frame li -- the same items in another order, without the
// dependent load of the list entry at every wave's start.
__device__ __forceinline__ ScoreItem resolve_item(int it, int tiles_max, const int32_t* __restrict__ list,
                                                  const FrameMeta* __restrict__ meta,
                                                  const FrameState* __restrict__ st, int h0, int H, bool ident) {
    ScoreItem r;
    const int li = it / tiles_max;
    const int t = it - li * tiles_max;
    const int f = ident ? li : __builtin_amdgcn_readfirstlane(list[li]);
    const FrameMeta m = meta[f];
    const bool ok = t < m.tiles;
    r.base = m.off + (ok ? (int64_t)t * kTile : 0);
    r.rem = ok ? (int32_t)min(m.n - (int64_t)t * kTile, (int64_t)kTile) : 0;
    r.f = f;
    r.t = t;
    int h = ok ? H : 0;
    if (ok && h0 > 0) {
        const double k = st[f].k;
        const int need = k < (double)(h0 + H) ? (int)ceil(k) - h0 : H;  // hypotheses hh < k
        h = max(0, min(h, min(need, st[f].n_avail - h0)));
    }
    r.h = __builtin_amdgcn_readfirstlane(h);
    return r;
}

// The same for a later chunk's item from its list slot (k_replay wrote the frame's limit there).
__device__ __forceinline__ ScoreItem resolve_slot(int it, int tiles_max, const ScoreSlot* __restrict__ slots, int H) {
    ScoreItem r;
    const int li = it / tiles_max;
    const int t = it - li * tiles_max;
    const ScoreSlot sl = slots[li];
    const bool ok = t < sl.tiles;
    r.base = sl.off + (ok ? (int64_t)t * kTile : 0);
    r.rem = ok ? (int32_t)min(sl.n - (int64_t)t * kTile, (int64_t)kTile) : 0;
    r.f = sl.f;
    r.t = t;
    r.h = __builtin_amdgcn_readfirstlane(ok ? min(sl.h, H) : 0);
    return r;
}

typedef float f4v __attribute__((ext_vector_type(4)));

// The surviving hypotheses of group GR, compacted in ascending order into its 16-entry LDS list
// (lb + 16 kListRows GR): entry k is scored in PCL's float order and its count written to lane 16 GR + k of
// vc (PCL order A3, no FMA).  Hand-scheduled (tools/gen_score_asm.py -> score_list_asm.inc): two
// entries per step as two interleaved chains, the next two rows already in flight, an odd list's
// first entry alone; the lane of every count is an immediate (no m0), so the scalar work per entry
// is its s_bcnt1 and half a loop test.
template <int ORDER, int GR>
__device__ __forceinline__ void score_list(uint32_t lb, int c, float x, float y, float z, float tv, int& vc) {
    if (c == 0) return;
    uint32_t base;  // ds_read's address operand lives in a VGPR
    asm("v_mov_b32 %0, %1" : "=v"(base) : "s"(lb + 16u * kListRows * GR));
    float d0, t0, d1, t1;
    uint64_t m0, m1;
    uint32_t n0, n1;
#define PITT_LIST_OPERANDS                                                                              \
    : [d0] "=&v"(d0), [t0] "=&v"(t0), [d1] "=&v"(d1), [t1] "=&v"(t1), [m0] "=&s"(m0), [m1] "=&s"(m1),  \
      [n0] "=&s"(n0), [n1] "=&s"(n1), [vc] "+v"(vc)                                                     \
    : [base] "v"(base), [c] "s"(c), [x] "v"(x), [y] "v"(y), [z] "v"(z), [tv] "v"(tv), [L] "n"(16 * GR) \
    : "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69",  \
      "v70", "v71", "scc", "memory"
    if constexpr (ORDER == 0) asm volatile(PITT_SCORE_LIST_ASM_0 PITT_LIST_OPERANDS);
    else if constexpr (ORDER == 1) asm volatile(PITT_SCORE_LIST_ASM_1 PITT_LIST_OPERANDS);
    else asm volatile(PITT_SCORE_LIST_ASM_2 PITT_LIST_OPERANDS);
#undef PITT_LIST_OPERANDS
}

// PITT_SCORE_MERGE: the same over a 32-entry list (two rounds' survivors of group GR, lb + 512 GR);
// entry k's count lands in lane 16 GR + k of vc (k < 16) or lane 16 GR + k - 16 of vc2.
template <int ORDER, int GR>
__device__ __forceinline__ void score_list32(uint32_t lb, int c, float x, float y, float z, float tv, int& vc,
                                             int& vc2) {
    if (c == 0) return;
    uint32_t base;
    asm("v_mov_b32 %0, %1" : "=v"(base) : "s"(lb + 512u * GR));
    float d0, t0, d1, t1;
    uint64_t m0, m1;
    uint32_t n0, n1;
#if PITT_LIST_PIPE
    // the software-pipelined walk (gen_score_asm.py, _P): a pair's count chain under the next pair's dots
    float e0, e1;
#define PITT_LIST_OPERANDS                                                                              \
    : [d0] "=&v"(d0), [t0] "=&v"(t0), [d1] "=&v"(d1), [t1] "=&v"(t1), [e0] "=&v"(e0), [e1] "=&v"(e1),  \
      [m0] "=&s"(m0), [m1] "=&s"(m1), [n0] "=&s"(n0), [n1] "=&s"(n1), [vc] "+v"(vc), [vc2] "+v"(vc2)    \
    : [base] "v"(base), [c] "s"(c), [x] "v"(x), [y] "v"(y), [z] "v"(z), [tv] "v"(tv), [L] "n"(16 * GR) \
    : "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69",  \
      "v70", "v71", "scc", "memory"
    if constexpr (ORDER == 0) asm volatile(PITT_SCORE_LIST32_ASM_P_0 PITT_LIST_OPERANDS);
    else if constexpr (ORDER == 1) asm volatile(PITT_SCORE_LIST32_ASM_P_1 PITT_LIST_OPERANDS);
    else asm volatile(PITT_SCORE_LIST32_ASM_P_2 PITT_LIST_OPERANDS);
#else
#define PITT_LIST_OPERANDS                                                                              \
    : [d0] "=&v"(d0), [t0] "=&v"(t0), [d1] "=&v"(d1), [t1] "=&v"(t1), [m0] "=&s"(m0), [m1] "=&s"(m1),  \
      [n0] "=&s"(n0), [n1] "=&s"(n1), [vc] "+v"(vc), [vc2] "+v"(vc2)                                    \
    : [base] "v"(base), [c] "s"(c), [x] "v"(x), [y] "v"(y), [z] "v"(z), [tv] "v"(tv), [L] "n"(16 * GR) \
    : "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69",  \
      "v70", "v71", "scc", "memory"
    if constexpr (ORDER == 0) asm volatile(PITT_SCORE_LIST32_ASM_0 PITT_LIST_OPERANDS);
    else if constexpr (ORDER == 1) asm volatile(PITT_SCORE_LIST32_ASM_1 PITT_LIST_OPERANDS);
    else asm volatile(PITT_SCORE_LIST32_ASM_2 PITT_LIST_OPERANDS);
#endif
#undef PITT_LIST_OPERANDS
}

// One sub-step: box, cull, score.  wc: the wave's LDS count row, [round][16 g + h'].
// INS: a pair whose box lies certainly inside the slab (box_inside) is not scored point by point;
// it counts the group's points with no NaN coordinate (gcnt, one ballot per group and sub-step).
// BOX, the last sub-step of an item (last): the item's staged boxes go to HBM here (gbox: its 32 group
// boxes, tbox: its tile box), before the sub-step's scoring.
template <int ORDER, bool BOX, bool INS>
__device__ __forceinline__ void score_sub(const float4* cl, float4* wl, int Hf, SubPts& P, int rem, float tv, int lane,
                                          int32_t* __restrict__ wc, float& tb, float* __restrict__ gbox,
                                          uint32_t gsrc, bool last = false, float* __restrict__ tbox = nullptr) {
    if (__builtin_expect(rem < kSub, 0)) {  // frame tail: points past it never count, never widen a box
#pragma unroll
        for (int g = 0; g < kGPS; ++g)
            if (g * kGrp + lane >= rem) P.x[g] = P.y[g] = P.z[g] = __builtin_nanf("");
    }
    // INS: this lane's group's points with three non-NaN coordinates, counted in the first round that
    // certifies a pair of the sub-step (x + y + z is NaN iff a coordinate is NaN, or when infinities of
    // both signs meet, and an infinite coordinate never lets its group's box certify)
    int gcnt = 0;
    bool have_gcnt = false;
    auto count_groups = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int g = 0; g < kGPS; ++g) {
            const float sxyz = P.x[g] + P.y[g] + P.z[g];
            const int cg = __builtin_popcountll(__builtin_amdgcn_ballot_w64(sxyz == sxyz));
            gcnt = (lane >> 4) == g ? cg : gcnt;
        }
    };
    RowBox B;
    if constexpr (BOX) {
        coord_box(P.x[0], P.x[1], P.x[2], P.x[3], B.lo[0], B.hi[0]);
        coord_box(P.y[0], P.y[1], P.y[2], P.y[3], B.lo[1], B.hi[1]);
        coord_box(P.z[0], P.z[1], P.z[2], P.z[3], B.lo[2], B.hi[2]);
        row_reduce(B);
        // the four groups' boxes, for the later chunks and the final selection: row g holds group g's
        // six values; its first lane stages them in the wave's LDS box rows (written to HBM once per
        // item: a global store here would sit in vmcnt between the sub-steps' loads, and every later
        // wait for a load would wait for its write acknowledgement too)
        if ((lane & 15) == 0) {
            typedef __attribute__((address_space(3))) float lf;
            lf* row = (lf*)(uintptr_t)(gsrc + 32u * (uint32_t)(lane >> 4));
            row[0] = B.lo[0];
            row[1] = B.lo[1];
            row[2] = B.lo[2];
            row[3] = B.hi[0];
            row[4] = B.hi[1];
            row[5] = B.hi[2];
        }
        const int i = lane & 15;
        (void)tb;
#if defined(PITT_SCORE_EXPERIMENT) && PITT_SCORE_EXPERIMENT == 3
        if (false) {  // measurement only: no box stores
#else
        if (last) {
#endif
            // the item's boxes are complete: write them now, before this sub-step's scoring, so the
            // stores are acknowledged while the wave still scores (a store left at the wave's end holds
            // its slot until the acknowledgement: ~10 % of the first chunk, tools/microbench/tile_stream)
            const uint32_t base = gsrc - 128u * (kSubs - 1);  // the item's staged rows, 32 groups x 8 floats
            const f4v q = *(const __attribute__((address_space(3))) f4v*)(uintptr_t)(base + 16u * (uint32_t)lane);
            reinterpret_cast<f4v*>(gbox)[lane] = q;  // 32 group boxes, 1 KB
            // the tile box: value i (< 6) folded over the 32 groups (NaN-free min / max, as the groups')
            float t = *(const __attribute__((address_space(3))) float*)(uintptr_t)(base + 4u * (uint32_t)(i < 6 ? i : 0));
#pragma unroll 8
            for (int j = 1; j < kTile / kGrp; ++j) {
                const float u = *(const __attribute__((address_space(3))) float*)(uintptr_t)(base + 32u * j + 4u * (uint32_t)(i < 6 ? i : 0));
                t = i < 3 ? vmin(t, u) : vmax(t, u);
            }
            if (lane < 8) tbox[lane] = t;  // the whole 32-byte sector (values 6, 7: padding)
        }
    } else {
        // later chunks: the boxes the first chunk stored, staged in LDS at the item's start (row g of
        // the row layout = group g: a broadcast read per row, no reduction)
        typedef float f2v __attribute__((ext_vector_type(2)));
        const uint32_t a = gsrc + 32u * (uint32_t)(lane >> 4);
        const f4v q = *(const __attribute__((address_space(3))) f4v*)(uintptr_t)a;
        const f2v r = *(const __attribute__((address_space(3))) f2v*)(uintptr_t)(a + 16u);
        B.lo[0] = q.x;
        B.lo[1] = q.y;
        B.lo[2] = q.z;
        B.hi[0] = q.w;
        B.hi[1] = r.x;
        B.hi[2] = r.y;
    }
    const RowGeo G = row_geo(B);
    const int rounds = (Hf + kRnd - 1) / kRnd;
    const uint32_t lrow = (uint32_t)(uintptr_t)wl + 16u * kListRows * (uint32_t)(lane >> 4);  // this lane's group list
#if defined(PITT_SCORE_EXPERIMENT) && PITT_SCORE_EXPERIMENT == 2
    // measurement only (wrong counts): the box and nothing else
    asm volatile("" ::"v"(G.c[0]), "v"(G.c[1]), "v"(G.c[2]), "v"(G.h[0]), "v"(G.h[1]), "v"(G.h[2]), "v"(G.m));
    return;
#endif
    if constexpr (kScoreMerge && !INS) {
        // rounds r, r + 1 in one pass: round r's survivors of group g take list slots 0.. in ascending
        // order, round r + 1's follow them (slot = round r's survivor count of the row + rank)
        const uint32_t lb = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uintptr_t)wl);
        for (int r = 0; r < rounds; r += 2) {
            const int hl = kRnd * r + (lane & (kRnd - 1));
            const float4 c0 = cl[min(hl, Hf - 1)];
            const float4 c1 = cl[min(hl + kRnd, Hf - 1)];
            const int nb0 = min(kRnd, Hf - kRnd * r);
            const int nb1 = max(0, min(kRnd, Hf - kRnd * (r + 1)));
            const uint64_t valid0 = (((uint64_t)1 << nb0) - 1) * 0x0001000100010001ull;
            const uint64_t valid1 = (((uint64_t)1 << nb1) - 1) * 0x0001000100010001ull;
            const uint64_t need0 = __builtin_amdgcn_ballot_w64(!box_clear(G, c0, tv)) & valid0;
            const uint64_t need1 = __builtin_amdgcn_ballot_w64(!box_clear(G, c1, tv)) & valid1;
            if ((need0 | need1) == 0) continue;
            const uint32_t below = (1u << (lane & 15)) - 1u;
            const uint32_t row0 = (uint32_t)(need0 >> (lane & 48)) & 0xFFFFu;
            const uint32_t row1 = (uint32_t)(need1 >> (lane & 48)) & 0xFFFFu;
            const bool mine0 = (row0 >> (lane & 15)) & 1u, mine1 = (row1 >> (lane & 15)) & 1u;
            const int k0 = __builtin_popcount(row0 & below);
            const int k1 = __builtin_popcount(row0) + __builtin_popcount(row1 & below);
            if (mine0) *(__attribute__((address_space(3))) f4v*)(uintptr_t)(lrow + 16u * (uint32_t)k0) = f4v{c0.x, c0.y, c0.z, c0.w};
            if (mine1) *(__attribute__((address_space(3))) f4v*)(uintptr_t)(lrow + 16u * (uint32_t)k1) = f4v{c1.x, c1.y, c1.z, c1.w};
            int vc = 0, vc2 = 0;
#define PITT_ROWC(g) (__builtin_popcount((uint32_t)(need0 >> (16 * (g))) & 0xFFFFu) + \
                      __builtin_popcount((uint32_t)(need1 >> (16 * (g))) & 0xFFFFu))
#if defined(PITT_SCORE_EXPERIMENT) && PITT_SCORE_EXPERIMENT == 1
            // measurement only (wrong counts): the cull and compaction without the list walks
            asm volatile("" : "+v"(vc), "+v"(vc2) : "s"(PITT_ROWC(0) + PITT_ROWC(1) + PITT_ROWC(2) + PITT_ROWC(3)), "v"(lb));
#else
            score_list32<ORDER, 0>(lb, PITT_ROWC(0), P.x[0], P.y[0], P.z[0], tv, vc, vc2);
            score_list32<ORDER, 1>(lb, PITT_ROWC(1), P.x[1], P.y[1], P.z[1], tv, vc, vc2);
            score_list32<ORDER, 2>(lb, PITT_ROWC(2), P.x[2], P.y[2], P.z[2], tv, vc, vc2);
            score_list32<ORDER, 3>(lb, PITT_ROWC(3), P.x[3], P.y[3], P.z[3], tv, vc, vc2);
#endif
#undef PITT_ROWC
            // back to the hypothesis lanes: round r's count from slot k0 (< 16, in vc), round r + 1's
            // from slot k1 (vc below 16, vc2 from 16)
            const int got0 = __builtin_amdgcn_ds_bpermute(4 * ((lane & 48) + k0), vc);
            const int ga = __builtin_amdgcn_ds_bpermute(4 * ((lane & 48) + (k1 & 15)), vc);
            const int gb = __builtin_amdgcn_ds_bpermute(4 * ((lane & 48) + (k1 & 15)), vc2);
            wc[64 * r + lane] += mine0 ? got0 : 0;
            if (r + 1 < rounds) wc[64 * (r + 1) + lane] += mine1 ? (k1 < 16 ? ga : gb) : 0;
        }
        return;
    }
    for (int r = 0; r < rounds; ++r) {
        const int hl = kRnd * r + (lane & (kRnd - 1));
        const float4 cr = cl[min(hl, Hf - 1)];
        const int nb = min(kRnd, Hf - kRnd * r);  // valid hypotheses of this round
        const uint64_t valid = (((uint64_t)1 << nb) - 1) * 0x0001000100010001ull;
        const bool clr = box_clear(G, cr, tv);
        bool ins = false;
        if constexpr (INS) {
            ins = !clr && ((valid >> lane) & 1u) && box_inside(G, cr, tv);
            if (!have_gcnt && __builtin_amdgcn_ballot_w64(ins) != 0) {  // wave-uniform
                count_groups();
                have_gcnt = true;
            }
        }
        const int add_in = ins ? gcnt : 0;
        const uint64_t need = __builtin_amdgcn_ballot_w64(!clr && !ins) & valid;
        if (need == 0) {
            if constexpr (INS)
                if (ins) wc[64 * r + lane] += add_in;
            continue;
        }
        // compaction: the surviving hypotheses of group g, in ascending order, into list slots
        // 16 g + k (k = the bit's rank inside its 16-lane row)
        const bool mine = (need >> lane) & 1u;
        const uint32_t rowbits = (uint32_t)(need >> (lane & 48));
        const int k = __builtin_popcount(rowbits & ((1u << (lane & 15)) - 1u));
        if (mine) *(__attribute__((address_space(3))) f4v*)(uintptr_t)(lrow + 16u * (uint32_t)k) = f4v{cr.x, cr.y, cr.z, cr.w};
        // each list in order; entry k's count lands in lane 16 g + k of vc
        int vc = 0;
        const uint32_t lb = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uintptr_t)wl);
        score_list<ORDER, 0>(lb, __builtin_popcount((uint32_t)need & 0xFFFFu), P.x[0], P.y[0], P.z[0], tv, vc);
        score_list<ORDER, 1>(lb, __builtin_popcount((uint32_t)(need >> 16) & 0xFFFFu), P.x[1], P.y[1], P.z[1], tv, vc);
        score_list<ORDER, 2>(lb, __builtin_popcount((uint32_t)(need >> 32) & 0xFFFFu), P.x[2], P.y[2], P.z[2], tv, vc);
        score_list<ORDER, 3>(lb, __builtin_popcount((uint32_t)(need >> 48)), P.x[3], P.y[3], P.z[3], tv, vc);
        // back to the hypothesis lanes: lane 16 g + h' reads lane 16 g + k
        const int got = __builtin_amdgcn_ds_bpermute(4 * ((lane & 48) + k), vc);
        wc[64 * r + lane] += (mine ? got : 0) + add_in;
    }
}

// First-chunk scoring with per-lane counters (H <= 32): the same box and certified cull as score_sub,
// then every surviving (group, hypothesis) pair is scored with full-rate VALU only -- PCL's six
// float ops, |d| - t (VOP3 abs modifier) and the sign bit added into lane-private counter cnt[h].
// Exact: with denormals kept, fl(|d| - t) < 0 iff |d| < t (a nonzero difference never rounds to
// zero; equality gives +0), and a NaN |d| (or t) gives a NaN with a clear sign bit.  The pairs are
// dispatched by scalar bit tests on the cull mask (hypotheses with no surviving group in the
// sub-step are skipped with one test), so no compaction, no SGPR count, no v_writelane; the
// counters are reduced across the wave once per item.
template <int ORDER>
__device__ __forceinline__ void score_sub_lane(const float4* cl, int Hf, SubPts& P, int rem, float tv, int lane,
                                               uint32_t (&cnt)[8], float& tb, float* __restrict__ gbox) {
    if (__builtin_expect(rem < kSub, 0)) {
#pragma unroll
        for (int g = 0; g < kGPS; ++g)
            if (g * kGrp + lane >= rem) P.x[g] = P.y[g] = P.z[g] = __builtin_nanf("");
    }
    RowBox B;
    coord_box(P.x[0], P.x[1], P.x[2], P.x[3], B.lo[0], B.hi[0]);
    coord_box(P.y[0], P.y[1], P.y[2], P.y[3], B.lo[1], B.hi[1]);
    coord_box(P.z[0], P.z[1], P.z[2], P.z[3], B.lo[2], B.hi[2]);
    row_reduce(B);
    {
        const int i = lane & 15;
        float v = B.lo[0];
        v = i == 1 ? B.lo[1] : v;
        v = i == 2 ? B.lo[2] : v;
        v = i == 3 ? B.hi[0] : v;
        v = i == 4 ? B.hi[1] : v;
        v = i == 5 ? B.hi[2] : v;
        if (i < 6) gbox[(lane >> 4) * 8 + i] = v;
        tb = i < 3 ? vmin(tb, v) : vmax(tb, v);
    }
    const RowGeo G = row_geo(B);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        if (kRnd * r >= Hf) break;
        const int hl = kRnd * r + (lane & (kRnd - 1));
        const float4 cr = cl[min(hl, Hf - 1)];
        const int nb = min(kRnd, Hf - kRnd * r);
        const uint64_t valid = (((uint64_t)1 << nb) - 1) * 0x0001000100010001ull;
        const uint64_t need = __builtin_amdgcn_ballot_w64(!box_clear(G, cr, tv)) & valid;
        // bit 16 g + h' of need: group g survives hypothesis 16 r + h'.  Word w holds groups 2 w, 2 w + 1.
        const uint32_t w0 = (uint32_t)need, w1 = (uint32_t)(need >> 32);
        const uint32_t hany = (w0 | (w0 >> 16) | w1 | (w1 >> 16)) & 0xFFFFu;
        if (hany == 0) continue;
        // coefficient rows read two hypotheses ahead (LDS broadcast), whether or not they are needed
        float4 c0 = lds_row_v((uint32_t)(uintptr_t)(cl + kRnd * r));
        float4 c1 = lds_row_v((uint32_t)(uintptr_t)(cl + kRnd * r + 1));
#pragma unroll
        for (int hh = 0; hh < kRnd; ++hh) {
            const float4 c = c0;
            c0 = c1;
            if (hh + 2 < kRnd) c1 = lds_row_v((uint32_t)(uintptr_t)(cl + kRnd * r + hh + 2));
            if (!((hany >> hh) & 1u)) continue;
            const int h = kRnd * r + hh;
#pragma unroll
            for (int g = 0; g < kGPS; ++g) {
                const uint32_t w = g < 2 ? w0 : w1;
                if ((w >> (16 * (g & 1) + hh)) & 1u) {
                    const float d = plane_dot<ORDER>(c, P.x[g], P.y[g], P.z[g]);
                    float sd;
                    asm("v_sub_f32_e64 %0, |%1|, %2" : "=v"(sd) : "v"(d), "v"(tv));
                    // the sign bit into byte h % 4 of counter word h / 4 (<= 32 per lane and item)
                    cnt[h >> 2] += (__float_as_uint(sd) >> 31) << (8 * (h & 3));
                }
            }
        }
    }
}

// The 32 lane-private counters reduced across the wave and stored: out[h] for h < Hf.  Folds with
// permlane32 / permlane16 swaps (32 -> 16 -> 8 registers, each row of 16 lanes one hypothesis), a
// row_ror all-reduce inside the rows, then lane 16 q + i (i < 8) stores hypothesis i + 8 q.
__device__ __forceinline__ uint32_t u32_swap_add32(uint32_t a, uint32_t b) {
    const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    return r[0] + r[1];
}
__device__ __forceinline__ uint32_t u32_swap_add16(uint32_t a, uint32_t b) {
    const auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    return r[0] + r[1];
}
__device__ __forceinline__ uint32_t row_allsum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false);  // row_ror:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xf, 0xf, false);  // row_ror:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x122, 0xf, 0xf, false);  // row_ror:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x121, 0xf, 0xf, false);  // row_ror:1
    return v;
}
__device__ __forceinline__ void store_lane_counts(const uint32_t (&packed)[8], int Hf, int lane, int32_t* __restrict__ out) {
    uint32_t cnt[32], c16[16], c8[8];
#pragma unroll
    for (int h = 0; h < 32; ++h) cnt[h] = (packed[h >> 2] >> (8 * (h & 3))) & 0xFFu;
#pragma unroll
    for (int j = 0; j < 16; ++j) c16[j] = u32_swap_add32(cnt[j], cnt[j + 16]);  // lanes < 32: hyp j; else j + 16
#pragma unroll
    for (int j = 0; j < 8; ++j) c8[j] = u32_swap_add16(c16[j], c16[j + 8]);     // row q: hyp j + 8 q
#pragma unroll
    for (int j = 0; j < 8; ++j) c8[j] = row_allsum(c8[j]);
    const int i = lane & 15, q = lane >> 4;
    uint32_t v = c8[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) v = i == j ? c8[j] : v;
    const int h = i + 8 * q;
    if (i < 8 && h < Hf) out[h] = (int32_t)v;
}

// The item's coefficients into the wave's LDS row (rows past H repeat the last: never counted).
template <int NST>
__device__ __forceinline__ void put_coefs(float4* cl, const float4* __restrict__ hc, int H, int lane) {
    float4 c[NST];
#pragma unroll
    for (int j = 0; j < NST; ++j) c[j] = hc[min(lane + 64 * j, max(H, 1) - 1)];
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < NST; ++j) cl[lane + 64 * j] = c[j];
    asm volatile("" ::: "memory");
}

// BOX (the first chunk only): also record each tile's bounding box -- NaN points never widen it
// -- for k_refine's tile skipping.
#ifndef PITT_SCORE_WPE
// k_score's register budget: 5 waves per SIMD (<= 96 VGPRs; without the bound the first chunk's
// in-loop box flush takes it to 98 and 4 waves)
#define PITT_SCORE_WPE 5
#endif
#if PITT_SCORE_WPE > 0
#define PITT_SCORE_ATTR __attribute__((amdgpu_waves_per_eu(PITT_SCORE_WPE, PITT_SCORE_WPE)))
#else
#define PITT_SCORE_ATTR
#endif
template <int ORDER, int NST, bool BOX, bool LANE = false, bool INS = false>
__global__ __launch_bounds__(64 * kScoreWaves) PITT_SCORE_ATTR void k_score(
    const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
    const FrameMeta* __restrict__ meta, const FrameState* __restrict__ st, const float4* __restrict__ hyp_coef,
    int hcap, int hstride, const int32_t* __restrict__ list, const int32_t* __restrict__ cnt, int tiles_max,
    int h0, int H, float thf, int32_t* __restrict__ tile_counts, float* __restrict__ tile_box,
    float* __restrict__ group_box, int nf, const ScoreSlot* __restrict__ slots) {
    PITT_DBG_GUARD();
    __shared__ float4 wcoef[kScoreWaves][NST * 64];
    __shared__ float4 wlist[kScoreWaves][4 * kListRows];  // four survivor lists, one per group
    __shared__ float4 wbox[kScoreWaves][64];  // the item's 32 group boxes (first chunk: staged for one store)
    __shared__ int32_t wcnt[kScoreWaves][NST * 64 * (64 / kRnd)];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    // The first chunk (BOX) scores every frame of the batch: its items are all nf x tiles_max (frame
    // f = list slot f), with no wait for the active count or the list at the wave's start -- a frame
    // that RANSAC cannot run (n < 3, no good sample) is scored too, and k_replay never reads its
    // counts.  Later chunks score the frames k_replay listed.
    const int nact = BOX ? nf : __builtin_amdgcn_readfirstlane(*cnt);
    const int items = nact * tiles_max;  // < 2^31 (validated)
    const bool ident = BOX;
    float4* cl = wcoef[w];
    float4* wl = wlist[w];
    int32_t* wc = wcnt[w];
    float tv;
    asm volatile("v_mov_b32 %0, %1" : "=v"(tv) : "s"(thf));  // threshold in a VGPR (full-rate v_cmp)
    // items strided over the grid: the grid is sized for the whole batch but capped near the chip's
    // resident capacity, so a later chunk with few active frames (or none) retires quickly
    for (int it = blockIdx.x * kScoreWaves + w; it < items; it += gridDim.x * kScoreWaves) {
    const ScoreItem cur = BOX ? resolve_item(it, tiles_max, list, meta, st, h0, H, ident) : resolve_slot(it, tiles_max, slots, H);
    const int Hf = cur.h;
    if (Hf <= 0) continue;  // an empty item, or a frame that needs none of this chunk
    const int rounds = (Hf + kRnd - 1) / kRnd;
    SubPts P[2];
    // the item's coefficient rows (and, later chunks, its group boxes) are requested before its first
    // points: vmcnt counts in issue order, so staging them into LDS then waits for them alone, not for
    // the points' HBM latency (the next sub-step's loads go out that much sooner)
    float* gb = group_box + ((int64_t)cur.f * tiles_max + cur.t) * (kTile / kGrp) * 8;
    float4 crow[NST], brow;
    {
        const float4* hc = hyp_coef + (int64_t)cur.f * hcap + h0;
#pragma unroll
        for (int j = 0; j < NST; ++j) crow[j] = hc[min(lane + 64 * j, max(Hf, 1) - 1)];  // rows past H repeat the last
        if constexpr (!BOX) brow = reinterpret_cast<const float4*>(gb)[lane];  // the 32 boxes the first chunk wrote
    }
    load_sub(X, Y, Z, cur.base, lane, P[0]);
#pragma unroll
    for (int j = 0; j < NST; ++j) cl[lane + 64 * j] = crow[j];
    if constexpr (!BOX) wbox[w][lane] = brow;
    (void)brow;
    // the count rows stored below: whole 32-count lines (rows past the rounds stay zero)
    const int hw = (Hf + 31) & ~31;
    for (int r = 0; r < hw / kRnd; ++r) wc[64 * r + lane] = 0;
    const uint32_t gsrc = (uint32_t)(uintptr_t)wbox[w];
    float tb = (lane & 15) < 3 ? __builtin_inff() : -__builtin_inff();  // BOX: this lane's tile-box value
    if constexpr (LANE) {  // the first chunk, H <= 32: lane-private counters (score_sub_lane)
        uint32_t cnt[8];  // 32 lane-private counters, 8 bits each
#pragma unroll
        for (int h = 0; h < 8; ++h) cnt[h] = 0;
        for (int s = 0; s < kSubs; s += 2) {
            load_sub(X, Y, Z, cur.base + (s + 1) * kSub, lane, P[1]);
            score_sub_lane<ORDER>(cl, Hf, P[0], cur.rem - s * kSub, tv, lane, cnt, tb, gb + s * kGPS * 8);
            load_sub(X, Y, Z, cur.base + min(s + 2, kSubs - 1) * kSub, lane, P[0]);  // unconditional: see below
            score_sub_lane<ORDER>(cl, Hf, P[1], cur.rem - (s + 1) * kSub, tv, lane, cnt, tb, gb + (s + 1) * kGPS * 8);
        }
        store_lane_counts(cnt, Hf, lane, tile_counts + ((int64_t)cur.f * tiles_max + cur.t) * hstride + h0);
        (void)rounds;
    } else {
#if PITT_SCORE_DEPTH == 3
    // three register sets: sub-steps s + 1 and s + 2 are in flight while s is scored
    static_assert(kSubs == 8, "the 3-deep rotation below is written for 8 sub-steps");
    SubPts P2;
    load_sub(X, Y, Z, cur.base + kSub, lane, P[1]);
    for (int s = 0; s < 6; s += 3) {
        load_sub(X, Y, Z, cur.base + (s + 2) * kSub, lane, P2);
        score_sub<ORDER, BOX, INS>(cl, wl, Hf, P[0], cur.rem - s * kSub, tv, lane, wc, tb, gb + s * kGPS * 8,
                              gsrc + 128u * s);
        load_sub(X, Y, Z, cur.base + (s + 3) * kSub, lane, P[0]);
        score_sub<ORDER, BOX, INS>(cl, wl, Hf, P[1], cur.rem - (s + 1) * kSub, tv, lane, wc, tb, gb + (s + 1) * kGPS * 8,
                              gsrc + 128u * (s + 1));
        load_sub(X, Y, Z, cur.base + (s + 4) * kSub, lane, P[1]);
        score_sub<ORDER, BOX, INS>(cl, wl, Hf, P2, cur.rem - (s + 2) * kSub, tv, lane, wc, tb, gb + (s + 2) * kGPS * 8,
                              gsrc + 128u * (s + 2));
    }
    score_sub<ORDER, BOX, INS>(cl, wl, Hf, P[0], cur.rem - 6 * kSub, tv, lane, wc, tb, gb + 6 * kGPS * 8, gsrc + 128u * 6);
    score_sub<ORDER, BOX, INS>(cl, wl, Hf, P[1], cur.rem - 7 * kSub, tv, lane, wc, tb, gb + 7 * kGPS * 8, gsrc + 128u * 7);
#else
    // sub-steps in pairs: the next sub-step loads into the other register set while this one is
    // scored (a runtime loop: unrolled 8 times the body would not fit the instruction cache).  The
    // second load is unconditional (the last pair reloads sub-step 7, an L2 hit): guarded by
    // s + 2 < kSubs, the compiler's vmcnt at the join had to assume it was not issued, so the
    // second half-step waited for sub-step s + 2's loads before scoring s + 1 (one exposed HBM
    // latency per pair of sub-steps).
    float* tbx = tile_box + ((int64_t)cur.f * tiles_max + cur.t) * 8;
    for (int s = 0; s < kSubs; s += 2) {
        load_sub(X, Y, Z, cur.base + (s + 1) * kSub, lane, P[1]);
        score_sub<ORDER, BOX, INS>(cl, wl, Hf, P[0], cur.rem - s * kSub, tv, lane, wc, tb, gb, gsrc + 128u * s);
        load_sub(X, Y, Z, cur.base + min(s + 2, kSubs - 1) * kSub, lane, P[0]);
        // BOX: the last sub-step writes the item's group and tile boxes before its scoring
        score_sub<ORDER, BOX, INS>(cl, wl, Hf, P[1], cur.rem - (s + 1) * kSub, tv, lane, wc, tb, gb,
                                   gsrc + 128u * (s + 1), s + 2 == kSubs, tbx);
    }
#endif
    // counts: hypothesis h = 16 r + h' sums its four groups' lanes of round r
    asm volatile("" ::: "memory");
    int32_t* out = tile_counts + ((int64_t)cur.f * tiles_max + cur.t) * hstride + h0;
#pragma unroll
    for (int j = 0; j < NST; ++j) {
        const int h = lane + 64 * j;
#if defined(PITT_SCORE_EXPERIMENT) && (PITT_SCORE_EXPERIMENT == 3 || PITT_SCORE_EXPERIMENT == 4)
        if (h < hw && wc[h] == 0x7fffffff) {  // measurement only: no count stores
#else
        if (h < hw) {
#endif
            const int32_t* row = wc + 64 * (h / kRnd) + (h % kRnd);
            out[h] = row[0] + row[16] + row[32] + row[48];
        }
    }
    }  // !LANE
#if PITT_SCORE_DEPTH == 3
    constexpr bool kBoxesAtEnd = true;
#else
    constexpr bool kBoxesAtEnd = LANE;  // the 2-deep loop writes them inside its last sub-step
#endif
    if constexpr (BOX && kBoxesAtEnd) {
        if constexpr (!LANE) reinterpret_cast<float4*>(gb)[lane] = wbox[w][lane];  // the item's 32 group boxes, 1 KB
        // rows -> tile: value i of the four rows combined (xor 16, xor 32)
#pragma unroll
        for (int off = 16; off <= 32; off <<= 1) {
            const float o = __shfl_xor(tb, off, 64);
            tb = (lane & 15) < 3 ? vmin(tb, o) : vmax(tb, o);
        }
        if (lane < 8) tile_box[((int64_t)cur.f * tiles_max + cur.t) * 8 + lane] = tb;
    }
    }
}

// ------------------------------------------------------------------------------------------
// k_replay: RandomSampleConsensus::computeModel's serial control over the chunk's counts.
// A frame that goes on to the next chunk first gets that chunk's hypotheses (hyp_extend up to
// target_next), so every scored hypothesis index is below n_avail unless generation has ended.
template <int ORDER, int DIV>
__global__ __launch_bounds__(kBlock) void k_replay(
    const int32_t* __restrict__ tile_counts, int hcap, int hstride, int tiles_max, int h0, int H, int max_iter,
    double log_probability, const FrameMeta* __restrict__ meta, FrameState* __restrict__ st,
    int32_t* __restrict__ hyp_total, int32_t* __restrict__ next_list, int32_t* __restrict__ next_cnt,
    ChunkStat* __restrict__ next_stat, const float* __restrict__ X, const float* __restrict__ Y,
    const float* __restrict__ Z, const int32_t* __restrict__ tables, int A, int target_next,
    float4* __restrict__ hyp_coef, int32_t* __restrict__ hyp_attempt, unsigned long long* __restrict__ acct,
    ScoreSlot* __restrict__ next_slot) {
    PITT_DBG_GUARD();
    __shared__ GenLds G;
    __shared__ int32_t part[kBlock / 64][kMaxChunk];
    __shared__ int32_t tot[kMaxChunk];
    const int f = blockIdx.x;
    if (st[f].done) return;
    const FrameMeta m = meta[f];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // the hypotheses k_score scored for this frame (resolve_item's limit); the loop below stops
    // before any later one
    int Hn = H;
    if (h0 > 0) {
        const double k = st[f].k;
        const int need = k < (double)(h0 + H) ? (int)ceil(k) - h0 : H;
        Hn = max(0, min(H, min(need, st[f].n_avail - h0)));
    }
    // per-tile count rows summed with lanes across hypotheses (coalesced rows), waves across tiles
    const int32_t* base = tile_counts + (int64_t)f * tiles_max * hstride + h0;
    for (int h = lane; h < Hn; h += 64) {
        int acc = 0;
        for (int t = w; t < m.tiles; t += kBlock / 64) acc += base[(int64_t)t * hstride + h];
        part[w][h] = acc;
    }
    __syncthreads();
    for (int h = threadIdx.x; h < Hn; h += kBlock) {
        int acc = 0;
#pragma unroll
        for (int k = 0; k < kBlock / 64; ++k) acc += part[k][h];
        tot[h] = acc;
    }
    __syncthreads();
    if (threadIdx.x == 0) G.s = st[f];
    __syncthreads();
    const int att0 = G.s.gen_att, avail0 = G.s.n_avail;
    if (threadIdx.x != 0) goto extend;
    {
    FrameState& s = G.s;
    const double one_over_indices = 1.0 / (double)m.n;
    const double eps = 2.220446049250313e-16;
    for (int h = 0; h < H; ++h) {
        const int hh = h0 + h;
        if (!((double)s.it < s.k)) { s.done = 1; break; }
        if (hh >= s.n_avail) {
            if (s.exhausted) s.status = PITT_E_SAMPLER;
            else s.pad0 = 1;  // getSamples: 1000 consecutive rejections, "No samples could be selected!"
            s.done = 1;
            break;
        }
        const int c = tot[h];
        hyp_total[(int64_t)f * hcap + hh] = c;
        if (c > s.best_count) {
            s.best_count = c;
            s.best_h = hh;
            const double w = (double)c * one_over_indices;
            // w^3 rounded once (pow(w, 3.0)): exact double-double cube, then one rounding.
            const double w2 = w * w, w2l = fma(w, w, -w2);
            const double w3 = w2 * w, w3l = fma(w2, w, -w3) + w2l * w;
            double p = 1.0 - (w3 + w3l);
            p = fmax(eps, p);
            p = fmin(1.0 - eps, p);
            s.k = log_probability / log(p);
            const double r = rint(s.k);
            if (fabs(s.k - r) <= 1e-9 * fmax(1.0, s.k) && r >= 1.0 && r <= (double)max_iter + 1.0)
                s.flags |= PITT_FLAG_K_NEAR_INTEGER;
        }
        s.it++;
        if (s.it > max_iter) { s.done = 1; break; }
    }
    if (!s.done && !((double)s.it < s.k)) s.done = 1;
    }
extend:
    __syncthreads();
    if (!G.s.done && G.s.n_avail < target_next)
        hyp_extend<ORDER, DIV>(G, f, m, X, Y, Z, tables + m.tab, A, hcap, target_next, hyp_coef, hyp_attempt);
    if (threadIdx.x == 0) {
        const FrameState s = G.s;
        st[f] = s;
        if (!s.done) {
            const int idx = atomicAdd(next_cnt, 1);
            next_list[idx] = f;
            // the next chunk's limit for this frame (resolve_item's, with the state just decided)
            const int hn0 = h0 + H, Hn1 = max(0, target_next - hn0);
            const int need = s.k < (double)(hn0 + Hn1) ? (int)ceil(s.k) - hn0 : Hn1;
            next_slot[idx] = ScoreSlot{m.off, m.n, f, m.tiles, max(0, min(Hn1, min(need, s.n_avail - hn0))), 0};
            atomicAdd(&next_stat->tiles, m.tiles);
            atomicAdd((unsigned long long*)&next_stat->points, (unsigned long long)m.n);
        }
        // count rows read, totals written, and the next chunk's hypotheses generated
        acct_add(acct, kAcReplay, (unsigned long long)Hn * (unsigned long long)m.tiles * 4ull + (unsigned long long)Hn * 4ull +
                                      (unsigned long long)(s.gen_att - att0) * 48ull +
                                      (unsigned long long)(s.n_avail - avail0) * 20ull);
    }
}

// ------------------------------------------------------------------------------------------
// After the chunks: decide model / refinement per frame (one thread per frame).  A batch may run its
// chunks in two phases (run_plane_batch: the chunks recent batches needed, then -- only when a frame is
// still running -- the rest): phase p decides the frames that have finished and are not decided yet
// (FrameState.pad1 = the phase that decided the frame), and k_refine refines only those.
__global__ void k_decide(const FrameMeta* __restrict__ meta, FrameState* __restrict__ st,
                         const float4* __restrict__ hyp_coef, int hcap, int n_frames, int optimize,
                         float4* __restrict__ best_coef, float4* __restrict__ final_coef, int phase) {
    PITT_DBG_GUARD();
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= n_frames) return;
    FrameState s = st[f];
    if (!s.done || s.pad1 != 0) return;  // still running (a later phase decides it), or decided already
    s.pad1 = phase;
    s.has_model = (s.best_h >= 0 && s.status == PITT_OK) ? 1 : 0;
    if (!s.has_model && s.status == PITT_OK) s.status = PITT_NO_MODEL;
    s.need_refine = (s.has_model && optimize && s.best_count >= 4) ? 1 : 0;
    if (s.has_model) {
        const float4 c = hyp_coef[(int64_t)f * hcap + s.best_h];
        best_coef[f] = c;
        final_coef[f] = c;  // overwritten by k_refine
    }
    st[f] = s;
    (void)meta;
}

// ------------------------------------------------------------------------------------------
// k_refine: optimizeModelCoefficients (A6/A7) for one frame, one (P + 2)-wave block per frame.
//
//   producers  P waves stream the frame's tiles that hold inliers of the winning hypothesis, step
//              s going to producer s % P (4 points per lane per 256-point step, a global_load_lds
//              ring kRDepth steps deep per producer); each selects the step's inliers on its own
//              and, in step order (a ticket in LDS), appends their coordinates -- ascending -- to
//              the inlier ring;
//   former     forms the six products of each full 256-inlier block (xx, xy, xz, yy, yz, zz, each
//              separately rounded as PCL) with all 64 lanes into a product slot;
//   chain      lanes 0..8 run the nine float accumulators of computeMeanAndCovarianceMatrix in
//              exact PCL order as pure dependent adds; lane 0 then divides (Eigen 3.2
//              `accu /= n`), runs eigen33 and writes the refined plane.
//
// The chain's 9 dependent float streams bound the frame at ~1.9 ns per inlier.  One producer
// (~0.45 us per step) stalls the chain across the runs of steps with few inliers, which one ring
// cannot buffer; P producers select P steps at once and serialise only the append.
// The waves hand over ring space through LDS counters (WS: step ticket | produced, F: formed,
// R: summed).  The final inlier list of every frame (refined or not) is the job of k_sel_mark /
// k_sel_write.
constexpr int kRChunk = 256;   // points per producer step (4 per lane)
constexpr int kRSlot = 3 * kRChunk;          // floats per raw ring slot (x, y, z)
#ifndef PITT_REFINE_DEPTH
#define PITT_REFINE_DEPTH 4
#endif
constexpr int kRDepth = PITT_REFINE_DEPTH;  // raw steps in flight per producer
#ifndef PITT_REFINE_RING
#define PITT_REFINE_RING 1024
#endif
constexpr int kRRing = PITT_REFINE_RING;  // compacted-inlier ring (points, a power of two)
#ifndef PITT_REFINE_BLK
#define PITT_REFINE_BLK 256
#endif
constexpr int kRBlk = PITT_REFINE_BLK;  // chain block (a multiple of 256): products formed by all lanes, then the chains
static_assert(kRBlk % 256 == 0 && kRRing % kRBlk == 0, "chain blocks of 256-element parts that tile the ring");
// producer waves: k_refine<.., P> is instantiated for P = 1..4, pitt_ctx::refine_producers picks

#ifndef PITT_REFINE_MAX_TILES
#define PITT_REFINE_MAX_TILES ((1 << 21) / kTile)
#endif
constexpr int kRMaxTiles = PITT_REFINE_MAX_TILES;  // tile list capacity (larger frames stream every tile)
constexpr int kRStepsPerTile = kTile / kRChunk;

// The nine chain lanes read nine different streams at the same offset in one ds_read_b128: the
// streams' strides are padded by 4 floats so that they start on different LDS banks (unpadded,
// all nine land on one bank group and each read serialises).
constexpr int kRS = kRRing + 4;  // ring stream stride (x | y | z), floats
constexpr int kPS = kRBlk + 4;   // product stream stride, floats

constexpr int kRProdSlots = 2;   // product blocks formed ahead of the chain

template <int P>
struct RefineLds {
    float pool[P * kRDepth * kRSlot + 3 * kRS];  // raw[P][kRDepth] | cx | cy | cz (stride kRS)
    float prod[kRProdSlots][6 * kPS];    // xx, xy, xz, yy, yz, zz of the next chain blocks
    int tl[kRMaxTiles];             // the pass's tiles that can hold inliers, ascending
    // produced inliers (low word) | steps appended (high word), written as one 64-bit LDS store:
    // the former and the chain read the low word, a producer waits for its step's ticket
    alignas(8) unsigned long long WS;
    int R, F, done, total, nact;    // consumed (chain), formed (products)
    float4 coef;
};

// True when no point in the tile's bounding box can satisfy |d| < thf for plane c: the extremes of
// the exact plane value over the box (double) clear the threshold by more than any rounding of
// PCL's float evaluation (<= 4 ulp of |a x| + |b y| + |c z| + |w|; the margin is 1e-5 of it).
// An empty box (no finite point) holds no inliers; boxes with infinities never clear.
__device__ __forceinline__ bool box_misses_slab(const float* __restrict__ b, float4 c, float thf) {
    const double lo[3] = {b[0], b[1], b[2]}, hi[3] = {b[3], b[4], b[5]};
    if (!(lo[0] <= hi[0])) return true;
    const double cc[3] = {c.x, c.y, c.z};
    double dmin = c.w, dmax = c.w, sc = fabs((double)c.w);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double a = cc[k] * lo[k], z = cc[k] * hi[k];
        dmin += fmin(a, z);
        dmax += fmax(a, z);
        sc += fabs(cc[k]) * fmax(fabs(lo[k]), fabs(hi[k]));
    }
    const double lim = (double)thf + 1e-5 * sc + 1e-30;
    return dmin > lim || dmax < -lim;
}

// The tile list in LDS (ascending): tiles where the winning hypothesis counted inliers during
// scoring (exact).  Returns the number of tiles, or -1 (stream every tile) for frames beyond the
// list's capacity.
template <class LDS>
__device__ __forceinline__ int refine_tiles(LDS& L, int tiles, int lane,
                                            const int32_t* __restrict__ best_counts, int hstride) {
    if (tiles > kRMaxTiles) return -1;
    int nact = 0;
    for (int g = 0; g < tiles; g += 64) {
        const int t = g + lane;
        bool act = false;
        if (t < tiles) act = best_counts[(int64_t)t * hstride] > 0;
        const uint64_t b = __builtin_amdgcn_ballot_w64(act);
        const int pre = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
        if (act) L.tl[nact + pre] = t;
        nact += __builtin_popcountll(b);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    return nact;
}

// Step s of the pass -> step of the frame, through a cursor that reads the tile list once per tile
// (tile: the list position it holds; base: that tile's first frame step).  The list is read in
// asm: a visible LDS read would make the compiler wait for the ring's in-flight global_load_lds
// writes.
struct StepCursor {
    int tile = -1;
    int base = 0;
};

template <class LDS>
__device__ __forceinline__ int refine_step(LDS& L, int s, int nact, StepCursor& cur) {
    if (nact < 0) return s;
    const int ti = s / kRStepsPerTile;
    if (ti != cur.tile) {
        const uint32_t a = (uint32_t)(uintptr_t)&L.tl[ti];
        int t;
        asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(t) : "v"(a) : "memory");
        cur.tile = ti;
        cur.base = __builtin_amdgcn_readfirstlane(t) * kRStepsPerTile;
    }
    return cur.base + s % kRStepsPerTile;
}

template <int P>
__device__ __forceinline__ float* ring_x(RefineLds<P>& L) { return L.pool + P * kRDepth * kRSlot; }

typedef __attribute__((address_space(3))) volatile int lds_vint;  // ds_read/ds_write, not flat

// Hand-over counters.  LDS executes each wave's operations in issue order, so a counter written
// after the data it covers is seen only after that data, and a counter read before a write is
// performed before it; compiler barriers keep the source order.  (Workgroup-scope acquire/release
// atomics would also wait for the ring's in-flight global loads: vmcnt(0).)
__device__ __forceinline__ int lds_acquire(int* p) {
    asm volatile("" ::: "memory");
    const int v = *(lds_vint*)(p);
    asm volatile("" ::: "memory");
    return v;
}
__device__ __forceinline__ void lds_release(int* p, int v) {
    asm volatile("" ::: "memory");
    *(lds_vint*)(p) = v;
    asm volatile("" ::: "memory");
}

// The 64-bit ticket word, read and written in asm (see refine_step: a visible LDS access in the
// producer would wait for its in-flight global_load_lds writes).
__device__ __forceinline__ unsigned long long lds_ticket_read(const unsigned long long* p) {
    unsigned long long v;
    asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((uint32_t)(uintptr_t)p) : "memory");
    return v;
}
__device__ __forceinline__ void lds_ticket_write(unsigned long long* p, unsigned long long v) {
    asm volatile("ds_write_b64 %0, %1" ::"v"((uint32_t)(uintptr_t)p), "v"(v) : "memory");
}
__device__ __forceinline__ int lds_read_asm(const int* p) {
    int v;
    asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((uint32_t)(uintptr_t)p) : "memory");
    return v;
}

// Producer q's local step j (pass step sb + q + j P) into its ring slot j % kRDepth; steps past
// the range re-read the pass's last step so that every iteration issues the same three loads (the
// waits below are fixed vmcnt counts).
template <class LDS>
__device__ __forceinline__ void refine_issue(LDS& L, float* raw, const float* xs, const float* ys,
                                             const float* zs, int j, int step, int se, int nact, int lane,
                                             StepCursor& cur) {
    typedef __attribute__((address_space(3))) void* lds_ptr;
    const int cc = refine_step(L, min(step, se - 1), nact, cur);
    float* b = raw + (j % kRDepth) * kRSlot;
    const int64_t o = (int64_t)cc * kRChunk + lane * 4;
    __builtin_amdgcn_global_load_lds(xs + o, (lds_ptr)(b), 16, 0, 0);
    __builtin_amdgcn_global_load_lds(ys + o, (lds_ptr)(b + kRChunk), 16, 0, 0);
    __builtin_amdgcn_global_load_lds(zs + o, (lds_ptr)(b + 2 * kRChunk), 16, 0, 0);
}

// Producer q of P: pass steps sb + q, sb + q + P, ... below se with plane c.  Each step's inliers
// are selected independently; the append waits for the step's ticket (the previous step's
// producer has appended), so the ring receives the inliers in ascending order.  The producer of
// the pass's last step publishes the total and `done`.
template <int ORDER, int P>
__device__ __forceinline__ void refine_stream(RefineLds<P>& L, int q, const float* xs, const float* ys,
                                              const float* zs, int64_t n, float4 c, float thf, int lane,
                                              int nact, int sb, int se, uint32_t& spin_ticket, uint32_t& spin_ring,
                                              bool masked) {
    const int nj = se - sb > q ? (se - sb - q + P - 1) / P : 0;
    if (nj == 0) return;
    float* raw = L.pool + q * kRDepth * kRSlot;
    float* rx = ring_x(L);
    float tv;  // threshold and plane in VGPRs: a VALU op reading an SGPR issues at half rate
    asm volatile("v_mov_b32 %0, %1" : "=v"(tv) : "s"(thf));
    asm volatile("" ::"v"(c.x), "v"(c.y), "v"(c.z), "v"(c.w));  // plane in registers before the ring starts
    StepCursor ic, pc;  // issue and process cursors
    int rfree = 0;      // the chain's ring position as last read
#pragma unroll
    for (int k = 0; k < kRDepth - 1; ++k) refine_issue(L, raw, xs, ys, zs, k, sb + q + k * P, se, nact, lane, ic);
    for (int j = 0; j < nj; ++j) {
        const int st = sb + q + j * P;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads of the slot refilled next are done
        refine_issue(L, raw, xs, ys, zs, j + kRDepth - 1, st + (kRDepth - 1) * P, se, nact, lane, ic);
        // step j landed: younger are the kRDepth - 1 steps issued since (3 loads each; the producer
        // issues no other vector-memory op, so the count is exact)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * (kRDepth - 1)) : "memory");
        __builtin_amdgcn_sched_barrier(0);
        const int ch = refine_step(L, st, nact, pc);  // the frame's step
        const uint32_t b = (uint32_t)(uintptr_t)(raw + (j % kRDepth) * kRSlot + lane * 4);
        float4 x4, y4, z4;
        asm volatile(
            "ds_read_b128 %0, %3\n"
            "ds_read_b128 %1, %3 offset:1024\n"
            "ds_read_b128 %2, %3 offset:2048\n"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(x4), "=&v"(y4), "=&v"(z4)
            : "v"(b)
            : "memory");
        float px[4] = {x4.x, x4.y, x4.z, x4.w};
        const float py[4] = {y4.x, y4.y, y4.z, y4.w};
        const float pz[4] = {z4.x, z4.y, z4.z, z4.w};
        const int64_t s0 = (int64_t)ch * kRChunk;
        const int p0 = lane * 4;  // point of the step
        if (s0 + kRChunk > n) {  // the frame's last step: points past its end never count
            const int lim = (int)(n - s0);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (p0 + k >= lim) px[k] = __builtin_nanf("");
        }
        uint32_t bits = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            bits |= (fabsf(plane_dot<ORDER>(c, px[k], py[k], pz[k])) < tv ? 1u : 0u) << k;
        // ascending positions: exclusive prefix of the per-lane counts (0..4) from their bit slices
        const int cnt = __builtin_popcount(bits);
        const uint64_t b0 = __builtin_amdgcn_ballot_w64((cnt & 1) != 0);
        const uint64_t b1 = __builtin_amdgcn_ballot_w64((cnt & 2) != 0);
        const uint64_t b2 = __builtin_amdgcn_ballot_w64((cnt & 4) != 0);
        const uint32_t lo = 0xFFFFFFFFu;
        const int pre = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)(b0 & lo), 0u)) +
                        2 * (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)(b1 & lo), 0u)) +
                        4 * (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b2 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)(b2 & lo), 0u));
        const int tot = __builtin_popcountll(b0) + 2 * __builtin_popcountll(b1) + 4 * __builtin_popcountll(b2);
        // the step's ticket: every earlier step has been appended
        const unsigned long long key = (unsigned long long)(uint32_t)(st - sb);
        unsigned long long ws;
        if constexpr (P == 1) {
            ws = (key << 32) | (uint32_t)lds_ticket_read(&L.WS);  // own previous step: no wait
        } else {
            // uniform (one LDS word): compared in SGPRs, no divergent loop
            while ((uint32_t)__builtin_amdgcn_readfirstlane((int)((ws = lds_ticket_read(&L.WS)) >> 32)) != (uint32_t)key)
            {
                __builtin_amdgcn_s_sleep(0);
                ++spin_ticket;
            }
        }
        const int wpos = (int)(uint32_t)ws;
        // ring space: the chain's position is re-read only when the cached one is too old
        if (wpos + tot - rfree > kRRing) {
            while (wpos + tot - (rfree = lds_read_asm(&L.R)) > kRRing) {
                __builtin_amdgcn_s_sleep(1);
                ++spin_ring;
            }
        }
        int k = wpos + pre;
        if (masked) {  // PITT_REFINE_MODE bit 1: only inlier lanes write (LDS cost per active lane)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if ((bits >> e) & 1u) {
                    const int r = k & (kRRing - 1);
                    rx[r] = px[e];
                    rx[kRS + r] = py[e];
                    rx[2 * kRS + r] = pz[e];
                    ++k;
                }
            }
        } else {
            // branch-free: a point that is not an inlier writes into the streams' padding (never read)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const bool in = (bits >> e) & 1u;
                const int r = in ? (k & (kRRing - 1)) : kRRing;
                rx[r] = px[e];
                rx[kRS + r] = py[e];
                rx[2 * kRS + r] = pz[e];
                k += in ? 1 : 0;
            }
        }
        // after the step's writes (LDS executes a wave's operations in order)
        if (lane == 0) {
            lds_ticket_write(&L.WS, ((key + 1) << 32) | (uint32_t)(wpos + tot));
            if (st == se - 1) {
                L.total = wpos + tot;
                lds_release(&L.done, 1);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the re-read steps land before the block ends
}

// 16 dependent adds, back to back, in order.
__device__ __forceinline__ void chain16(float& s, const float4& a, const float4& b, const float4& c, const float4& d) {
    asm volatile(
        "v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %2\n v_add_f32 %0, %0, %3\n v_add_f32 %0, %0, %4\n"
        "v_add_f32 %0, %0, %5\n v_add_f32 %0, %0, %6\n v_add_f32 %0, %0, %7\n v_add_f32 %0, %0, %8\n"
        "v_add_f32 %0, %0, %9\n v_add_f32 %0, %0, %10\n v_add_f32 %0, %0, %11\n v_add_f32 %0, %0, %12\n"
        "v_add_f32 %0, %0, %13\n v_add_f32 %0, %0, %14\n v_add_f32 %0, %0, %15\n v_add_f32 %0, %0, %16"
        : "+v"(s)
        : "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w), "v"(c.x), "v"(c.y),
          "v"(c.z), "v"(c.w), "v"(d.x), "v"(d.y), "v"(d.z), "v"(d.w));
}

// 8 x ds_read_b128 (32 consecutive floats from LDS byte address a), issued back to back.
__device__ __forceinline__ void lds_read32(f4v (&v)[8], uint32_t a) {
    asm volatile(
        "ds_read_b128 %0, %8\n ds_read_b128 %1, %8 offset:16\n ds_read_b128 %2, %8 offset:32\n"
        "ds_read_b128 %3, %8 offset:48\n ds_read_b128 %4, %8 offset:64\n ds_read_b128 %5, %8 offset:80\n"
        "ds_read_b128 %6, %8 offset:96\n ds_read_b128 %7, %8 offset:112"
        : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7])
        : "v"(a)
        : "memory");
}

// 32 dependent adds, in order.
__device__ __forceinline__ void chain32(float& s, const f4v (&v)[8]) {
#pragma unroll
    for (int t = 0; t < 8; t += 4)
        chain16(s, make_float4(v[t].x, v[t].y, v[t].z, v[t].w), make_float4(v[t + 1].x, v[t + 1].y, v[t + 1].z, v[t + 1].w),
                make_float4(v[t + 2].x, v[t + 2].y, v[t + 2].z, v[t + 2].w),
                make_float4(v[t + 3].x, v[t + 3].y, v[t + 3].z, v[t + 3].w));
}

// The six product streams of the kRBlk ring entries from position r (a multiple of kRBlk: the block
// does not wrap), 256 per pass, each lane four consecutive entries, separately rounded as PCL.
__device__ __forceinline__ void form_block(const float* rx, int r, float* prod, int lane) {
    const int q = r & (kRRing - 1);
#pragma unroll
    for (int h = 0; h < kRBlk / 256; ++h) {
        const int e = q + 256 * h + 4 * lane;
        const float4 x = *reinterpret_cast<const float4*>(rx + e);
        const float4 y = *reinterpret_cast<const float4*>(rx + kRS + e);
        const float4 z = *reinterpret_cast<const float4*>(rx + 2 * kRS + e);
        float4* o = reinterpret_cast<float4*>(prod + 256 * h) + lane;
        constexpr int S = kPS / 4;
        o[0 * S] = make_float4(x.x * x.x, x.y * x.y, x.z * x.z, x.w * x.w);
        o[1 * S] = make_float4(x.x * y.x, x.y * y.y, x.z * y.z, x.w * y.w);
        o[2 * S] = make_float4(x.x * z.x, x.y * z.y, x.z * z.z, x.w * z.w);
        o[3 * S] = make_float4(y.x * y.x, y.y * y.y, y.z * y.z, y.w * y.w);
        o[4 * S] = make_float4(y.x * z.x, y.y * z.y, y.z * z.z, y.w * z.w);
        o[5 * S] = make_float4(z.x * z.x, z.y * z.y, z.z * z.z, z.w * z.w);
    }
}

// Former wave: the six product streams of each full kRBlk-inlier block (formed by all 64 lanes,
// separately rounded as PCL) into a product slot, up to kRProdSlots blocks ahead of the chain.
template <int P>
__device__ __forceinline__ void refine_form(RefineLds<P>& L, int lane, uint32_t& spins) {
    float* rx = ring_x(L);
    int rf = 0, rc = 0;  // formed; the chain's position as last read
    while (true) {
        const int w = lds_acquire(reinterpret_cast<int*>(&L.WS));
        if (w - rf >= kRBlk) {
            if (rf - rc >= kRProdSlots * kRBlk) {  // the slot is still being summed
                rc = lds_acquire(&L.R);
                if (rf - rc >= kRProdSlots * kRBlk) {
                    __builtin_amdgcn_s_sleep(1);
                    ++spins;
                    continue;
                }
            }
            form_block(rx, rf, &L.prod[(rf / kRBlk) % kRProdSlots][0], lane);
            rf += kRBlk;
            if (lane == 0) lds_release(&L.F, rf);  // after the block's writes (in-order LDS)
            continue;
        }
        if (lds_acquire(&L.done) && lds_acquire(reinterpret_cast<int*>(&L.WS)) - rf < kRBlk) break;  // the rest is the chain's tail
        __builtin_amdgcn_s_sleep(1);
        spins += 1u << 16;  // waiting for inliers (high half) vs for a free product slot (low half)
    }
}

// Chain wave: lane k < 9 accumulates stream k of computeMeanAndCovarianceMatrix (xx, xy, xz, yy,
// yz, zz, x, y, z) in ascending inlier order as pure dependent adds, 64 elements per batched read:
// the products from the former's slots, x, y, z from the inlier ring.  Lanes >= 9 repeat lane 0's
// stream (uniform control flow: limiting the reads to 9 active lanes measured slower,
// tools/microbench/chain_rate.hip).  The last partial block goes element by element.
// NOADD (PITT_REFINE_MODE bit 2, a measurement only, results wrong): the reads without the adds.
// PF (bit 3): the former's count is read during the block's second-to-last 64 elements; when the next
// block is formed by then, its first 32 elements load under this block's last 32 adds, so the block
// boundary costs neither the count's round trip nor the first reads' latency.
template <int P>
__device__ __forceinline__ uint32_t chain_addr(RefineLds<P>& L, int k, int r) {
    const int q = r & (kRRing - 1);
    const float* p = k < 6 ? &L.prod[(r / kRBlk) % kRProdSlots][k * kPS] : ring_x(L) + (k - 6) * kRS + q;
    return (uint32_t)(uintptr_t)p;
}

template <int P, bool NOADD = false, bool PF = false>
__device__ __forceinline__ float refine_chain(RefineLds<P>& L, int lane, uint32_t& spins, long long& busy, bool timed) {
    const int k = lane < 9 ? lane : 0;
    float* rx = ring_x(L);
    float s = 0.0f;
    int r = 0;
    f4v A[8], B[8];
    bool pre = false;  // PF: the block at r is formed and its first 32 elements are in flight in A
    while (true) {
        const int formed = pre ? r + kRBlk : lds_acquire(&L.F);
        if (formed - r >= kRBlk) {
            const long long tb = timed ? clock64() : 0;
            // the next 32 elements' reads are in flight while these 32 are added (reads and waits
            // in asm: the compiler would otherwise sink each read to just before its use)
            const uint32_t pa = chain_addr(L, k, r);
            if (!pre) lds_read32(A, pa);
            pre = false;
            bool nxt = false;
#pragma unroll
            for (int i = 0; i < kRBlk / 32; i += 2) {
                lds_read32(B, pa + 128u * (i + 1));
                asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
                if constexpr (NOADD) s += A[0].x; else chain32(s, A);
                if (i + 2 < kRBlk / 32) {
                    int fn = 0;
                    if (PF && i + 4 == kRBlk / 32)
                        asm volatile("ds_read_b32 %0, %1" : "=v"(fn) : "v"((uint32_t)(uintptr_t)&L.F) : "memory");
                    lds_read32(A, pa + 128u * (i + 2));
                    asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");  // B (and the count) landed
                    if (PF && i + 4 == kRBlk / 32) {
                        int fs;
                        asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(fs) : "v"(fn));
                        nxt = fs - (r + kRBlk) >= kRBlk;
                    }
                } else if (PF && nxt) {
                    lds_read32(A, chain_addr(L, k, r + kRBlk));
                    asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");  // B landed; the next A in flight
                } else {
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                }
                if constexpr (NOADD) s += B[0].x; else chain32(s, B);
            }
            r += kRBlk;
            if (lane == 0) lds_release(&L.R, r);
            if (timed) busy += clock64() - tb;
            pre = PF && nxt;
            continue;
        }
        if (lds_acquire(&L.done)) {
            const int wf = lds_acquire(reinterpret_cast<int*>(&L.WS));
            if (wf - r < kRBlk) {  // every full block summed: the tail element by element
                const float* U = (k == 0 || k == 1 || k == 2 || k == 6) ? rx : (k == 3 || k == 4 || k == 7) ? rx + kRS : rx + 2 * kRS;
                const float* V = k == 0 ? rx : (k == 1 || k == 3) ? rx + kRS : rx + 2 * kRS;
                for (; r < wf; ++r) {
                    const int q = r & (kRRing - 1);
                    s += k >= 6 ? U[q] : U[q] * V[q];
                }
                break;
            }
        }
        __builtin_amdgcn_s_sleep(1);
        ++spins;
    }
    return s;
}

// The refined plane from the nine normalised accumulators (accu / n): PCL's float covariance, eigen33
// and d = -(e, 0) . (centroid, 1) (A6/A7).
template <int ORDER>
__device__ float4 refine_plane_mean(const float a9[9]) {
    float cov[9];
    cov[0] = a9[0] - a9[6] * a9[6];
    cov[1] = a9[1] - a9[6] * a9[7];
    cov[2] = a9[2] - a9[6] * a9[8];
    cov[4] = a9[3] - a9[7] * a9[7];
    cov[5] = a9[4] - a9[7] * a9[8];
    cov[8] = a9[5] - a9[8] * a9[8];
    cov[3] = cov[1];
    cov[6] = cov[2];
    cov[7] = cov[5];
    float e[3];
    eigen33(cov, e);
    const float d = -1.0f * red4<ORDER>(e[0] * a9[6], e[1] * a9[7], e[2] * a9[8], 0.0f * 1.0f);
    return make_float4(e[0], e[1], e[2], d);
}

// The refined plane from the nine accumulators (Eigen 3.2 `accu /= n`, then eigen33, A6/A7/A9).
template <int ORDER, int DIV>
__device__ float4 refine_plane(float a9[9], int n) {
    const float fn = (float)n;
    if constexpr (DIV == 0) {  // Eigen 3.2: accu /= n  ==>  accu * (1/n)
        const float r = 1.0f / fn;
#pragma unroll
        for (int k = 0; k < 9; ++k) a9[k] = a9[k] * r;
    } else {
#pragma unroll
        for (int k = 0; k < 9; ++k) a9[k] = a9[k] / fn;
    }
    return refine_plane_mean<ORDER>(a9);
}

template <int ORDER, int DIV, int P>
__global__ __launch_bounds__(64 * (P + 2)) void k_refine(
    const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
    const FrameMeta* __restrict__ meta, const FrameState* __restrict__ st,
    const float4* __restrict__ best_coef, float thf, const int32_t* __restrict__ tile_counts, int hstride,
    int tiles_max, float4* __restrict__ final_coef, unsigned long long* __restrict__ acct,
    unsigned long long* __restrict__ rdbg, int mode, const int32_t* __restrict__ only, int phase) {
    PITT_DBG_GUARD();
    __shared__ RefineLds<P> L;
    const long long t_start = rdbg ? clock64() : 0;
    const int f = blockIdx.x;
    const FrameState s = st[f];
    if (!s.has_model || !s.need_refine || s.pad1 != phase) return;
    if (only && !only[f]) return;  // after k_xrefine: only the frames it handed back
    const FrameMeta m = meta[f];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const float* xs = X + m.off;
    const float* ys = Y + m.off;
    const float* zs = Z + m.off;
    if (wave == 0) {
        const int nact = refine_tiles(L, m.tiles, lane, tile_counts + (int64_t)f * tiles_max * hstride + s.best_h,
                                      hstride);
        const int nsteps = nact < 0 ? (int)((m.n + kRChunk - 1) / kRChunk) : nact * kRStepsPerTile;
        if (lane == 0) {
            L.WS = 0ull;
            L.R = 0;
            L.F = 0;
            L.done = nsteps == 0 ? 1 : 0;  // nothing to stream: no producer publishes
            L.total = 0;
            L.nact = nact;
            L.coef = best_coef[f];
            // the listed tiles' points, their count words, the plane in and out
            acct_add(acct, kAcRefine, (unsigned long long)nsteps * kRChunk * 12ull + (unsigned long long)m.tiles * 4ull + 32ull);
        }
    }
    __syncthreads();
    if (wave < P) {
        const int nact = L.nact;
        const int nsteps = nact < 0 ? (int)((m.n + kRChunk - 1) / kRChunk) : nact * kRStepsPerTile;
        uint32_t spin_ticket = 0, spin_ring = 0;
        refine_stream<ORDER, P>(L, wave, xs, ys, zs, m.n, L.coef, thf, lane, nact, 0, nsteps, spin_ticket, spin_ring,
                                (mode & 2) != 0);
        if (rdbg && lane == 0 && wave < 2) {  // PITT_REFINE_DEBUG: cycles and spin counts per role
            unsigned long long* d = rdbg + (int64_t)f * 16 + 4 + 4 * wave;
            d[0] = (unsigned long long)(clock64() - t_start);
            d[1] = spin_ticket;
            d[2] = spin_ring;
            d[3] = (unsigned long long)nsteps;
        }
    } else if (wave == P) {
        __builtin_amdgcn_s_setprio(2);
        uint32_t spins = 0;
        refine_form(L, lane, spins);
        if (rdbg && lane == 0) {
            rdbg[(int64_t)f * 16 + 2] = (unsigned long long)(clock64() - t_start);
            rdbg[(int64_t)f * 16 + 3] = spins;
        }
    } else {
        // the chain bounds the frame: first call on its SIMD's issue slots
        __builtin_amdgcn_s_setprio(3);
        uint32_t spins = 0;
        long long busy = 0;
#ifdef PITT_AB_VARIANTS
        const float acc = (mode & 4) ? refine_chain<P, true>(L, lane, spins, busy, rdbg != nullptr)
                        : (mode & 8) ? refine_chain<P, false, true>(L, lane, spins, busy, rdbg != nullptr)
                                     : refine_chain<P>(L, lane, spins, busy, rdbg != nullptr);
#else
        const float acc = refine_chain<P>(L, lane, spins, busy, false);  // the product: the exact chain only
#endif
        float a9[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) a9[k] = __shfl(acc, k, 64);
        const int n_in = lds_acquire(reinterpret_cast<int*>(&L.WS));
        if (lane == 0) final_coef[f] = refine_plane<ORDER, DIV>(a9, n_in);
        if (rdbg && lane == 0) {
            rdbg[(int64_t)f * 16 + 0] = (unsigned long long)(clock64() - t_start);
            rdbg[(int64_t)f * 16 + 1] = spins;
            rdbg[(int64_t)f * 16 + 12] = (unsigned long long)n_in;
            rdbg[(int64_t)f * 16 + 13] = (unsigned long long)busy;
        }
    }
}

// ------------------------------------------------------------------------------------------
// k_refine_multi: k_refine for F frames per block with one chain wave for all of them.  What the
// serial chain costs the pipelined chip is its instruction count -- one wave64 v_add per inlier
// with nine useful lanes (measured: the chain's reads without its adds, PITT_REFINE_MODE bit 2,
// took 362k to 430k frames/s at four batches in flight, while k_refine itself only went from 670
// to 554 us).  Here lanes 9 j + k (j < F) run stream k of frame j, so one v_add advances F frames.
// Per frame: a producer wave (refine_stream, unchanged) and its own ring and product slots; one
// former wave forms every frame's product blocks, round robin; the chain takes the next block of
// every frame that has one formed (the others sit out under the exec mask), then each frame's tail
// element by element.  Per frame the same values are added in the same
// order as k_refine: bit-exact with it.
constexpr int kRL1Words = (int)(sizeof(RefineLds<1>) / 4);
// frame j's LDS starts 36 j banks on (nine 4-bank streams per frame): the frames' reads of one
// stream never land on one bank group
constexpr int kRL1Pad = (36 - kRL1Words % 64 + 64) % 64 + 64;
struct RefineLdsP {
    RefineLds<1> L;
    float pad[kRL1Pad];
};

template <int F>
__device__ __forceinline__ void refine_form_multi(RefineLdsP (&LL)[F], int lane) {
    int rf[F], rc[F];
    bool fin[F];
#pragma unroll
    for (int j = 0; j < F; ++j) {
        rf[j] = rc[j] = 0;
        fin[j] = false;
    }
    while (true) {
        bool progress = false, all = true;
#pragma unroll
        for (int j = 0; j < F; ++j) {
            if (fin[j]) continue;
            all = false;
            RefineLds<1>& L = LL[j].L;
            const int w = lds_acquire(reinterpret_cast<int*>(&L.WS));
            if (w - rf[j] >= kRBlk) {
                if (rf[j] - rc[j] >= kRProdSlots * kRBlk) {  // both slots still being summed
                    rc[j] = lds_acquire(&L.R);
                    if (rf[j] - rc[j] >= kRProdSlots * kRBlk) continue;
                }
                form_block(ring_x(L), rf[j], &L.prod[(rf[j] / kRBlk) % kRProdSlots][0], lane);
                rf[j] += kRBlk;
                if (lane == 0) lds_release(&L.F, rf[j]);  // after the block's writes (in-order LDS)
                progress = true;
            } else if (lds_acquire(&L.done) && lds_acquire(reinterpret_cast<int*>(&L.WS)) - rf[j] < kRBlk) {
                fin[j] = true;  // the rest is the chain's tail
            }
        }
        if (all) break;
        if (!progress) __builtin_amdgcn_s_sleep(1);
    }
}

template <int F, bool NOADD>
__device__ __forceinline__ float refine_chain_multi(RefineLdsP (&LL)[F], int lane) {
    const int j = lane < 9 * F ? lane / 9 : 0;
    const int k = lane < 9 * F ? lane - 9 * j : 0;  // lanes >= 9 F repeat frame 0's stream 0
    RefineLds<1>& L = LL[j].L;
    float* rx = ring_x(L);
    float s = 0.0f;
    int r = 0;
    bool fin = false;
    while (true) {
        bool has = false;
        if (!fin) {
            if (lds_acquire(&L.F) - r >= kRBlk) has = true;
            else if (lds_acquire(&L.done) && lds_acquire(reinterpret_cast<int*>(&L.WS)) - r < kRBlk) fin = true;
        }
        // the frames whose next block is formed go on (the others sit out under the exec mask): no
        // frame waits for another's producer
        if (__builtin_amdgcn_ballot_w64(has) == 0) {
            if (__builtin_amdgcn_ballot_w64(!fin) == 0) break;
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        if (has) {
            const int q = r & (kRRing - 1);
            const float* p = k < 6 ? &L.prod[(r / kRBlk) % kRProdSlots][k * kPS] : rx + (k - 6) * kRS + q;
            const uint32_t pa = (uint32_t)(uintptr_t)p;
            f4v A[8], B[8];
            lds_read32(A, pa);
#pragma unroll
            for (int i = 0; i < kRBlk / 32; i += 2) {
                lds_read32(B, pa + 128u * (i + 1));
                asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
                if constexpr (NOADD) s += A[0].x; else chain32(s, A);
                if (i + 2 < kRBlk / 32) {
                    lds_read32(A, pa + 128u * (i + 2));
                    asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
                } else {
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                }
                if constexpr (NOADD) s += B[0].x; else chain32(s, B);
            }
            r += kRBlk;
            if (k == 0 && lane < 9 * F) lds_release(&L.R, r);
        }
    }
    // every full block summed: each frame's tail element by element
    const int wf = lds_acquire(reinterpret_cast<int*>(&L.WS));
    const float* U = (k == 0 || k == 1 || k == 2 || k == 6) ? rx : (k == 3 || k == 4 || k == 7) ? rx + kRS : rx + 2 * kRS;
    const float* V = k == 0 ? rx : (k == 1 || k == 3) ? rx + kRS : rx + 2 * kRS;
    for (; r < wf; ++r) {
        const int q = r & (kRRing - 1);
        s += k >= 6 ? U[q] : U[q] * V[q];
    }
    return s;
}

template <int ORDER, int DIV, int F>
__global__ __launch_bounds__(64 * (F + 2)) void k_refine_multi(
    const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
    const FrameMeta* __restrict__ meta, const FrameState* __restrict__ st,
    const float4* __restrict__ best_coef, float thf, const int32_t* __restrict__ tile_counts, int hstride,
    int tiles_max, int n_frames, float4* __restrict__ final_coef, unsigned long long* __restrict__ acct, int mode) {
    PITT_DBG_GUARD();
    __shared__ RefineLdsP LL[F];
    __shared__ int act[F];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int f0 = blockIdx.x * F;
    int nact = 0, nsteps = 0;
    if (wave < F) {  // wave j: frame f0 + j's tile list and ring state, then its producer
        RefineLds<1>& L = LL[wave].L;
        const int f = f0 + wave;
        bool a = false;
        FrameState s;
        if (f < n_frames) {
            s = st[f];
            a = s.has_model && s.need_refine;
        }
        if (a) {
            const FrameMeta m = meta[f];
            nact = refine_tiles(L, m.tiles, lane, tile_counts + (int64_t)f * tiles_max * hstride + s.best_h, hstride);
            nsteps = nact < 0 ? (int)((m.n + kRChunk - 1) / kRChunk) : nact * kRStepsPerTile;
        }
        if (lane == 0) {
            L.WS = 0ull;
            L.R = 0;
            L.F = 0;
            L.done = nsteps == 0 ? 1 : 0;  // nothing to stream (or no refinement): no producer publishes
            L.total = 0;
            L.nact = nact;
            act[wave] = a ? 1 : 0;
            if (a) {
                L.coef = best_coef[f];
                acct_add(acct, kAcRefine,
                         (unsigned long long)nsteps * kRChunk * 12ull + (unsigned long long)meta[f].tiles * 4ull + 32ull);
            }
        }
    }
    __syncthreads();
    if (wave < F) {
        if (nsteps > 0) {
            RefineLds<1>& L = LL[wave].L;
            const FrameMeta m = meta[f0 + wave];
            uint32_t spin_ticket = 0, spin_ring = 0;
            refine_stream<ORDER, 1>(L, 0, X + m.off, Y + m.off, Z + m.off, m.n, L.coef, thf, lane, nact, 0, nsteps,
                                    spin_ticket, spin_ring, (mode & 2) != 0);
        }
    } else if (wave == F) {
        __builtin_amdgcn_s_setprio(2);
        refine_form_multi<F>(LL, lane);
    } else {
        __builtin_amdgcn_s_setprio(3);
        const float acc = (mode & 4) ? refine_chain_multi<F, true>(LL, lane) : refine_chain_multi<F, false>(LL, lane);
        // lane j < F: frame j's nine sums (lanes 9 j .. 9 j + 8), its plane
        float a9[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) a9[k] = __shfl(acc, (9 * lane + k) & 63, 64);
        if (lane < F && act[lane]) {
            const int n_in = lds_acquire(reinterpret_cast<int*>(&LL[lane].L.WS));
            final_coef[f0 + lane] = refine_plane<ORDER, DIV>(a9, n_in);
        }
    }
}

// ------------------------------------------------------------------------------------------
// k_xrefine: the same nine exact-order float sums (A6: accu[k] += v in ascending inlier order,
// computeMeanAndCovarianceMatrix, called from optimizeModelCoefficients at
// plane_segmentation_srv.cpp:55,67) without one dependent add per inlier ("binade runs").
//
// While a float sum s stays inside one binade [2^e, 2^(e+1)) (or its negative), every add rounds
// to the same grid u = 2^(e-23), and s is a multiple of u.  So fl(s + v) = s + q u with
// q = rint(v / u) whenever the exact sum is not a tie (|v/u - q| != 1/2) and the result stays
// at least one u inside the binade: the rounding does not depend on s.  A run of elements then
// advances s by R u with R = sum q, an integer computed in parallel, and it is valid for the actual
// s exactly when every partial sum s + (q_1 + ... + q_m) u, m = 0..len, lies in
// [2^e + u, 2^(e+1) - u] -- one integer range test on s / u against the run's prefix minimum and
// maximum.  Only the elements where the sum crosses a binade (near zero, or at a power of two) or
// hits a tie still need their own rounded add.
//
// One block per refined frame, kXW waves; per iteration each wave takes one listed tile (the tiles
// where the winning hypothesis counted inliers, as k_refine) and lane l its 32 consecutive points.
//   phase 1  per stream k (xx, xy, xz, yy, yz, zz, x, y, z): the lane's sum and absolute sum, a wave
//            scan, the block's wave totals: an estimate P of the chain value at the lane's start
//            (from the walk's exact value at the iteration start);
//   phase 2  a lane whose estimated partial-sum range [P + neg, P + pos] (widened by a margin)
//            stays inside one binade scores its elements on that grid: q, R, the prefix min / max
//            and the tie test -> a RUN term (R u, the range limits); any other lane with inliers
//            -> a SEQ term whose values are laid out in order for the walk;
//   walk     wave 0, lane k = stream k: s += R u after the range test, or s = fl(s + v) per SEQ
//            value, in lane-segment order (= ascending inlier order).
// A RUN whose range test fails (an estimate off by more than the margin) marks the frame; such
// frames are refined again by k_refine's serial chain (the fallback launch after this one), so
// the result never depends on the estimate.  Bit-exact with k_refine by construction.
constexpr int kXW = 4;              // waves per block = listed tiles per iteration
constexpr int kXSeg = kTile / 64;   // points per lane segment (32)
constexpr int kXLanes = 64 * kXW;   // lane segments (terms per stream) per iteration
constexpr int kXCap = 1024;         // add-list entries per stream per window
constexpr int kXVS = kXCap + 8;     // entry stride per stream (floats): streams on distinct banks

struct XRefineLds {
    int tl[kRMaxTiles];
    float seqv[9][kXVS];  // a window of each stream's add list (then: the chain value before each entry)
    float wsum[kXW][9];  // the waves' stream sums (estimates)
    float wabs[kXW][9];  // and absolute sums
    int wseq[kXW][9];    // add-list entries per wave and stream
    float sx[9];         // the walk's exact chain value at the iteration start
    int nact, n_in, fail;
};

// Stream k of computeMeanAndCovarianceMatrix's accumulator (PCL order): products rounded to float.
__device__ __forceinline__ float xval(int k, float x, float y, float z) {
    switch (k) {
        case 0: return x * x;
        case 1: return x * y;
        case 2: return x * z;
        case 3: return y * y;
        case 4: return y * z;
        case 5: return z * z;
        case 6: return x;
        case 7: return y;
        default: return z;
    }
}

__device__ __forceinline__ float wave_incl_f(float v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const float t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}
__device__ __forceinline__ int wave_incl_i(int v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}
__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// The points, opaque to the compiler: products are recomputed per phase instead of kept live.
__device__ __forceinline__ void xopaque(float (&px)[kXSeg], float (&py)[kXSeg], float (&pz)[kXSeg]) {
#pragma unroll
    for (int j = 0; j < kXSeg; ++j) asm volatile("" : "+v"(px[j]), "+v"(py[j]), "+v"(pz[j]));
}

template <int ORDER, int DIV>
__global__ __launch_bounds__(64 * kXW) void k_xrefine(
    const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
    const FrameMeta* __restrict__ meta, const FrameState* __restrict__ st, const float4* __restrict__ best_coef,
    float thf, const int32_t* __restrict__ tile_counts, int hstride, int tiles_max, float4* __restrict__ final_coef,
    int32_t* __restrict__ fallback, int32_t* __restrict__ fallback_count, unsigned long long* __restrict__ acct,
    int force_fallback, unsigned long long* __restrict__ rdbg) {
    PITT_DBG_GUARD();
    __shared__ XRefineLds L;
    const long long t_start = rdbg ? clock64() : 0;
    unsigned long long n_seq = 0, n_run = 0, n_wait = 0;
    const int f = blockIdx.x;
    const FrameState s = st[f];
    if (!s.has_model || !s.need_refine) return;
    const FrameMeta m = meta[f];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    if (wave == 0) {
        const int nact = refine_tiles(L, m.tiles, lane, tile_counts + (int64_t)f * tiles_max * hstride + s.best_h,
                                      hstride);
        if (lane == 0) {
            L.nact = nact;
            L.n_in = 0;
            L.fail = 0;
            const int nsteps = nact < 0 ? (int)((m.n + kRChunk - 1) / kRChunk) : nact * kRStepsPerTile;
            acct_add(acct, kAcRefine, (unsigned long long)nsteps * kRChunk * 12ull + (unsigned long long)m.tiles * 4ull + 32ull);
        }
        if (lane < 9) L.sx[lane] = 0.0f;
    }
    __syncthreads();
    const int nact = L.nact;
    const int npass = nact < 0 ? m.tiles : nact;
    const float4 c = best_coef[f];
    float tv;
    asm volatile("v_mov_b32 %0, %1" : "=v"(tv) : "s"(thf));
    const int wk = lane < 9 ? lane : 0;  // the walk: wave 0, lane k = stream k
    float ws = 0.0f;
    for (int it = 0; it < npass; it += kXW) {
        const int ti = it + wave;
        const bool valid = ti < npass;
        const int tile = valid ? (nact < 0 ? ti : L.tl[ti]) : 0;
        const int64_t q0 = (int64_t)tile * kTile + lane * kXSeg;  // the segment's first point (in the frame)
        float px[kXSeg], py[kXSeg], pz[kXSeg];
        uint32_t msk = 0;
        if (valid) {
            const float4* gx = reinterpret_cast<const float4*>(X + m.off + q0);
            const float4* gy = reinterpret_cast<const float4*>(Y + m.off + q0);
            const float4* gz = reinterpret_cast<const float4*>(Z + m.off + q0);
#pragma unroll
            for (int i = 0; i < kXSeg / 4; ++i) {
                const float4 a = gx[i], b = gy[i], d = gz[i];
                px[4 * i] = a.x; px[4 * i + 1] = a.y; px[4 * i + 2] = a.z; px[4 * i + 3] = a.w;
                py[4 * i] = b.x; py[4 * i + 1] = b.y; py[4 * i + 2] = b.z; py[4 * i + 3] = b.w;
                pz[4 * i] = d.x; pz[4 * i + 1] = d.y; pz[4 * i + 2] = d.z; pz[4 * i + 3] = d.w;
            }
#pragma unroll
            for (int j = 0; j < kXSeg; ++j) {
                const bool in = (q0 + j < m.n) & (fabsf(plane_dot<ORDER>(c, px[j], py[j], pz[j])) < tv);
                msk |= (in ? 1u : 0u) << j;  // NaN never counts
            }
        } else {
#pragma unroll
            for (int j = 0; j < kXSeg; ++j) px[j] = py[j] = pz[j] = 0.0f;
        }
        const int cnt = __builtin_popcount(msk);
        // phase 1: sums per stream (estimates)
        float sv[9], sa[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) sv[k] = sa[k] = 0.0f;
#pragma unroll
        for (int j = 0; j < kXSeg; ++j) {
            const bool in = (msk >> j) & 1u;
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                const float v = in ? xval(k, px[j], py[j], pz[j]) : 0.0f;
                sv[k] += v;
                sa[k] += fabsf(v);
            }
        }
        float pre[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const float inc = wave_incl_f(sv[k], lane);
            pre[k] = inc - sv[k];
            if (lane == 63) L.wsum[wave][k] = inc;
            const float ab = wave_sum_f(sa[k]);
            if (lane == 0) L.wabs[wave][k] = ab;
        }
        {
            const int wc = __shfl(wave_incl_i(cnt, lane), 63, 64);
            if (lane == 0) atomicAdd(&L.n_in, wc);
        }
        __syncthreads();
        xopaque(px, py, pz);  // phase 2 recomputes the products (kept from phase 1: 288 live VGPRs)
        // phase 2: RUN or SEQ per (lane segment, stream)
        int ent[9], rlo[9], rhi[9], rex[9];
        float ra[9];
        uint32_t runbits = 0;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            float P = L.sx[k], A = fabsf(L.sx[k]);
#pragma unroll
            for (int w = 0; w < kXW; ++w) {
                if (w < wave) P += L.wsum[w][k];
                A += L.wabs[w][k];
            }
            P += pre[k];
            const float mg = A * 0x1p-14f;
            const float pos = 0.5f * (sv[k] + sa[k]), neg = 0.5f * (sv[k] - sa[k]);
            const float lo = (P + neg) - mg, hi = (P + pos) + mg;
            const bool up = lo > 0.0f;
            bool cand = cnt > 0 && (up || hi < 0.0f) && __builtin_isfinite(lo) && __builtin_isfinite(hi);
            const float a0 = up ? lo : -hi, b0 = up ? hi : -lo;
            int ex = 0;
            (void)frexpf(a0, &ex);  // a0 in [2^(ex-1), 2^ex): binade e = ex - 1
            const int e = ex - 1;
            cand = cand && e >= -100 && e <= 125 && b0 < ldexpf(1.0f, e + 1);
            float R = 0.0f, mn = 0.0f, mx = 0.0f, T = 0.0f;
            if (cand) {
                const float scale = ldexpf(1.0f, 23 - e);
#pragma unroll
                for (int j = 0; j < kXSeg; ++j) {
                    const float v = ((msk >> j) & 1u) ? xval(k, px[j], py[j], pz[j]) : 0.0f;
                    const float t = v * scale;
                    const float q = rintf(t);
                    T = fmaxf(T, fabsf(t - q));
                    R += q;
                    mn = fminf(mn, R);
                    mx = fmaxf(mx, R);
                }
            }
            const bool clean = cand && T < 0.5f && fabsf(mn) <= 0x1p25f && fabsf(mx) <= 0x1p25f;
            // the lane's entries in the stream's add list: a RUN is one entry (R u), SEQ its values
            ent[k] = cnt == 0 ? 0 : clean ? 1 : cnt;
            runbits |= (cnt > 0 && clean ? 1u : 0u) << k;
            ra[k] = clean ? ldexpf(R, e - 23) : 0.0f;  // exact: |R| <= 2^25, e >= -100
            rlo[k] = (up ? (1 << 23) + 1 : -((1 << 24) - 1)) - (clean ? (int)mn : 0);
            rhi[k] = (up ? (1 << 24) - 1 : -((1 << 23) + 1)) - (clean ? (int)mx : 0);
            rex[k] = e;
        }
        int eoff[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const int inc = wave_incl_i(ent[k], lane);
            eoff[k] = inc - ent[k];
            if (lane == 63) L.wseq[wave][k] = inc;
        }
        __syncthreads();
        int ntot[9], nmax = 0;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            ntot[k] = 0;
#pragma unroll
            for (int w = 0; w < kXW; ++w) {
                if (w < wave) eoff[k] += L.wseq[w][k];
                ntot[k] += L.wseq[w][k];
            }
            nmax = max(nmax, ntot[k]);
        }
        // windows of kXCap entries per stream: laid out, walked (each entry replaced by the chain
        // value before it), then the window's RUN entries checked by the lanes that made them
        for (int wb = 0; wb < nmax; wb += kXCap) {
            xopaque(px, py, pz);
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                if (ent[k] > 0 && eoff[k] < wb + kXCap && eoff[k] + ent[k] > wb) {
                    if ((runbits >> k) & 1u) {
                        L.seqv[k][eoff[k] - wb] = ra[k];
                    } else {
                        int r = eoff[k] - wb;
#pragma unroll
                        for (int j = 0; j < kXSeg; ++j) {
                            if ((msk >> j) & 1u) {
                                if (r >= 0 && r < kXCap) L.seqv[k][r] = xval(k, px[j], py[j], pz[j]);
                                ++r;
                            }
                        }
                    }
                }
            }
            __syncthreads();
            if (wave == 0 && lane < 9) {
                int nk = 0;
#pragma unroll
                for (int k = 0; k < 9; ++k) nk = wk == k ? ntot[k] : nk;
                const int hi = min(nk - wb, kXCap);
                float4* v = reinterpret_cast<float4*>(&L.seqv[wk][0]);
                float4 cur = v[0], nxt = v[1];
                for (int j = 0; j < hi; j += 4) {
                    const float4 nn = v[(j >> 2) + 2];  // within the stride's padding at the end
                    float4 pz4;
                    const float a0 = j < hi ? cur.x : 0.0f, a1 = j + 1 < hi ? cur.y : 0.0f;
                    const float a2 = j + 2 < hi ? cur.z : 0.0f, a3 = j + 3 < hi ? cur.w : 0.0f;
                    pz4.x = ws;
                    ws = ws + a0;
                    pz4.y = ws;
                    ws = ws + a1;
                    pz4.z = ws;
                    ws = ws + a2;
                    pz4.w = ws;
                    ws = ws + a3;
                    v[j >> 2] = pz4;
                    cur = nxt;
                    nxt = nn;
                }
                n_seq += (unsigned long long)max(hi, 0);
                if (wb + kXCap >= nk) L.sx[wk] = ws;
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                if (((runbits >> k) & 1u) && eoff[k] >= wb && eoff[k] < wb + kXCap) {
                    const float sb = L.seqv[k][eoff[k] - wb];  // the chain value before the run
                    const float ts = sb * ldexpf(1.0f, 23 - rex[k]);  // s / u, exact when in range
                    const bool ok = fabsf(ts) < 0x1p26f && (int)ts >= rlo[k] && (int)ts <= rhi[k];
                    if (!ok) L.fail = 1;
                    ++n_run;
                }
            }
            __syncthreads();  // the window's checks read the values the next window replaces
            ++n_wait;
        }
    }
    if (wave == 0) {
        float a9[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) a9[k] = __shfl(ws, k, 64);
        const bool fail = force_fallback || L.fail != 0;
        if (rdbg && lane < 9) {
            rdbg[(int64_t)f * 16 + 3 + lane] = n_seq;  // 3..11: SEQ values per stream
            if (lane == 0) rdbg[(int64_t)f * 16 + 13] = n_run;
        }
        if (lane == 0) {
            if (rdbg) {  // PITT_REFINE_DEBUG: cycles, windows, RUN terms and SEQ values (stream 0, max)
                rdbg[(int64_t)f * 16 + 0] = (unsigned long long)(clock64() - t_start);
                rdbg[(int64_t)f * 16 + 1] = (unsigned long long)npass;
                rdbg[(int64_t)f * 16 + 2] = n_wait;
                rdbg[(int64_t)f * 16 + 12] = (unsigned long long)L.n_in;
            }
            if (!fail) final_coef[f] = refine_plane<ORDER, DIV>(a9, L.n_in);
            else atomicAdd(fallback_count, 1);
            fallback[f] = fail ? 1 : 0;
        }
    }
}

// ------------------------------------------------------------------------------------------
// A6 fast mode (PITT_COV_FAST): the winning model's inlier covariance in double, tree-reduced over
// the whole chip instead of nine serial float chains per frame.
//   k_cov_tiles  one wave per (frame, tile) where the winning hypothesis counted inliers (exact, from
//                the scoring counts; other tiles hold none): PCL's predicate |d| < t (ORDER), then per
//                lane sequential double sums of x, y, z, xx, xy, xz, yy, yz, zz over its 32 points
//                (float products are exact in double), a fixed xor-shuffle tree over the wave, and
//                the tile's partial [f][t] (9 sums + count) stored;
//   k_cov_final  one wave per refined frame: lane l sums tiles l, l + 64, ... in order, the same tree,
//                then accu_k = (float)(S_k / n) into PCL's float covariance and eigen33.
// Deterministic (fixed association); differs from PCL's sequential float sums by their rounding only.
struct CovPart {
    double s[9];  // x, y, z, xx, xy, xz, yy, yz, zz
    int32_t n;
    int32_t pad;
};

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

template <int ORDER>
__global__ __launch_bounds__(kBlock) void k_cov_tiles(
    const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
    const FrameMeta* __restrict__ meta, const FrameState* __restrict__ st, const float4* __restrict__ best_coef,
    float thf, const int32_t* __restrict__ tile_counts, int hstride, int n_frames, int tiles_max,
    CovPart* __restrict__ part) {
    PITT_DBG_GUARD();
    const int lane = threadIdx.x & 63;
    const int it = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * kWaves + (threadIdx.x >> 6)));
    const int f = it / tiles_max, t = it - f * tiles_max;
    if (f >= n_frames) return;
    const FrameState s = st[f];
    const FrameMeta m = meta[f];
    if (t >= m.tiles || !s.has_model || !s.need_refine) return;
    CovPart* out = part + (int64_t)f * tiles_max + t;
    double a[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    int cnt = 0;
    if (tile_counts[((int64_t)f * tiles_max + t) * hstride + s.best_h] > 0) {
        const float4 c = best_coef[f];
        float tv;
        asm volatile("v_mov_b32 %0, %1" : "=v"(tv) : "s"(thf));
        const int rem = (int)min(m.n - (int64_t)t * kTile, (int64_t)kTile);
        const int64_t p0 = m.off + (int64_t)t * kTile + lane;
#pragma unroll 4
        for (int g = 0; g < kTile / 64; ++g) {
            const float x = X[p0 + 64 * g], y = Y[p0 + 64 * g], z = Z[p0 + 64 * g];
            if (64 * g + lane < rem && fabsf(plane_dot<ORDER>(c, x, y, z)) < tv) {
                const double dx = x, dy = y, dz = z;
                a[0] += dx;
                a[1] += dy;
                a[2] += dz;
                a[3] += dx * dx;
                a[4] += dx * dy;
                a[5] += dx * dz;
                a[6] += dy * dy;
                a[7] += dy * dz;
                a[8] += dz * dz;
                ++cnt;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) a[k] = wave_sum_d(a[k]);
    cnt = wave_sum_i(cnt);
    if (lane < 9) {
        double v = a[0];
#pragma unroll
        for (int k = 1; k < 9; ++k) v = lane == k ? a[k] : v;
        out->s[lane] = v;
    }
    if (lane == 0) out->n = cnt;
}

template <int ORDER>
__global__ __launch_bounds__(64) void k_cov_final(const FrameMeta* __restrict__ meta,
                                                  const FrameState* __restrict__ st, const CovPart* __restrict__ part,
                                                  int n_frames, int tiles_max, float4* __restrict__ final_coef) {
    PITT_DBG_GUARD();
    const int f = blockIdx.x;
    const int lane = threadIdx.x;
    if (f >= n_frames) return;
    const FrameState s = st[f];
    if (!s.has_model || !s.need_refine) return;
    const int tiles = meta[f].tiles;
    double a[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    int cnt = 0;
    for (int t = lane; t < tiles; t += 64) {
        const CovPart& p = part[(int64_t)f * tiles_max + t];
#pragma unroll
        for (int k = 0; k < 9; ++k) a[k] += p.s[k];
        cnt += p.n;
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) a[k] = wave_sum_d(a[k]);
    cnt = wave_sum_i(cnt);
    if (lane == 0 && cnt > 0) {
        // accu order of computeMeanAndCovarianceMatrix: xx, xy, xz, yy, yz, zz, x, y, z
        const double n = (double)cnt;
        float a9[9] = {(float)(a[3] / n), (float)(a[4] / n), (float)(a[5] / n), (float)(a[6] / n),
                       (float)(a[7] / n), (float)(a[8] / n), (float)(a[0] / n), (float)(a[1] / n),
                       (float)(a[2] / n)};
        final_coef[f] = refine_plane_mean<ORDER>(a9);
    }
}

// ------------------------------------------------------------------------------------------
// Final selection: selectWithinDistance on each frame's final model (the refined plane, or the
// winning hypothesis without refinement) -> the ascending inlier list.  Two launches, one wave per
// (frame, tile), the whole chip on the batch instead of one streaming wave per frame:
//   k_sel_mark   the tile's predicate bits (lane l, bit g <=> point 64 g + l of the tile is an
//                inlier) and its inlier count; a tile whose bounding box certainly misses the
//                model's slab (box_misses_slab) is marked empty without reading a point;
//   k_sel_write  the tile's output offset (the frame's earlier tile counts) and its inliers'
//                indices, ascending, from the predicate bits alone.
constexpr int kSelGroups = kTile / 64;  // 32 predicate bits per lane

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

template <int ORDER>
__global__ __launch_bounds__(kBlock) void k_sel_mark(
    const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
    const FrameMeta* __restrict__ meta, const FrameState* __restrict__ st, const float4* __restrict__ final_coef,
    float thf, int n_frames, int tiles_max, const float* __restrict__ tile_box, const float* __restrict__ group_box,
    uint32_t* __restrict__ sel_bits, int32_t* __restrict__ sel_cnt, uint32_t* __restrict__ acct_tile) {
    PITT_DBG_GUARD();
    (void)tile_box;
    const int lane = threadIdx.x & 63;
    const int it = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * kWaves + (threadIdx.x >> 6)));
    const int f = it / tiles_max, t = it - f * tiles_max;
    if (f >= n_frames) return;
    const int64_t row = (int64_t)f * tiles_max + t;
    // the tile's 32 group boxes (lane g: group g), requested with the frame's metadata rather than
    // behind it and behind a tile-box test: one dependent memory latency per wave instead of three
    // (a tile whose box misses the slab has every group box missing it too)
    const float4* gbp = reinterpret_cast<const float4*>(group_box + (row * kSelGroups + (lane & (kSelGroups - 1))) * 8);
    const float4 b0 = gbp[0], b1 = gbp[1];
    const FrameMeta m = meta[f];
    if (t >= m.tiles || !st[f].has_model) return;
    const float4 c = final_coef[f];
    uint32_t word = 0;
    const int rem = (int)min(m.n - (int64_t)t * kTile, (int64_t)kTile);
    const int64_t p0 = m.off + (int64_t)t * kTile + lane;
    float tv;
    asm volatile("v_mov_b32 %0, %1" : "=v"(tv) : "s"(thf));
    // groups whose box certainly misses the slab hold no inlier: not read (lane g tests group g)
    const float gb6[6] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y};
    const bool gact = lane < kSelGroups && !box_misses_slab(gb6, c, thf);
    const uint32_t gm = (uint32_t)__builtin_amdgcn_ballot_w64(gact);
    const unsigned long long moved = 32ull * kSelGroups + 12ull * 64ull * (unsigned long long)__builtin_popcount(gm) +
                                     256ull + 4ull;  // group boxes and live groups in; bits and count out
    if (gm) {
        float px[kSelGroups], py[kSelGroups], pz[kSelGroups];  // the tile's live groups in flight
#pragma unroll
        for (int g = 0; g < kSelGroups; ++g) {
            px[g] = py[g] = pz[g] = __builtin_nanf("");
            if ((gm >> g) & 1u) {
                px[g] = X[p0 + 64 * g];
                py[g] = Y[p0 + 64 * g];
                pz[g] = Z[p0 + 64 * g];
            }
        }
#pragma unroll
        for (int g = 0; g < kSelGroups; ++g) {
            const bool in = (64 * g + lane < rem) & (fabsf(plane_dot<ORDER>(c, px[g], py[g], pz[g])) < tv);
            word |= (in ? 1u : 0u) << g;  // no branch per group (NaN never counts)
        }
    }
    sel_bits[row * 64 + lane] = word;
    const int n = wave_sum(__builtin_popcount(word));
    if (lane == 0) {
        sel_cnt[row] = n;
        if (acct_tile) acct_tile[row] = (uint32_t)moved;  // profiling: a plain store per tile, no atomics
    }
}

__global__ __launch_bounds__(kBlock) void k_sel_write(
    const FrameMeta* __restrict__ meta, const FrameState* __restrict__ st, int n_frames, int tiles_max,
    const uint32_t* __restrict__ sel_bits, const int32_t* __restrict__ sel_cnt, int32_t* __restrict__ inliers,
    int32_t* __restrict__ n_final, uint32_t* __restrict__ acct_tile) {
    PITT_DBG_GUARD();
    const int lane = threadIdx.x & 63;
    const int it = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * kWaves + (threadIdx.x >> 6)));
    const int f = it / tiles_max, t = it - f * tiles_max;
    if (f >= n_frames) return;
    // the tile's predicate bits, requested with the metadata (valid memory for every tile slot)
    const uint32_t word = sel_bits[((int64_t)f * tiles_max + t) * 64 + lane];
    const FrameMeta m = meta[f];
    if (t >= m.tiles || !st[f].has_model) return;
    const int32_t* cnt = sel_cnt + (int64_t)f * tiles_max;
    int pre = 0;
    for (int j = lane; j < t; j += 64) pre += cnt[j];
    pre = __builtin_amdgcn_readfirstlane(wave_sum(pre));
    const int mine = cnt[t];
    if (t == m.tiles - 1 && lane == 0) n_final[f] = pre + mine;
    // the earlier tiles' counts, then the tile's bits and its indices
    if (lane == 0 && acct_tile)
        acct_tile[(int64_t)f * tiles_max + t] = 4u * (uint32_t)(t + 1) + (inliers && mine ? 256u + 4u * (uint32_t)mine : 0u);
    if (!inliers || mine == 0) return;
    int32_t* out = inliers + m.off + pre;
    const int32_t i0 = t * kTile + lane;
#pragma unroll
    for (int g = 0; g < kSelGroups; ++g) {
        const bool in = (word >> g) & 1u;
        const uint64_t b = __builtin_amdgcn_ballot_w64(in);
        if (in) out[__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u))] = i0 + 64 * g;
        out += __builtin_popcountll(b);
    }
}

__global__ void k_finalize(const FrameState* __restrict__ st, const int32_t* __restrict__ hyp_attempt,
                           const float4* __restrict__ final_coef, const int32_t* __restrict__ n_final,
                           int hcap, int n_frames, pitt_plane_result* __restrict__ res) {
    PITT_DBG_GUARD();
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= n_frames) return;
    const FrameState s = st[f];
    pitt_plane_result r;
    r.status = s.status;
    r.hypotheses = s.it;
    r.best_hypothesis = s.best_h;
    r.best_count = s.best_h >= 0 ? s.best_count : 0;
    r.flags = s.flags;
    // rejections before the last evaluated hypothesis; + 1000 when getSamples gave up
    int rej = 0;
    if (s.it > 0) rej = hyp_attempt[(int64_t)f * hcap + s.it - 1] - (s.it - 1);
    if (s.pad0) rej += 1000;
    r.rejected_samples = rej;
    if (s.has_model) {
        const float4 c = final_coef[f];
        r.coefficients[0] = c.x;
        r.coefficients[1] = c.y;
        r.coefficients[2] = c.z;
        r.coefficients[3] = c.w;
        r.n_coeff = 4;
        r.n_inliers = n_final[f];
    } else {
        r.coefficients[0] = r.coefficients[1] = r.coefficients[2] = r.coefficients[3] = 0.0f;
        r.n_coeff = 0;
        r.n_inliers = 0;
    }
    res[f] = r;
}

// ------------------------------------------------------------------------------------------
// Small batches (a service call, a support-loop iteration, one camera frame): optimizeModelCoefficients'
// nine exact-order sums by the block-parallel exact walk (xsum.hpp) over the whole chip instead of one
// frame's serial chain in k_refine -- the same float sums, so the same refined plane, at a fraction of
// the latency (a 600k-inlier support plane: ~2.5 ms of chain).  The winning model's inliers, ascending,
// become nine product streams (PCL's separately rounded xx, xy, xz, yy, yz, zz, then x, y, z) in one
// 256-aligned segment per frame.
__device__ __forceinline__ bool xr_eligible(const FrameState& s, int phase) {
    return s.has_model && s.need_refine && s.pad1 == phase;
}

// per (frame, tile) wave: the tile's inliers of the winning model
// The walk's producers take each tile in kXrSplit parts, one wave each (a one-frame batch has only ~150
// tiles: whole-tile waves left the chip nearly idle and each wave walked 32 dependent groups).
#ifndef PITT_XR_SPLIT
#define PITT_XR_SPLIT 8
#endif
constexpr int kXrSplit = PITT_XR_SPLIT;
constexpr int kXrGroups = kTile / 64 / kXrSplit;  // 64-point groups per part

template <int ORDER>
__global__ __launch_bounds__(kBlock) void k_xr_count(const float* __restrict__ X, const float* __restrict__ Y,
                                                     const float* __restrict__ Z, const FrameMeta* __restrict__ meta,
                                                     const FrameState* __restrict__ st, const float4* __restrict__ best_coef,
                                                     float thf, int n_frames, int tiles_max, int32_t* __restrict__ tcnt,
                                                     int phase) {
    PITT_DBG_GUARD();
    const int lane = threadIdx.x & 63;
    const int it = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * kWaves + (threadIdx.x >> 6)));
    const int ts = tiles_max * kXrSplit;  // items per frame: kXrSplit parts of each tile
    const int f = it / ts, q = it - f * ts, t = q / kXrSplit, part = q - t * kXrSplit;
    if (f >= n_frames) return;
    const FrameMeta m = meta[f];
    int cnt = 0;
    if (t < m.tiles && xr_eligible(st[f], phase)) {
        const float4 c = best_coef[f];
        float tv;
        asm volatile("v_mov_b32 %0, %1" : "=v"(tv) : "s"(thf));
        for (int g = part * kXrGroups; g < (part + 1) * kXrGroups; ++g) {
            const int64_t i = (int64_t)t * kTile + 64 * g + lane;
            const bool in = i < m.n && fabsf(plane_dot<ORDER>(c, X[m.off + i], Y[m.off + i], Z[m.off + i])) < tv;
            cnt += __builtin_popcountll(__builtin_amdgcn_ballot_w64(in));
        }
    }
    if (lane == 0) tcnt[(int64_t)f * ts + q] = cnt;
}

// one block per frame: the tiles' inlier offsets, the frame's segment (first block: the previous frames'
// point spans, 256-aligned) and its length, and the block -> segment map of its span
__global__ __launch_bounds__(256) void k_xr_scan(const FrameMeta* __restrict__ meta, int tiles_max,
                                                 int32_t* __restrict__ tcnt, XsSeg* __restrict__ seg,
                                                 int32_t* __restrict__ blk_seg) {
    PITT_DBG_GUARD();
    const int f = blockIdx.x;
    __shared__ int64_t base;
    __shared__ int32_t part[256];
    const FrameMeta m = meta[f];
    if (threadIdx.x == 0) {
        int64_t b = 0;
        for (int g = 0; g < f; ++g) b += (meta[g].n + kXsBlk - 1) / kXsBlk;
        base = b;
    }
    int32_t* c = tcnt + (int64_t)f * tiles_max * kXrSplit;
    const int parts = m.tiles * kXrSplit;
    const int per = (parts + 255) / 256;
    const int a = (int)threadIdx.x * per, e = min(a + per, parts);
    int acc = 0;
    for (int i = a; i < e; ++i) acc += c[i];
    part[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        int run = 0;
        for (int i = 0; i < 256; ++i) {
            const int t = part[i];
            part[i] = run;
            run += t;
        }
        seg[f] = XsSeg{base, (int64_t)run};
    }
    __syncthreads();
    acc = part[threadIdx.x];
    for (int i = a; i < e; ++i) {  // in place: count -> exclusive offset
        const int t = c[i];
        c[i] = acc;
        acc += t;
    }
    const int64_t nb = (m.n + kXsBlk - 1) / kXsBlk;
    for (int64_t b = threadIdx.x; b < nb; b += 256) blk_seg[base + b] = f;
}

// per (frame, tile) wave: the tile's inliers' nine products at their ascending positions
template <int ORDER>
__global__ __launch_bounds__(kBlock) void k_xr_write(const float* __restrict__ X, const float* __restrict__ Y,
                                                     const float* __restrict__ Z, const FrameMeta* __restrict__ meta,
                                                     const FrameState* __restrict__ st, const float4* __restrict__ best_coef,
                                                     float thf, int n_frames, int tiles_max, const int32_t* __restrict__ toff,
                                                     const XsSeg* __restrict__ seg, float* __restrict__ V, int64_t T,
                                                     int phase) {
    PITT_DBG_GUARD();
    const int lane = threadIdx.x & 63;
    const int it = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * kWaves + (threadIdx.x >> 6)));
    const int ts = tiles_max * kXrSplit;
    const int f = it / ts, q = it - f * ts, t = q / kXrSplit, part = q - t * kXrSplit;
    if (f >= n_frames) return;
    const FrameMeta m = meta[f];
    if (t >= m.tiles || !xr_eligible(st[f], phase)) return;
    const float4 c = best_coef[f];
    float tv;
    asm volatile("v_mov_b32 %0, %1" : "=v"(tv) : "s"(thf));
    int64_t pos = seg[f].blk0 * kXsBlk + toff[(int64_t)f * ts + q];
    for (int g = part * kXrGroups; g < (part + 1) * kXrGroups; ++g) {
        const int64_t i = (int64_t)t * kTile + 64 * g + lane;
        float x = 0.0f, y = 0.0f, z = 0.0f;
        bool in = false;
        if (i < m.n) {
            x = X[m.off + i];
            y = Y[m.off + i];
            z = Z[m.off + i];
            in = fabsf(plane_dot<ORDER>(c, x, y, z)) < tv;
        }
        const uint64_t b = __builtin_amdgcn_ballot_w64(in);
        if (in) {
            const int64_t p = pos + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
            V[p] = x * x;
            V[T + p] = x * y;
            V[2 * T + p] = x * z;
            V[3 * T + p] = y * y;
            V[4 * T + p] = y * z;
            V[5 * T + p] = z * z;
            V[6 * T + p] = x;
            V[7 * T + p] = y;
            V[8 * T + p] = z;
        }
        pos += __builtin_popcountll(b);
    }
}

// one thread per frame: the refined plane from the nine sums (k_refine's refine_plane)
template <int ORDER, int DIV>
__global__ void k_xr_plane(const FrameState* __restrict__ st, const XsSeg* __restrict__ seg,
                           const float* __restrict__ sums, int n_frames, float4* __restrict__ final_coef, int phase) {
    PITT_DBG_GUARD();
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= n_frames || !xr_eligible(st[f], phase)) return;
    float a9[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) a9[k] = sums[f * 9 + k];
    final_coef[f] = refine_plane<ORDER, DIV>(a9, (int)seg[f].len);
}

// ------------------------------------------------------------------------------------------
// Host orchestration.

template <typename T>
static T* as(void* p) { return static_cast<T*>(p); }

// k_refine_multi's instantiations that fit the CU's LDS (160 KB)
constexpr bool kRefineMulti3 = 3 * sizeof(RefineLdsP) + 64 <= 160 * 1024;
template <int ORDER, int DIV>
static auto refine_multi_kernel(int F) {
    if constexpr (kRefineMulti3)
        if (F == 3) return k_refine_multi<ORDER, DIV, 3>;
    return k_refine_multi<ORDER, DIV, 2>;
}

// Debug builds only (tools/build_variant.sh <name> -DPITT_SYNC_CHECK): synchronise
// after every launch of a batch so that a faulting kernel is named on stderr.
#ifdef PITT_SYNC_CHECK
#define PITT_CHECK_LAUNCH(what, c, phase)                                                                    \
    do {                                                                                                   \
        hipStreamCaptureStatus cs_ = hipStreamCaptureStatusNone;                                           \
        (void)hipStreamIsCapturing(sm, &cs_);                                                              \
        if (cs_ != hipStreamCaptureStatusNone) break;                                                      \
        const hipError_t e_ = hipStreamSynchronize(sm);                                                    \
        std::fprintf(stderr, "PITT_SYNC_CHECK %s chunk %d phase %d: %s\n", what, c, phase,                \
                     hipGetErrorString(e_));                                                               \
        if (e_ != hipSuccess) return ctx->fail(PITT_E_HIP, what);                                          \
    } while (0)
#else
#define PITT_CHECK_LAUNCH(what, c, phase) \
    do {                                  \
    } while (0)
#endif

template <int ORDER, int DIV>
static int run_plane_batch(pitt_ctx* ctx, const pitt_frames* fr, const pitt_sac_params* p,
                           pitt_plane_result* results, int32_t* inliers_dev) {
    const int nf = fr->n_frames;
    hipStream_t sm = ctx->stream;
#ifdef PITT_SYNC_CHECK
    ctx->check_canaries("plane batch entry");
#endif
    // --- sizes ---
    int tiles_max = 1;
    for (int f = 0; f < nf; ++f) tiles_max = std::max<int>(tiles_max, (int)((fr->counts[f] + kTile - 1) / kTile));
    const int max_iter = p->max_iterations;
    const int hcap = max_iter >= 0 ? max_iter + 1 : 1;
    const int runnable_all = ((unsigned)max_iter * 10u) != 0u ? 1 : 0;
    // getSamples gives up after 1000 consecutive rejected draws (sac_model.hpp); the table always
    // covers that run past the last hypothesis, so a degenerate cloud ends in PCL's "no samples"
    // outcome rather than in an exhausted table.
    const int64_t A64 = (int64_t)hcap + std::max(1000, p->sampler_slack);
    if (A64 > kMaxAttempts) return ctx->fail(PITT_E_INVALID, "max_iterations + sampler_slack exceeds 2^24");
    const int A = (int)A64;
    const float thf = float_threshold(p->threshold);
    if ((int64_t)nf * tiles_max >= ((int64_t)1 << 31) || (int64_t)nf * hcap * tiles_max >= ((int64_t)1 << 40))
        return ctx->fail(PITT_E_INVALID, "batch too large (frames x tiles must stay below 2^31)");

    // --- sampler tables: one per distinct point count ---
    std::vector<int64_t> distinct;
    for (int f = 0; f < nf; ++f)
        if (fr->counts[f] >= 3 &&
            std::find(distinct.begin(), distinct.end(), fr->counts[f]) == distinct.end())
            distinct.push_back(fr->counts[f]);
    const size_t tab_ints = (size_t)A * 3;
    int32_t* tables = as<int32_t>(ctx->buf("tables", std::max<size_t>(1, distinct.size()) * tab_ints * 4));
    {
        std::vector<std::tuple<int64_t, uint32_t, int64_t>> keys;
        for (int64_t n : distinct) keys.emplace_back(n, p->seed, (int64_t)A);
        if (keys != ctx->pool_keys) {
            int32_t* hp = as<int32_t>(ctx->pinned("tables_h", std::max<size_t>(1, distinct.size()) * tab_ints * 4));
            for (size_t i = 0; i < distinct.size(); ++i) {
                const std::vector<int32_t>& t = sampler_table(ctx, distinct[i], p->seed, A);
                std::memcpy(hp + i * tab_ints, t.data(), tab_ints * 4);
            }
            if (!distinct.empty())
                PITT_HIP_TRY(hipMemcpyAsync(tables, hp, distinct.size() * tab_ints * 4, hipMemcpyHostToDevice, sm));
            ctx->pool_keys = keys;
        }
    }
    // --- frame metadata ---
    const uint32_t seq = ++ctx->call_seq;
    unsigned int* dbg_seq = nullptr;  // the debug build's pinned copy of the stamp (k_hypothesize compares)
#ifdef PITT_SYNC_CHECK
    dbg_seq = as<unsigned int>(ctx->pinned("dbg_seq_h", 16));
    if (!dbg_seq) return ctx->fail(PITT_E_NOMEM, "pinned stamp");
#endif
    FrameMeta* hm = as<FrameMeta>(ctx->pinned("meta_h", (size_t)nf * sizeof(FrameMeta)));
    for (int f = 0; f < nf; ++f) {
        hm[f].off = fr->offsets[f];
        hm[f].n = fr->counts[f];
        hm[f].tiles = (int32_t)((fr->counts[f] + kTile - 1) / kTile);
        hm[f].pad = (int32_t)seq;
        int64_t ti = 0;
        for (size_t i = 0; i < distinct.size(); ++i)
            if (distinct[i] == fr->counts[f]) ti = (int64_t)(i * tab_ints);
        hm[f].tab = ti;
    }
    FrameMeta* meta = as<FrameMeta>(ctx->buf("meta", (size_t)nf * sizeof(FrameMeta)));
    PITT_HIP_TRY(hipMemcpyAsync(meta, hm, (size_t)nf * sizeof(FrameMeta), hipMemcpyHostToDevice, sm));

    // --- chunk schedule: a culled first chunk that finishes most table frames (T <= 32 for 64 % of
    //     them, tools/make_golden-style oracle runs), then geometric chunks ---
    std::vector<int> chunks;
#ifndef PITT_FIRST_CHUNK
#define PITT_FIRST_CHUNK 32
#endif
    for (int h0 = 0, i = 0; h0 < hcap; ++i) {
        int H = i == 0 ? PITT_FIRST_CHUNK : std::min(kMaxScoreChunk, 64 << (i - 1));
        H = std::min(H, hcap - h0);
        chunks.push_back(H);
        h0 += H;
    }
    const int nchunks = (int)chunks.size();

    // --- scratch ---
    float4* hyp_coef = as<float4>(ctx->buf("hyp_coef", (size_t)nf * hcap * sizeof(float4)));
    int32_t* hyp_attempt = as<int32_t>(ctx->buf("hyp_attempt", (size_t)nf * hcap * 4));
    int32_t* hyp_total = as<int32_t>(ctx->buf("hyp_total", (size_t)nf * hcap * 4));
    // rows padded by 64 counts (k_score's stores may cover up to ceil(H / 64) * 64 entries) and aligned
    // to 128 B: a chunk's counts (h0 and its stores' extent multiples of 32) fill whole cache lines
    const int hstride = (hcap + 64 + 31) & ~31;
    int32_t* tile_counts = as<int32_t>(ctx->buf("tile_counts", (size_t)nf * hstride * tiles_max * 4));
    FrameState* st = as<FrameState>(ctx->buf("state", (size_t)nf * sizeof(FrameState)));
    int32_t* lists = as<int32_t>(ctx->buf("lists", (size_t)(nchunks + 1) * nf * 4));
    ScoreSlot* slots = as<ScoreSlot>(ctx->buf("score_slots", (size_t)(nchunks + 1) * nf * sizeof(ScoreSlot)));
    // counters + chunk stats in one zeroed block
    const size_t cnt_bytes = (size_t)(nchunks + 2) * 4;  // + k_xrefine's fallback count
    const size_t stat_off = (cnt_bytes + 15) & ~(size_t)15;
    const size_t acct_off = stat_off + (size_t)(nchunks + 1) * sizeof(ChunkStat);
    const size_t acct_bytes = (size_t)kAcKernels * kAcShards * sizeof(unsigned long long);
    const size_t zero_bytes = acct_off + acct_bytes;
    char* zblock = as<char>(ctx->buf("zblock", zero_bytes));
    int32_t* counters = as<int32_t>(zblock);
    ChunkStat* cstat = as<ChunkStat>(zblock + stat_off);
    // per-kernel byte accounting, only while profiling (the kernels skip the atomics otherwise)
    unsigned long long* acct = ctx->prof ? as<unsigned long long>(zblock + acct_off) : nullptr;
    // the per-tile kernels store their bytes per tile instead (two arrays of nf x tiles_max words)
    const size_t tile_words = (size_t)nf * tiles_max;
    uint32_t* acct_tiles = nullptr;
    if (ctx->prof) {
        acct_tiles = as<uint32_t>(ctx->buf("acct_tiles", tile_words * 2 * 4));
        if (!acct_tiles) return ctx->fail(PITT_E_NOMEM, "profiling scratch");
        PITT_HIP_TRY(hipMemsetAsync(acct_tiles, 0, tile_words * 2 * 4, sm));
    }
    float4* best_coef = as<float4>(ctx->buf("best_coef", (size_t)nf * sizeof(float4)));
    float4* final_coef = as<float4>(ctx->buf("final_coef", (size_t)nf * sizeof(float4)));
    int32_t* n_final = as<int32_t>(ctx->buf("n_final", (size_t)nf * 4));
    float* tile_box = as<float>(ctx->buf("tile_box", (size_t)nf * tiles_max * 8 * sizeof(float)));
    float* group_box = as<float>(ctx->buf("group_box", (size_t)nf * tiles_max * (kTile / kGrp) * 8 * sizeof(float)));
    uint32_t* sel_bits = as<uint32_t>(ctx->buf("sel_bits", (size_t)nf * tiles_max * 64 * 4));
    int32_t* sel_cnt = as<int32_t>(ctx->buf("sel_cnt", (size_t)nf * tiles_max * 4));
    pitt_plane_result* dres = as<pitt_plane_result>(ctx->buf("results", (size_t)nf * sizeof(pitt_plane_result)));
    if (!slots || !hyp_coef || !tile_counts || !n_final || !tile_box || !group_box || !sel_bits || !sel_cnt || !dres) return ctx->fail(PITT_E_NOMEM, "device allocation failed");
    int32_t* xfallback = ctx->xrefine ? as<int32_t>(ctx->buf("xfallback", (size_t)nf * 4)) : nullptr;
    if (ctx->xrefine && !xfallback) return ctx->fail(PITT_E_NOMEM, "refinement flags");
    CovPart* part = nullptr;
    if (p->cov_mode == PITT_COV_FAST) {
        part = as<CovPart>(ctx->buf("cov_part", (size_t)nf * tiles_max * sizeof(CovPart)));
        if (!part) return ctx->fail(PITT_E_NOMEM, "covariance partials");
    }
    pitt_plane_result* hres = as<pitt_plane_result>(ctx->pinned("results_h", (size_t)nf * sizeof(pitt_plane_result)));
    ChunkStat* hstat = as<ChunkStat>(ctx->pinned("cstat_h", (size_t)(nchunks + 1) * sizeof(ChunkStat)));
    int32_t* hxfb = as<int32_t>(ctx->pinned("xfb_h", 16));
    if (!hxfb) return ctx->fail(PITT_E_NOMEM, "pinned results");
    void* hacct = acct ? ctx->pinned("acct_h", acct_bytes + tile_words * 2 * 4) : nullptr;
    if (!hres || !hstat || (acct && !hacct)) return ctx->fail(PITT_E_NOMEM, "pinned results");
    // $PITT_REFINE_DEBUG: k_refine's per-role cycles and spin counts, summarised on stderr by pitt_wait
    unsigned long long* rdbg = nullptr;
    if (ctx->refine_debug) {
        rdbg = as<unsigned long long>(ctx->buf("refine_dbg", (size_t)nf * 16 * 8));
        ctx->refine_dbg_h = ctx->pinned("refine_dbg_h", (size_t)nf * 16 * 8);
        if (!rdbg || !ctx->refine_dbg_h) return ctx->fail(PITT_E_NOMEM, "refine debug");
    }

    // small batches refine through the chip-wide exact walk (k_xr_*, xsum.hpp) instead of k_refine's chain
    bool xs = p->optimize && p->cov_mode != PITT_COV_FAST && nf <= ctx->xs_max_frames;
    if constexpr (pitt_ctx::kVariants)  // the A/B build keeps k_refine whenever one of its variants is asked for
        xs = xs && ctx->refine_producers == 1 && ctx->refine_frames == 1 && ctx->xrefine == 0 &&
             ctx->refine_mode == 2 && !ctx->refine_debug;
    int64_t xs_blocks = 0;
    for (int f = 0; f < nf; ++f) xs_blocks += (fr->counts[f] + kXsBlk - 1) / kXsBlk;
    if (xs_blocks == 0) xs = false;  // every frame empty: nothing to refine (and no block -> segment map)
    const int64_t xs_T = std::max<int64_t>(1, xs_blocks) * kXsBlk;
    float* xr_v = nullptr;
    int32_t *xr_tcnt = nullptr, *xr_bseg = nullptr;
    XsSeg* xr_seg = nullptr;
    float* xr_sums = nullptr;
    XsScratch xr_scr;
    if (xs) {
        xr_v = as<float>(ctx->buf("xr_v", (size_t)9 * xs_T * 4));
        xr_tcnt = as<int32_t>(ctx->buf("xr_tcnt", (size_t)nf * tiles_max * kXrSplit * 4));
        xr_bseg = as<int32_t>(ctx->buf("xr_bseg", (size_t)(xs_T / kXsBlk) * 4));
        xr_seg = as<XsSeg>(ctx->buf("xr_seg", (size_t)nf * sizeof(XsSeg)));
        xr_sums = as<float>(ctx->buf("xr_sums", (size_t)nf * 9 * 4));
        if (!xr_v || !xr_tcnt || !xr_bseg || !xr_seg || !xr_sums) return ctx->fail(PITT_E_NOMEM, "refinement streams");
        if (int rc = xs_scratch(ctx, xs_T / kXsBlk, 9, "xr", &xr_scr)) return rc;
    }

    // Everything below is stream-ordered device work with device-built work lists: no host
    // synchronisation until the results are copied back (pitt_wait / finish_batch).
    const int sel_blocks = (int)(((int64_t)nf * tiles_max + kWaves - 1) / kWaves);
    const double log_prob = std::log(1.0 - p->probability);
    std::vector<int> acct_recs((size_t)kAcKernels, -1);
    std::vector<int> score_recs;
    // Adaptive chunk schedule: launch only the scoring chunks that recent batches of this layout needed
    // (table scenes finish after 2 of 7; every launch past that would find no active frame).  A frame
    // still running after them is finished by a continuation in finish_batch (the remaining chunks, then
    // the decision, refinement and selection of the frames it finished): exact either way.
    const std::array<uint64_t, 4> hint_key = {(uint64_t)(uintptr_t)fr->x, (uint64_t)nf, (uint64_t)hcap,
                                              (uint64_t)tiles_max};
    const int K = ctx->adaptive_chunks ? std::min(nchunks, ctx->chunk_hint(hint_key, nchunks)) : nchunks;
    // everything the launches use, by value: a continuation runs after this call has returned
    const float *fx = fr->x, *fy = fr->y, *fz = fr->z;
    const int optimize = p->optimize ? 1 : 0, cov_mode = p->cov_mode;
    // early refinement (ctx.hpp): the first chunk's finished frames refine on side[0] during the later chunks
#ifdef PITT_AB_VARIANTS
    const bool er_refine_default = ctx->refine_producers == 1 && ctx->refine_frames == 1 && !ctx->xrefine && !rdbg;
#else
    const bool er_refine_default = true;
#endif
    const bool er_base = ctx->early_refine && er_refine_default && !ctx->prof && K >= 2 && optimize &&
                         cov_mode != PITT_COV_FAST && !xs;
    if (er_base) {
        if (!ctx->side[0]) PITT_HIP_TRY(hipStreamCreateWithFlags(&ctx->side[0], hipStreamNonBlocking));
        for (hipEvent_t& e : ctx->er_ev)
            if (!e) PITT_HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    // chunks [c0, c1) with their replays (front: the state reset and first hypotheses before them), then
    // phase `phase`'s decisions, refinements, the final selection and the result copies
    auto enqueue = [=](int c0, int c1, int phase, bool front, std::vector<int>& acct_recs,
                       std::vector<int>& score_recs, bool er = false) -> int {
    int rec;
    bool er_launched = false;
    if (front) {
    PITT_HIP_TRY(hipMemsetAsync(zblock, 0, zero_bytes, sm));
    rec = ctx->prof_begin("k_hypothesize", 0.0);
    acct_recs[kAcHyp] = rec;
    hipLaunchKernelGGL((k_hypothesize<ORDER, DIV>), dim3(nf), dim3(kBlock), 0, sm, fx, fy, fz, meta,
                       tables, A, hcap, std::min(chunks[0], hcap), runnable_all, hyp_coef, hyp_attempt, st, lists,
                       counters, cstat, acct, dbg_seq);
    PITT_CHECK_LAUNCH("k_hypothesize", -1, phase);
    ctx->prof_end(rec);
    }
    int h0 = 0;
    for (int c = 0; c < c0; ++c) h0 += chunks[(size_t)c];
    for (int c = c0; c < c1; h0 += chunks[(size_t)c], ++c) {
        const int H = chunks[(size_t)c];
        rec = ctx->prof_begin("k_score", 0.0);
        if (c == 0) ctx->prof_alias(rec, "k_score.first");  // the first chunk: every frame, H hypotheses
        score_recs.push_back(rec);
#ifdef PITT_AB_VARIANTS
        const bool ins = ctx->inside_cull;
        auto kern = c == 0 ? (H <= 32 && ctx->lane_score ? k_score<ORDER, 1, true, true>
                              : ins ? (H <= 64 ? k_score<ORDER, 1, true, false, true> : H <= 128 ? k_score<ORDER, 2, true, false, true>
                                                : k_score<ORDER, 4, true, false, true>)
                                    : (H <= 64 ? k_score<ORDER, 1, true> : H <= 128 ? k_score<ORDER, 2, true> : k_score<ORDER, 4, true>))
                           : ins ? (H <= 64 ? k_score<ORDER, 1, false, false, true> : H <= 128 ? k_score<ORDER, 2, false, false, true>
                                             : k_score<ORDER, 4, false, false, true>)
                                 : (H <= 64 ? k_score<ORDER, 1, false> : H <= 128 ? k_score<ORDER, 2, false> : k_score<ORDER, 4, false>);
#else
        auto kern = c == 0 ? (H <= 64 ? k_score<ORDER, 1, true> : H <= 128 ? k_score<ORDER, 2, true> : k_score<ORDER, 4, true>)
                           : (H <= 64 ? k_score<ORDER, 1, false> : H <= 128 ? k_score<ORDER, 2, false> : k_score<ORDER, 4, false>);
#endif
        // the first chunk scores every frame (one item per wave); later ones stride over a capped grid
        const int64_t all_blocks = ((int64_t)nf * tiles_max + kScoreWaves - 1) / kScoreWaves;
        const int score_blocks = (int)(c == 0 ? all_blocks : std::min<int64_t>(all_blocks, kScoreGridCap));
        hipLaunchKernelGGL(kern, dim3(score_blocks), dim3(64 * kScoreWaves), 0, sm, fx, fy, fz, meta, st, hyp_coef,
                           hcap, hstride, lists + (size_t)c * nf, counters + c, tiles_max, h0, H, thf, tile_counts,
                           tile_box, group_box, nf, slots + (size_t)c * nf);
    PITT_CHECK_LAUNCH("k_score", c, phase);
        ctx->prof_end(rec);
        rec = ctx->prof_begin("k_replay", 0.0);
        if (c == 0) acct_recs[kAcReplay] = rec;  // every replay launch's bytes are counted in this one
        const int target_next = c + 1 < nchunks ? std::min(h0 + H + chunks[(size_t)c + 1], hcap) : 0;
        hipLaunchKernelGGL((k_replay<ORDER, DIV>), dim3(nf), dim3(kBlock), 0, sm, tile_counts, hcap, hstride,
                           tiles_max, h0, H, max_iter, log_prob, meta, st, hyp_total, lists + (size_t)(c + 1) * nf,
                           counters + c + 1, cstat + c + 1, fx, fy, fz, tables, A, target_next, hyp_coef,
                           hyp_attempt, acct, slots + (size_t)(c + 1) * nf);
    PITT_CHECK_LAUNCH("k_replay", c, phase);
        ctx->prof_end(rec);
        if (er && c == 0 && c1 >= 2) {
            // the frames done after the first chunk (the ones with the most inliers: they need the fewest
            // hypotheses) are decided now, as phase 3, and refined on the side stream while the later
            // chunks score the rest.  Nothing later on this stream touches them: k_replay and k_score
            // skip done frames, k_decide skips decided ones, k_refine below takes phase 1 only; the
            // selection waits for the side stream.
            hipLaunchKernelGGL(k_decide, dim3((nf + 255) / 256), dim3(256), 0, sm, meta, st, hyp_coef, hcap, nf,
                               optimize, best_coef, final_coef, 3);
            PITT_CHECK_LAUNCH("k_decide", -1, 3);
            PITT_HIP_TRY(hipEventRecord(ctx->er_ev[0], sm));
            PITT_HIP_TRY(hipStreamWaitEvent(ctx->side[0], ctx->er_ev[0], 0));
            hipLaunchKernelGGL((k_refine<ORDER, DIV, 1>), dim3(nf), dim3(64 * 3), 0, ctx->side[0], fx, fy, fz, meta,
                               st, best_coef, thf, tile_counts, hstride, tiles_max, final_coef, acct,
                               (unsigned long long*)nullptr, 2, (const int32_t*)nullptr, 3);
            PITT_CHECK_LAUNCH("k_refine", -1, 3);
            PITT_HIP_TRY(hipEventRecord(ctx->er_ev[1], ctx->side[0]));
            er_launched = true;
        }
    }
    hipLaunchKernelGGL(k_decide, dim3((nf + 255) / 256), dim3(256), 0, sm, meta, st, hyp_coef, hcap, nf,
                       optimize, best_coef, final_coef, phase);
    PITT_CHECK_LAUNCH("k_decide", -1, phase);
    // refinement (pass 1 over refined frames), then the final selection over every frame's tiles
    if (cov_mode == PITT_COV_FAST) {  // A6 fast mode: double sums over the chip, fixed tree
        rec = ctx->prof_begin("k_cov_tiles", 0.0);
        hipLaunchKernelGGL((k_cov_tiles<ORDER>), dim3(sel_blocks), dim3(kBlock), 0, sm, fx, fy, fz, meta, st,
                           best_coef, thf, tile_counts, hstride, nf, tiles_max, part);
        ctx->prof_end(rec);
        rec = ctx->prof_begin("k_cov_final", 0.0);
        hipLaunchKernelGGL((k_cov_final<ORDER>), dim3(nf), dim3(64), 0, sm, meta, st, part, nf, tiles_max, final_coef);
        ctx->prof_end(rec);
    } else if (xs) {  // small batch: the nine sums by the exact walk over the chip
        rec = ctx->prof_begin("k_refine:xsum", 0.0);
        const int xr_blocks = (int)(((int64_t)nf * tiles_max * kXrSplit + kWaves - 1) / kWaves);
        hipLaunchKernelGGL((k_xr_count<ORDER>), dim3(xr_blocks), dim3(kBlock), 0, sm, fx, fy, fz, meta, st, best_coef,
                           thf, nf, tiles_max, xr_tcnt, phase);
    PITT_CHECK_LAUNCH("k_xr_count", -1, phase);
        hipLaunchKernelGGL(k_xr_scan, dim3(nf), dim3(256), 0, sm, meta, tiles_max, xr_tcnt, xr_seg, xr_bseg);
    PITT_CHECK_LAUNCH("k_xr_scan", -1, phase);
        hipLaunchKernelGGL((k_xr_write<ORDER>), dim3(xr_blocks), dim3(kBlock), 0, sm, fx, fy, fz, meta, st, best_coef,
                           thf, nf, tiles_max, xr_tcnt, xr_seg, xr_v, xs_T, phase);
    PITT_CHECK_LAUNCH("k_xr_write", -1, phase);
        xs_enqueue(sm, xr_v, xs_T, 9, nf, xr_seg, xr_bseg, xr_sums, xr_scr);
    PITT_CHECK_LAUNCH("xs_enqueue", -1, phase);
        hipLaunchKernelGGL((k_xr_plane<ORDER, DIV>), dim3((nf + 63) / 64), dim3(64), 0, sm, st, xr_seg, xr_sums, nf,
                           final_coef, phase);
    PITT_CHECK_LAUNCH("k_xr_plane", -1, phase);
        ctx->prof_end(rec);
    } else {
#ifndef PITT_AB_VARIANTS
        rec = ctx->prof_begin("k_refine", 0.0);
        acct_recs[kAcRefine] = rec;
        hipLaunchKernelGGL((k_refine<ORDER, DIV, 1>), dim3(nf), dim3(64 * 3), 0, sm, fx, fy, fz, meta, st,
                           best_coef, thf, tile_counts, hstride, tiles_max, final_coef, acct,
                           (unsigned long long*)nullptr, 2, (const int32_t*)nullptr, phase);
    PITT_CHECK_LAUNCH("k_refine", -1, phase);
        ctx->prof_end(rec);
#else
        const int P = ctx->refine_producers;
        auto kern = P == 1 ? k_refine<ORDER, DIV, 1> : P == 2 ? k_refine<ORDER, DIV, 2>
                  : P == 3 ? k_refine<ORDER, DIV, 3> : k_refine<ORDER, DIV, 4>;
        if (ctx->xrefine) {  // binade runs; k_refine's chain only for frames it hands back
            rec = ctx->prof_begin("k_xrefine", 0.0);
            acct_recs[kAcRefine] = rec;
            hipLaunchKernelGGL((k_xrefine<ORDER, DIV>), dim3(nf), dim3(64 * kXW), 0, sm, fx, fy, fz, meta, st,
                               best_coef, thf, tile_counts, hstride, tiles_max, final_coef, xfallback,
                               counters + nchunks + 1, acct, ctx->xrefine == 2 ? 1 : 0, rdbg);
            ctx->prof_end(rec);
            rec = ctx->prof_begin("k_refine:fallback", 0.0);
            hipLaunchKernelGGL(kern, dim3(nf), dim3(64 * (P + 2)), 0, sm, fx, fy, fz, meta, st, best_coef,
                               thf, tile_counts, hstride, tiles_max, final_coef, nullptr, rdbg, ctx->refine_mode,
                               xfallback, phase);
            ctx->prof_end(rec);
        } else if (ctx->refine_frames > 1 && P == 1 && !rdbg) {  // F frames per block, one chain wave
            rec = ctx->prof_begin("k_refine", 0.0);
            acct_recs[kAcRefine] = rec;
            const int F = ctx->refine_frames == 3 && kRefineMulti3 ? 3 : 2;
            auto mk = refine_multi_kernel<ORDER, DIV>(F);
            hipLaunchKernelGGL(mk, dim3((nf + F - 1) / F), dim3(64 * (F + 2)), 0, sm, fx, fy, fz, meta, st,
                               best_coef, thf, tile_counts, hstride, tiles_max, nf, final_coef, acct, ctx->refine_mode);
            ctx->prof_end(rec);
        } else {
            rec = ctx->prof_begin("k_refine", 0.0);
            acct_recs[kAcRefine] = rec;
            hipLaunchKernelGGL(kern, dim3(nf), dim3(64 * (P + 2)), 0, sm, fx, fy, fz, meta, st, best_coef,
                               thf, tile_counts, hstride, tiles_max, final_coef, acct, rdbg, ctx->refine_mode,
                               nullptr, phase);
            ctx->prof_end(rec);
        }
#endif
    }
    if (er_launched) PITT_HIP_TRY(hipStreamWaitEvent(sm, ctx->er_ev[1], 0));  // the early refinements
    rec = ctx->prof_begin("k_sel_mark", 0.0);
    acct_recs[kAcSelMark] = rec;
    hipLaunchKernelGGL((k_sel_mark<ORDER>), dim3(sel_blocks), dim3(kBlock), 0, sm, fx, fy, fz, meta, st,
                       final_coef, thf, nf, tiles_max, tile_box, group_box, sel_bits, sel_cnt, acct_tiles);
    PITT_CHECK_LAUNCH("k_sel_mark", -1, phase);
    ctx->prof_end(rec);
    rec = ctx->prof_begin("k_sel_write", 0.0);
    acct_recs[kAcSelWrite] = rec;
    hipLaunchKernelGGL(k_sel_write, dim3(sel_blocks), dim3(kBlock), 0, sm, meta, st, nf, tiles_max, sel_bits, sel_cnt,
                       inliers_dev, n_final, acct_tiles ? acct_tiles + tile_words : nullptr);
    PITT_CHECK_LAUNCH("k_sel_write", -1, phase);
    ctx->prof_end(rec);
    hipLaunchKernelGGL(k_finalize, dim3((nf + 255) / 256), dim3(256), 0, sm, st, hyp_attempt, final_coef, n_final,
                       hcap, nf, dres);
    PITT_CHECK_LAUNCH("k_finalize", -1, phase);
    PITT_HIP_TRY(hipGetLastError());
    PITT_HIP_TRY(hipMemcpyAsync(hres, dres, (size_t)nf * sizeof(pitt_plane_result), hipMemcpyDeviceToHost, sm));
    PITT_HIP_TRY(hipMemcpyAsync(hstat, cstat, (size_t)(nchunks + 1) * sizeof(ChunkStat), hipMemcpyDeviceToHost, sm));
    PITT_HIP_TRY(hipMemcpyAsync(hxfb, counters + nchunks + 1, 4, hipMemcpyDeviceToHost, sm));
    if (rdbg) PITT_HIP_TRY(hipMemcpyAsync(ctx->refine_dbg_h, rdbg, (size_t)nf * 16 * 8, hipMemcpyDeviceToHost, sm));
    if (acct) {
        PITT_HIP_TRY(hipMemcpyAsync(hacct, acct, acct_bytes, hipMemcpyDeviceToHost, sm));
        PITT_HIP_TRY(hipMemcpyAsync((char*)hacct + acct_bytes, acct_tiles, tile_words * 2 * 4, hipMemcpyDeviceToHost, sm));
    }
    return PITT_OK;
    };
    auto enqueue_front = [&](bool er) -> int { return enqueue(0, K, 1, true, acct_recs, score_recs, er); };
#ifdef PITT_SYNC_CHECK
    *(volatile unsigned int*)dbg_seq = seq;
#endif
    {
        const int erc = enqueue_front(er_base);
        if (erc) return erc;
    }
#ifdef PITT_SYNC_CHECK
    std::fprintf(stderr, "PITT_SYNC_CHECK call seq %u nf %d n0 %lld K %d/%d xs %d xs_T %lld tiles_max %d gen %llu\n",
                 seq, nf, (long long)fr->counts[0], K, nchunks, (int)xs, (long long)xs_T, tiles_max,
                 (unsigned long long)ctx->arena_gen);
#endif
    // the continuation, should a frame still be running after the K chunks (finish_batch)
    ctx->inflight_k = K;
    ctx->inflight_hint_key = hint_key;
    ctx->inflight_cont = nullptr;
    if (K < nchunks)
        ctx->inflight_cont = [enqueue, K, nchunks](std::vector<int>& ar, std::vector<int>& sr) -> int {
            return enqueue(K, nchunks, 2, false, ar, sr);
        };
    // completion (pitt_wait): copy results out, price the score launches
    ctx->inflight = true;
    ctx->inflight_results = results;
    ctx->inflight_frames = nf;
    ctx->inflight_hres = hres;
    ctx->inflight_stat.assign((size_t)(nchunks + 1), {0, 0});
    ctx->inflight_score_recs = score_recs;
    ctx->inflight_chunks = chunks;
    ctx->inflight_hstat = hstat;
    ctx->inflight_xfb = (ctx->xrefine && p->optimize && p->cov_mode != PITT_COV_FAST) ? hxfb : nullptr;
    ctx->inflight_acct = hacct;
    ctx->inflight_acct_tiles = (int64_t)tile_words;
    ctx->inflight_acct_recs = acct_recs;
    ctx->last_hcap = hcap;
    ctx->last_frames = nf;
    return PITT_OK;
}

// Completes the batch enqueued on ctx (if any): waits for the stream, copies the per-frame results
// to the caller's array and fills in the algorithmic bytes of each k_score launch (12 B per point
// of every active frame's tiles + the per-tile count words written).
int finish_batch(pitt_ctx* ctx) {
    if (!ctx->inflight) return PITT_OK;
    ctx->inflight = false;
    PITT_HIP_TRY(hipStreamSynchronize(ctx->stream));
#ifdef PITT_SYNC_CHECK
    {
        unsigned int stale = 0, seen[4] = {0, 0, 0, 0};
        (void)hipMemcpyFromSymbol(&stale, HIP_SYMBOL(g_dbg_stale), sizeof stale);
        if (stale) {
            (void)hipMemcpyFromSymbol(seen, HIP_SYMBOL(g_dbg_seen), sizeof seen);
            std::fprintf(stderr, "PITT_SYNC_CHECK STALE METADATA: k_hypothesize read stamp %u (n %u, frame %u), host wrote %u\n",
                         seen[0], seen[2], seen[3], seen[1]);
            const unsigned int zero = 0;
            (void)hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_stale), &zero, sizeof zero);
            return ctx->fail(PITT_E_HIP, "sync check: a batch read stale frame metadata");
        }
    }
#endif
    const ChunkStat* cs = (const ChunkStat*)ctx->inflight_hstat;
    const int nchunks = (int)ctx->inflight_chunks.size();
    if (ctx->inflight_cont && cs[ctx->inflight_k].tiles > 0) {
        // frames still running after the scheduled chunks: the rest of the chunks, then their frames'
        // decisions, refinements and the selection (direct launches; rare once the hint has learnt)
#ifdef PITT_SYNC_CHECK
        std::fprintf(stderr, "PITT_SYNC_CHECK continuation after %d of %d chunks\n", ctx->inflight_k, nchunks);
#endif
        std::function<int(std::vector<int>&, std::vector<int>&)> cont = std::move(ctx->inflight_cont);
        ctx->inflight_cont = nullptr;
        const int rc = cont(ctx->inflight_acct_recs, ctx->inflight_score_recs);
        if (rc) return rc;
        PITT_HIP_TRY(hipStreamSynchronize(ctx->stream));
        ++ctx->continuations;
    }
    ctx->inflight_cont = nullptr;
    {  // chunks with active frames: the schedule the next batches of this layout launch
        int need = 1;
        for (int c = 1; c < nchunks; ++c)
            if (cs[c].tiles > 0) need = c + 1;  // (a listed frame adds its tiles)
        ctx->chunk_hint_update(ctx->inflight_hint_key, need);
    }
    std::memcpy(ctx->inflight_results, ctx->inflight_hres, (size_t)ctx->inflight_frames * sizeof(pitt_plane_result));
    if (ctx->inflight_xfb) {
        ++ctx->xrefine_batches;
        ctx->xrefine_fallbacks += *(const int32_t*)ctx->inflight_xfb;
    }
    if (ctx->refine_debug && ctx->refine_dbg_h) {  // mean / max over the refined frames, cycles
        const unsigned long long* d = (const unsigned long long*)ctx->refine_dbg_h;
        double sum[16] = {0}, mx[16] = {0};
        int cnt = 0;
        for (int f = 0; f < ctx->inflight_frames; ++f) {
            if (d[f * 16] == 0) continue;
            ++cnt;
            for (int k = 0; k < 16; ++k) {
                sum[k] += (double)d[f * 16 + k];
                mx[k] = std::max(mx[k], (double)d[f * 16 + k]);
            }
        }
        if (cnt) {
            static const char* names[14] = {"chain_cyc", "chain_spin", "form_cyc", "form_spin(hi:data lo:slot)",
                                            "p0_cyc", "p0_ticket", "p0_ring", "steps", "p1_cyc", "p1_ticket",
                                            "p1_ring", "p1_steps", "inliers", "chain_busy"};
            static const char* xnames[14] = {"cyc", "tiles", "windows", "list_xx", "list_xy", "list_xz", "list_yy",
                                             "list_yz", "list_zz", "list_x", "list_y", "list_z", "inliers", "-"};
            const char* const* nm = ctx->xrefine ? xnames : names;
            std::fprintf(stderr, "[refine_debug] frames %d producers %d xrefine %d\n", cnt, ctx->refine_producers,
                         ctx->xrefine);
            for (int k = 0; k < 14; ++k)
                std::fprintf(stderr, "[refine_debug] %-28s mean %14.1f max %14.1f\n", nm[k], sum[k] / cnt, mx[k]);
        }
    }
    const ChunkStat* hstat = (const ChunkStat*)ctx->inflight_hstat;
    for (size_t c = 0; c < ctx->inflight_score_recs.size(); ++c)
        ctx->prof_set_bytes(ctx->inflight_score_recs[c],
                            (double)hstat[c].tiles * kTile * 12.0 + (double)hstat[c].tiles * ctx->inflight_chunks[c] * 4.0);
    if (ctx->inflight_acct) {  // the data-dependent kernels: bytes they actually moved
        const unsigned long long* a = (const unsigned long long*)ctx->inflight_acct;
        const uint32_t* tw = (const uint32_t*)(a + kAcKernels * kAcShards);
        const int64_t nt = ctx->inflight_acct_tiles;
        for (int k = 0; k < kAcKernels; ++k) {
            double b = 0;
            if (k == kAcSelMark || k == kAcSelWrite) {
                const uint32_t* v = tw + (k == kAcSelMark ? 0 : nt);
                for (int64_t i = 0; i < nt; ++i) b += (double)v[i];
            } else {
                for (int j = 0; j < kAcShards; ++j) b += (double)a[k * kAcShards + j];
            }
            ctx->prof_set_bytes(ctx->inflight_acct_recs[(size_t)k], b);
        }
        ctx->inflight_acct = nullptr;
    }
    return PITT_OK;
}

int plane_segment_batch_impl(pitt_ctx* ctx, const pitt_frames* fr, const pitt_sac_params* p,
                             pitt_plane_result* results, int32_t* inliers_dev) {
    int rc = finish_batch(ctx);  // one batch in flight per context
    if (rc) return rc;
    const int key = p->reduce_order * 2 + (p->div_mode ? 1 : 0);
    switch (key) {
    case 0: return run_plane_batch<0, 0>(ctx, fr, p, results, inliers_dev);
    case 1: return run_plane_batch<0, 1>(ctx, fr, p, results, inliers_dev);
    case 2: return run_plane_batch<1, 0>(ctx, fr, p, results, inliers_dev);
    case 3: return run_plane_batch<1, 1>(ctx, fr, p, results, inliers_dev);
    case 4: return run_plane_batch<2, 0>(ctx, fr, p, results, inliers_dev);
    case 5: return run_plane_batch<2, 1>(ctx, fr, p, results, inliers_dev);
    default: return ctx->fail(PITT_E_INVALID, "reduce_order / div_mode out of range");
    }
}

}  // namespace pitt
