// ctx.hpp -- pitt_ctx: device, stream, scratch arena, sampler-table cache, kernel profiler.
#pragma once
#include <cstdlib>
#include <hip/hip_runtime.h>

#include <array>
#include <chrono>
#include <cstdint>
#include <functional>
#include <map>
#include <tuple>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/pitt_seg.h"

#define PITT_HIP_TRY(expr)                                                          \
    do {                                                                            \
        hipError_t e_ = (expr);                                                     \
        if (e_ != hipSuccess) {                                                     \
            return ctx->fail(PITT_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
        }                                                                           \
    } while (0)

namespace pitt {

inline double wall_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// One growable device buffer.
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

struct ProfRec {
    std::string name;
    std::string alias;  // optional second total the launch is also counted in (e.g. one chunk)
    hipEvent_t a = nullptr, b = nullptr;
    double bytes = 0;
};

struct ProfTotal {
    int64_t launches = 0;
    double ms = 0;
    double bytes = 0;
};

}  // namespace pitt

#ifndef PITT_REFINE_PRODUCERS_DEFAULT
#define PITT_REFINE_PRODUCERS_DEFAULT 1
#endif

// A boolean knob from the environment ("0" / "1"), read when a context is created.
inline bool pitt_env_flag(const char* name, bool dflt) {
    const char* v = std::getenv(name);
    return v && *v ? (v[0] != '0') : dflt;
}
// A small integer knob from the environment, clamped to [lo, hi].
inline int pitt_env_int(const char* name, int dflt, int lo, int hi) {
    const char* v = std::getenv(name);
    const int x = v && *v ? std::atoi(v) : dflt;
    return x < lo ? lo : x > hi ? hi : x;
}

struct pitt_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    // a second context on its own stream for work that overlaps this one's (pitt_classify_clusters runs
    // the plane service's batch there beside the other services); created on first use
    pitt_ctx* aux = nullptr;
    // two more streams for independent service runs (pitt_classify_clusters), created on first use
    hipStream_t side[2] = {nullptr, nullptr};
    std::string err;

    // scratch arena: named growable buffers (contents undefined between calls)
    std::unordered_map<std::string, pitt::DevBuf> bufs;
    std::unordered_map<std::string, std::pair<void*, size_t>> host_pinned;

    // sampler tables (host) keyed by (n, seed, attempts)
    std::map<std::tuple<int64_t, uint32_t, int64_t, int>, std::vector<int32_t>> tables;
    // device pool of the last batch's tables
    std::vector<std::tuple<int64_t, uint32_t, int64_t>> pool_keys;

    // Kernel variants kept for A/B measurements.  Only a library built with
    // -DPITT_AB_VARIANTS (`make ab`: libpitt_seg_ab.so, loaded by tools/ and the variant tests through
    // $PITT_LIB_PATH) reads them from the environment and instantiates their kernels.  The product
    // library fixes them at the defaults below and ignores the environment, so no setting can make
    // it run a variant -- in particular not the chain-without-adds measurement (refine_mode bit 2).
#ifdef PITT_AB_VARIANTS
    static constexpr bool kVariants = true;
    // first scoring chunk with lane-private counters (k_score LANE); $PITT_LANE_SCORE overrides
    bool lane_score = pitt_env_flag("PITT_LANE_SCORE", false);
    // k_score: pairs whose group box lies certainly inside the slab count the group without scoring
    // (exact; measured 1-3 % slower on the table batch, so off by default)
    bool inside_cull = pitt_env_flag("PITT_INSIDE_CULL", false);
    // producer waves of k_refine (1..4); $PITT_REFINE_PRODUCERS overrides
    int refine_producers = pitt_env_int("PITT_REFINE_PRODUCERS", PITT_REFINE_PRODUCERS_DEFAULT, 1, 4);
    // frames per k_refine block (1: k_refine; 2, 3: k_refine_multi, one chain wave for all of them)
    int refine_frames = pitt_env_int("PITT_REFINE_FRAMES", 1, 1, 3);
    // k_refine variant (bit 1: producers write inlier lanes only, as masked stores)
    // bit 2: chain without adds (a measurement: WRONG planes); bit 3: the chain prefetches across
    // block boundaries
    int refine_mode = pitt_env_int("PITT_REFINE_MODE", 2, 0, 15);
    // $PITT_XREFINE=1: optimizeModelCoefficients' sums by binade runs (k_xrefine, bit-exact, measured
    // slower than k_refine's chain: DESIGN.md s6); 2: k_xrefine hands every frame back (tests)
    int xrefine = pitt_env_int("PITT_XREFINE", 0, 0, 2);
    // $PITT_REFINE_DEBUG=1: k_refine records per-role cycles and spins, printed at completion
    bool refine_debug = pitt_env_flag("PITT_REFINE_DEBUG", false);
#else
    static constexpr bool kVariants = false;
    static constexpr bool lane_score = false;
    static constexpr bool inside_cull = false;
    static constexpr int refine_producers = 1;
    static constexpr int refine_frames = 1;
    static constexpr int refine_mode = 2;
    static constexpr int xrefine = 0;
    static constexpr bool refine_debug = false;
#endif
    int64_t xrefine_batches = 0, xrefine_fallbacks = 0;  // frames k_xrefine handed back to k_refine
    void* refine_dbg_h = nullptr;

    // Adaptive chunk schedule (plane_ransac.hip): a batch launches the scoring chunks that the last
    // batches of its layout needed; a frame still running after them is finished by a continuation.
    // Exact either way; $PITT_ADAPTIVE_CHUNKS=0 always launches the whole schedule.
    bool adaptive_chunks = pitt_env_flag("PITT_ADAPTIVE_CHUNKS", true);
    // batches of up to this many frames refine through the chip-wide exact walk (xsum.hpp) instead of
    // k_refine's per-frame chain (same sums, lower latency); $PITT_XS_MAX_FRAMES=0 keeps the chain always
    int xs_max_frames = pitt_env_int("PITT_XS_MAX_FRAMES", 8, 0, 1 << 30);
    // Early refinement ($PITT_EARLY_REFINE=1, off by default): when a batch launches two or more scoring
    // chunks, the frames that finished in the first are decided and refined on side[0] while the later
    // chunks score the rest (profiled runs keep one stream).
    // Bit-exact, but measured slower on the pipelined headline.
    bool early_refine = pitt_env_flag("PITT_EARLY_REFINE", false);
    hipEvent_t er_ev[2] = {nullptr, nullptr};  // first-chunk decisions made | early refinement done
    // pitt_plane_segment: points converted (AoS -> SoA) per staged H2D copy; 0 = one copy of the cloud.
    // $PITT_HOST_TIMING=1 prints its host phases to stderr.
    int64_t single_chunk = pitt_env_int("PITT_SINGLE_CHUNK", 1 << 16, 0, 1 << 30);
    // $PITT_SINGLE_MODE bit 0: the caller's AoS bytes go up in one pageable copy and the device deinterleaves
    // them (else the host deinterleaves into pinned chunks); bit 1: the inliers come down straight into the
    // caller's memory (else through a pinned copy behind the batch)
    int single_mode = pitt_env_int("PITT_SINGLE_MODE", 3, 0, 3);
    bool host_timing = pitt_env_flag("PITT_HOST_TIMING", false);
    struct ChunkHint {
        std::array<uint64_t, 4> key;  // frame planes, frames, hypothesis cap, tiles
        int need[16];                 // chunks with active frames in the last batches (0: none yet)
        int pos;
        uint64_t last_use;
    };
    std::vector<ChunkHint> chunk_hints;
    uint64_t hint_clock = 0;
    int64_t continuations = 0;        // batches that ran past their scheduled chunks
    // chunks to launch for a layout: the most the last sixteen batches needed (all of them when unknown).
    // A long window: a continuation re-runs the decision / refinement / selection launches for the frames
    // it finishes, which costs about one refinement latency (~0.7 ms on the table batch), while a
    // scoring chunk with no active frame costs ~10 us -- a layout that needed more chunks once in a
    // while keeps launching them (bench.py streaming: a cluttered batch in every five).
    int chunk_hint(const std::array<uint64_t, 4>& key, int all) {
        for (ChunkHint& h : chunk_hints)
            if (h.key == key) {
                h.last_use = ++hint_clock;
                int k = 0;
                for (int v : h.need) k = v > k ? v : k;
                return k > 0 ? k : all;
            }
        return all;
    }
    void chunk_hint_update(const std::array<uint64_t, 4>& key, int need) {
        ChunkHint* h = nullptr;
        for (ChunkHint& e : chunk_hints)
            if (e.key == key) h = &e;
        if (!h) {
            if (chunk_hints.size() >= 16) {
                size_t lru = 0;
                for (size_t i = 1; i < chunk_hints.size(); ++i)
                    if (chunk_hints[i].last_use < chunk_hints[lru].last_use) lru = i;
                chunk_hints.erase(chunk_hints.begin() + (long)lru);
            }
            chunk_hints.push_back(ChunkHint{key, {}, 0, ++hint_clock});
            h = &chunk_hints.back();
        }
        h->need[h->pos] = need;
        h->pos = (h->pos + 1) & 15;
    }
    uint64_t arena_gen = 0;  // bumped whenever an arena buffer moves (memoised device tables hold its pointers)
    // prim_ransac.hpp: which sampler table each cloud slot of a model's device table buffer holds (the
    // buffer's address, arena generation and slot stride when they were uploaded), so a repeat skips
    // the upload
    struct PrimTableMemo {
        const void* dev = nullptr;
        uint64_t gen = 0;
        int64_t stride = -1;  // attempts per slot (A): slot c starts at c * A * kSample
        std::vector<std::tuple<int64_t, uint32_t, int64_t>> keys;
    };
    std::unordered_map<std::string, PrimTableMemo> prim_tables;
    uint32_t call_seq = 0;  // plane batches enqueued; stamped into each frame's metadata (FrameMeta.pad)

    // profiling
    bool prof = false;
    std::vector<pitt::ProfRec> pending;
    std::vector<hipEvent_t> event_pool;
    std::map<std::string, pitt::ProfTotal> totals;

    // batch in flight (pitt_plane_segment_batch_async until pitt_wait)
    bool inflight = false;
    pitt_plane_result* inflight_results = nullptr;
    int inflight_frames = 0;
    void* inflight_hres = nullptr;
    void* inflight_hstat = nullptr;
    void* inflight_xfb = nullptr;   // k_xrefine fallback count (pinned), when it ran
    std::vector<std::pair<int64_t, int64_t>> inflight_stat;
    std::vector<int> inflight_score_recs;
    std::vector<int> inflight_chunks;
    void* inflight_acct = nullptr;        // pinned copy of the device byte counters (profiling)
    std::vector<int> inflight_acct_recs;  // profiler record per counted kernel (-1: none)
    int64_t inflight_acct_tiles = 0;      // per-tile byte words following the counters
    int inflight_k = 0;                   // scoring chunks the batch launched
    std::array<uint64_t, 4> inflight_hint_key = {0, 0, 0, 0};
    std::function<int(std::vector<int>&, std::vector<int>&)> inflight_cont;  // the rest of the chunks, if any

    // support loop: z sums that could not be certified and ran the sequential loop (diagnostic)
    int64_t zsum_sequential = 0;

    // last batch (debug / parity hooks)
    int32_t last_hcap = 0;
    int32_t last_frames = 0;

    // results kept alive for list-returning calls
    std::vector<pitt_support> keep_supports;
    std::vector<pitt_support_dev> keep_supports_dev;
    std::vector<pitt_cluster> keep_clusters;
    std::vector<pitt_cluster_dev> keep_clusters_dev;
    std::vector<pitt_object> keep_objects;

    int fail(int code, const std::string& msg) {
        err = msg;
        return code;
    }
    // Waits for the work queued on the context's stream and its side streams.
    void drain();
    // Debug builds (-DPITT_SYNC_CHECK): every arena block carries a 256 KB canary past its rounded size,
    // and a 256 MB sentinel block catches wild writes; check_canaries names any corrupted one (a no-op
    // in the product build).
    void check_canaries(const char* where);
    void* sentinel = nullptr;
    // Device scratch buffer `name` of at least `bytes` (grows, never shrinks).  A block that moves
    // is freed only after drain(), and bumps arena_gen (memoised device contents are then stale).
    void* buf(const std::string& name, size_t bytes);
    // Pinned host buffer (the same rules: drain() before a free, arena_gen bumped on a move).
    void* pinned(const std::string& name, size_t bytes);

    // Profiler hooks around a launch.
    int prof_begin(const char* name, double bytes);
    void prof_end(int rec);
    void prof_set_bytes(int rec, double bytes) {
        if (rec >= 0 && rec < (int)pending.size()) pending[(size_t)rec].bytes = bytes;
    }
    void prof_alias(int rec, const char* alias) {
        if (rec >= 0 && rec < (int)pending.size()) pending[(size_t)rec].alias = alias;
    }
    int prof_collect();
};

namespace pitt {
// Host sampler table (A2): attempts*3 indices of drawIndexSample for n points.
// (k = 4: the sphere model's samples)
const std::vector<int32_t>& sampler_table(pitt_ctx* ctx, int64_t n, uint32_t seed, int64_t attempts, int k = 3);
// Smallest float t with (double)|d| < th  <=>  |d| < t for every float d (A4).
float float_threshold(double th);
}  // namespace pitt
