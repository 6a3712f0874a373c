// exact_sum_proto.cpp -- CPU prototype of the block-parallel exact sequential float sum (the algorithm
// csrc/xsum.hpp runs on the device).  s_{i+1} = fl(s_i + v_i), s_0 = +0, reproduced bit for bit:
//
//   phase 1  (parallel)  an estimate of every block's entry sum: double prefix sums of the blocks;
//   phase 2  (parallel)  per block of B elements, for the binade (and sign) of its estimated entry:
//                        q_j = round-to-nearest(v_j / u) with u the binade's float spacing, R = sum q_j,
//                        the prefix minimum / maximum of the partial q sums, and whether any v_j / u is
//                        a tie (fractional part exactly 1/2) or out of range;
//   phase 3  (serial over blocks)  with the exact running float s: when s lies in the block's assumed
//                        binade with the right sign, s = K u, and every partial K + P_m stays inside the
//                        binade's interior [2^23 + 1, 2^24 - 1] with no tie, every rounding of the block
//                        is the integer step q_j, so s = (K + R) u; otherwise the block is added element by
//                        element (exact by construction).
//
// g++ -O2 -ffp-contract=off -std=c++17 tools/exact_sum_proto.cpp -o /tmp/xsum && /tmp/xsum
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

struct Blk {
    int e;          // binade exponent of the assumed entry (|s| in [2^e, 2^(e+1))), or INT32_MIN: no assumption
    int neg;        // entry sign
    int64_t R, mn, mx;
    int bad;        // a tie or an out-of-range quotient: never valid
};

static float seq_sum(const std::vector<float>& v) {
    float s = 0.0f;
    for (float x : v) s = s + x;
    return s;
}

static int binade(double a) {  // floor(log2 |a|) for a normal float magnitude
    int e;
    std::frexp(a, &e);
    return e - 1;
}

struct Stats {
    int64_t blocks = 0, dirty = 0;
};

static float block_sum(const std::vector<float>& v, int B, Stats* st) {
    const int64_t n = (int64_t)v.size();
    const int64_t nb = (n + B - 1) / B;
    // phase 1: block entry estimates (double prefix)
    std::vector<double> est((size_t)nb);
    double acc = 0.0;
    for (int64_t b = 0; b < nb; ++b) {
        est[(size_t)b] = acc;
        for (int64_t i = b * B; i < std::min(n, (b + 1) * B); ++i) acc += (double)v[(size_t)i];
    }
    // phase 2: per block integer steps for the estimated binade
    std::vector<Blk> blk((size_t)nb);
    for (int64_t b = 0; b < nb; ++b) {
        Blk& k = blk[(size_t)b];
        const double a = est[(size_t)b];
        if (!(std::fabs(a) >= (double)FLT_MIN) || !(std::fabs(a) <= (double)FLT_MAX)) {
            k.e = INT32_MIN;
            continue;
        }
        k.e = binade(a);
        k.neg = a < 0;
        const double scale = std::ldexp(1.0, 23 - k.e);  // 1 / u
        int64_t P = 0, mn = 0, mx = 0;
        k.bad = 0;
        for (int64_t i = b * B; i < std::min(n, (b + 1) * B); ++i) {
            double x = (double)v[(size_t)i] * scale;  // exact (a float times a power of two, in range)
            if (k.neg) x = -x;                        // steps in magnitude
            if (!(std::fabs(x) < 4.0e15)) {
                k.bad = 1;
                break;
            }
            const double fl = std::floor(x);
            if (x - fl == 0.5) {
                k.bad = 1;
                break;
            }
            P += (int64_t)std::nearbyint(x);
            mn = std::min(mn, P);
            mx = std::max(mx, P);
        }
        k.R = P;
        k.mn = mn;
        k.mx = mx;
    }
    // phase 3: the exact walk over blocks
    float s = 0.0f;
    for (int64_t b = 0; b < nb; ++b) {
        const Blk& k = blk[(size_t)b];
        bool ok = k.e != INT32_MIN && !k.bad && s != 0.0f && std::isfinite(s);
        if (ok) {
            const double a = std::fabs((double)s);
            ok = binade(a) == k.e && ((s < 0) == (k.neg != 0));
            if (ok) {
                const int64_t K = (int64_t)std::ldexp(a, 23 - k.e);  // exact integer in [2^23, 2^24)
                const int64_t lo = (1ll << 23) + 1, hi = (1ll << 24) - 1;
                ok = K + k.mn >= lo && K + k.mx <= hi && K >= lo && K <= hi;
                if (ok) {
                    const double r = std::ldexp((double)(K + k.R), k.e - 23);
                    s = (float)(k.neg ? -r : r);
                }
            }
        }
        ++st->blocks;
        if (!ok) {
            ++st->dirty;
            for (int64_t i = b * B; i < std::min(n, (b + 1) * B); ++i) s = s + v[(size_t)i];
        }
    }
    return s;
}

int main() {
    std::mt19937_64 rng(7);
    std::normal_distribution<double> N(0.0, 1.0);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    int fails = 0;
    struct Case {
        const char* name;
        std::vector<float> v;
    };
    std::vector<Case> cases;
    const int n = 600000;
    {  // table-like: x around -0.3..0.3 (sum oscillates), x*x, x*z, z ~ 1.2
        std::vector<float> x(n), xx(n), xz(n), z(n);
        for (int i = 0; i < n; ++i) {
            const float xi = (float)(-0.4 + 0.8 * ((i % 640) / 640.0) + 0.001 * N(rng));
            const float zi = (float)(1.1 + 0.05 * U(rng));
            x[i] = xi;
            z[i] = zi;
            xx[i] = xi * xi;
            xz[i] = xi * zi;
        }
        cases.push_back({"x (oscillating)", x});
        cases.push_back({"x*x", xx});
        cases.push_back({"x*z", xz});
        cases.push_back({"z", z});
    }
    {
        std::vector<float> v(n);
        for (int i = 0; i < n; ++i) v[i] = (float)N(rng);
        cases.push_back({"normal", v});
        for (int i = 0; i < n; ++i) v[i] = (float)((i & 1) ? -1.0 : 1.0) * (float)(0.25 + 0.5 * U(rng));
        cases.push_back({"alternating", v});
        for (int i = 0; i < n; ++i) v[i] = (float)((int)(U(rng) * 1024) - 512) / 256.0f;
        cases.push_back({"dyadic", v});
        for (int i = 0; i < n; ++i) v[i] = 1.0f + (float)(i % 7) * std::ldexp(1.0f, -20);
        cases.push_back({"powers-of-two walk", v});
        for (int i = 0; i < n; ++i) v[i] = (float)(1000.0 + U(rng));
        cases.push_back({"large", v});
        for (int i = 0; i < n; ++i) v[i] = (float)((U(rng) - 0.3) * 1e-38);
        cases.push_back({"denormal-ish", v});
        v.assign(5000, 0.0f);
        for (int i = 0; i < 5000; ++i) v[i] = (float)(U(rng) - 0.5);
        cases.push_back({"short", v});
    }
    for (int B : {16, 32, 64, 256}) {
        for (const Case& c : cases) {
            Stats st;
            const float a = seq_sum(c.v), b = block_sum(c.v, B, &st);
            uint32_t ua, ub;
            std::memcpy(&ua, &a, 4);
            std::memcpy(&ub, &b, 4);
            const bool eq = ua == ub;
            fails += !eq;
            std::printf("B %4d %-22s seq %.9g block %.9g %s  dirty %lld / %lld\n", B, c.name, a, b, eq ? "EQUAL" : "DIFF",
                        (long long)st.dirty, (long long)st.blocks);
        }
    }
    std::printf("%s\n", fails ? "FAILURES" : "all bit-exact");
    return fails ? 1 : 0;
}
