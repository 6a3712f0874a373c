// synth.cpp -- deterministic synthetic organised clouds.
//
// A Kinect-like pinhole camera (fx = fy = 525, cx = 319.5, cy = 239.5; camera optical frame:
// x right, y down, z forward) ray-casts a room with a floor, walls, a table top and objects on
// the table (boxes, vertical cylinders, spheres).  Depth noise is Gaussian-like with
// sigma = 1.5 mm + 0.0019 z^2 (Irwin-Hall of 4 hashed uniforms), so every point is a pure
// function of (scene_seed, pixel): no sequential RNG, reproducible across hosts.
// Pixel (u, v) -> point index v * width + u, which is what fromROSMsg yields for an organised
// PointCloud2 (reference pc_manager.cpp:85-89).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <vector>

#include "../../include/pitt_seg.h"

namespace {

inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
inline double hash_uniform(uint64_t seed, uint64_t a, uint64_t b) {
    return (double)(mix64(seed ^ mix64(a * 0x100000001B3ull + b)) >> 11) * 0x1.0p-53;
}

struct Rng {
    uint64_t s;
    double uni() { s = mix64(s); return (double)(s >> 11) * 0x1.0p-53; }
    double range(double a, double b) { return a + (b - a) * uni(); }
};

struct V3 {
    double x, y, z;
};
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator*(V3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
inline double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

enum ObjType { BOX, CYL, SPH };
struct Obj {
    ObjType t;
    double cx, cy, cz;   // footprint centre (cz = base height; sphere: centre height)
    double a, b, h;      // box: half x, half y, height; cyl: radius, -, height; sph: radius
};

struct Scene {
    bool room = true;             // floor + walls
    double wall_x = 2.2, wall_y = 3.0, wall_back = -1.5, ceil_z = 3.0;
    bool bg_sphere = false;       // clutter: curved background instead of a room
    V3 bg_c{0, 0, 0};
    double bg_r = 6.0;
    double table_h = 0.75, tx0 = -0.7, tx1 = 0.7, ty0 = 0.4, ty1 = 1.3;
    std::vector<Obj> objs;
    V3 cam;
    V3 ax, ay, az;                // camera optical axes in world
};

// Objects on the table top, pairwise separated by > 6 cm and > 8 cm from the edges.
void place_objects(Scene& s, Rng& r, int count) {
    int tries = 0;
    while ((int)s.objs.size() < count && tries < 500) {
        ++tries;
        Obj o;
        int k = (int)(r.uni() * 3.0);
        o.t = k == 0 ? BOX : (k == 1 ? CYL : SPH);
        if (o.t == BOX) { o.a = r.range(0.03, 0.08); o.b = r.range(0.03, 0.08); o.h = r.range(0.05, 0.20); }
        if (o.t == CYL) { o.a = r.range(0.025, 0.06); o.b = o.a; o.h = r.range(0.06, 0.25); }
        if (o.t == SPH) { o.a = r.range(0.03, 0.08); o.b = o.a; o.h = 2 * o.a; }
        double ext = std::max(o.a, o.b) * 1.5;
        o.cx = r.range(s.tx0 + 0.08 + ext, s.tx1 - 0.08 - ext);
        o.cy = r.range(s.ty0 + 0.08 + ext, s.ty1 - 0.08 - ext);
        o.cz = o.t == SPH ? s.table_h + o.a : s.table_h;
        bool ok = true;
        for (const Obj& q : s.objs) {
            double need = ext + std::max(q.a, q.b) * 1.5 + 0.06;
            if (std::hypot(o.cx - q.cx, o.cy - q.cy) < need) { ok = false; break; }
        }
        if (ok) s.objs.push_back(o);
    }
}

void look_at(Scene& s, V3 cam, double yaw, double pitch) {
    s.cam = cam;
    // forward in world: yaw about +z, pitch below the horizon
    V3 f{std::sin(yaw) * std::cos(pitch), std::cos(yaw) * std::cos(pitch), -std::sin(pitch)};
    V3 rgt{std::cos(yaw), -std::sin(yaw), 0.0};
    // y_c = z_c x x_c (down)
    V3 dn{f.y * rgt.z - f.z * rgt.y, f.z * rgt.x - f.x * rgt.z, f.x * rgt.y - f.y * rgt.x};
    s.ax = rgt;
    s.ay = dn;
    s.az = f;
}

Scene make_scene(int kind, uint64_t seed) {
    Scene s;
    Rng r{mix64(seed * 0x2545F4914F6CDD1Dull + 17)};
    if (kind == PITT_SCENE_CLUTTER) {
        // No dominant plane: a small table (~8 % of pixels) inside a curved background,
        // surrounded by many spheres and cylinders.
        s.room = false;
        s.bg_sphere = true;
        s.table_h = 0.75;
        s.tx0 = -0.22; s.tx1 = 0.22; s.ty0 = 1.0; s.ty1 = 1.35;
        s.bg_c = {r.range(-0.3, 0.3), r.range(1.0, 1.6), r.range(0.4, 1.0)};
        s.bg_r = r.range(3.5, 4.5);
        place_objects(s, r, 2);
        int extra = 60;
        for (int i = 0; i < extra; ++i) {
            Obj o;
            o.t = (i % 3 == 0) ? CYL : SPH;
            o.a = r.range(0.04, 0.16);
            o.b = o.a;
            o.h = r.range(0.2, 1.6);
            o.cx = r.range(-1.6, 1.6);
            o.cy = r.range(1.5, 3.2);
            o.cz = o.t == SPH ? r.range(0.0, 1.9) : r.range(-0.2, 0.8);
            s.objs.push_back(o);
        }
        look_at(s, {0.0, 0.0, s.table_h + 0.55}, r.range(-0.05, 0.05), r.range(0.45, 0.55));
        return s;
    }
    // Table-dominant: the table top covers about half of the pixels.
    s.table_h = r.range(0.72, 0.78);
    double w = r.range(1.3, 1.7);
    s.tx0 = -w / 2;
    s.tx1 = w / 2;
    s.ty0 = r.range(0.35, 0.45);
    s.ty1 = s.ty0 + r.range(0.75, 0.95);
    place_objects(s, r, 3 + (int)(r.uni() * 4.0));  // 3-6 objects
    double pitch = r.range(30.0, 40.0) * M_PI / 180.0;
    double yaw = r.range(-8.0, 8.0) * M_PI / 180.0;
    look_at(s, {r.range(-0.05, 0.05), 0.0, s.table_h + r.range(0.58, 0.68)}, yaw, pitch);
    return s;
}

// Ray cast: returns the parameter t of the nearest hit (inf if none).
double cast(const Scene& s, V3 o, V3 d) {
    const double inf = std::numeric_limits<double>::infinity();
    double best = inf;
    auto take = [&](double t) { if (t > 1e-6 && t < best) best = t; };
    if (s.room) {
        if (d.z < 0) take(-o.z / d.z);
        if (d.z > 0) take((s.ceil_z - o.z) / d.z);
        if (d.y > 0) take((s.wall_y - o.y) / d.y);
        if (d.y < 0) take((s.wall_back - o.y) / d.y);
        if (d.x > 0) take((s.wall_x - o.x) / d.x);
        if (d.x < 0) take((-s.wall_x - o.x) / d.x);
    }
    if (s.bg_sphere) {
        V3 oc = o - s.bg_c;
        double b = dot(oc, d), c = dot(oc, oc) - s.bg_r * s.bg_r, dd = dot(d, d);
        double disc = b * b - dd * c;
        if (disc >= 0) take((-b + std::sqrt(disc)) / dd);
    }
    // table top (thin slab seen from above)
    if (d.z < 0 && o.z > s.table_h) {
        double t = (s.table_h - o.z) / d.z;
        V3 p = o + d * t;
        if (p.x >= s.tx0 && p.x <= s.tx1 && p.y >= s.ty0 && p.y <= s.ty1) take(t);
    }
    for (const Obj& ob : s.objs) {
        if (ob.t == SPH) {
            V3 c{ob.cx, ob.cy, ob.cz};
            V3 oc = o - c;
            double b = dot(oc, d), cc = dot(oc, oc) - ob.a * ob.a, dd = dot(d, d);
            double disc = b * b - dd * cc;
            if (disc >= 0) take((-b - std::sqrt(disc)) / dd);
        } else if (ob.t == CYL) {
            double ox = o.x - ob.cx, oy = o.y - ob.cy;
            double A = d.x * d.x + d.y * d.y, B = ox * d.x + oy * d.y, C = ox * ox + oy * oy - ob.a * ob.a;
            double disc = B * B - A * C;
            if (A > 0 && disc >= 0) {
                double t = (-B - std::sqrt(disc)) / A;
                double z = o.z + t * d.z;
                if (z >= ob.cz && z <= ob.cz + ob.h) take(t);
            }
            if (d.z != 0) {  // top cap
                double t = (ob.cz + ob.h - o.z) / d.z;
                double px = o.x + t * d.x - ob.cx, py = o.y + t * d.y - ob.cy;
                if (px * px + py * py <= ob.a * ob.a) take(t);
            }
        } else {  // axis-aligned box [cx-a, cx+a] x [cy-b, cy+b] x [cz, cz+h] (slab test)
            double lo[3] = {ob.cx - ob.a, ob.cy - ob.b, ob.cz};
            double hi[3] = {ob.cx + ob.a, ob.cy + ob.b, ob.cz + ob.h};
            double oo[3] = {o.x, o.y, o.z}, dv[3] = {d.x, d.y, d.z};
            double t0 = -inf, t1 = inf;
            bool miss = false;
            for (int k = 0; k < 3; ++k) {
                if (dv[k] == 0) {
                    if (oo[k] < lo[k] || oo[k] > hi[k]) { miss = true; break; }
                    continue;
                }
                double ta = (lo[k] - oo[k]) / dv[k], tb = (hi[k] - oo[k]) / dv[k];
                if (ta > tb) std::swap(ta, tb);
                t0 = std::max(t0, ta);
                t1 = std::min(t1, tb);
            }
            if (!miss && t0 <= t1) take(t0);
        }
    }
    return best;
}

// Render one view.  world == false: points in the camera optical frame; else world frame.
void render(const Scene& s, uint64_t seed, int W, int H, bool world, bool with_nan, float* X,
            float* Y, float* Z) {
    // Kinect intrinsics at 640x480 (fx = fy = 525, cx = 319.5, cy = 239.5), scaled with the
    // resolution so smaller test clouds see the same scene.
    const double fx = 525.0 * W / 640.0, fy = 525.0 * H / 480.0;
    const double cx = 0.5 * (W - 1), cy = 0.5 * (H - 1);
    for (int v = 0; v < H; ++v) {
        for (int u = 0; u < W; ++u) {
            const uint64_t pix = (uint64_t)v * (uint64_t)W + (uint64_t)u;
            const double dcx = (u - cx) / fx, dcy = (v - cy) / fy;  // d_c = (dcx, dcy, 1)
            V3 d = s.ax * dcx + s.ay * dcy + s.az;
            double t = cast(s, s.cam, d);
            float px, py, pz;
            bool invalid = !std::isfinite(t) || (with_nan && hash_uniform(seed, pix, 7) < 0.05);
            if (invalid) {
                px = py = pz = std::numeric_limits<float>::quiet_NaN();
            } else {
                double g = hash_uniform(seed, pix, 0) + hash_uniform(seed, pix, 1) +
                           hash_uniform(seed, pix, 2) + hash_uniform(seed, pix, 3) - 2.0;
                g *= std::sqrt(3.0);  // Irwin-Hall(4): unit variance
                double zc = t * (1.0 + 0.0);  // depth along the optical axis (d_c.z == 1)
                double sigma = 0.0015 + 0.0019 * zc * zc;
                zc += sigma * g;
                if (!world) {
                    px = (float)(dcx * zc);
                    py = (float)(dcy * zc);
                    pz = (float)zc;
                } else {
                    V3 p = s.cam + (s.ax * dcx + s.ay * dcy + s.az) * zc;
                    px = (float)p.x;
                    py = (float)p.y;
                    pz = (float)p.z;
                }
            }
            X[pix] = px;
            Y[pix] = py;
            Z[pix] = pz;
        }
    }
}

}  // namespace

extern "C" int pitt_synth_frame(int32_t scene, uint64_t scene_seed, int32_t width, int32_t height,
                                float* x, float* y, float* z) {
    if (!x || !y || !z || width <= 0 || height <= 0) return PITT_E_INVALID;
    if (scene < 0 || scene > PITT_SCENE_TABLE_NAN) return PITT_E_INVALID;
    Scene s = make_scene(scene == PITT_SCENE_CLUTTER ? PITT_SCENE_CLUTTER : PITT_SCENE_TABLE,
                         scene_seed);
    render(s, scene_seed, width, height, false, scene == PITT_SCENE_TABLE_NAN, x, y, z);
    return PITT_OK;
}

// Fused scene (config 5): `views` cameras around one table, world frame (z up), concatenated.
extern "C" int pitt_synth_fused(uint64_t scene_seed, int32_t views, int32_t width, int32_t height,
                                float* x, float* y, float* z) {
    if (!x || !y || !z || views <= 0 || width <= 0 || height <= 0) return PITT_E_INVALID;
    Scene s = make_scene(PITT_SCENE_TABLE, scene_seed);
    Rng r{mix64(scene_seed ^ 0xF05E5EEDull)};
    const double mx = 0.5 * (s.tx0 + s.tx1), my = 0.5 * (s.ty0 + s.ty1);
    const int64_t per = (int64_t)width * height;
    for (int vw = 0; vw < views; ++vw) {
        double ang = 2.0 * M_PI * vw / views + r.range(-0.1, 0.1);
        double dist = r.range(0.75, 0.9);
        V3 cam{mx - dist * std::sin(ang), my - dist * std::cos(ang), s.table_h + r.range(0.6, 0.7)};
        double pitch = r.range(38.0, 45.0) * M_PI / 180.0;
        look_at(s, cam, ang, pitch);
        render(s, scene_seed * 31 + vw, width, height, true, false, x + vw * per, y + vw * per,
               z + vw * per);
    }
    return PITT_OK;
}
