// mpenv_core.h — the "Madrona layer" this build has to DEFINE itself.
//
// The reference (shacklettbp/madrona-mp-env) calls into the Madrona engine for
// vector/quaternion math, the counter-based RNG and three geo:: helpers
// (SURVEY.md §8a row 35).  Madrona is not vendored under /root/reference, so
// its exact arithmetic is unavailable (parity to the reference bitstream is
// unpinned).  This header is the build's single definition of
// that layer.  It is compiled unchanged by g++ (the CPU oracle) and by hipcc
// (the gfx950 kernels) with -ffp-contract=off on both sides, so that every
// float operation rounds identically on host and device:
//   * only +, -, *, /, sqrtf and explicit fmaf are used (IEEE correctly
//     rounded on x86-64 SSE and on gfx950 with HIP's default
//     correctly-rounded f32 div/sqrt);
//   * sinf/cosf/atan2f/asinf/logf are own float-only polynomial
//     implementations (cephes-style), never the platform libm / ocml;
//   * the RNG is Threefry-2x32-20 keyed like Madrona's rand::split_i.
// Call sites in the reference: utils.cpp:45-47,156-160; mesh_bvh.inl:929-930,
// 946,1120; sim.cpp:743-749; level_gen.cpp:345.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define MP_HD __host__ __device__ inline
#else
#define MP_HD inline
#endif

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace mp {

// ---------------------------------------------------------------- constants
static constexpr float kPi = 3.14159265358979323846f;
static constexpr float kFltMax = 3.40282346638528859812e+38f;

// IEEE minNum/maxNum (v_min_f32 / v_max_f32 on gfx950).  The choice between
// -0 and +0 on ties is platform-defined, so these are used only where the
// result feeds comparisons (BVH slab tests, mesh_bvh.inl:180-183).
MP_HD float fmin_(float a, float b) { return __builtin_fminf(a, b); }
MP_HD float fmax_(float a, float b) { return __builtin_fmaxf(a, b); }
// Deterministic minNum/maxNum (ties return the first operand) for results
// that flow into arithmetic or outputs.
MP_HD float fminD(float a, float b)
{
    if (a != a) return b;
    if (b != b) return a;
    return (b < a) ? b : a;
}
MP_HD float fmaxD(float a, float b)
{
    if (a != a) return b;
    if (b != b) return a;
    return (a < b) ? b : a;
}
MP_HD float fabs_(float a) { return __builtin_fabsf(a); }
MP_HD float sqrt_(float a) { return __builtin_sqrtf(a); }
MP_HD float fma_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
MP_HD float copysign_(float a, float b) { return __builtin_copysignf(a, b); }
MP_HD float clampf(float v, float lo, float hi) { return v < lo ? lo : (hi < v ? hi : v); }

MP_HD uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
MP_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }

// ---------------------------------------------------------------- Vector3
struct Vec3 {
    float x, y, z;
};

MP_HD Vec3 v3(float x, float y, float z) { Vec3 r; r.x = x; r.y = y; r.z = z; return r; }
MP_HD Vec3 operator+(Vec3 a, Vec3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
MP_HD Vec3 operator-(Vec3 a, Vec3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
MP_HD Vec3 operator-(Vec3 a) { return v3(-a.x, -a.y, -a.z); }
MP_HD Vec3 operator*(Vec3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
MP_HD Vec3 operator*(float s, Vec3 a) { return v3(s * a.x, s * a.y, s * a.z); }
MP_HD Vec3 operator/(Vec3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
MP_HD float dot(Vec3 a, Vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
MP_HD Vec3 cross(Vec3 a, Vec3 b)
{
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
MP_HD float length2(Vec3 a) { return dot(a, a); }
MP_HD float length(Vec3 a) { return sqrt_(length2(a)); }
MP_HD float distance(Vec3 a, Vec3 b) { return length(a - b); }
// Madrona Vector3::normalize(): defined here as v * (1 / |v|).
MP_HD Vec3 normalize(Vec3 a) { return a * (1.f / sqrt_(length2(a))); }
MP_HD float comp(Vec3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

static constexpr Vec3 kUp = { 0.f, 0.f, 1.f };
static constexpr Vec3 kFwd = { 0.f, 1.f, 0.f };
static constexpr Vec3 kRight = { 1.f, 0.f, 0.f };

struct AABB {
    Vec3 pMin, pMax;
};

// madrona::math::AABB::contains (inclusive bounds)
MP_HD bool aabbContains(AABB b, Vec3 p)
{
    return b.pMin.x <= p.x && b.pMin.y <= p.y && b.pMin.z <= p.z &&
           b.pMax.x >= p.x && b.pMax.y >= p.y && b.pMax.z >= p.z;
}

// ------------------------------------------------------ transcendentals
// Float-only cephes-style kernels.  Accuracy ~1-2 ulp on the ranges used by
// the sim (|x| < 1e4); identical bits on host and device.
static constexpr float kFOPI = 1.27323954473516f;
static constexpr float kDP1 = 0.78515625f;
static constexpr float kDP2 = 2.4187564849853515625e-4f;
static constexpr float kDP3 = 3.77489497744594108e-8f;

MP_HD float sinPoly_(float x, float z)
{
    return ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * x + x;
}

MP_HD float cosPoly_(float z)
{
    return ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z * z -
           0.5f * z + 1.0f;
}

MP_HD float sinf_(float xx)
{
    float x = xx;
    if (!(fabs_(x) <= 1.0e6f)) return u2f(0x7fc00000u); // NaN/inf/huge: defined as NaN
    bool neg = false;
    if (x < 0.f) { neg = true; x = -x; }
    int32_t j = (int32_t)(kFOPI * x);
    float y = (float)j;
    if (j & 1) { j += 1; y += 1.0f; }
    j &= 7;
    if (j > 3) { neg = !neg; j -= 4; }
    x = ((x - y * kDP1) - y * kDP2) - y * kDP3;
    float z = x * x;
    float r = (j == 1 || j == 2) ? cosPoly_(z) : sinPoly_(x, z);
    return neg ? -r : r;
}

MP_HD float cosf_(float xx)
{
    float x = xx < 0.f ? -xx : xx;
    if (!(x <= 1.0e6f)) return u2f(0x7fc00000u);
    int32_t j = (int32_t)(kFOPI * x);
    float y = (float)j;
    if (j & 1) { j += 1; y += 1.0f; }
    j &= 7;
    bool neg = false;
    if (j > 3) { j -= 4; neg = true; }
    if (j > 1) { neg = !neg; }
    x = ((x - y * kDP1) - y * kDP2) - y * kDP3;
    float z = x * x;
    float r = (j == 1 || j == 2) ? sinPoly_(x, z) : cosPoly_(z);
    return neg ? -r : r;
}

MP_HD float atanf_(float xx)
{
    float x = xx;
    bool neg = false;
    if (x < 0.f) { neg = true; x = -x; }
    float y;
    if (x > 2.414213562373095f) {
        y = 1.5707963267948966192f;
        x = -(1.0f / x);
    } else if (x > 0.4142135623730950f) {
        y = 0.7853981633974483096f;
        x = (x - 1.0f) / (x + 1.0f);
    } else {
        y = 0.0f;
    }
    float z = x * x;
    y += (((8.05374449538e-2f * z - 1.38776856032e-1f) * z + 1.99777106478e-1f) * z -
          3.33329491539e-1f) * z * x + x;
    return neg ? -y : y;
}

MP_HD float atan2f_(float y, float x)
{
    if (x == 0.f) {
        if (y < 0.f) return -1.5707963267948966192f;
        if (y == 0.f) return 0.f;
        return 1.5707963267948966192f;
    }
    if (y == 0.f) {
        return x < 0.f ? kPi : 0.f;
    }
    float w;
    if (x < 0.f) {
        w = y < 0.f ? -kPi : kPi;
    } else {
        w = 0.f;
    }
    return w + atanf_(y / x);
}

MP_HD float asinf_(float xx)
{
    float a = xx < 0.f ? -xx : xx;
    if (a > 1.0f) return u2f(0x7fc00000u);
    float x, z;
    bool flag = false;
    if (a < 1.0e-4f) {
        return xx;
    } else if (a > 0.5f) {
        z = 0.5f * (1.0f - a);
        x = sqrt_(z);
        flag = true;
    } else {
        x = a;
        z = x * x;
    }
    z = ((((4.2163199048e-2f * z + 2.4181311049e-2f) * z + 4.5470025998e-2f) * z +
          7.4953002686e-2f) * z + 1.6666752422e-1f) * z * x + x;
    if (flag) {
        z = z + z;
        z = 1.5707963267948966192f - z;
    }
    return xx < 0.f ? -z : z;
}

MP_HD float logf_(float xin)
{
    uint32_t u = f2u(xin);
    if (xin != xin) return xin;
    if (xin <= 0.f) {
        return xin == 0.f ? u2f(0xff800000u) : u2f(0x7fc00000u);
    }
    if (u == 0x7f800000u) return xin;
    int32_t e = 0;
    if ((u & 0x7f800000u) == 0) { // subnormal: scale up by 2^23
        xin = xin * 8388608.0f;
        u = f2u(xin);
        e = -23;
    }
    e += (int32_t)((u >> 23) & 0xff) - 126;
    float x = u2f((u & 0x007fffffu) | 0x3f000000u); // [0.5, 1)
    if (x < 0.707106781186547524f) {
        e -= 1;
        x = x + x - 1.0f;
    } else {
        x = x - 1.0f;
    }
    float z = x * x;
    float y = ((((((((7.0376836292e-2f * x - 1.1514610310e-1f) * x + 1.1676998740e-1f) * x -
                    1.2420140846e-1f) * x + 1.4249322787e-1f) * x - 1.6668057665e-1f) * x +
                 2.0000714765e-1f) * x - 2.4999993993e-1f) * x + 3.3333331174e-1f) * x * z;
    float fe = (float)e;
    if (e != 0) y += -2.12194440e-4f * fe;
    y += -0.5f * z;
    z = x + y;
    if (e != 0) z += 0.693359375f * fe;
    return z;
}

// ---------------------------------------------------------------- Quat
struct Quat {
    float w, x, y, z;
};

MP_HD Quat quat(float w, float x, float y, float z) { Quat q; q.w = w; q.x = x; q.y = y; q.z = z; return q; }

// Madrona Quat::angleAxis
MP_HD Quat angleAxis(float angle, Vec3 axis)
{
    float h = 0.5f * angle;
    float s = sinf_(h);
    return quat(cosf_(h), axis.x * s, axis.y * s, axis.z * s);
}

MP_HD Quat operator*(Quat a, Quat b)
{
    return quat(a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z,
                a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
                a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x,
                a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w);
}

MP_HD Quat qnormalize(Quat q)
{
    float inv = 1.f / sqrt_(q.w * q.w + q.x * q.x + q.y * q.y + q.z * q.z);
    return quat(q.w * inv, q.x * inv, q.y * inv, q.z * inv);
}

MP_HD Quat qinv(Quat q) { return quat(q.w, -q.x, -q.y, -q.z); }

// Madrona Quat::rotateVec: v + 2 * ((pure x v) * w + pure x (pure x v))
MP_HD Vec3 rotateVec(Quat q, Vec3 v)
{
    Vec3 pure = v3(q.x, q.y, q.z);
    Vec3 pxv = cross(pure, v);
    Vec3 pxpxv = cross(pure, pxv);
    return v + 2.f * (pxv * q.w + pxpxv);
}

// ---------------------------------------------------------------- RNG
// Threefry-2x32, 20 rounds (Salmon et al. 2011; the construction Madrona's
// rand:: API is modelled on).  RandKey = {a, b}.
struct RandKey {
    uint32_t a, b;
};

MP_HD uint32_t rotl32(uint32_t v, uint32_t r) { return (v << r) | (v >> (32u - r)); }

MP_HD RandKey threefry2x32(RandKey k, uint32_t c0, uint32_t c1)
{
    const uint32_t ks0 = k.a, ks1 = k.b, ks2 = 0x1BD11BDAu ^ k.a ^ k.b;
    uint32_t x0 = c0 + ks0, x1 = c1 + ks1;
#define MP_TF_ROUND(r) { x0 += x1; x1 = rotl32(x1, r); x1 ^= x0; }
    MP_TF_ROUND(13) MP_TF_ROUND(15) MP_TF_ROUND(26) MP_TF_ROUND(6)
    x0 += ks1; x1 += ks2 + 1u;
    MP_TF_ROUND(17) MP_TF_ROUND(29) MP_TF_ROUND(16) MP_TF_ROUND(24)
    x0 += ks2; x1 += ks0 + 2u;
    MP_TF_ROUND(13) MP_TF_ROUND(15) MP_TF_ROUND(26) MP_TF_ROUND(6)
    x0 += ks0; x1 += ks1 + 3u;
    MP_TF_ROUND(17) MP_TF_ROUND(29) MP_TF_ROUND(16) MP_TF_ROUND(24)
    x0 += ks1; x1 += ks2 + 4u;
    MP_TF_ROUND(13) MP_TF_ROUND(15) MP_TF_ROUND(26) MP_TF_ROUND(6)
    x0 += ks2; x1 += ks0 + 5u;
#undef MP_TF_ROUND
    RandKey r; r.a = x0; r.b = x1;
    return r;
}

// rand::initKey(seed, upper)
MP_HD RandKey initKey(uint32_t seed, uint32_t upper = 0) { RandKey k; k.a = seed; k.b = upper; return k; }
// rand::split_i(src, idx, idx_upper)
MP_HD RandKey splitI(RandKey src, uint32_t idx, uint32_t idx_upper = 0)
{
    return threefry2x32(src, idx, idx_upper);
}
// rand::sampleUniform(key): 24 random mantissa bits -> [0, 1)
MP_HD float keyUniform(RandKey k) { return (float)(k.a >> 8) * 5.9604644775390625e-8f; }
// rand::sampleI32(key, a, b): uniform in [a, b) by 32x32->64 multiply-high
MP_HD int32_t keyI32(RandKey k, int32_t a, int32_t b)
{
    uint32_t n = (uint32_t)(b - a);
    return a + (int32_t)(((uint64_t)k.a * (uint64_t)n) >> 32);
}

// madrona::RNG: key + draw counter; every draw consumes one split.
struct RNG {
    RandKey key;
    uint32_t ctr;
};

MP_HD RNG makeRNG(RandKey k) { RNG r; r.key = k; r.ctr = 0; return r; }
MP_HD RandKey rngAdvance(RNG &r) { RandKey k = splitI(r.key, r.ctr); r.ctr += 1; return k; }
MP_HD float rngUniform(RNG &r) { return keyUniform(rngAdvance(r)); }
MP_HD int32_t rngI32(RNG &r, int32_t a, int32_t b) { return keyI32(rngAdvance(r), a, b); }

// ----------------------------------------------------------- geo helpers
// madrona::geo::intersectRayZOriginCapsule(o, d, r, h): capsule whose axis
// runs from (0,0,0) to (0,0,h).  Defined here as: the smallest t > 0 at which
// the ray enters the capsule; 0 if the ray misses or starts inside (the
// reference relies on a ray cast from inside the caster's own capsule not
// hitting it, utils.cpp:49 / utils.cpp:218 — SURVEY.md §8c).
MP_HD float intersectRayZOriginCapsule(Vec3 o, Vec3 d, float r, float h)
{
    const float r2 = r * r;
    float zc = clampf(o.z, 0.f, h);
    float dz0 = o.z - zc;
    if (o.x * o.x + o.y * o.y + dz0 * dz0 <= r2) {
        return 0.f;
    }

    float t_best = kFltMax;

    float a = d.x * d.x + d.y * d.y;
    if (a > 0.f) {
        float b = o.x * d.x + o.y * d.y;
        float c = o.x * o.x + o.y * o.y - r2;
        float disc = b * b - a * c;
        if (disc >= 0.f) {
            float t = (-b - sqrt_(disc)) / a;
            if (t > 0.f) {
                float z = o.z + t * d.z;
                if (z >= 0.f && z <= h) {
                    t_best = t;
                }
            }
        }
    }

    float dd = dot(d, d);
    for (int cap = 0; cap < 2; cap++) {
        Vec3 m = v3(o.x, o.y, o.z - (cap == 0 ? 0.f : h));
        float b = dot(m, d);
        float c = dot(m, m) - r2;
        if (c > 0.f && b > 0.f) continue;
        float disc = b * b - dd * c;
        if (disc < 0.f) continue;
        float t = (-b - sqrt_(disc)) / dd;
        if (t > 0.f && t < t_best) t_best = t;
    }

    return t_best == kFltMax ? 0.f : t_best;
}

// madrona::geo::triangleClosestPointToOrigin(a, b, c, ab, ac)
// (Ericson, Real-Time Collision Detection 5.1.5 with p = 0)
MP_HD Vec3 triangleClosestPointToOrigin(Vec3 a, Vec3 b, Vec3 c, Vec3 ab, Vec3 ac)
{
    Vec3 ap = -a;
    float d1 = dot(ab, ap);
    float d2 = dot(ac, ap);
    if (d1 <= 0.f && d2 <= 0.f) return a;

    Vec3 bp = -b;
    float d3 = dot(ab, bp);
    float d4 = dot(ac, bp);
    if (d3 >= 0.f && d4 <= d3) return b;

    float vc = d1 * d4 - d3 * d2;
    if (vc <= 0.f && d1 >= 0.f && d3 <= 0.f) {
        float v = d1 / (d1 - d3);
        return a + v * ab;
    }

    Vec3 cp = -c;
    float d5 = dot(ab, cp);
    float d6 = dot(ac, cp);
    if (d6 >= 0.f && d5 <= d6) return c;

    float vb = d5 * d2 - d1 * d6;
    if (vb <= 0.f && d2 >= 0.f && d6 <= 0.f) {
        float w = d2 / (d2 - d6);
        return a + w * ac;
    }

    float va = d3 * d6 - d5 * d4;
    if (va <= 0.f && (d4 - d3) >= 0.f && (d5 - d6) >= 0.f) {
        float w = (d4 - d3) / ((d4 - d3) + (d5 - d6));
        return b + w * (c - b);
    }

    float denom = 1.f / (va + vb + vc);
    float v = vb * denom;
    float w = vc * denom;
    return a + ab * v + ac * w;
}

// madrona::geo::computeTriangleGeoNormal(ab, ac, bc): unnormalised normal.
MP_HD Vec3 computeTriangleGeoNormal(Vec3 ab, Vec3 ac, Vec3 /*bc*/)
{
    return cross(ab, ac);
}

// ------------------------------------------------------ synthetic inputs
// Counter-hash action tape: h(seed, step, global agent,
// field).  Shared by the benchmark, the parity tests and the CPU baseline so
// that every rank/thread sees the same actions regardless of sharding.
MP_HD uint32_t tapeHash(uint32_t seed, uint32_t step, uint32_t agent, uint32_t field)
{
    return threefry2x32(initKey(seed, 0x5eed7a9eu), step, agent * 8u + field).a;
}

MP_HD int32_t mulhi(uint32_t h, uint32_t n) { return (int32_t)(((uint64_t)h * n) >> 32); }

// out: discrete[4] = {moveAmount, moveAngle, fire, stand}; aim[2] = {yaw, pitch}
MP_HD void tapeActions(uint32_t seed, uint32_t step, uint32_t agent, int32_t *discrete, int32_t *aim)
{
    discrete[0] = mulhi(tapeHash(seed, step, agent, 0), 3);
    discrete[1] = mulhi(tapeHash(seed, step, agent, 1), 8);
    uint32_t hf = tapeHash(seed, step, agent, 2);
    discrete[2] = hf < 1932735283u ? 0 : (hf < 4080218931u ? 1 : 2);   // .45 / .50 / .05
    uint32_t hs = tapeHash(seed, step, agent, 3);
    discrete[3] = hs < 3865470566u ? 0 : (hs < 4166118277u ? 1 : 2);   // .90 / .07 / .03
    aim[0] = mulhi(tapeHash(seed, step, agent, 4), 13);
    aim[1] = mulhi(tapeHash(seed, step, agent, 5), 7);
}

// ----------------------------------------------------------- spawn helpers
// hardcodedSpawnPoint table (utils.cpp:503-541; hardcodedSpawnIdx is always
// 0, sim.cpp:795-798): index (team A ? 0 : 3) + offset.  The literals are
// doubles narrowed to float, as in the reference's brace initialisers; pitch
// is 0 for every entry.  With more than 3 agents per team the reference
// reads past the 6-entry table for the other team's offsets 3..5 (undefined
// behaviour; jax_train.py's ZoneCaptureDefend setup does this at team size
// 6): defined here as index - 3, i.e. they reuse that team's entries.
MP_HD void hardcodedSpawn(int idx, Vec3 &pos, float &yaw)
{
    if (idx >= 6) idx -= 3;
    switch (idx) {
    case 0: pos = v3((float)510.0, (float)179.1, -64.f); yaw = (float)-2.05; break;
    case 1: pos = v3((float)525.8, (float)17.1, -64.f); yaw = (float)-0.80; break;
    case 2: pos = v3((float)434.3, (float)184.7, -64.f); yaw = (float)-1.80; break;
    case 3: pos = v3((float)1037.2, (float)449.0, -56.f); yaw = (float)2.37; break;
    case 4: pos = v3((float)1094.3, (float)200.1, -56.f); yaw = (float)1.41; break;
    default: pos = v3((float)1045.8, (float)416.8, -56.f); yaw = 2.37f; break;
    }
}

// level_gen.cpp:282-326: sub-zones 0 and 1 are zones 1 and 2, the rest
// fixed boxes (sub-zone 7's x range is inverted, so it never contains a
// point).
template <typename Z>
inline void subZoneTable(const AABB *zones, const float *rots, Z *out)
{
    out[0] = { zones[1].pMin, zones[1].pMax, rots[1] };
    out[1] = { zones[2].pMin, zones[2].pMax, rots[2] };
    out[2] = { v3(-950.f, -500.f, 0.f), v3(-50.f, 500.f, 1000.f), 0.f };
    out[3] = { v3(50.f, -500.f, 0.f), v3(950.f, 500.f, 1000.f), 0.f };
    out[4] = { v3(-1000.f, -1650.f, 0.f), v3(-50.f, -600.f, 1000.f), 0.f };
    out[5] = { v3(50.f, -1650.f, 0.f), v3(1000.f, -600.f, 1000.f), 0.f };
    out[6] = { v3(-1000.f, 600.f, 0.f), v3(-50.f, 1650.f, 1000.f), 0.f };
    out[7] = { v3(1000.f, 600.f, 0.f), v3(50.f, 1650.f, 1000.f), 0.f };
}

// Navmesh::samplePoint(RandKey) (called at utils.cpp:808) lives in Madrona,
// which is not vendored: parity to the reference's bitstream is unpinned and
// the sampler is DEFINED here as area-uniform sampling over the deduplicated
// fan-triangulated navmesh (navmesh.cpp):
//   triangle = first t with u0 * cdf[T-1] < cdf[t], u0 = uniform(split_i(key, 0))
//   (cdf[t] = float running sum of triangle areas 0.5 |(b-a) x (c-a)|, in order)
//   b1, b2 = uniform(split_i(key, 1)), uniform(split_i(key, 2)); reflected
//   into the triangle when b1 + b2 > 1; point = a + (b-a) b1 + (c-a) b2.
// tris: 9 floats per triangle.
MP_HD float navTriArea(const float *t)
{
    const Vec3 a = v3(t[0], t[1], t[2]), b = v3(t[3], t[4], t[5]), c = v3(t[6], t[7], t[8]);
    return 0.5f * length(cross(b - a, c - a));
}

inline void navAreaCDF(const float *tris, int T, float *cdf)
{
    float run = 0.f;
    for (int t = 0; t < T; t++) {
        run += navTriArea(tris + 9 * t);
        cdf[t] = run;
    }
}

MP_HD Vec3 navSamplePoint(const float *tris, const float *cdf, int T, RandKey key)
{
    const float u = keyUniform(splitI(key, 0)) * cdf[T - 1];
    int lo = 0, hi = T - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (u < cdf[mid]) hi = mid;
        else lo = mid + 1;
    }
    float b1 = keyUniform(splitI(key, 1)), b2 = keyUniform(splitI(key, 2));
    if (b1 + b2 > 1.f) {
        b1 = 1.f - b1;
        b2 = 1.f - b2;
    }
    const float *t = tris + 9 * lo;
    const Vec3 a = v3(t[0], t[1], t[2]), b = v3(t[3], t[4], t[5]), c = v3(t[6], t[7], t[8]);
    return a + (b - a) * b1 + (c - a) * b2;
}

} // namespace mp
