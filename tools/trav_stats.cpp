// trav_stats — CPU analysis of BVH traversal work on a ray set (not a
// correctness tool): nodes popped, child boxes tested, triangles tested per
// ray for the reference child order and for front-to-back order.
//
//   trav_stats SCENE_DIR RAYS.f32   (RAYS: n x 6 floats, origin + direction)
//   TRAV_TREES=1 trav_stats SCENE_DIR RAYS.f32
//       k_lidar's lockstep cost on candidate trees (treesMain)
//   TRAV_HINT=PREV.f32 trav_stats SCENE_DIR RAYS.f32
//       temporal-hint model: PREV holds the same ray slots one step earlier
//       (tools/dump_lidar_rays.py at step s - 1); each ray first tests the
//       triangle its slot hit then and starts with t_max = that hit's t
#include <algorithm>
#include <array>
#include <atomic>
#include <map>
#include <thread>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mpenv.h"

struct Node {
    float minX, minY, minZ;
    int8_t expX, expY, expZ;
    uint8_t internalNodes;
    uint8_t triSize[4];
    uint8_t qMinX[4], qMinY[4], qMinZ[4], qMaxX[4], qMaxY[4], qMaxZ[4];
    int32_t children[4];
    int32_t parentID;
};

struct Stats {
    double pops = 0, boxes = 0, tris = 0, maxStack = 0;
    std::vector<std::array<int, 4>> slotTris; // per popped node: tris tested in each child slot
};

static std::vector<Node> nodes;
static std::vector<float> verts;

static bool tri(const float *v, const float *o, const float *d, float tmax, float &t)
{
    // Moller-Trumbore (analysis only)
    float e1[3], e2[3], p[3], q[3], s[3];
    for (int k = 0; k < 3; k++) { e1[k] = v[3 + k] - v[k]; e2[k] = v[6 + k] - v[k]; s[k] = o[k] - v[k]; }
    p[0] = d[1] * e2[2] - d[2] * e2[1]; p[1] = d[2] * e2[0] - d[0] * e2[2]; p[2] = d[0] * e2[1] - d[1] * e2[0];
    float det = e1[0] * p[0] + e1[1] * p[1] + e1[2] * p[2];
    if (std::fabs(det) < 1e-12f) return false;
    float inv = 1.f / det;
    float u = (s[0] * p[0] + s[1] * p[1] + s[2] * p[2]) * inv;
    if (u < 0 || u > 1) return false;
    q[0] = s[1] * e1[2] - s[2] * e1[1]; q[1] = s[2] * e1[0] - s[0] * e1[2]; q[2] = s[0] * e1[1] - s[1] * e1[0];
    float vv = (d[0] * q[0] + d[1] * q[1] + d[2] * q[2]) * inv;
    if (vv < 0 || u + vv > 1) return false;
    t = (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]) * inv;
    return t > 0 && t < tmax;
}

struct Visit {
    std::vector<int> nodes;
    std::vector<int> leaves; // first triangle ids of leaves whose box passed
};

static void traceVisits(const float *o, const float *d, Visit &v)
{
    float inv[3];
    for (int k = 0; k < 3; k++) inv[k] = d[k] == 0 ? 1e7f : 1.f / d[k];
    float tmax = 3.4e38f;
    std::vector<int> stack = { 0 };
    while (!stack.empty()) {
        int ni = stack.back();
        stack.pop_back();
        v.nodes.push_back(ni);
        const Node &n = nodes[ni];
        for (int i = 0; i < 4; i++) {
            if (n.children[i] == -1) continue;
            float sx = std::ldexp(1.f, n.expX), sy = std::ldexp(1.f, n.expY), sz = std::ldexp(1.f, n.expZ);
            float lo[3] = { n.minX + sx * n.qMinX[i], n.minY + sy * n.qMinY[i], n.minZ + sz * n.qMinZ[i] };
            float hi[3] = { n.minX + sx * n.qMaxX[i], n.minY + sy * n.qMaxY[i], n.minZ + sz * n.qMaxZ[i] };
            float tn = 0, tf = tmax;
            for (int k = 0; k < 3; k++) {
                float a = (lo[k] - o[k]) * inv[k], b = (hi[k] - o[k]) * inv[k];
                tn = std::max(tn, std::min(a, b));
                tf = std::min(tf, std::max(a, b));
            }
            if (tn > tf) continue;
            if (n.children[i] & 0x80000000) {
                int leaf = n.children[i] & 0x7fffffff;
                v.leaves.push_back(leaf * 4 + n.triSize[i]);
                for (int k = 0; k < n.triSize[i]; k++) {
                    float t;
                    if (tri(&verts[(leaf + k) * 9], o, d, tmax, t)) tmax = t;
                }
            } else {
                stack.push_back(n.children[i]);
            }
        }
    }
}

// Octant-ordered mode: per node, a static child order for each ray-direction
// octant (children sorted by their box centre projected on the octant's
// diagonal), so the nearer side is visited first without a per-ray sort.
static std::vector<std::array<std::array<int, 4>, 8>> octOrder;

static void buildOctOrder()
{
    octOrder.resize(nodes.size());
    for (size_t ni = 0; ni < nodes.size(); ni++) {
        const Node &n = nodes[ni];
        float c[4][3];
        for (int i = 0; i < 4; i++) {
            float sx = std::ldexp(1.f, n.expX), sy = std::ldexp(1.f, n.expY), sz = std::ldexp(1.f, n.expZ);
            c[i][0] = n.minX + sx * 0.5f * (n.qMinX[i] + n.qMaxX[i]);
            c[i][1] = n.minY + sy * 0.5f * (n.qMinY[i] + n.qMaxY[i]);
            c[i][2] = n.minZ + sz * 0.5f * (n.qMinZ[i] + n.qMaxZ[i]);
        }
        for (int oct = 0; oct < 8; oct++) {
            float sgn[3] = { (oct & 1) ? -1.f : 1.f, (oct & 2) ? -1.f : 1.f, (oct & 4) ? -1.f : 1.f };
            std::array<int, 4> ord = { 0, 1, 2, 3 };
            std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) {
                float ka = c[a][0] * sgn[0] + c[a][1] * sgn[1] + c[a][2] * sgn[2];
                float kb = c[b][0] * sgn[0] + c[b][1] * sgn[1] + c[b][2] * sgn[2];
                return ka < kb;
            });
            octOrder[ni][oct] = ord;
        }
    }
}

static int g_lastTri = -1; // closest-hit triangle of the last trace() (-1: none)

static void trace(const float *o, const float *d, int mode, Stats &st, float tmax0 = 3.4e38f)
{
    const bool ftb = mode == 1;
    const int oct = (d[0] < 0 ? 1 : 0) | (d[1] < 0 ? 2 : 0) | (d[2] < 0 ? 4 : 0);
    float inv[3];
    for (int k = 0; k < 3; k++) inv[k] = d[k] == 0 ? 1e7f : 1.f / d[k];
    float tmax = tmax0;
    g_lastTri = -1;
    std::vector<int> stack = { 0 };
    while (!stack.empty()) {
        st.maxStack = std::max(st.maxStack, (double)stack.size());
        int ni = stack.back();
        stack.pop_back();
        st.pops++;
        const Node &n = nodes[ni];
        std::pair<float, int> kids[4];
        int nk = 0;
        st.slotTris.push_back({ 0, 0, 0, 0 });
        for (int ii = 0; ii < 4; ii++) {
            const int i = mode == 2 ? octOrder[ni][oct][ii] : mode == 3 ? octOrder[ni][oct][3 - ii] : ii;
            if (n.children[i] == -1) continue;
            st.boxes++;
            float sx = std::ldexp(1.f, n.expX), sy = std::ldexp(1.f, n.expY), sz = std::ldexp(1.f, n.expZ);
            float lo[3] = { n.minX + sx * n.qMinX[i], n.minY + sy * n.qMinY[i], n.minZ + sz * n.qMinZ[i] };
            float hi[3] = { n.minX + sx * n.qMaxX[i], n.minY + sy * n.qMaxY[i], n.minZ + sz * n.qMaxZ[i] };
            float tn = 0, tf = tmax;
            for (int k = 0; k < 3; k++) {
                float a = (lo[k] - o[k]) * inv[k], b = (hi[k] - o[k]) * inv[k];
                tn = std::max(tn, std::min(a, b));
                tf = std::min(tf, std::max(a, b));
            }
            if (tn > tf) continue;
            if (n.children[i] & 0x80000000) {
                int leaf = n.children[i] & 0x7fffffff;
                for (int k = 0; k < n.triSize[i]; k++) {
                    st.tris++;
                    st.slotTris.back()[i]++;
                    float t;
                    if (tri(&verts[(leaf + k) * 9], o, d, tmax, t)) {
                        tmax = t;
                        g_lastTri = leaf + k;
                    }
                }
            } else {
                kids[nk++] = { tn, n.children[i] };
            }
        }
        if (ftb) std::sort(kids, kids + nk, [](auto a, auto b) { return a.first > b.first; });
        if (mode == 2) std::reverse(kids, kids + nk); // nearest (first in order) popped first
        for (int k = 0; k < nk; k++) stack.push_back(kids[k].second);
    }
}

// While-while traversal with postponed triangles (Aila & Laine 2009), one
// wave of up to 64 lanes in lockstep.  Each lane keeps its octant-order
// stack and a FIFO of discovered-but-untested triangles.  Node phase: every
// lane with stack entries and fewer than `cap` pending triangles pops one
// node per lockstep iteration (boxes tested with its current t_max; leaf
// children's triangles queued in slot order); the phase ends when fewer
// than `need` lanes still pop.  Triangle phase: every lane tests its queued
// triangles, one per lockstep iteration (t_max updated).  Closest-hit
// results are order-independent under the min-over-candidates definition,
// so only the work differs.  Returns lockstep (node iterations, triangle
// iterations, phases) summed over the wave, and the per-lane totals.
struct WW {
    double nodeIters = 0, triIters = 0, phases = 0, pops = 0, tris = 0;
};

static void traceWaveWW(const float *rays, size_t r0, size_t n, int cap, int need, WW &out)
{
    struct Lane {
        std::vector<int> stack;
        std::vector<int> pending;
        float o[3], d[3], inv[3], tmax;
        int oct;
    };
    std::vector<Lane> L(n);
    for (size_t k = 0; k < n; k++) {
        Lane &l = L[k];
        for (int j = 0; j < 3; j++) {
            l.o[j] = rays[6 * (r0 + k) + j];
            l.d[j] = rays[6 * (r0 + k) + 3 + j];
            l.inv[j] = l.d[j] == 0 ? 1e7f : 1.f / l.d[j];
        }
        l.tmax = 3.4e38f;
        l.oct = (l.d[0] < 0 ? 1 : 0) | (l.d[1] < 0 ? 2 : 0) | (l.d[2] < 0 ? 4 : 0);
        l.stack = { 0 };
    }
    auto popNode = [&](Lane &l) {
        int ni = l.stack.back();
        l.stack.pop_back();
        out.pops++;
        const Node &nd = nodes[ni];
        int kids[4], nk = 0;
        for (int ii = 0; ii < 4; ii++) {
            const int i = octOrder[ni][l.oct][ii];
            if (nd.children[i] == -1) continue;
            float sx = std::ldexp(1.f, nd.expX), sy = std::ldexp(1.f, nd.expY), sz = std::ldexp(1.f, nd.expZ);
            float lo[3] = { nd.minX + sx * nd.qMinX[i], nd.minY + sy * nd.qMinY[i], nd.minZ + sz * nd.qMinZ[i] };
            float hi[3] = { nd.minX + sx * nd.qMaxX[i], nd.minY + sy * nd.qMaxY[i], nd.minZ + sz * nd.qMaxZ[i] };
            float tn = 0, tf = l.tmax;
            for (int k = 0; k < 3; k++) {
                float a = (lo[k] - l.o[k]) * l.inv[k], b = (hi[k] - l.o[k]) * l.inv[k];
                tn = std::max(tn, std::min(a, b));
                tf = std::min(tf, std::max(a, b));
            }
            if (tn > tf) continue;
            if (nd.children[i] & 0x80000000) {
                int leaf = nd.children[i] & 0x7fffffff;
                for (int k = 0; k < nd.triSize[i]; k++) l.pending.push_back(leaf + k);
            } else {
                kids[nk++] = nd.children[i];
            }
        }
        for (int k = nk - 1; k >= 0; k--) l.stack.push_back(kids[k]);
    };
    for (;;) {
        bool any = false;
        for (auto &l : L) any = any || !l.stack.empty() || !l.pending.empty();
        if (!any) break;
        out.phases++;
        for (;;) {
            int popping = 0;
            for (auto &l : L)
                if (!l.stack.empty() && (int)l.pending.size() < cap) popping++;
            if (popping == 0) break;
            out.nodeIters++;
            for (auto &l : L)
                if (!l.stack.empty() && (int)l.pending.size() < cap) popNode(l);
            if (popping < need) break;
        }
        size_t mx = 0;
        for (auto &l : L) mx = std::max(mx, l.pending.size());
        out.triIters += mx;
        for (auto &l : L) {
            for (int t : l.pending) {
                out.tris++;
                float th;
                if (tri(&verts[t * 9], l.o, l.d, l.tmax, th)) l.tmax = th;
            }
            l.pending.clear();
        }
    }
}

// Packet traversal: one wave-uniform stack per wave of up to 64 rays.  A
// popped node is box-tested by every lane against its own t_max; a child is
// pushed if any lane enters it, a leaf's triangles are tested (lockstep:
// the leaf's triSize iterations) by the lanes that entered it.  Child order
// from the octant of lane `ref`'s direction (mode 0) or of the wave's mean
// direction (mode 1).  Returns lockstep node iterations and triangle
// iterations summed over the wave, and the per-lane box / triangle tests.
struct PK {
    double nodeIters = 0, triIters = 0, laneBoxes = 0, laneTris = 0;
};

static void traceWavePacket(const float *rays, size_t r0, size_t n, int mode, PK &out)
{
    std::vector<float> tmax(n, 3.4e38f), inv(3 * n);
    for (size_t k = 0; k < n; k++)
        for (int j = 0; j < 3; j++) {
            const float d = rays[6 * (r0 + k) + 3 + j];
            inv[3 * k + j] = d == 0 ? 1e7f : 1.f / d;
        }
    float md[3] = { 0, 0, 0 };
    for (size_t k = 0; k < n; k++)
        for (int j = 0; j < 3; j++) md[j] += rays[6 * (r0 + k) + 3 + j];
    const float *rd = mode == 0 ? &rays[6 * r0 + 3] : md;
    const int oct = (rd[0] < 0 ? 1 : 0) | (rd[1] < 0 ? 2 : 0) | (rd[2] < 0 ? 4 : 0);
    std::vector<int> stack = { 0 };
    while (!stack.empty()) {
        const int ni = stack.back();
        stack.pop_back();
        out.nodeIters++;
        const Node &nd = nodes[ni];
        int kids[4], nk = 0;
        for (int ii = 0; ii < 4; ii++) {
            const int i = octOrder[ni][oct][ii];
            if (nd.children[i] == -1) continue;
            float sx = std::ldexp(1.f, nd.expX), sy = std::ldexp(1.f, nd.expY), sz = std::ldexp(1.f, nd.expZ);
            float lo[3] = { nd.minX + sx * nd.qMinX[i], nd.minY + sy * nd.qMinY[i], nd.minZ + sz * nd.qMinZ[i] };
            float hi[3] = { nd.minX + sx * nd.qMaxX[i], nd.minY + sy * nd.qMaxY[i], nd.minZ + sz * nd.qMaxZ[i] };
            std::vector<int> in;
            for (size_t k = 0; k < n; k++) {
                out.laneBoxes++;
                const float *o = &rays[6 * (r0 + k)];
                float tn = 0, tf = tmax[k];
                for (int j = 0; j < 3; j++) {
                    float a = (lo[j] - o[j]) * inv[3 * k + j], b = (hi[j] - o[j]) * inv[3 * k + j];
                    tn = std::max(tn, std::min(a, b));
                    tf = std::min(tf, std::max(a, b));
                }
                if (tn <= tf) in.push_back((int)k);
            }
            if (in.empty()) continue;
            if (nd.children[i] & 0x80000000) {
                const int leaf = nd.children[i] & 0x7fffffff;
                out.triIters += nd.triSize[i];
                for (int k : in)
                    for (int q = 0; q < nd.triSize[i]; q++) {
                        out.laneTris++;
                        float th;
                        if (tri(&verts[(leaf + q) * 9], &rays[6 * (r0 + k)], &rays[6 * (r0 + k) + 3], tmax[k], th))
                            tmax[k] = th;
                    }
            } else {
                kids[nk++] = nd.children[i];
            }
        }
        for (int k = nk - 1; k >= 0; k--) stack.push_back(kids[k]);
    }
}

// Per-fan candidate lists (forward waves only: one agent's 64 rays, two
// sheets of 32 rays from one xy origin at two heights, each sheet in the
// plane spanned by the aim frame's right and forward axes).  Cull per
// (triangle, sheet): back faces (the sheet origin behind the triangle's
// plane: rayTri accepts one winding only), triangles with no point within
// `eps` of the sheet plane, then the angular span (seen from the sheet
// origin) of the triangle's band |s| <= eps gives the candidate rays (plus
// `delta` rad each side); the exact distance from the origin to the
// triangle bounds any hit's t from below.  Entries (triangle, sheet, 32-ray
// mask, bound) are walked in lockstep in one of three orders -- sorted by
// bound, bucketed by bound (counting sort on log2 buckets), or unsorted --
// an entry costs a full triangle test when some ray of its mask still has
// t > bound (order-independent closest hit: the minimum of (t, triangle)),
// else a skip.  Compared with brute force over every triangle.
struct FanStats {
    double waves = 0, entries = 0, walked = 0, full = 0, laneTests = 0;
    double wrong = 0, bigLists = 0;
    double planeTests = 0, straddle = 0; // per (triangle, sheet): after the back-face cull, after the band test
};
static int g_frontSign = 0; // +1 / -1: the origin side rayTri accepts; 0: no back-face cull

static double closestDist(const double *a, const double *b, const double *c) // RTCD 5.1.5, p = origin
{
    auto dot = [](const double *x, const double *y) { return x[0] * y[0] + x[1] * y[1] + x[2] * y[2]; };
    double ab[3], ac[3], ap[3], bp[3], cp[3], r[3];
    for (int k = 0; k < 3; k++) { ab[k] = b[k] - a[k]; ac[k] = c[k] - a[k]; ap[k] = -a[k]; bp[k] = -b[k]; cp[k] = -c[k]; }
    auto len = [&](const double *x) { return std::sqrt(dot(x, x)); };
    double d1 = dot(ab, ap), d2 = dot(ac, ap);
    if (d1 <= 0 && d2 <= 0) return len(a);
    double d3 = dot(ab, bp), d4 = dot(ac, bp);
    if (d3 >= 0 && d4 <= d3) return len(b);
    double vc = d1 * d4 - d3 * d2;
    if (vc <= 0 && d1 >= 0 && d3 <= 0) { double v = d1 / (d1 - d3); for (int k = 0; k < 3; k++) r[k] = a[k] + v * ab[k]; return len(r); }
    double d5 = dot(ab, cp), d6 = dot(ac, cp);
    if (d6 >= 0 && d5 <= d6) return len(c);
    double vb = d5 * d2 - d1 * d6;
    if (vb <= 0 && d2 >= 0 && d6 <= 0) { double w = d2 / (d2 - d6); for (int k = 0; k < 3; k++) r[k] = a[k] + w * ac[k]; return len(r); }
    double va = d3 * d6 - d5 * d4;
    if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) {
        double w = (d4 - d3) / ((d4 - d3) + (d5 - d6));
        for (int k = 0; k < 3; k++) r[k] = b[k] + w * (c[k] - b[k]);
        return len(r);
    }
    double den = 1.0 / (va + vb + vc), v = vb * den, w = vc * den;
    for (int k = 0; k < 3; k++) r[k] = a[k] + ab[k] * v + ac[k] * w;
    return len(r);
}

static void fanWave(const float *rays, size_t r0, int order, FanStats &fs)
{
    const double kPi = 3.14159265358979323846;
    const double eps = 0.05, delta = 1e-3;
    double R[3], F[3], N[3], O[2][3];
    {
        const float *d0 = &rays[6 * r0 + 3], *d31 = &rays[6 * (r0 + 31) + 3];
        for (int k = 0; k < 3; k++) {
            F[k] = (d0[k] + d31[k]) / (2.0 * std::sin(kPi / 8));
            R[k] = (d31[k] - d0[k]) / (2.0 * std::cos(kPi / 8));
        }
        N[0] = R[1] * F[2] - R[2] * F[1]; N[1] = R[2] * F[0] - R[0] * F[2]; N[2] = R[0] * F[1] - R[1] * F[0];
        for (int h = 0; h < 2; h++)
            for (int k = 0; k < 3; k++) O[h][k] = rays[6 * (r0 + 32 * h) + k];
    }
    struct Ent { int tri, sheet; uint32_t mask; double nearB; };
    std::vector<Ent> ents;
    const int ntri = (int)(verts.size() / 9);
    const double step = 0.75 * kPi / 31, off = 0.125 * kPi;
    for (int t = 0; t < ntri; t++) {
        const float *tv = &verts[t * 9];
        double e1[3], e2[3], tn[3];
        for (int k = 0; k < 3; k++) { e1[k] = tv[3 + k] - tv[k]; e2[k] = tv[6 + k] - tv[k]; }
        tn[0] = e1[1] * e2[2] - e1[2] * e2[1]; tn[1] = e1[2] * e2[0] - e1[0] * e2[2]; tn[2] = e1[0] * e2[1] - e1[1] * e2[0];
        const double tnl = std::sqrt(tn[0] * tn[0] + tn[1] * tn[1] + tn[2] * tn[2]);
        for (int h = 0; h < 2; h++) {
            double v[3][3], s[3];
            for (int i = 0; i < 3; i++) {
                for (int k = 0; k < 3; k++) v[i][k] = tv[3 * i + k] - O[h][k];
                s[i] = v[i][0] * N[0] + v[i][1] * N[1] + v[i][2] * N[2];
            }
            if (g_frontSign != 0) {
                const double so = -(tn[0] * v[0][0] + tn[1] * v[0][1] + tn[2] * v[0][2]);
                if (so * g_frontSign < -1e-3 * tnl) continue;
            }
            fs.planeTests++;
            if ((s[0] > eps && s[1] > eps && s[2] > eps) || (s[0] < -eps && s[1] < -eps && s[2] < -eps)) continue;
            fs.straddle++;
            // the band |s| <= eps: vertices inside it, edge crossings of s = +-eps
            double pts[9][2];
            int np = 0;
            auto addP = [&](const double *p) {
                pts[np][0] = p[0] * R[0] + p[1] * R[1] + p[2] * R[2];
                pts[np][1] = p[0] * F[0] + p[1] * F[1] + p[2] * F[2];
                np++;
            };
            // TRAV_FAN_TRI: the angular span of the whole projected triangle
            // (3 vertices) instead of its band strip
            static const bool triSpan = getenv("TRAV_FAN_TRI") != nullptr;
            if (triSpan)
                for (int i = 0; i < 3; i++) addP(v[i]);
            for (int i = 0; i < 3 && !triSpan; i++) {
                if (std::fabs(s[i]) <= eps) addP(v[i]);
                const int j = (i + 1) % 3;
                for (double bnd : { eps, -eps }) {
                    if ((s[i] - bnd) * (s[j] - bnd) < 0) {
                        const double a = (s[i] - bnd) / (s[i] - s[j]);
                        double p[3];
                        for (int k = 0; k < 3; k++) p[k] = v[i][k] + (v[j][k] - v[i][k]) * a;
                        addP(p);
                    }
                }
            }
            if (np == 0) continue;
            double lo = 0, hi = 0;
            bool full = false;
            // TRAV_FAN_MID: the cut segment of the sheet's own plane (s = 0),
            // widened by the band's reach along the triangle, eps / sin of
            // the angle between the planes (+0.5), seen from its distance;
            // a triangle in the band that does not cross the plane, or a
            // near-parallel one (sin < 0.1), takes every ray
            static const bool midSeg = getenv("TRAV_FAN_MID") != nullptr;
            double widen = 0;
            if (midSeg) {
                const double cosT = std::fabs(tn[0] * N[0] + tn[1] * N[1] + tn[2] * N[2]) / tnl;
                const double sinT = std::sqrt(std::max(0.0, 1 - cosT * cosT));
                np = 0;
                for (int i = 0; i < 3; i++) {
                    const int j = (i + 1) % 3;
                    if (s[i] == 0) addP(v[i]);
                    if ((s[i] < 0 && s[j] > 0) || (s[i] > 0 && s[j] < 0)) {
                        const double a = s[i] / (s[i] - s[j]);
                        double p[3];
                        for (int k = 0; k < 3; k++) p[k] = v[i][k] + (v[j][k] - v[i][k]) * a;
                        addP(p);
                    }
                }
                if (np < 2 || sinT < 0.1) {
                    full = true;
                    np = np ? np : 1;
                    if (!np) pts[0][0] = pts[0][1] = 1;
                } else {
                    const double e = eps / sinT + 0.5;
                    const double ex = pts[1][0] - pts[0][0], ey = pts[1][1] - pts[0][1], L = ex * ex + ey * ey;
                    double tt = L > 0 ? -(pts[0][0] * ex + pts[0][1] * ey) / L : 0;
                    tt = std::min(1.0, std::max(0.0, tt));
                    const double cx = pts[0][0] + tt * ex, cy = pts[0][1] + tt * ey, dseg = std::sqrt(cx * cx + cy * cy);
                    if (dseg < e + 16) full = true;
                    else widen = std::asin(e / dseg);
                }
            }
            const double a0 = std::atan2(pts[0][1], -pts[0][0]);
            for (int p = 0; p < np; p++) {
                if (pts[p][0] * pts[p][0] + pts[p][1] * pts[p][1] < 1.0) full = true;
                double d = std::atan2(pts[p][1], -pts[p][0]) - a0;
                while (d > kPi) d -= 2 * kPi;
                while (d <= -kPi) d += 2 * kPi;
                lo = std::min(lo, d);
                hi = std::max(hi, d);
            }
            if (hi - lo >= kPi - 1e-3) full = true;
            uint32_t m = 0;
            for (int x = 0; x < 32; x++) {
                const double th = off + step * x;
                for (double wrap : { -2 * kPi, 0.0, 2 * kPi })
                    if (full || (th + wrap >= a0 + lo - delta - widen && th + wrap <= a0 + hi + delta + widen)) m |= 1u << x;
            }
            if (!m) continue;
            double nb = closestDist(v[0], v[1], v[2]);
            if (getenv("TRAV_FAN_CHEAPNB")) {
                // max(distance to the triangle's plane, distance to its bounding sphere)
                double c[3], r2 = 0;
                for (int k = 0; k < 3; k++) c[k] = (v[0][k] + v[1][k] + v[2][k]) / 3;
                for (int i = 0; i < 3; i++) {
                    double d2 = 0;
                    for (int k = 0; k < 3; k++) d2 += (v[i][k] - c[k]) * (v[i][k] - c[k]);
                    r2 = std::max(r2, d2);
                }
                const double pd = std::fabs(tn[0] * v[0][0] + tn[1] * v[0][1] + tn[2] * v[0][2]) / tnl;
                const double cd = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]) - std::sqrt(r2);
                nb = std::max(pd, cd);
            }
            ents.push_back({ t, h, m, std::max(0.0, nb * (1 - 1e-5) - 0.01) });
        }
    }
    fs.waves++;
    float tl[64];
    int il[64];
    for (int l = 0; l < 64; l++) { tl[l] = 3.4e38f; il[l] = -1; }
    if (order >= 3) {
        // one entry per triangle: both sheets' masks (64 lanes) and bounds;
        // 3: 8 log2 buckets of the smaller bound, 4: sorted by it.  Every
        // entry is walked (no termination test); an entry with no lane
        // still above its bound is a skip.
        struct M { int tri; uint64_t mask; double nb[2]; double key; };
        std::vector<M> ms;
        for (const Ent &e : ents) {
            if (ms.empty() || ms.back().tri != e.tri) ms.push_back({ e.tri, 0ull, { 1e30, 1e30 }, 1e30 });
            ms.back().mask |= (uint64_t)e.mask << (32 * e.sheet);
            ms.back().nb[e.sheet] = e.nearB;
            ms.back().key = std::min(ms.back().key, e.nearB);
        }
        auto bk = [](double nb) { return nb < 32 ? 0 : std::min(7, 1 + (int)std::floor(std::log2(nb / 32))); };
        if (order == 3)
            std::stable_sort(ms.begin(), ms.end(), [&](const M &a, const M &b) { return bk(a.key) < bk(b.key); });
        else
            std::stable_sort(ms.begin(), ms.end(), [](const M &a, const M &b) { return a.key < b.key; });
        fs.entries += ms.size();
        if (ms.size() > 64) fs.bigLists++;
        for (const M &c : ms) {
            fs.walked++;
            bool act = false;
            for (int l = 0; l < 64; l++) {
                if (!((c.mask >> l) & 1) || !(c.nb[l >> 5] < tl[l])) continue;
                act = true;
                fs.laneTests++;
                float th;
                if (tri(&verts[c.tri * 9], &rays[6 * (r0 + l)], &rays[6 * (r0 + l) + 3], 3.4e38f, th) &&
                    (th < tl[l] || (th == tl[l] && c.tri < il[l]))) { tl[l] = th; il[l] = c.tri; }
            }
            if (act) fs.full++;
        }
    } else {
    if (order == 0) {
        std::stable_sort(ents.begin(), ents.end(), [](const Ent &a, const Ent &b) { return a.nearB < b.nearB; });
    } else if (order == 1) {
        // counting sort on 16 buckets: log2 of the bound (bucket 0: < 64 units)
        auto bk = [](double nb) { return nb < 64 ? 0 : std::min(15, 1 + (int)std::floor(std::log2(nb / 64) * 2)); };
        std::stable_sort(ents.begin(), ents.end(), [&](const Ent &a, const Ent &b) { return bk(a.nearB) < bk(b.nearB); });
    }
    fs.entries += ents.size();
    if (ents.size() > 64) fs.bigLists++;
    for (size_t ci = 0; ci < ents.size(); ci++) {
        bool anyLater = false;
        for (size_t cj = ci; cj < ents.size() && !anyLater; cj++)
            for (int x = 0; x < 32; x++)
                if (((ents[cj].mask >> x) & 1) && ents[cj].nearB < tl[32 * ents[cj].sheet + x]) { anyLater = true; break; }
        if (!anyLater) break;
        fs.walked++;
        const Ent &c = ents[ci];
        bool act = false;
        for (int x = 0; x < 32; x++) {
            const int l = 32 * c.sheet + x;
            if (!((c.mask >> x) & 1) || !(c.nearB < tl[l])) continue;
            act = true;
            fs.laneTests++;
            float th;
            if (tri(&verts[c.tri * 9], &rays[6 * (r0 + l)], &rays[6 * (r0 + l) + 3], 3.4e38f, th) &&
                (th < tl[l] || (th == tl[l] && c.tri < il[l]))) { tl[l] = th; il[l] = c.tri; }
        }
        if (act) fs.full++;
    }
    }
    // brute force: min (t, triangle) over every triangle
    for (int l = 0; l < 64; l++) {
        float tb = 3.4e38f;
        int ib = -1;
        for (int t = 0; t < ntri; t++) {
            float th;
            if (tri(&verts[t * 9], &rays[6 * (r0 + l)], &rays[6 * (r0 + l) + 3], 3.4e38f, th) && (th < tb || (th == tb && t < ib))) { tb = th; ib = t; }
        }
        if (tb != tl[l] || ib != il[l]) fs.wrong++;
    }
}

// Ray-pair traversal (TRAV_PAIR): one lane walks the two sheet rays of one
// fan angle -- same direction, origins differing only in z -- through one
// union traversal in the shared octant order: a node carries a 2-bit mask of
// the rays that entered it, each child box is tested per ray against that
// ray's own t_max, a leaf's triangles are tested for each ray that entered
// it (A's, then B's), an internal child is pushed with the mask of the rays
// that entered it.  Each ray sees exactly the node sequence and t_max of its
// solo traversal, so the closest hits are the same; what changes is the
// lockstep work.  Per node iteration: slotTris[it][i] = A's tests in slot i,
// slotTrisB = B's.
struct PairStats {
    int pops = 0, boxesA = 0, boxesB = 0, trisA = 0, trisB = 0, solo = 0;
    std::vector<std::array<int, 4>> slotA, slotB;
};

static void tracePair(const float *oA, const float *oB, const float *d, PairStats &st)
{
    const int oct = (d[0] < 0 ? 1 : 0) | (d[1] < 0 ? 2 : 0) | (d[2] < 0 ? 4 : 0);
    float inv[3];
    for (int k = 0; k < 3; k++) inv[k] = d[k] == 0 ? 1e7f : 1.f / d[k];
    float tmax[2] = { 3.4e38f, 3.4e38f };
    const float *o[2] = { oA, oB };
    std::vector<std::pair<int, int>> stack = { { 0, 3 } };
    while (!stack.empty()) {
        auto [ni, mask] = stack.back();
        stack.pop_back();
        st.pops++;
        if (mask != 3) st.solo++;
        const Node &n = nodes[ni];
        std::pair<int, int> kids[4];
        int nk = 0;
        st.slotA.push_back({ 0, 0, 0, 0 });
        st.slotB.push_back({ 0, 0, 0, 0 });
        for (int ii = 0; ii < 4; ii++) {
            const int i = octOrder[ni][oct][ii];
            if (n.children[i] == -1) continue;
            float sx = std::ldexp(1.f, n.expX), sy = std::ldexp(1.f, n.expY), sz = std::ldexp(1.f, n.expZ);
            float lo[3] = { n.minX + sx * n.qMinX[i], n.minY + sy * n.qMinY[i], n.minZ + sz * n.qMinZ[i] };
            float hi[3] = { n.minX + sx * n.qMaxX[i], n.minY + sy * n.qMaxY[i], n.minZ + sz * n.qMaxZ[i] };
            int enter = 0;
            for (int r = 0; r < 2; r++) {
                if (!((mask >> r) & 1)) continue;
                (r ? st.boxesB : st.boxesA)++;
                float tn = 0, tf = tmax[r];
                for (int k = 0; k < 3; k++) {
                    float a = (lo[k] - o[r][k]) * inv[k], b = (hi[k] - o[r][k]) * inv[k];
                    tn = std::max(tn, std::min(a, b));
                    tf = std::min(tf, std::max(a, b));
                }
                if (tn <= tf) enter |= 1 << r;
            }
            if (!enter) continue;
            if (n.children[i] & 0x80000000) {
                int leaf = n.children[i] & 0x7fffffff;
                for (int r = 0; r < 2; r++) {
                    if (!((enter >> r) & 1)) continue;
                    for (int k = 0; k < n.triSize[i]; k++) {
                        (r ? st.trisB : st.trisA)++;
                        (r ? st.slotB : st.slotA).back()[i]++;
                        float t;
                        if (tri(&verts[(leaf + k) * 9], o[r], d, tmax[r], t)) tmax[r] = t;
                    }
                }
            } else {
                kids[nk++] = { n.children[i], enter };
            }
        }
        std::reverse(kids, kids + nk); // nearest (first in order) popped first
        for (int k = 0; k < nk; k++) stack.push_back(kids[k]);
    }
}

// Lockstep cost of one wave of lanes: node iterations (max pops) and
// triangle-test iterations (per iteration and slot, the max over lanes).
struct Lockstep {
    double nodeIters = 0, triIters = 0;
};

static void lockSolo(const std::vector<Stats> &lanes, Lockstep &ls)
{
    double mp = 0;
    for (auto &L : lanes) mp = std::max(mp, L.pops);
    ls.nodeIters += mp;
    for (int it = 0; it < (int)mp; it++)
        for (int i = 0; i < 4; i++) {
            int m = 0;
            for (auto &L : lanes)
                if (it < (int)L.slotTris.size()) m = std::max(m, L.slotTris[it][i]);
            ls.triIters += m;
        }
}

static void lockPair(const std::vector<PairStats> &lanes, Lockstep &ls)
{
    int mp = 0;
    for (auto &L : lanes) mp = std::max(mp, L.pops);
    ls.nodeIters += mp;
    for (int it = 0; it < mp; it++)
        for (int i = 0; i < 4; i++) {
            int ma = 0, mb = 0;
            for (auto &L : lanes)
                if (it < (int)L.slotA.size()) {
                    ma = std::max(ma, L.slotA[it][i]);
                    mb = std::max(mb, L.slotB[it][i]);
                }
            ls.triIters += ma + mb;
        }
}

static int pairMain(const std::vector<float> &rays)
{
    // dump_lidar_rays order: per 4-agent unit, each agent's 64 forward rays
    // (k = h * 32 + x), then the 4 agents' 16 rear rays (k = h * 8 + x)
    const size_t n = rays.size() / 6, units = n / 320;
    auto R = [&](size_t r) { return &rays[6 * r]; };
    Lockstep soloF, soloR, pairF, pairR;
    double soloFw = 0, soloRw = 0, pairFw = 0, pairRw = 0, dirMismatch = 0, pops = 0, solo = 0, lanesP = 0;
    double trisSolo = 0, trisPair = 0;
    std::vector<PairStats> rearLanes;
    for (size_t u = 0; u < units; u++) {
        const size_t base = u * 320;
        // solo: 4 forward waves (one agent each) + 1 rear wave (4 x 16)
        for (int a = 0; a < 4; a++) {
            std::vector<Stats> lanes(64);
            for (int k = 0; k < 64; k++) trace(R(base + a * 64 + k), R(base + a * 64 + k) + 3, 2, lanes[k]);
            for (auto &L : lanes) trisSolo += L.tris;
            lockSolo(lanes, soloF);
            soloFw++;
        }
        {
            std::vector<Stats> lanes(64);
            for (int k = 0; k < 64; k++) trace(R(base + 256 + k), R(base + 256 + k) + 3, 2, lanes[k]);
            for (auto &L : lanes) trisSolo += L.tris;
            lockSolo(lanes, soloR);
            soloRw++;
        }
        // pairs: forward waves of 2 agents x 32 angles
        for (int a0 = 0; a0 < 4; a0 += 2) {
            std::vector<PairStats> lanes(64);
            for (int l = 0; l < 64; l++) {
                const int a = a0 + l / 32, x = l % 32;
                const float *ra = R(base + a * 64 + x), *rb = R(base + a * 64 + 32 + x);
                for (int k = 0; k < 3; k++) dirMismatch += ra[3 + k] != rb[3 + k];
                tracePair(ra, rb, ra + 3, lanes[l]);
                pops += lanes[l].pops; solo += lanes[l].solo; lanesP++;
                trisPair += lanes[l].trisA + lanes[l].trisB;
            }
            lockPair(lanes, pairF);
            pairFw++;
        }
        // rear pairs: 4 agents x 8 angles per unit; a wave takes two units
        for (int l = 0; l < 32; l++) {
            const int a = l / 8, x = l % 8;
            const float *ra = R(base + 256 + a * 16 + x), *rb = R(base + 256 + a * 16 + 8 + x);
            rearLanes.emplace_back();
            tracePair(ra, rb, ra + 3, rearLanes.back());
            trisPair += rearLanes.back().trisA + rearLanes.back().trisB;
        }
        if (rearLanes.size() == 64) {
            lockPair(rearLanes, pairR);
            pairRw++;
            rearLanes.clear();
        }
    }
    printf("rays %zu (%zu units), direction mismatches within pairs %.0f\n", n, units, dirMismatch);
    printf("solo  forward: %.0f waves, lockstep node iters/wave %.2f tri iters/wave %.2f | rear: %.0f waves, %.2f / %.2f\n",
           soloFw, soloF.nodeIters / soloFw, soloF.triIters / soloFw, soloRw, soloR.nodeIters / soloRw, soloR.triIters / soloRw);
    printf("pairs forward: %.0f waves, lockstep node iters/wave %.2f tri iters/wave %.2f | rear: %.0f waves, %.2f / %.2f\n",
           pairFw, pairF.nodeIters / pairFw, pairF.triIters / pairFw, pairRw, pairR.nodeIters / std::max(pairRw, 1.0),
           pairR.triIters / std::max(pairRw, 1.0));
    printf("pair lanes: union pops/lane %.2f (single-ray nodes %.1f%%); lane tri tests solo %.0f pair %.0f\n",
           pops / lanesP, 100.0 * solo / pops, trisSolo, trisPair);
    // instruction model: per node iteration ~110 VALU solo, ~150 paired
    // (shared decode and x/y slabs, two z slabs / t_near / t_far), ~45 per
    // triangle test
    const double cs = soloF.nodeIters * 110 + soloF.triIters * 45 + soloR.nodeIters * 110 + soloR.triIters * 45;
    const double cp = pairF.nodeIters * 150 + pairF.triIters * 45 + (pairR.nodeIters * 150 + pairR.triIters * 45);
    printf("model VALU per unit: solo %.0f, pairs %.0f (%.2fx)\n", cs / units, cp / units, cp / cs);
    return 0;
}

// ---- TRAV_TREES: k_lidar's traversal, modelled exactly, over candidate
// trees (mpenv_scene_bvh_variant).  Per node and ray octant the slot order
// of scene.h octantNodeImages (leaves by ascending key, then internal
// children by descending key -- the nearest popped first -- then empty
// slots); a popped node tests its slots in that order against the lane's
// t_max, a passing leaf runs its triangle tests (slot k's unrolled pair), a
// passing internal child is pushed.  Lockstep per 64-lane wave (k_lidar's
// waves: one agent's 64 forward rays, or 4 agents' 16 rear rays): node
// iterations = the longest lane's pops; triangle iterations = per iteration
// and slot, the most tests any lane runs there.  Weighted cost = 110 VALU
// per node iteration + 45 per triangle iteration (DESIGN.md §4 model).
struct KM {
    double waves = 0, nodeIters = 0, triIters = 0, pops = 0, tris = 0, wrong = 0;
    double triItersMerged = 0; // per iteration: the most triangle tests any lane runs over all its slots
};

static bool g_deferTris = false; // TRAV_DEFER: every slot's box test at the node's entry t_max, then the triangles

static void kernelModel(const std::vector<Node> &nd, const std::vector<float> &vt, const std::vector<float> &rays,
                        bool fwd_waves, KM &km, const std::vector<float> *ref_t = nullptr, std::vector<float> *out_t = nullptr)
{
    const size_t n = rays.size() / 6;
    // octant slot orders
    std::vector<std::array<std::array<int, 4>, 8>> ord(nd.size());
    for (size_t ni = 0; ni < nd.size(); ni++) {
        const Node &x = nd[ni];
        for (int oct = 0; oct < 8; oct++) {
            const double sgn[3] = { (oct & 1) ? -1.0 : 1.0, (oct & 2) ? -1.0 : 1.0, (oct & 4) ? -1.0 : 1.0 };
            double key[4];
            const int8_t ex[3] = { x.expX, x.expY, x.expZ };
            const float mn[3] = { x.minX, x.minY, x.minZ };
            const uint8_t *qlo[3] = { x.qMinX, x.qMinY, x.qMinZ }, *qhi[3] = { x.qMaxX, x.qMaxY, x.qMaxZ };
            for (int i = 0; i < 4; i++) {
                key[i] = 0;
                for (int a = 0; a < 3; a++)
                    key[i] += sgn[a] * ((double)mn[a] + std::ldexp(0.5 * ((double)qlo[a][i] + (double)qhi[a][i]), ex[a]));
            }
            std::vector<int> lv, in, em;
            for (int i = 0; i < 4; i++) {
                if (x.children[i] == -1) em.push_back(i);
                else if (x.children[i] & 0x80000000) lv.push_back(i);
                else in.push_back(i);
            }
            std::stable_sort(lv.begin(), lv.end(), [&](int a, int b) { return key[a] < key[b]; });
            std::stable_sort(in.begin(), in.end(), [&](int a, int b) { return key[a] > key[b]; });
            std::vector<int> o = lv;
            o.insert(o.end(), in.begin(), in.end());
            o.insert(o.end(), em.begin(), em.end());
            for (int k = 0; k < 4; k++) ord[ni][oct][k] = o[k];
        }
    }
    for (size_t w0 = 0; w0 + 64 <= n; w0 += 64) {
        const bool fwd = ((w0 / 64) % 5) != 4;
        if (fwd != fwd_waves) continue;
        km.waves++;
        std::vector<std::vector<std::array<int, 4>>> lanes(64);
        size_t mp = 0;
        for (int l = 0; l < 64; l++) {
            const float *o = &rays[6 * (w0 + l)], *d = o + 3;
            const int oct = (d[0] < 0 ? 1 : 0) | (d[1] < 0 ? 2 : 0) | (d[2] < 0 ? 4 : 0);
            float inv[3];
            for (int k = 0; k < 3; k++) inv[k] = d[k] == 0 ? 1e7f : 1.f / d[k];
            float tmax = 3.4e38f;
            std::vector<int> st = { 0 };
            while (!st.empty()) {
                const int ni = st.back();
                st.pop_back();
                km.pops++;
                lanes[l].push_back({ 0, 0, 0, 0 });
                const Node &x = nd[ni];
                const float sx = std::ldexp(1.f, x.expX), sy = std::ldexp(1.f, x.expY), sz = std::ldexp(1.f, x.expZ);
                const float tmax_entry = tmax;
                std::vector<std::pair<int, int>> deferred; // (leaf, ntri, slot) of passing leaves
                std::vector<int> dslot;
                for (int k = 0; k < 4; k++) {
                    const int i = ord[ni][oct][k];
                    if (x.children[i] == -1) continue;
                    const float lo[3] = { x.minX + sx * x.qMinX[i], x.minY + sy * x.qMinY[i], x.minZ + sz * x.qMinZ[i] };
                    const float hi[3] = { x.minX + sx * x.qMaxX[i], x.minY + sy * x.qMaxY[i], x.minZ + sz * x.qMaxZ[i] };
                    float tn = 0, tf = g_deferTris ? tmax_entry : tmax;
                    for (int a = 0; a < 3; a++) {
                        const float p = (lo[a] - o[a]) * inv[a], q = (hi[a] - o[a]) * inv[a];
                        tn = std::max(tn, std::min(p, q));
                        tf = std::min(tf, std::max(p, q));
                    }
                    if (tn > tf) continue;
                    if (x.children[i] & 0x80000000) {
                        const int leaf = x.children[i] & 0x7fffffff;
                        if (g_deferTris) {
                            deferred.push_back({ leaf, x.triSize[i] });
                            dslot.push_back(k);
                            continue;
                        }
                        for (int q = 0; q < x.triSize[i]; q++) {
                            lanes[l].back()[k]++;
                            km.tris++;
                            float th;
                            if (tri(&vt[(leaf + q) * 9], o, d, tmax, th)) tmax = th;
                        }
                    } else {
                        st.push_back(x.children[i]);
                    }
                }
                for (size_t e = 0; e < deferred.size(); e++)
                    for (int q = 0; q < deferred[e].second; q++) {
                        lanes[l].back()[dslot[e]]++;
                        km.tris++;
                        float th;
                        if (tri(&vt[(deferred[e].first + q) * 9], o, d, tmax, th)) tmax = th;
                    }
            }
            mp = std::max(mp, lanes[l].size());
            if (out_t) (*out_t)[w0 + l] = tmax;
            if (ref_t && (*ref_t)[w0 + l] != tmax) {
                const float a = (*ref_t)[w0 + l];
                if (std::fabs(a - tmax) > 1e-4f * std::max(1.f, std::fabs(a))) km.wrong++;
            }
        }
        km.nodeIters += mp;
        for (size_t it = 0; it < mp; it++) {
            for (int k = 0; k < 4; k++) {
                int m = 0;
                for (auto &L : lanes)
                    if (it < L.size()) m = std::max(m, L[it][k]);
                km.triIters += m;
            }
            int mm = 0;
            for (auto &L : lanes)
                if (it < L.size()) mm = std::max(mm, L[it][0] + L[it][1] + L[it][2] + L[it][3]);
            km.triItersMerged += mm;
        }
    }
}

static int treesMain(const char *scene, const std::vector<float> &rays)
{
    struct V { const char *name; std::vector<int32_t> o; };
    const std::vector<V> vs = {
        { "collision tree: SAH 16 bins, leaf 2", { 2, 16, 0, 400, 0 } },
        { "product lidar tree (scene.h lidarBVHOpts)", { 2, 12, 1, 400, 10 } },
        { "SAH 16 bins, leaf 1", { 1, 16, 0, 400, 0 } },
        { "SAH full sweep, leaf 2", { 2, 0, 0, 400, 0 } },
        { "SAH full sweep, leaf 1", { 1, 0, 0, 400, 0 } },
        { "SAH full sweep, leaf 2, trav 1", { 2, 0, 0, 100, 0 } },
        { "SAH full sweep, leaf 2, trav 2", { 2, 0, 0, 200, 0 } },
        { "SAH full sweep, leaf 2, trav 8", { 2, 0, 0, 800, 0 } },
        { "lidar measure, 16 bins, leaf 2", { 2, 16, 1, 400, 0 } },
        { "lidar measure, full sweep, leaf 2", { 2, 0, 1, 400, 0 } },
        { "lidar measure, full sweep, leaf 1", { 1, 0, 1, 400, 0 } },
        { "lidar measure + 0.05 floor, full sweep, leaf 2", { 2, 0, 1, 400, 5 } },
        { "lidar measure + 0.2 floor, full sweep, leaf 2", { 2, 0, 1, 400, 20 } },
        { "lidar measure + 0.2 floor, full sweep, leaf 1", { 1, 0, 1, 400, 20 } },
        { "lidar measure, full sweep, leaf 2, trav 2", { 2, 0, 1, 200, 0 } },
        { "lidar measure, full sweep, leaf 2, trav 8", { 2, 0, 1, 800, 0 } },
    };
    std::vector<V> custom;
    if (const char *e = getenv("TRAV_OPTS")) { // "a,b,c,d,e|a,b,..." (mpenv_scene_bvh_variant opts)
        static std::vector<std::string> names;
        std::string all = e;
        size_t p = 0;
        custom.push_back(vs[0]);
        while (p <= all.size()) {
            size_t q = all.find('|', p);
            if (q == std::string::npos) q = all.size();
            std::string one = all.substr(p, q - p);
            if (!one.empty()) {
                V v;
                names.push_back(one);
                size_t a = 0;
                while (a <= one.size()) {
                    size_t b = one.find(',', a);
                    if (b == std::string::npos) b = one.size();
                    v.o.push_back(std::atoi(one.substr(a, b - a).c_str()));
                    a = b + 1;
                }
                custom.push_back(v);
            }
            p = q + 1;
        }
        for (size_t i = 1; i < custom.size(); i++) custom[i].name = names[i - 1].c_str();
    }
    const std::vector<V> &list = custom.empty() ? vs : custom;
    std::vector<float> ref_t(rays.size() / 6);
    double base = 0;
    for (size_t vi = 0; vi < list.size(); vi++) {
        const V &cv = list[vi];
        int32_t nn = 0, nv = 0, ms = 0;
        if (mpenv_scene_bvh_variant(scene, cv.o.data(), (int32_t)cv.o.size(), nullptr, &nn, nullptr, &nv, &ms))
            return 1;
        std::vector<Node> nd(nn);
        std::vector<float> vt((size_t)nv * 3);
        mpenv_scene_bvh_variant(scene, cv.o.data(), (int32_t)cv.o.size(), nd.data(), &nn, vt.data(), &nv, &ms);
        KM f, r;
        kernelModel(nd, vt, rays, true, f, vi ? &ref_t : nullptr, vi ? nullptr : &ref_t);
        kernelModel(nd, vt, rays, false, r, vi ? &ref_t : nullptr, vi ? nullptr : &ref_t);
        const double units = f.waves / 4;
        const double cost = (110 * (f.nodeIters + r.nodeIters) + 45 * (f.triIters + r.triIters)) / units;
        if (vi == 0) base = cost;
        if (getenv("TRAV_MERGED")) {
            const double cm = (110 * (f.nodeIters + r.nodeIters) + 45 * (f.triItersMerged + r.triItersMerged)) / units;
            printf("   merged triangle loop: fwd tri it %5.2f rear %5.2f, cost/unit %6.0f (%+.1f%% vs this tree per-slot)\n",
                   f.triItersMerged / f.waves, r.triItersMerged / r.waves, cm, 100.0 * (cm / cost - 1));
        }
        printf("%-48s nodes %3d stack %2d | fwd wave: node it %5.2f tri it %5.2f | rear wave: %5.2f / %5.2f | "
               "lane pops/ray %.2f tris/ray %.2f | cost/unit %6.0f (%+.1f%%)%s\n",
               cv.name, nn, ms, f.nodeIters / f.waves, f.triIters / f.waves, r.nodeIters / r.waves,
               r.triIters / r.waves, (f.pops + r.pops) / (rays.size() / 6), (f.tris + r.tris) / (rays.size() / 6), cost,
               100.0 * (cost / base - 1), (f.wrong + r.wrong) ? " hits differ" : "");
        if (f.wrong + r.wrong) printf("    rays whose closest hit differs from the product tree: %.0f of %zu\n", f.wrong + r.wrong, rays.size() / 6);
    }
    return 0;
}

// ---- TRAV_TUNE: ray-driven tuning of the lidar tree.  Coordinate descent
// over BVHBuildOpts::splitRank (per binary build node down to depth
// TRAV_TUNE_DEPTH, the rank among its distinct SAH candidate splits, up to
// TRAV_TUNE_RANKS) and collapseChoice (key -hid: which inner children the
// 4-wide node rooted there opens): each move is scored by kernelModel's lockstep cost
// summed over the TRAIN ray sets (each relative to the untuned tree), kept
// if it lowers it; trees over TRAV_TUNE_NODES nodes or a stack over 14 are
// rejected.  The VAL sets are reported, never optimised.
//   TRAV_TUNE=1 trav_stats SCENE TRAIN1.f32,TRAIN2.f32 VAL1.f32,VAL2.f32
static std::vector<float> readRays(const std::string &path)
{
    std::vector<float> r;
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) return r;
    float buf[6];
    while (fread(buf, 4, 6, f) == 6) r.insert(r.end(), buf, buf + 6);
    fclose(f);
    return r;
}

static std::vector<std::string> splitList(const std::string &s)
{
    std::vector<std::string> v;
    size_t p = 0;
    while (p <= s.size()) {
        size_t q = s.find(',', p);
        if (q == std::string::npos) q = s.size();
        if (q > p) v.push_back(s.substr(p, q - p));
        p = q + 1;
    }
    return v;
}

struct TuneEval {
    std::vector<double> cost; // per ray set
    int nodes = 0, stack = 0;
    bool ok = false, same = false; // same: the tree of `skip_if` (not evaluated)
    std::string bytes;             // node + vertex bytes
};

static TuneEval tuneEval(const char *scene, const std::vector<int32_t> &opts, const std::vector<std::vector<float>> &sets,
                         const std::string *skip_if = nullptr)
{
    TuneEval e;
    int32_t nn = 0, nv = 0, ms = 0;
    if (mpenv_scene_bvh_variant(scene, opts.data(), (int32_t)opts.size(), nullptr, &nn, nullptr, &nv, &ms)) return e;
    std::vector<Node> nd(nn);
    std::vector<float> vt((size_t)nv * 3);
    mpenv_scene_bvh_variant(scene, opts.data(), (int32_t)opts.size(), nd.data(), &nn, vt.data(), &nv, &ms);
    e.nodes = nn;
    e.stack = ms;
    e.bytes.assign(reinterpret_cast<const char *>(nd.data()), nd.size() * sizeof(Node));
    e.bytes.append(reinterpret_cast<const char *>(vt.data()), vt.size() * 4);
    if (skip_if && *skip_if == e.bytes) {
        e.same = true;
        return e;
    }
    for (const auto &rays : sets) {
        KM f, r;
        kernelModel(nd, vt, rays, true, f);
        kernelModel(nd, vt, rays, false, r);
        e.cost.push_back((110 * (f.nodeIters + r.nodeIters) + 45 * (f.triIters + r.triIters)) / (f.waves / 4));
    }
    e.ok = true;
    return e;
}

static int tuneMain(const char *scene, const char *train_list, const char *val_list)
{
    std::vector<std::vector<float>> train, val;
    // TRAV_TUNE_SUB=k: train on every k-th 4-agent unit (320 rays: 4 forward
    // waves + 1 rear wave) of each set, for speed
    const int sub = getenv("TRAV_TUNE_SUB") ? std::max(1, atoi(getenv("TRAV_TUNE_SUB"))) : 1;
    for (const auto &p : splitList(train_list)) {
        std::vector<float> r = readRays(p), t;
        for (size_t u = 0; (u + 1) * 320 * 6 <= r.size(); u += sub)
            t.insert(t.end(), r.begin() + u * 320 * 6, r.begin() + (u + 1) * 320 * 6);
        train.push_back(t);
    }
    for (const auto &p : splitList(val_list)) val.push_back(readRays(p));
    const int depth = getenv("TRAV_TUNE_DEPTH") ? atoi(getenv("TRAV_TUNE_DEPTH")) : 7;
    const int ranks = getenv("TRAV_TUNE_RANKS") ? atoi(getenv("TRAV_TUNE_RANKS")) : 6;
    const int maxNodes = getenv("TRAV_TUNE_NODES") ? atoi(getenv("TRAV_TUNE_NODES")) : 64;
    const int passes = getenv("TRAV_TUNE_PASSES") ? atoi(getenv("TRAV_TUNE_PASSES")) : 3;
    const std::vector<int32_t> base = { 2, 12, 1, 400, 10 };
    std::map<int64_t, int> cur;
    if (const char *init = getenv("TRAV_TUNE_INIT")) { // "hid:rank hid:rank ..." (a previous run's splitRank line)
        std::string t = init;
        size_t p = 0;
        while (p < t.size()) {
            size_t q = t.find(' ', p);
            if (q == std::string::npos) q = t.size();
            const std::string one = t.substr(p, q - p);
            const size_t c = one.find(':');
            if (c != std::string::npos) cur[(int64_t)std::stoll(one.substr(0, c))] = std::stoi(one.substr(c + 1));
            p = q + 1;
        }
    }
    auto optsOf = [&](const std::map<int64_t, int> &m) {
        std::vector<int32_t> o = base;
        for (auto &kv : m) {
            if (kv.second == 0) continue;
            o.push_back((int32_t)kv.first);
            o.push_back(kv.second);
        }
        return o;
    };
    const TuneEval b0 = tuneEval(scene, base, train), v0 = tuneEval(scene, base, val);
    auto score = [&](const TuneEval &e) {
        double s = 0;
        for (size_t i = 0; i < e.cost.size(); i++) s += e.cost[i] / b0.cost[i];
        return s / (double)e.cost.size();
    };
    const TuneEval s0 = tuneEval(scene, optsOf(cur), train);
    double best = score(s0);
    std::string bestBytes = s0.bytes;
    printf("start %.4f; untuned: train", best);
    for (double c : b0.cost) printf(" %.0f", c);
    printf(" | val");
    for (double c : v0.cost) printf(" %.0f", c);
    printf(" | nodes %d stack %d\n", b0.nodes, b0.stack);
    fflush(stdout);
    const unsigned nth = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    for (int pass = 0; pass < passes; pass++) {
        bool improved = false;
        for (uint32_t hid = 1; hid < (1u << depth); hid++) {
            std::vector<std::map<int64_t, int>> cands;
            // split ranks at hid, then (key -hid) the collapse choices of the
            // 4-wide node whose binary root is hid
            for (const int64_t key : { (int64_t)hid, -(int64_t)hid }) {
                const int have = cur.count(key) ? cur[key] : 0;
                for (int r = 0; r < (key > 0 ? ranks : 4); r++) {
                    if (r == have) continue;
                    auto m = cur;
                    m[key] = r;
                    cands.push_back(m);
                }
            }
            std::vector<TuneEval> res(cands.size());
            std::vector<std::thread> th;
            std::atomic<size_t> next { 0 };
            for (unsigned t = 0; t < nth; t++)
                th.emplace_back([&] {
                    for (size_t i; (i = next++) < cands.size();)
                        res[i] = tuneEval(scene, optsOf(cands[i]), train, &bestBytes);
                });
            for (auto &t : th) t.join();
            int pick = -1;
            for (size_t i = 0; i < cands.size(); i++) {
                if (!res[i].ok || res[i].same || res[i].nodes > maxNodes || res[i].stack > 14) continue;
                const double sc = score(res[i]);
                if (sc < best - 1e-4) {
                    best = sc;
                    pick = (int)i;
                }
            }
            if (pick >= 0) {
                cur = cands[pick];
                bestBytes = res[pick].bytes;
                improved = true;
                printf("pass %d hid %u: split %d collapse %d: train %.4f (nodes %d stack %d)\n", pass, hid, cur[(int64_t)hid], cur[-(int64_t)hid], best,
                       res[pick].nodes, res[pick].stack);
                fflush(stdout);
            }
        }
        if (!improved) break;
    }
    // TRAV_TUNE_KICKS=n: iterated local search -- n times, re-rank 3 random
    // nodes of the best tree (depth <= TRAV_TUNE_DEPTH), descend one pass
    // from there, keep the result if it beats the best
    const int kicks = getenv("TRAV_TUNE_KICKS") ? atoi(getenv("TRAV_TUNE_KICKS")) : 0;
    uint64_t rng = 0x9e3779b97f4a7c15ull;
    auto rnd = [&](uint32_t n) {
        rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
        return (uint32_t)(rng % n);
    };
    for (int kk = 0; kk < kicks; kk++) {
        auto m = cur;
        for (int j = 0; j < 3; j++) m[1 + rnd((1u << std::min(depth, 7)) - 1)] = (int)rnd((uint32_t)ranks);
        TuneEval e = tuneEval(scene, optsOf(m), train);
        if (!e.ok || e.nodes > maxNodes || e.stack > 14) continue;
        double sc = score(e);
        std::string bytes = e.bytes;
        for (uint32_t hid = 1; hid < (1u << depth); hid++) {
            std::vector<std::map<int64_t, int>> cands;
            for (const int64_t key : { (int64_t)hid, -(int64_t)hid }) {
                const int have = m.count(key) ? m[key] : 0;
                for (int r = 0; r < (key > 0 ? ranks : 4); r++) {
                    if (r == have) continue;
                    auto c = m;
                    c[key] = r;
                    cands.push_back(c);
                }
            }
            std::vector<TuneEval> res(cands.size());
            std::vector<std::thread> th;
            std::atomic<size_t> next { 0 };
            for (unsigned t = 0; t < nth; t++)
                th.emplace_back([&] {
                    for (size_t i; (i = next++) < cands.size();) res[i] = tuneEval(scene, optsOf(cands[i]), train, &bytes);
                });
            for (auto &t : th) t.join();
            for (size_t i = 0; i < cands.size(); i++) {
                if (!res[i].ok || res[i].same || res[i].nodes > maxNodes || res[i].stack > 14) continue;
                const double c = score(res[i]);
                if (c < sc - 1e-4) {
                    sc = c;
                    m = cands[i];
                    bytes = res[i].bytes;
                }
            }
        }
        printf("kick %d: %.4f (best %.4f)\n", kk, sc, best);
        fflush(stdout);
        if (sc < best - 1e-4) {
            best = sc;
            cur = m;
            bestBytes = bytes;
            printf("  kept:");
            for (auto &kv : cur)
                if (kv.second) printf(" %lld:%d", (long long)kv.first, kv.second);
            printf("\n");
        }
    }
    const TuneEval ft = tuneEval(scene, optsOf(cur), train), fv = tuneEval(scene, optsOf(cur), val);
    printf("tuned: train");
    for (size_t i = 0; i < ft.cost.size(); i++) printf(" %.0f (%+.1f%%)", ft.cost[i], 100.0 * (ft.cost[i] / b0.cost[i] - 1));
    printf(" | val");
    for (size_t i = 0; i < fv.cost.size(); i++) printf(" %.0f (%+.1f%%)", fv.cost[i], 100.0 * (fv.cost[i] / v0.cost[i] - 1));
    printf(" | nodes %d stack %d\nsplitRank:", ft.nodes, ft.stack);
    for (auto &kv : cur)
        if (kv.second) printf(" %lld:%d", (long long)kv.first, kv.second);
    printf("\n");
    return 0;
}

int main(int argc, char **argv)
{
    if (getenv("TRAV_TUNE") && argc >= 4) return tuneMain(argv[1], argv[2], argv[3]);
    if (argc < 3) {
        fprintf(stderr, "%s SCENE RAYS.f32\n", argv[0]);
        return 1;
    }
    int32_t nn = 0, nv = 0, ms = 0;
    mpenv_scene_bvh(argv[1], nullptr, &nn, nullptr, &nv, &ms);
    nodes.resize(nn);
    verts.resize((size_t)nv * 3);
    mpenv_scene_bvh(argv[1], nodes.data(), &nn, verts.data(), &nv, &ms);
    FILE *f = fopen(argv[2], "rb");
    std::vector<float> rays;
    float buf[6];
    while (fread(buf, 4, 6, f) == 6) rays.insert(rays.end(), buf, buf + 6);
    fclose(f);
    size_t n = rays.size() / 6;
    g_deferTris = getenv("TRAV_DEFER") != nullptr;
    if (getenv("TRAV_TREES")) return treesMain(argv[1], rays);
    {
        double un = 0, ut = 0;
        for (size_t w0 = 0; w0 < n; w0 += 64) {
            std::vector<char> seen_n(nodes.size(), 0);
            std::vector<int> leafset;
            for (size_t r = w0; r < std::min(n, w0 + 64); r++) {
                Visit v;
                traceVisits(&rays[6 * r], &rays[6 * r + 3], v);
                for (int x : v.nodes) seen_n[x] = 1;
                for (int x : v.leaves) leafset.push_back(x);
            }
            std::sort(leafset.begin(), leafset.end());
            leafset.erase(std::unique(leafset.begin(), leafset.end()), leafset.end());
            for (char c : seen_n) un += c;
            for (int x : leafset) ut += x & 3;
        }
        double waves = (double)((n + 63) / 64);
        printf("packet (64 consecutive rays): union nodes/wave %.2f, union tris/wave %.2f\n", un / waves, ut / waves);
    }
    buildOctOrder();
    if (getenv("TRAV_PAIR")) return pairMain(rays);
    if (getenv("TRAV_FAN")) {
        // forward waves only (dump_lidar_rays order: 4 forward waves, then 1 rear)
        // which side of a triangle does an accepted hit come from?
        {
            long pos = 0, neg = 0;
            for (size_t r = 0; r < n; r += 7) {
                Stats one;
                trace(&rays[6 * r], &rays[6 * r + 3], 2, one);
                if (g_lastTri < 0) continue;
                const float *tv = &verts[g_lastTri * 9], *o = &rays[6 * r];
                const double e1[3] = { tv[3] - tv[0], tv[4] - tv[1], tv[5] - tv[2] };
                const double e2[3] = { tv[6] - tv[0], tv[7] - tv[1], tv[8] - tv[2] };
                const double nn[3] = { e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0] };
                const double so = nn[0] * (o[0] - tv[0]) + nn[1] * (o[1] - tv[1]) + nn[2] * (o[2] - tv[2]);
                (so > 0 ? pos : neg)++;
            }
            printf("accepted hits: origin on the +normal side %ld, on the -normal side %ld\n", pos, neg);
            g_frontSign = getenv("TRAV_FAN_NOBF") ? 0 : (pos > neg ? 1 : -1);
        }
        for (int order = 0; order < 5; order++) {
            FanStats fs;
            double octNode = 0, octTri = 0;
            size_t nf = 0;
            for (size_t w0 = 0; w0 + 64 <= n; w0 += 64) {
                if ((w0 / 64) % 5 == 4) continue;
                fanWave(rays.data(), w0, order, fs);
                nf += 64;
                if (order) continue;
                double mp = 0;
                std::vector<Stats> lanes;
                for (size_t r = w0; r < w0 + 64; r++) {
                    Stats one;
                    trace(&rays[6 * r], &rays[6 * r + 3], 2, one);
                    lanes.push_back(one);
                    mp = std::max(mp, one.pops);
                }
                octNode += mp;
                for (int it = 0; it < (int)mp; it++)
                    for (int i = 0; i < 4; i++) {
                        int m = 0;
                        for (auto &L : lanes)
                            if (it < (int)L.slotTris.size()) m = std::max(m, L.slotTris[it][i]);
                        octTri += m;
                    }
            }
            printf("fan lists, %s: per forward wave: (tri, sheet) entries %.1f (lists > 64: %.3f), walked %.1f, "
                   "lockstep full tests %.1f, lane tests/ray %.2f | per sheet: front-facing %.1f, in the band %.1f | "
                   "closest hits differing from brute force %.0f of %zu",
                   order == 0 ? "sorted  " : order == 1 ? "bucketed" : order == 2 ? "unsorted" : order == 3 ? "merged, 8 buckets, walk all" : "merged, sorted, walk all", fs.entries / fs.waves,
                   fs.bigLists / fs.waves, fs.walked / fs.waves, fs.full / fs.waves, fs.laneTests / nf,
                   fs.planeTests / fs.waves / 2, fs.straddle / fs.waves / 2, fs.wrong, nf);
            if (!order) printf(" | octant BVH lockstep: node iters %.2f, tri tests %.2f", octNode / fs.waves, octTri / fs.waves);
            printf("\n");
        }
        return 0;
    }
    for (int ftb = 0; ftb < 4; ftb++) {
        Stats st;
        double wave_pops = 0, wave_tris = 0, simt_slot = 0, simt_merged = 0;
        for (size_t w0 = 0; w0 < n; w0 += 64) {
            double mp = 0, mt = 0;
            std::vector<Stats> lanes;
            for (size_t r = w0; r < std::min(n, w0 + 64); r++) {
                Stats one;
                trace(&rays[6 * r], &rays[6 * r + 3], ftb, one);
                lanes.push_back(one);
                mp = std::max(mp, one.pops);
                mt = std::max(mt, one.tris);
                st.pops += one.pops; st.boxes += one.boxes; st.tris += one.tris;
                st.maxStack = std::max(st.maxStack, one.maxStack);
            }
            wave_pops += mp * 64; wave_tris += mt * 64;
            // lockstep: iteration it runs slot i's tri loop max_lanes(slotTris[it][i]) times
            for (int it = 0; it < (int)mp; it++) {
                int merged = 0;
                for (int i = 0; i < 4; i++) {
                    int m = 0;
                    for (auto &L : lanes)
                        if (it < (int)L.slotTris.size()) m = std::max(m, L.slotTris[it][i]);
                    simt_slot += m * 64;
                }
                for (auto &L : lanes)
                    if (it < (int)L.slotTris.size())
                        merged = std::max(merged, L.slotTris[it][0] + L.slotTris[it][1] + L.slotTris[it][2] + L.slotTris[it][3]);
                simt_merged += merged * 64;
            }
        }
        printf("   SIMT tri executions/ray: per-slot loops %.2f, merged loop %.2f\n", simt_slot / n, simt_merged / n);
        printf("%s: rays %zu  pops/ray %.2f  boxes/ray %.2f  tris/ray %.2f  maxStack %.0f | wave-max pops/ray %.2f tris %.2f\n",
               ftb == 1 ? "front-to-back" : ftb == 2 ? "octant order " : ftb == 3 ? "octant rev 1L" : "reference    ", n, st.pops / n, st.boxes / n, st.tris / n, st.maxStack,
               wave_pops / n, wave_tris / n);
    }
    for (int mode = 0; mode < 2; mode++) {
        PK fw, rr;
        size_t nf = 0, nr = 0;
        for (size_t w0 = 0; w0 < n; w0 += 64) {
            // dump_lidar_rays order: per 320-ray unit, 4 forward waves then 1 rear wave
            const bool fwd = ((w0 / 64) % 5) != 4;
            traceWavePacket(rays.data(), w0, std::min<size_t>(64, n - w0), mode, fwd ? fw : rr);
            (fwd ? nf : nr) += std::min<size_t>(64, n - w0);
        }
        printf("packet (%s order) forward waves: lockstep node iters/ray %.2f tri iters/ray %.2f | lane boxes/ray %.2f lane tris/ray %.2f\n",
               mode ? "mean-dir" : "lane-0  ", fw.nodeIters * 64 / nf, fw.triIters * 64 / nf, fw.laneBoxes / nf, fw.laneTris / nf);
        printf("packet (%s order) rear waves:    lockstep node iters/ray %.2f tri iters/ray %.2f | lane boxes/ray %.2f lane tris/ray %.2f\n",
               mode ? "mean-dir" : "lane-0  ", rr.nodeIters * 64 / nr, rr.triIters * 64 / nr, rr.laneBoxes / nr, rr.laneTris / nr);
    }
    if (const char *hp = getenv("TRAV_HINT")) {
        // Temporal hint: HP holds the same ray slots one step earlier; each
        // ray first tests the triangle its slot hit then (one test), and the
        // octant traversal starts with t_max = that hit's t.  Also the ideal
        // bound (t_max0 = the ray's own closest hit).
        FILE *hf = fopen(hp, "rb");
        std::vector<float> prev;
        while (fread(buf, 4, 6, hf) == 6) prev.insert(prev.end(), buf, buf + 6);
        fclose(hf);
        if (prev.size() != rays.size()) { fprintf(stderr, "hint file size differs\n"); return 1; }
        for (int variant = 0; variant < 3; variant++) {
            double lsPops = 0, lsTris = 0, lanePops = 0, laneTris = 0, hintHits = 0;
            for (size_t w0 = 0; w0 < n; w0 += 64) {
                std::vector<Stats> lanes;
                double mp = 0;
                for (size_t r = w0; r < std::min(n, w0 + 64); r++) {
                    float t0 = 3.4e38f;
                    if (variant == 1) {
                        Stats tmp;
                        trace(&prev[6 * r], &prev[6 * r + 3], 2, tmp);
                        const int ht = g_lastTri;
                        float th;
                        if (ht >= 0 && tri(&verts[ht * 9], &rays[6 * r], &rays[6 * r + 3], 3.4e38f, th)) {
                            t0 = th;
                            hintHits++;
                        }
                    } else if (variant == 2) {
                        Stats tmp;
                        trace(&rays[6 * r], &rays[6 * r + 3], 2, tmp);
                        if (g_lastTri >= 0) {
                            float th;
                            tri(&verts[g_lastTri * 9], &rays[6 * r], &rays[6 * r + 3], 3.4e38f, th);
                            t0 = th * 1.000001f;
                        }
                    }
                    Stats one;
                    trace(&rays[6 * r], &rays[6 * r + 3], 2, one, t0);
                    lanes.push_back(one);
                    mp = std::max(mp, one.pops);
                    lanePops += one.pops;
                    laneTris += one.tris;
                }
                lsPops += mp * 64;
                for (int it = 0; it < (int)mp; it++)
                    for (int i = 0; i < 4; i++) {
                        int m = 0;
                        for (auto &L : lanes)
                            if (it < (int)L.slotTris.size()) m = std::max(m, L.slotTris[it][i]);
                        lsTris += m * 64;
                    }
            }
            printf("%s: lockstep node iters/ray %.2f tri tests/ray %.2f | lane pops/ray %.2f tris/ray %.2f | hint hits %.3f\n",
                   variant == 0 ? "octant, no hint   " : variant == 1 ? "octant, prev hint " : "octant, ideal t0  ",
                   lsPops / n, lsTris / n, lanePops / n, laneTris / n, hintHits / n);
        }
        return 0;
    }
    if (getenv("TRAV_PACKET_ONLY")) return 0;
    // while-while with postponed triangles, octant order
    const int caps[] = { 1, 2, 3, 4, 8 };
    for (int cap : caps) {
        for (int need : { 64, 48, 32, 16, 1 }) {
            WW ww;
            for (size_t w0 = 0; w0 < n; w0 += 64) traceWaveWW(rays.data(), w0, std::min<size_t>(64, n - w0), cap, need, ww);
            printf("while-while cap %d need %2d: lockstep node iters/ray %.2f, tri iters/ray %.2f, phases/wave %.2f | "
                   "pops/ray %.2f tris/ray %.2f\n", cap, need, ww.nodeIters * 64 / n, ww.triIters * 64 / n,
                   ww.phases * 64 / n, ww.pops / n, ww.tris / n);
        }
    }
    return 0;
}
