// trav_stats — CPU analysis of BVH traversal work on a ray set (not a
// correctness tool): nodes popped, child boxes tested, triangles tested per
// ray for the reference child order and for front-to-back order.
//
//   trav_stats SCENE_DIR RAYS.f32   (RAYS: n x 6 floats, origin + direction)
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
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

static void trace(const float *o, const float *d, bool ftb, Stats &st)
{
    float inv[3];
    for (int k = 0; k < 3; k++) inv[k] = d[k] == 0 ? 1e7f : 1.f / d[k];
    float tmax = 3.4e38f;
    std::vector<int> stack = { 0 };
    while (!stack.empty()) {
        st.maxStack = std::max(st.maxStack, (double)stack.size());
        int ni = stack.back();
        stack.pop_back();
        st.pops++;
        const Node &n = nodes[ni];
        std::pair<float, int> kids[4];
        int nk = 0;
        for (int i = 0; i < 4; i++) {
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
                    float t;
                    if (tri(&verts[(leaf + k) * 9], o, d, tmax, t)) tmax = t;
                }
            } else {
                kids[nk++] = { tn, n.children[i] };
            }
        }
        if (ftb) std::sort(kids, kids + nk, [](auto a, auto b) { return a.first > b.first; });
        for (int k = 0; k < nk; k++) stack.push_back(kids[k].second);
    }
}

int main(int argc, char **argv)
{
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
    for (int ftb = 0; ftb < 2; ftb++) {
        Stats st;
        double wave_pops = 0, wave_tris = 0;
        for (size_t w0 = 0; w0 < n; w0 += 64) {
            double mp = 0, mt = 0;
            for (size_t r = w0; r < std::min(n, w0 + 64); r++) {
                Stats one;
                trace(&rays[6 * r], &rays[6 * r + 3], ftb, one);
                mp = std::max(mp, one.pops);
                mt = std::max(mt, one.tris);
                st.pops += one.pops; st.boxes += one.boxes; st.tris += one.tris;
                st.maxStack = std::max(st.maxStack, one.maxStack);
            }
            wave_pops += mp * 64; wave_tris += mt * 64;
        }
        printf("%s: rays %zu  pops/ray %.2f  boxes/ray %.2f  tris/ray %.2f  maxStack %.0f | wave-max pops/ray %.2f tris %.2f\n",
               ftb ? "front-to-back" : "reference    ", n, st.pops / n, st.boxes / n, st.tris / n, st.maxStack,
               wave_pops / n, wave_tris / n);
    }
    return 0;
}
