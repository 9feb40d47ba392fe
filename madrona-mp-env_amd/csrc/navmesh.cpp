// navmesh.cpp — navigation mesh and the all-pairs A* next-hop table used by
// the scripted bots (planAStarAISystem, sim.cpp:5041-5172).
//
// Host-side setup, run once per Manager:
//   * vertex dedup of navmesh.bin (mgr.cpp:1301-1318 runs
//     meshopt_generateVertexRemap): bitwise-identical positions share one
//     index, numbered in first-occurrence order;
//   * Navmesh::initFromPolygons (Madrona, not vendored — defined here):
//     polygons are fanned into triangles (v0, vk, vk+1); triangle t's
//     neighbour across edge k (vk -> vk+1) is the lowest-numbered other
//     triangle with the same undirected deduplicated edge, else -1;
//   * buildAStarLookup (mgr.cpp:1155-1211): table[start * T + goal] = the
//     first triangle after `start` on the A* path to `goal` (goal itself if
//     adjacent, -1 if unreachable), with the reference's open set — an
//     ordered set keyed by the node's current score, so equal-score inserts
//     are dropped and re-scored entries stay where they were inserted — and
//     its far-goal early-out for meshes over 400 triangles
//     (mgr.cpp:1005-1153).  A "<navmesh>.astar" cache next to navmesh.bin is
//     read when present with the right size (mgr.cpp:1157-1180); it is never
//     written (scene directories may be read-only).
#include <cfloat>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <set>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "scene.h"

namespace mpenv {

using mp::Vec3;

namespace {

Vec3 triCenter(const NavMesh &nm, int tri)
{
    Vec3 c = mp::v3(0.f, 0.f, 0.f);
    for (int k = 0; k < 3; k++) c = c + nm.verts[nm.tris[3 * tri + k]] / 3.0f;
    return c;
}

float dist(Vec3 a, Vec3 b) { return mp::length(a - b); }

// A* over triangle centres (mgr.cpp:1055-1114).
struct AStar {
    const NavMesh &nm;
    std::vector<float> gScore, fScore;
    std::vector<int> parent;
    // early-out state (mgr.cpp:1005-1053, 1116-1153)
    bool farEnabled = false;
    float span = 0.f, nearDist2 = 0.f;
    int farHop[9];

    explicit AStar(const NavMesh &m) : nm(m)
    {
        const int T = (int)nm.numTris();
        gScore.resize(T);
        fScore.resize(T);
        parent.resize(T);
        const int kReasonable = 400;
        if (T > kReasonable) {
            Vec3 lo = mp::v3(FLT_MAX, FLT_MAX, FLT_MAX), hi = mp::v3(-FLT_MAX, -FLT_MAX, -FLT_MAX);
            for (const Vec3 &v : nm.verts) {
                lo = mp::v3(std::min(lo.x, v.x), std::min(lo.y, v.y), std::min(lo.z, v.z));
                hi = mp::v3(std::max(hi.x, v.x), std::max(hi.y, v.y), std::max(hi.z, v.z));
            }
            span = mp::length(hi - lo);
            nearDist2 = span * (float)kReasonable / (float)T;
            nearDist2 *= nearDist2;
            farEnabled = true;
        }
    }

    int farGoalHop(Vec3 from, Vec3 to) const
    {
        if (!farEnabled) return -1;
        if (mp::length2(from - to) < nearDist2) return -1;
        Vec3 d = mp::normalize(to - from);
        int dx = (int)(d.x * 1.9f), dy = (int)(d.y * 1.9f);
        return farHop[(dx + 1) + (dy + 1) * 3];
    }

    int nextHop(int start, int goal)
    {
        const Vec3 s = triCenter(nm, start), gpos = triCenter(nm, goal);
        int far = farGoalHop(s, gpos);
        if (far != -1) return far;
        const int T = (int)nm.numTris();
        for (int t = 0; t < T; t++) {
            parent[t] = -1;
            gScore[t] = FLT_MAX;
            fScore[t] = FLT_MAX;
        }
        gScore[start] = 0.f;
        // Ordered by the node's *current* fScore, like the reference's
        // std::set<int, cmp(score)>; keys are mutated in place on relaxation.
        auto cmp = [this](int a, int b) { return fScore[a] < fScore[b]; };
        std::set<int, decltype(cmp)> open(cmp);
        open.insert(start);
        while (!open.empty()) {
            const int cur = *open.begin();
            if (cur == goal) {
                for (int n = cur; n != start && n != -1; n = parent[n])
                    if (parent[n] == start) return n;
                return goal;
            }
            open.erase(open.begin());
            const Vec3 c = cur == start ? s : triCenter(nm, cur);
            for (int k = 0; k < 3; k++) {
                const int nb = nm.adj[3 * cur + k];
                if (nb == -1) continue;
                const Vec3 np = triCenter(nm, nb);
                const float g = gScore[cur] + dist(c, np);
                if (g < gScore[nb]) {
                    parent[nb] = cur;
                    gScore[nb] = g;
                    fScore[nb] = g + dist(np, gpos);
                    open.insert(nb);
                }
            }
        }
        return -1;
    }

    void prepareFarHops(int start)
    {
        if (!farEnabled) return;
        farEnabled = false; // the hops themselves are computed without early-out
        const int T = (int)nm.numTris();
        for (int dx = -1; dx <= 1; dx++) {
            for (int dy = -1; dy <= 1; dy++) {
                if (dx == 0 && dy == 0) continue;
                Vec3 dir = mp::normalize(mp::v3((float)dx, (float)dy, 0.f));
                Vec3 s = triCenter(nm, start);
                Vec3 end = s + dir * span * 2.0f;
                float best = FLT_MAX;
                int best_tri = -1;
                for (int t = 0; t < T; t++) {
                    float d = mp::length(triCenter(nm, t) - end);
                    if (d < best) {
                        best = d;
                        best_tri = t;
                    }
                }
                farHop[(dx + 1) + (dy + 1) * 3] = nextHop(start, best_tri);
            }
        }
        farEnabled = true;
    }
};

} // namespace

void buildNavMesh(Scene &s, const std::string &navmesh_path)
{
    NavMesh &nm = s.nav;
    nm = NavMesh {};
    // dedup (first-occurrence numbering of bitwise-identical positions)
    std::unordered_map<std::string, uint32_t> seen;
    std::vector<uint32_t> remap(s.navVerts.size());
    for (size_t i = 0; i < s.navVerts.size(); i++) {
        std::string key(reinterpret_cast<const char *>(&s.navVerts[i]), sizeof(Vec3));
        auto it = seen.find(key);
        if (it == seen.end()) {
            uint32_t id = (uint32_t)nm.verts.size();
            seen.emplace(key, id);
            nm.verts.push_back(s.navVerts[i]);
            remap[i] = id;
        } else {
            remap[i] = it->second;
        }
    }
    // fan triangulation
    size_t off = 0;
    for (uint32_t cnt : s.navFaceCounts) {
        if (off + cnt > s.navIndices.size()) throw std::runtime_error("navmesh.bin: face indices out of range");
        for (uint32_t k = 1; k + 1 < cnt; k++) {
            const uint32_t a = s.navIndices[off], b = s.navIndices[off + k], c = s.navIndices[off + k + 1];
            if (a >= remap.size() || b >= remap.size() || c >= remap.size())
                throw std::runtime_error("navmesh.bin: vertex index out of range");
            nm.tris.push_back(remap[a]);
            nm.tris.push_back(remap[b]);
            nm.tris.push_back(remap[c]);
        }
        off += cnt;
    }
    const int T = (int)nm.numTris();
    // adjacency through undirected edges
    std::unordered_map<uint64_t, std::vector<int>> edges;
    auto ekey = [](uint32_t a, uint32_t b) {
        return a < b ? ((uint64_t)a << 32) | b : ((uint64_t)b << 32) | a;
    };
    for (int t = 0; t < T; t++)
        for (int k = 0; k < 3; k++) edges[ekey(nm.tris[3 * t + k], nm.tris[3 * t + (k + 1) % 3])].push_back(t);
    nm.adj.assign((size_t)T * 3, -1);
    for (int t = 0; t < T; t++) {
        for (int k = 0; k < 3; k++) {
            for (int u : edges[ekey(nm.tris[3 * t + k], nm.tris[3 * t + (k + 1) % 3])]) {
                if (u != t) {
                    nm.adj[3 * t + k] = u;
                    break;
                }
            }
        }
    }
    // A* next-hop table: cached file or build
    nm.astar.assign((size_t)T * T, -1);
    std::string cache = navmesh_path;
    const size_t dot = cache.find_last_of('.');
    const size_t slash = cache.find_last_of('/');
    if (dot != std::string::npos && (slash == std::string::npos || dot > slash)) cache.resize(dot);
    cache += ".astar";
    if (FILE *f = std::fopen(cache.c_str(), "rb")) {
        std::fseek(f, 0, SEEK_END);
        long size = std::ftell(f);
        std::fseek(f, 0, SEEK_SET);
        bool ok = size == (long)(sizeof(int32_t) * (size_t)T * T) &&
                  std::fread(nm.astar.data(), sizeof(int32_t), (size_t)T * T, f) == (size_t)T * T;
        std::fclose(f);
        if (ok) {
            nm.astarFromCache = true;
            return;
        }
    }
    AStar search(nm);
    for (int start = 0; start < T; start++) {
        search.prepareFarHops(start);
        for (int goal = 0; goal < T; goal++) nm.astar[(size_t)start * T + goal] = search.nextHop(start, goal);
    }
}

} // namespace mpenv
