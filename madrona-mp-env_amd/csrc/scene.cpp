// scene.cpp — .bin loaders (map_importer.cpp:35-567, mgr.cpp:1229-1339) and
// an own binned-SAH 4-wide BVH builder that emits the reference's compressed
// node layout (mesh_bvh_builder.cpp:218-737 builds the same layout with
// Embree; Embree is not available, and every traversal result except exact
// ties is independent of the tree topology).
#include "scene.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <stdexcept>

namespace mpenv {

using mp::AABB;
using mp::Vec3;

namespace {

template <typename T>
void readPod(std::ifstream &f, T *dst, size_t n, const std::string &path)
{
    f.read(reinterpret_cast<char *>(dst), (std::streamsize)(sizeof(T) * n));
    if (!f) {
        throw std::runtime_error("mpenv: truncated file " + path);
    }
}

std::ifstream openOrThrow(const std::string &path)
{
    std::ifstream f(path, std::ios::binary);
    if (!f.is_open()) {
        throw std::runtime_error("mpenv: failed to open " + path);
    }
    return f;
}

// ------------------------------------------------------------ BVH builder
struct Box {
    double lo[3], hi[3];
    void reset() { for (int i = 0; i < 3; i++) { lo[i] = 1e300; hi[i] = -1e300; } }
    void grow(const Box &b) { for (int i = 0; i < 3; i++) { lo[i] = std::min(lo[i], b.lo[i]); hi[i] = std::max(hi[i], b.hi[i]); } }
    double area() const
    {
        double d[3];
        for (int i = 0; i < 3; i++) d[i] = std::max(0.0, hi[i] - lo[i]);
        return 2.0 * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0]);
    }
    // BVHBuildOpts::measure
    double measure(int m, double floor_w) const
    {
        if (m == 0) return area();
        double d[3];
        for (int i = 0; i < 3; i++) d[i] = std::max(0.0, hi[i] - lo[i]);
        return (d[0] + d[1]) * d[2] + floor_w * d[0] * d[1];
    }
};

struct BNode {            // binary build node
    Box box;
    int left = -1, right = -1;
    uint64_t hid = 0;      // heap index (root 1; 0 below depth 62)
    std::vector<int> tris; // leaf only
};

struct Builder {
    const std::vector<Vec3> &v;
    std::vector<Box> triBox;
    std::vector<Vec3> centroid;
    std::vector<BNode> bnodes;
    BVHBuildOpts o;
    int maxLeaf = 2;

    Builder(const std::vector<Vec3> &verts, const BVHBuildOpts &opts) : v(verts), o(opts)
    {
        maxLeaf = std::max(1, std::min(2, o.maxLeaf));
    }

    double meas(const Box &b) const { return b.measure(o.measure, o.floorWeight); }
    static double cen(const Vec3 &c, int ax) { return ax == 0 ? c.x : (ax == 1 ? c.y : c.z); }

    struct Cand {
        double cost;
        int axis, split;
    };

    // hid: heap index of this binary node (root 1), for o.splitRank
    int build(std::vector<int> tris, uint64_t hid = 1)
    {
        BNode node;
        node.box.reset();
        for (int t : tris) node.box.grow(triBox[t]);
        int id = (int)bnodes.size();
        node.hid = hid;
        bnodes.push_back(node);

        if ((int)tris.size() <= maxLeaf) { // maxLeafSize = numTrisPerLeaf (mesh_bvh_builder.cpp:345-346)
            bnodes[id].tris = tris;
            return id;
        }

        // SAH over centroids, intersection cost 1, traversal cost
        // o.travCost (4: mesh_bvh_builder.cpp:347-348), under o.measure:
        // binned (o.bins per axis) or a full sweep over sorted centroids.
        // Every candidate split is kept; the cheapest is taken unless
        // o.splitRank asks for another rank at this node.
        Box cbox; cbox.reset();
        for (int t : tris) {
            Box b; b.lo[0] = b.hi[0] = centroid[t].x; b.lo[1] = b.hi[1] = centroid[t].y;
            b.lo[2] = b.hi[2] = centroid[t].z; cbox.grow(b);
        }
        std::vector<Cand> cands;
        const int n = (int)tris.size();
        auto axisOrder = [&](int ax) {
            std::vector<int> ord = tris;
            std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return cen(centroid[a], ax) < cen(centroid[b], ax); });
            return ord;
        };
        const int kBins = std::min(64, std::max(1, o.bins));
        if (o.bins <= 0) {
            // full sweep: split after position s of the centroid order
            std::vector<double> right(n + 1);
            for (int ax = 0; ax < 3; ax++) {
                const std::vector<int> ord = axisOrder(ax);
                Box acc; acc.reset();
                for (int i = n - 1; i >= 1; i--) { acc.grow(triBox[ord[i]]); right[i] = meas(acc); }
                acc.reset();
                for (int i = 0; i + 1 < n; i++) {
                    acc.grow(triBox[ord[i]]);
                    cands.push_back({ o.travCost * meas(node.box) + meas(acc) * (i + 1) + right[i + 1] * (n - i - 1), ax, i + 1 });
                }
            }
        } else {
            for (int ax = 0; ax < 3; ax++) {
                double ext = cbox.hi[ax] - cbox.lo[ax];
                if (ext <= 0.0) continue;
                Box bins[64]; int cnt[64];
                for (int b = 0; b < kBins; b++) { bins[b].reset(); cnt[b] = 0; }
                for (int t : tris) {
                    double c = cen(centroid[t], ax);
                    int b = std::min(kBins - 1, (int)((c - cbox.lo[ax]) / ext * kBins));
                    bins[b].grow(triBox[t]); cnt[b]++;
                }
                for (int s = 1; s < kBins; s++) {
                    Box l, r; l.reset(); r.reset(); int nl = 0, nr = 0;
                    for (int b = 0; b < s; b++) { if (cnt[b]) { l.grow(bins[b]); nl += cnt[b]; } }
                    for (int b = s; b < kBins; b++) { if (cnt[b]) { r.grow(bins[b]); nr += cnt[b]; } }
                    if (nl == 0 || nr == 0) continue;
                    cands.push_back({ o.travCost * meas(node.box) + meas(l) * nl + meas(r) * nr, ax, s });
                }
            }
        }
        // cheapest first; ties keep generation order (axis, then split), so
        // rank 0 is the first strict minimum
        std::stable_sort(cands.begin(), cands.end(), [](const Cand &a, const Cand &b) { return a.cost < b.cost; });

        std::vector<int> lt, rt;
        if (cands.empty()) { // degenerate centroids: median split by index
            size_t h = tris.size() / 2;
            lt.assign(tris.begin(), tris.begin() + h);
            rt.assign(tris.begin() + h, tris.end());
        } else {
            auto partition = [&](const Cand &c, std::vector<int> &l, std::vector<int> &r) {
                l.clear();
                r.clear();
                if (o.bins <= 0) {
                    const std::vector<int> ord = axisOrder(c.axis);
                    l.assign(ord.begin(), ord.begin() + c.split);
                    r.assign(ord.begin() + c.split, ord.end());
                } else {
                    const double ext = cbox.hi[c.axis] - cbox.lo[c.axis];
                    for (int t : tris) {
                        int b = std::min(kBins - 1, (int)((cen(centroid[t], c.axis) - cbox.lo[c.axis]) / ext * kBins));
                        (b < c.split ? l : r).push_back(t);
                    }
                }
            };
            int rank = 0;
            const auto it = o.splitRank.find(hid);
            if (it != o.splitRank.end()) rank = std::max(0, it->second);
            // rank among the DISTINCT partitions (bins with nothing between
            // them give the same one), the last one when there are fewer
            std::vector<std::vector<int>> seen;
            for (const Cand &c : cands) {
                std::vector<int> l, r;
                partition(c, l, r);
                std::vector<int> key = l;
                std::sort(key.begin(), key.end());
                if (std::find(seen.begin(), seen.end(), key) != seen.end()) continue;
                seen.push_back(key);
                lt = l;
                rt = r;
                if ((int)seen.size() > rank) break;
            }
        }
        // heap index of the children (saturates below depth 62; no overrides there)
        const uint64_t hl = hid < (1ull << 62) ? 2 * hid : 0, hr = hid < (1ull << 62) ? 2 * hid + 1 : 0;
        int l = build(lt, hl);
        int r = build(rt, hr);
        bnodes[id].left = l;
        bnodes[id].right = r;
        return id;
    }
};

struct WNode { // 4-wide node before quantisation
    Box box;
    std::vector<int> kids;   // indices into bnodes (each is a child subtree root)
};

} // namespace

void buildBVH(const std::vector<Vec3> &tri_verts, Scene &out, const BVHBuildOpts &opts)
{
    const int num_tris = (int)(tri_verts.size() / 3);
    out.nodes.clear();
    out.bvhVerts.clear();
    if (num_tris == 0) {
        throw std::runtime_error("mpenv: scene has no collision triangles");
    }

    Builder b(tri_verts, opts);
    b.triBox.resize(num_tris);
    b.centroid.resize(num_tris);
    for (int t = 0; t < num_tris; t++) {
        Box bx; bx.reset();
        for (int k = 0; k < 3; k++) {
            const Vec3 &p = tri_verts[3 * t + k];
            bx.lo[0] = std::min(bx.lo[0], (double)p.x); bx.hi[0] = std::max(bx.hi[0], (double)p.x);
            bx.lo[1] = std::min(bx.lo[1], (double)p.y); bx.hi[1] = std::max(bx.hi[1], (double)p.y);
            bx.lo[2] = std::min(bx.lo[2], (double)p.z); bx.hi[2] = std::max(bx.hi[2], (double)p.z);
        }
        b.triBox[t] = bx;
        b.centroid[t] = mp::v3((float)(0.5 * (bx.lo[0] + bx.hi[0])), (float)(0.5 * (bx.lo[1] + bx.hi[1])),
                               (float)(0.5 * (bx.lo[2] + bx.hi[2])));
    }
    std::vector<int> all(num_tris);
    for (int t = 0; t < num_tris; t++) all[t] = t;
    int root = b.build(all);

    // Collapse the binary tree into a 4-wide tree: repeatedly open the
    // largest-area inner child until 4 children.
    auto isLeaf = [&](int n) { return b.bnodes[n].left < 0; };

    struct Pending { int bnode; int depth; };
    std::vector<int> wide_of; // output node index per expansion order
    // Each output inner node is identified by a binary subtree root.
    std::vector<std::vector<int>> kids_of;
    std::vector<int> order;   // binary roots of output inner nodes, DFS order
    std::vector<int> depth_of;

    // opts.collapseChoice[hid of broot] bit k: at the k-th opening, open the
    // inner child of second-largest measure instead of the largest
    auto collapse = [&](int broot) {
        std::vector<int> kids;
        if (isLeaf(broot)) { kids.push_back(broot); return kids; }
        kids.push_back(b.bnodes[broot].left);
        kids.push_back(b.bnodes[broot].right);
        const auto cit = opts.collapseChoice.find(b.bnodes[broot].hid);
        const int choice = cit == opts.collapseChoice.end() || b.bnodes[broot].hid == 0 ? 0 : cit->second;
        for (int step = 0; kids.size() < 4; step++) {
            int best = -1, second = -1; double best_area = -1, second_area = -1;
            for (int i = 0; i < (int)kids.size(); i++) {
                if (isLeaf(kids[i])) continue;
                double a = b.meas(b.bnodes[kids[i]].box);
                if (a > best_area) { second = best; second_area = best_area; best_area = a; best = i; }
                else if (a > second_area) { second_area = a; second = i; }
            }
            if (best < 0) break;
            if (((choice >> step) & 1) && second >= 0) best = second;
            int n = kids[best];
            kids.erase(kids.begin() + best);
            kids.insert(kids.begin() + best, b.bnodes[n].right);
            kids.insert(kids.begin() + best, b.bnodes[n].left);
        }
        return kids;
    };

    // Assign output inner-node ids in DFS pre-order (root = 0); leaves get
    // triangle offsets in the order they are first reached.
    std::vector<int> stack_b = { root };
    std::vector<int> stack_d = { 1 };
    std::vector<int> out_id_of_b(b.bnodes.size(), -1);
    out_id_of_b[root] = 0;
    order.push_back(root);
    depth_of.push_back(1);
    kids_of.push_back(collapse(root));
    // BFS-free explicit DFS to keep ids compact and deterministic.
    {
        std::vector<std::pair<int, int>> st; // (output node id, depth)
        st.push_back({0, 1});
        while (!st.empty()) {
            auto [oid, d] = st.back();
            st.pop_back();
            const std::vector<int> kids = kids_of[oid];
            for (int c : kids) {
                if (isLeaf(c)) continue;
                int nid = (int)order.size();
                out_id_of_b[c] = nid;
                order.push_back(c);
                depth_of.push_back(d + 1);
                kids_of.push_back(collapse(c));
                st.push_back({nid, d + 1});
            }
        }
    }

    const int num_inner = (int)order.size();
    out.nodes.resize(num_inner);
    out.maxDepth = 0;
    for (int d : depth_of) out.maxDepth = std::max(out.maxDepth, d);

    // Leaf triangle offsets: walk output nodes in id order, children in slot
    // order (deterministic).
    int tri_cursor = 0;
    out.numLeaves = 0;
    std::vector<int> leaf_off(b.bnodes.size(), -1);
    for (int oid = 0; oid < num_inner; oid++) {
        for (int c : kids_of[oid]) {
            if (!isLeaf(c)) continue;
            leaf_off[c] = tri_cursor;
            for (int t : b.bnodes[c].tris) {
                out.bvhVerts.push_back(tri_verts[3 * t + 0]);
                out.bvhVerts.push_back(tri_verts[3 * t + 1]);
                out.bvhVerts.push_back(tri_verts[3 * t + 2]);
                tri_cursor++;
            }
            out.numLeaves++;
        }
    }

    float root_max[3] = { -mp::kFltMax, -mp::kFltMax, -mp::kFltMax };
    for (int oid = 0; oid < num_inner; oid++) {
        BVHNode &n = out.nodes[oid];
        std::memset(&n, 0, sizeof(n));
        const std::vector<int> &kids = kids_of[oid];
        Box nb; nb.reset();
        for (int c : kids) nb.grow(b.bnodes[c].box);
        // Node origin in float, rounded down so that (min - child_lo) <= 0.
        float mn[3];
        for (int a = 0; a < 3; a++) {
            float f = (float)nb.lo[a];
            if ((double)f > nb.lo[a]) f = std::nextafter(f, -mp::kFltMax);
            mn[a] = f;
            root_max[a] = std::max(root_max[a], (float)nb.hi[a]);
        }
        n.minX = mn[0]; n.minY = mn[1]; n.minZ = mn[2];
        int8_t ex[3];
        for (int a = 0; a < 3; a++) {
            double range = nb.hi[a] - (double)mn[a];
            int e = -100;
            if (range > 0.0) {
                e = (int)std::ceil(std::log2(range / 253.0));
                while (std::ldexp(253.0, e) < range) e++;
            }
            e = std::max(-100, std::min(100, e));
            ex[a] = (int8_t)e;
        }
        n.expX = ex[0]; n.expY = ex[1]; n.expZ = ex[2];
        n.parentID = -1;
        int internal = 0;
        for (int i = 0; i < 4; i++) {
            if (i >= (int)kids.size()) {
                n.children[i] = -1;
                n.triSize[i] = 0;
                continue;
            }
            int c = kids[i];
            const Box &cb = b.bnodes[c].box;
            uint8_t *qmin[3] = { n.qMinX, n.qMinY, n.qMinZ };
            uint8_t *qmax[3] = { n.qMaxX, n.qMaxY, n.qMaxZ };
            for (int a = 0; a < 3; a++) {
                double s = std::ldexp(1.0, ex[a]);
                double lo = std::floor((cb.lo[a] - (double)mn[a]) / s) - 1.0;
                double hi = std::ceil((cb.hi[a] - (double)mn[a]) / s) + 1.0;
                lo = std::max(0.0, lo);
                hi = std::min(255.0, hi);
                qmin[a][i] = (uint8_t)lo;
                qmax[a][i] = (uint8_t)hi;
                // Conservativeness check (the traversal dequantises as
                // min + 2^e * q).
                if ((double)mn[a] + s * lo > cb.lo[a] || (double)mn[a] + s * hi < cb.hi[a]) {
                    throw std::runtime_error("mpenv: BVH quantisation not conservative");
                }
            }
            if (isLeaf(c)) {
                n.children[i] = (int32_t)(0x80000000u | (uint32_t)leaf_off[c]);
                n.triSize[i] = (uint8_t)b.bnodes[c].tris.size();
            } else {
                n.children[i] = out_id_of_b[c];
                n.triSize[i] = 0;
                internal++;
            }
        }
        n.internalNodes = (uint8_t)internal;
    }

    out.rootAABB.pMin = mp::v3(out.nodes[0].minX, out.nodes[0].minY, out.nodes[0].minZ);
    out.rootAABB.pMax = mp::v3(root_max[0], root_max[1], root_max[2]);
    // Exact worst-case occupancy of the LIFO traversal stack (mesh_bvh.inl
    // push order): after popping node X its k internal children are pushed
    // in slot order; child j (0-based) is processed with j entries below it.
    std::vector<int> occ(num_inner, 0);
    for (int oid = num_inner - 1; oid >= 0; oid--) { // children have larger ids (DFS pre-order)
        const BVHNode &n = out.nodes[oid];
        int k = 0, best = 0;
        for (int i = 0; i < 4; i++) {
            if (n.children[i] == -1 || (n.children[i] & 0x80000000)) continue;
            best = std::max(best, k + occ[n.children[i]]);
            k++;
        }
        occ[oid] = std::max(k, best);
    }
    out.maxStack = std::max(1, occ[0]);
    // Worst case over every push order (the front-to-back traversal pushes in
    // t_near order): the first-popped child can sit on all k-1 siblings.
    std::vector<int> occ_any(num_inner, 0);
    for (int oid = num_inner - 1; oid >= 0; oid--) {
        const BVHNode &n = out.nodes[oid];
        int k = 0, deepest = 0;
        for (int i = 0; i < 4; i++) {
            if (n.children[i] == -1 || (n.children[i] & 0x80000000)) continue;
            deepest = std::max(deepest, occ_any[n.children[i]]);
            k++;
        }
        occ_any[oid] = k == 0 ? 0 : std::max(k, (k - 1) + deepest);
    }
    out.maxStackAnyOrder = std::max(1, occ_any[0]);
}

std::vector<BVHNode> octantNodeImages(const std::vector<BVHNode> &nodes)
{
    const size_t n = nodes.size();
    std::vector<BVHNode> out(8 * n);
    for (int oct = 0; oct < 8; oct++) {
        const double sgn[3] = { (oct & 1) ? -1.0 : 1.0, (oct & 2) ? -1.0 : 1.0, (oct & 4) ? -1.0 : 1.0 };
        for (size_t ni = 0; ni < n; ni++) {
            const BVHNode &nd = nodes[ni];
            const int8_t ex[3] = { nd.expX, nd.expY, nd.expZ };
            const float mn[3] = { nd.minX, nd.minY, nd.minZ };
            const uint8_t *qlo[3] = { nd.qMinX, nd.qMinY, nd.qMinZ };
            const uint8_t *qhi[3] = { nd.qMaxX, nd.qMaxY, nd.qMaxZ };
            double key[4];
            for (int i = 0; i < 4; i++) {
                key[i] = 0.0;
                for (int a = 0; a < 3; a++)
                    key[i] += sgn[a] * ((double)mn[a] + std::ldexp(0.5 * ((double)qlo[a][i] + (double)qhi[a][i]), ex[a]));
            }
            std::vector<int> leaves, inner, empty;
            for (int i = 0; i < 4; i++) {
                if (nd.children[i] == -1) empty.push_back(i);
                else if (nd.children[i] & 0x80000000) leaves.push_back(i);
                else inner.push_back(i);
            }
            std::stable_sort(leaves.begin(), leaves.end(), [&](int a, int b) { return key[a] < key[b]; });
            std::stable_sort(inner.begin(), inner.end(), [&](int a, int b) { return key[a] > key[b]; });
            std::vector<int> ord = leaves;
            ord.insert(ord.end(), inner.begin(), inner.end());
            ord.insert(ord.end(), empty.begin(), empty.end());
            BVHNode p = nd;
            for (int k = 0; k < 4; k++) {
                const int i = ord[k];
                p.triSize[k] = nd.triSize[i];
                p.qMinX[k] = nd.qMinX[i]; p.qMinY[k] = nd.qMinY[i]; p.qMinZ[k] = nd.qMinZ[i];
                p.qMaxX[k] = nd.qMaxX[i]; p.qMaxY[k] = nd.qMaxY[i]; p.qMaxZ[k] = nd.qMaxZ[i];
                p.children[k] = nd.children[i];
                // near slab first for this octant's direction signs
                if (oct & 1) std::swap(p.qMinX[k], p.qMaxX[k]);
                if (oct & 2) std::swap(p.qMinY[k], p.qMaxY[k]);
                if (oct & 4) std::swap(p.qMinZ[k], p.qMaxZ[k]);
            }
            out[oct * n + ni] = p;
        }
    }
    return out;
}

QuirkGrid quirkGrid(const std::vector<Vec3> &verts, float r, float margin, float cell)
{
    QuirkGrid q;
    q.cell = cell;
    if (verts.empty()) return q;
    float lo[2] = { verts[0].x, verts[0].y }, hi[2] = { verts[0].x, verts[0].y };
    for (const Vec3 &v : verts) {
        lo[0] = std::min(lo[0], v.x); lo[1] = std::min(lo[1], v.y);
        hi[0] = std::max(hi[0], v.x); hi[1] = std::max(hi[1], v.y);
    }
    const float reach = r + margin;
    q.minX = std::floor((lo[0] - reach - cell) / cell) * cell;
    q.minY = std::floor((lo[1] - reach - cell) / cell) * cell;
    q.w = (int32_t)std::ceil((hi[0] + reach + cell - q.minX) / cell) + 1;
    q.h = (int32_t)std::ceil((hi[1] + reach + cell - q.minY) / cell) + 1;
    q.bits.assign(((size_t)q.w * q.h + 31) / 32, 0u);
    for (const Vec3 &v : verts) {
        const int x0 = (int)std::floor((v.x - reach - q.minX) / cell), x1 = (int)std::floor((v.x + reach - q.minX) / cell);
        const int y0 = (int)std::floor((v.y - reach - q.minY) / cell), y1 = (int)std::floor((v.y + reach - q.minY) / cell);
        for (int y = std::max(0, y0); y <= std::min(q.h - 1, y1); y++)
            for (int x = std::max(0, x0); x <= std::min(q.w - 1, x1); x++) {
                // distance from v to the square, in double
                const double cx0 = q.minX + (double)x * cell, cy0 = q.minY + (double)y * cell;
                const double dx = std::max({ cx0 - v.x, 0.0, (double)v.x - (cx0 + cell) });
                const double dy = std::max({ cy0 - v.y, 0.0, (double)v.y - (cy0 + cell) });
                if (dx * dx + dy * dy <= (double)reach * reach) {
                    const size_t bit = (size_t)y * q.w + x;
                    q.bits[bit >> 5] |= 1u << (bit & 31);
                }
            }
    }
    return q;
}

// lidar_tree.txt (optional, next to the .bin files): k_lidar's tree tuned
// for this scene -- BVHBuildOpts::splitRank entries ("split HID RANK") that
// tools/trav_stats.cpp TRAV_TUNE found against recorded lidar fans, and
// BVHBuildOpts::collapseChoice entries ("collapse HID CHOICE")
// (tools/write_lidar_tree.py writes the file).  Any ranks give a valid BVH
// (only the traversal cost changes), but they were tuned for one triangle
// set: the file names the FNV-1a 64 of its collisions.bin and is ignored
// for any other.
static uint64_t fnv1a64File(const std::string &path)
{
    std::ifstream f(path, std::ios::binary);
    uint64_t h = 1469598103934665603ull;
    char buf[4096];
    while (f) {
        f.read(buf, sizeof(buf));
        for (std::streamsize i = 0; i < f.gcount(); i++) {
            h ^= (uint8_t)buf[i];
            h *= 1099511628211ull;
        }
    }
    return h;
}

static void readLidarTuning(const std::string &dir, BVHBuildOpts &o)
{
    std::ifstream f(dir + "/lidar_tree.txt");
    if (!f) return;
    std::map<uint64_t, int> ranks, collapses;
    uint64_t want = 0;
    bool have_hash = false;
    std::string line;
    while (std::getline(f, line)) {
        if (line.empty() || line[0] == '#') continue;
        char key[32] = {};
        unsigned long long a = 0;
        int r = 0;
        if (std::sscanf(line.c_str(), "%31s %llx", key, &a) == 2 && std::strcmp(key, "collisions_fnv1a64") == 0) {
            want = a;
            have_hash = true;
        } else if (std::sscanf(line.c_str(), "%31s %llu %d", key, &a, &r) == 3 && std::strcmp(key, "split") == 0) {
            ranks[a] = r;
        } else if (std::sscanf(line.c_str(), "%31s %llu %d", key, &a, &r) == 3 && std::strcmp(key, "collapse") == 0) {
            collapses[a] = r;
        } else {
            throw std::runtime_error(dir + "/lidar_tree.txt: malformed line: " + line);
        }
    }
    if (have_hash && want == fnv1a64File(dir + "/collisions.bin")) {
        o.splitRank = ranks;
        o.collapseChoice = collapses;
    }
}

Scene loadScene(const std::string &dir, bool spawn_in_middle)
{
    Scene s;

    // ---- collisions.bin (map_importer.cpp:223-256, 35-124, 126-221)
    {
        const std::string path = dir + "/collisions.bin";
        std::ifstream f = openOrThrow(path);
        float wb[6];
        readPod(f, wb, 6, path);
        s.worldBounds.pMin = mp::v3(wb[0], wb[1], wb[2]);
        s.worldBounds.pMax = mp::v3(wb[3], wb[4], wb[5]);

        uint64_t num_materials = 0, num_name_bytes = 0;
        readPod(f, &num_materials, 1, path);
        readPod(f, &num_name_bytes, 1, path);
        std::vector<char> names(num_name_bytes);
        if (num_name_bytes) readPod(f, names.data(), num_name_bytes, path);
        std::vector<uint32_t> mat_flags(num_materials);
        if (num_materials) readPod(f, mat_flags.data(), num_materials, path);

        uint64_t num_meshes = 0, total_verts = 0, total_tris = 0;
        readPod(f, &num_meshes, 1, path);
        readPod(f, &total_verts, 1, path);
        readPod(f, &total_tris, 1, path);
        std::vector<Vec3> verts(total_verts);
        std::vector<uint32_t> idx(total_tris * 3);
        std::vector<uint32_t> tri_mats(total_tris);
        std::vector<uint32_t> mesh_info(num_meshes * 4); // vertexOffset, numVertices, triOffset, numTris
        readPod(f, verts.data(), total_verts, path);
        readPod(f, idx.data(), idx.size(), path);
        readPod(f, tri_mats.data(), tri_mats.size(), path);
        readPod(f, mesh_info.data(), mesh_info.size(), path);

        // mapOffset = 0, mapRotation = 0 (bindings.cpp:79-80): the
        // Quat::angleAxis(0).inv().rotateVec(v - 0) of map_importer.cpp:238-243
        // is the identity, applied here explicitly for fidelity.
        mp::Quat rot = mp::qinv(mp::angleAxis(0.f, mp::kUp));
        for (Vec3 &v : verts) v = mp::rotateVec(rot, v - mp::v3(0.f, 0.f, 0.f));

        // filterMeshes: drop BulletsOnly (flag value 1) triangles.
        for (uint64_t m = 0; m < num_meshes; m++) {
            const uint64_t voff = mesh_info[4 * m + 0], nv = mesh_info[4 * m + 1];
            const uint64_t toff = mesh_info[4 * m + 2], nt = mesh_info[4 * m + 3];
            if (voff + nv > total_verts || toff + nt > total_tris)
                throw std::runtime_error(path + ": mesh " + std::to_string(m) +
                                         " range outside the vertex/triangle arrays (truncated or malformed file)");
            for (uint64_t i = 0; i < nt; i++) {
                uint32_t mat = tri_mats[toff + i];
                if (mat < mat_flags.size() && mat_flags[mat] == 1u) continue;
                for (int k = 0; k < 3; k++) {
                    const uint64_t vi = idx[3 * (toff + i) + k];
                    if (vi >= nv)
                        throw std::runtime_error(path + ": mesh " + std::to_string(m) +
                                                 " vertex index out of range (truncated or malformed file)");
                    s.triVerts.push_back(verts[voff + vi]);
                }
            }
        }
    }

    buildBVH(s.triVerts, s);
    {
        Scene t;
        BVHBuildOpts lo = lidarBVHOpts();
        readLidarTuning(dir, lo);
        s.lidarTuned = !lo.splitRank.empty() || !lo.collapseChoice.empty();
        buildBVH(s.triVerts, t, lo);
        s.lidarNodes = std::move(t.nodes);
        s.lidarVerts = std::move(t.bvhVerts);
        s.lidarMaxStack = std::max(t.maxStack, t.maxStackAnyOrder);
    }

    // ---- navmesh.bin (map_importer.cpp:421-506)
    {
        const std::string path = dir + "/navmesh.bin";
        std::ifstream f = openOrThrow(path);
        uint32_t nv = 0, nf = 0, ni = 0;
        readPod(f, &nv, 1, path);
        s.navVerts.resize(nv);
        readPod(f, s.navVerts.data(), nv, path);
        readPod(f, &nf, 1, path);
        s.navFaceCounts.resize(nf);
        readPod(f, s.navFaceCounts.data(), nf, path);
        readPod(f, &ni, 1, path);
        s.navIndices.resize(ni);
        readPod(f, s.navIndices.data(), ni, path);
        buildNavMesh(s, path);
    }

    // ---- spawns.bin (map_importer.cpp:508-543)
    {
        const std::string path = dir + "/spawns.bin";
        std::ifstream f = openOrThrow(path);
        std::vector<Spawn> *dst[3] = { &s.aSpawns, &s.bSpawns, &s.commonRespawns };
        for (int k = 0; k < 3; k++) {
            uint32_t n = 0;
            readPod(f, &n, 1, path);
            dst[k]->resize(n);
            if (n) readPod(f, dst[k]->data(), n, path);
        }
        s.numDefaultASpawns = (uint32_t)s.aSpawns.size();
        s.numDefaultBSpawns = (uint32_t)s.bSpawns.size();
    }

    // SpawnInMiddle cell spawns (mgr.cpp:1251-1299).  The reference tests the
    // cell against BVH leaf boxes via findOverlaps; here against triangle
    // AABBs (builder-independent).
    if (spawn_in_middle) {
        AABB region = { mp::v3(-280.f, -200.f, 0.5f), mp::v3(280.f, 200.f, 0.5f) };
        Vec3 diff = region.pMax - region.pMin;
        const int cell_dim = 20;
        float cw = diff.x / cell_dim, ch = diff.y / cell_dim;
        for (int y = 0; y < cell_dim; y++) {
            for (int x = 0; x < cell_dim; x++) {
                Vec3 cmin = region.pMin + mp::v3(cw * x, ch * y, 0.5f);
                Vec3 cmax = cmin + mp::v3(cw, ch, 0.5f);
                bool overlaps = false;
                for (size_t t = 0; t + 2 < s.triVerts.size() && !overlaps; t += 3) {
                    float lo[3], hi[3];
                    for (int a = 0; a < 3; a++) {
                        float v0 = mp::comp(s.triVerts[t], a), v1 = mp::comp(s.triVerts[t + 1], a),
                              v2 = mp::comp(s.triVerts[t + 2], a);
                        lo[a] = std::min(v0, std::min(v1, v2));
                        hi[a] = std::max(v0, std::max(v1, v2));
                    }
                    overlaps = lo[0] <= cmax.x && hi[0] >= cmin.x && lo[1] <= cmax.y && hi[1] >= cmin.y &&
                               lo[2] <= cmax.z && hi[2] >= cmin.z;
                }
                if (!overlaps) {
                    Spawn sp;
                    sp.region.pMin = cmin; sp.region.pMax = cmax;
                    sp.yawMin = 0.f; sp.yawMax = 2.f * mp::kPi;
                    (x >= cell_dim / 2 ? s.bSpawns : s.aSpawns).push_back(sp);
                }
            }
        }
    }

    // ---- zones.bin (map_importer.cpp:545-567)
    {
        const std::string path = dir + "/zones.bin";
        std::ifstream f = openOrThrow(path);
        uint32_t n = 0;
        readPod(f, &n, 1, path);
        s.zoneAABBs.resize(n);
        s.zoneRotations.resize(n);
        if (n) {
            readPod(f, s.zoneAABBs.data(), n, path);
            readPod(f, s.zoneRotations.data(), n, path);
        }
    }

    // ---- hardcodedGoalRegions (mgr.cpp:913-944)
    {
        const float top = -56.f + 65.f * 1.5f;
        GoalRegion g0 = {};
        g0.subRegions[0] = { mp::v3(625.f, 510.f, -64.f), mp::v3(900.f, 540.f, top), 0.f };
        g0.numSubRegions = 1;
        g0.attackerTeam = 1;
        g0.rewardStrength = 1.f;
        GoalRegion g1 = {};
        g1.subRegions[0] = { mp::v3(938.f, 440.f, -56.f), mp::v3(1030.f, 539.f, top), 0.f };
        g1.subRegions[1] = { mp::v3(545.f, 102.f, -64.f), mp::v3(630.f, 134.f, top), 0.f };
        g1.numSubRegions = 2;
        g1.attackerTeam = 1;
        g1.rewardStrength = 1.f;
        s.goalRegions = { g0, g1 };
    }

    return s;
}

} // namespace mpenv
