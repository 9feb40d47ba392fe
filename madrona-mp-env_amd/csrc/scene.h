// scene.h — host-side map data: the four .bin formats of
// map_importer.cpp:35-567 and the compressed 4-wide BVH of mesh_bvh.hpp:56-86,
// built by our own SAH builder (the reference uses Embree's rtcBuildBVH,
// mesh_bvh_builder.cpp:218-737; Embree is absent here, and hit results are
// builder-independent up to exact ties).
#pragma once

#include <cstdint>
#include <string>
#include <map>
#include <vector>

#include "mpenv_core.h"

namespace mpenv {

// mesh_bvh.hpp:61-86 (MeshBVH::Node, 64 bytes).  Quantised child boxes:
// child AABB = min + 2^exp * q.  children[i] has bit 31 set for a leaf whose
// low bits give the leaf's first triangle; sentinel = -1.
struct BVHNode {
    float minX, minY, minZ;
    int8_t expX, expY, expZ;
    uint8_t internalNodes;
    uint8_t triSize[4];
    uint8_t qMinX[4];
    uint8_t qMinY[4];
    uint8_t qMinZ[4];
    uint8_t qMaxX[4];
    uint8_t qMaxY[4];
    uint8_t qMaxZ[4];
    int32_t children[4];
    int32_t parentID;
};
static_assert(sizeof(BVHNode) == 64, "BVHNode must be 64 bytes");

// Spawn (types.hpp:60-64): 32 bytes on disk.
struct Spawn {
    mp::AABB region;
    float yawMin, yawMax;
};
static_assert(sizeof(Spawn) == 32, "Spawn must be 32 bytes");

struct GoalZOBB {
    mp::Vec3 pMin, pMax;
    float rotation;
};

// GoalRegion (types.hpp:798-806) as filled by hardcodedGoalRegions
// (mgr.cpp:913-944).
struct GoalRegion {
    GoalZOBB subRegions[3];
    int32_t numSubRegions;
    int32_t attackerTeam; // bool in the reference
    float rewardStrength;
};

// Navigation mesh after vertex dedup + triangulation, with triangle
// adjacency and the A* next-hop table (navmesh.cpp).
struct NavMesh {
    std::vector<mp::Vec3> verts;
    std::vector<uint32_t> tris;   // 3 per triangle
    std::vector<int32_t> adj;     // 3 per triangle (neighbour across edge k, or -1)
    std::vector<int32_t> astar;   // [T][T] next triangle toward goal, -1 unreachable
    bool astarFromCache = false;
    size_t numTris() const { return tris.size() / 3; }
};

struct Scene {
    mp::AABB worldBounds;

    // Collision triangles after filterMeshes (map_importer.cpp:126-221),
    // de-indexed: tri i = verts[3i..3i+2].
    std::vector<mp::Vec3> triVerts;

    // BVH (nodes + per-leaf de-indexed vertices, 3 per triangle).
    std::vector<BVHNode> nodes;
    std::vector<mp::Vec3> bvhVerts;
    mp::AABB rootAABB;
    int32_t numLeaves = 0;
    int32_t maxDepth = 0;      // deepest inner-node level (root = 1)
    int32_t maxStack = 0;      // bound on traversal stack occupancy (reference order)
    int32_t maxStackAnyOrder = 0; // bound for any child push order

    // k_lidar's own tree over the same triangles (kLidarBVHOpts): closest
    // hits do not depend on the tree (up to ties between coplanar
    // overlapping triangles, DESIGN.md §2 definition 12), so pvpLidar walks
    // the tree that suits its near-horizontal fans while every other query
    // (sphere casts, line of sight, shots) keeps the collision tree above.
    std::vector<BVHNode> lidarNodes;
    std::vector<mp::Vec3> lidarVerts;
    int32_t lidarMaxStack = 0; // any push order
    bool lidarTuned = false;   // built with the scene's lidar_tree.txt split ranks

    std::vector<Spawn> aSpawns, bSpawns, commonRespawns;
    uint32_t numDefaultASpawns = 0, numDefaultBSpawns = 0;

    std::vector<mp::AABB> zoneAABBs;
    std::vector<float> zoneRotations;

    std::vector<mp::Vec3> navVerts;
    std::vector<uint32_t> navFaceCounts;
    std::vector<uint32_t> navIndices;

    std::vector<GoalRegion> goalRegions;

    NavMesh nav;
};

// Loads <dir>/{collisions,navmesh,spawns,zones}.bin (bindings.cpp:56-81) and
// builds the BVH.  Throws std::runtime_error on I/O failure (the reference
// FATALs, map_importer.cpp:229-231).
Scene loadScene(const std::string &scene_dir, bool spawn_in_middle = false);

// Dedups, triangulates and links the navmesh and builds/reads its A* table.
void buildNavMesh(Scene &s, const std::string &navmesh_path);

// Builder options.  The defaults are the collision tree every query but
// the lidar uses: 16-bin SAH over centroids (surface area, traversal cost 4,
// mesh_bvh_builder.cpp:347-348), leaves of <= 2 triangles, the binary tree
// collapsed to 4-wide by opening the largest child.
struct BVHBuildOpts {
    int maxLeaf = 2;        // 1 or 2 (the traversals unroll a 2-triangle leaf)
    int bins = 16;          // 0: full sweep (every centroid split on every axis)
    int measure = 0;        // 0: surface area; 1: lidar-weighted (below)
    float travCost = 4.f;   // SAH cost of an inner node relative to one triangle test
    float floorWeight = 0.f; // measure 1: weight of the horizontal (xy) face
    // Per binary build node, addressed by its heap index (root 1, children
    // 2i / 2i + 1): take the split of this rank in SAH-cost order instead of
    // the cheapest (rank 0).  A ray-driven tuning of the tree
    // (tools/trav_stats.cpp TRAV_TUNE) writes these.
    std::map<uint64_t, int> splitRank;
    // Per 4-wide node, by the heap index of its binary root: bit k set = at
    // the k-th child opening of the collapse take the inner child of
    // second-largest measure instead of the largest.
    std::map<uint64_t, int> collapseChoice;
};
// measure 1: the mean area a box shows to near-horizontal rays, (2/pi)
// (dx + dy) dz for uniformly distributed horizontal directions (the constant
// drops out of the SAH comparison), plus floorWeight * dx dy for the rays
// the aim pitch tilts -- what pvpLidar's fans (sim.cpp:3324-3506) see.

// The lidar tree's build (round 6, tools/trav_stats.cpp TRAV_TREES: the
// lockstep model of k_lidar's waves over recorded lidar fans):
// 12-bin SAH under the lidar measure with a 0.1 floor weight.
inline BVHBuildOpts lidarBVHOpts()
{
    BVHBuildOpts o;
    o.maxLeaf = 2;
    o.bins = 12;
    o.measure = 1;
    o.travCost = 4.f;
    o.floorWeight = 0.1f;
    return o;
}

// Builds the compressed 4-wide BVH over de-indexed triangles.
void buildBVH(const std::vector<mp::Vec3> &tri_verts, Scene &out, const BVHBuildOpts &opts = BVHBuildOpts {});

// Octant node images for closest-hit rays (k_lidar): 8 copies of the node
// array, copy o for rays whose direction sign bits are o (bit 0 x, bit 1 y,
// bit 2 z; a -0 component counts as negative, like the copysign'd inverse
// the slab test uses).  In each copy a node's child slots are permuted --
// leaf children first, nearest first, then internal children farthest
// first, then empty slots -- where "near" orders the child boxes' centres
// by their projection on the octant's diagonal (computed in double, ties
// by slot).  The reference's traversal loop over such a copy (slots in
// order, internal children pushed on a LIFO stack) therefore tests a
// node's leaves near-to-far and pops its nearest internal child first.
// Per axis whose bit is set, the copy also swaps the qMin / qMax bytes, so
// a ray of that octant finds its near slab in qMin and its far slab in qMax
// (mesh_bvh.inl:165-183 takes the min / max of the two; the slab t is
// monotonic in q with the slope's sign, so the values are the same).
// Node indices, unquantised bounds and leaves are unchanged.
std::vector<BVHNode> octantNodeImages(const std::vector<BVHNode> &nodes);

// The sphere cast's vertex test (mesh_bvh.inl:1073-1104) subtracts a vertex
// already taken relative to the origin o from o again, and returns t = 0
// for any visited triangle with a vertex v within the cast radius r of 2o
// (|2o - v| <= r, up to rounding).  quirkGrid marks, on a grid of `cell`
// x `cell` squares of the xy plane starting at (minX, minY), every square
// within xy distance r + margin of a vertex: when the square holding 2o is
// clear, no triangle can trigger the quirk for a cast from o, so the
// cast's result does not depend on which far triangles it visits.
struct QuirkGrid {
    float minX = 0.f, minY = 0.f, cell = 16.f;
    int32_t w = 0, h = 0;
    std::vector<uint32_t> bits; // row-major, w * h bits
};
QuirkGrid quirkGrid(const std::vector<mp::Vec3> &verts, float r, float margin, float cell);

} // namespace mpenv
