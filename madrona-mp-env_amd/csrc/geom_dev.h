// geom_dev.h — gfx950 device geometry: compressed 4-wide BVH traversal with
// nodes and triangles staged in LDS, a register-resident byte stack, and the
// agent-capsule test (mesh_bvh.inl:110-1127, utils.cpp:10-138).
//
// Design:
//   * the whole collision BVH (simple_map: 61 x 64 B nodes + 756 x 12 B
//     vertices = 13 KB) is copied into LDS once per workgroup; every
//     traversal reads LDS only (ds_read), never HBM;
//   * the traversal stack is a 16-entry byte stack held in two 64-bit
//     registers (node indices < 256) — no scratch memory, no LDS stack;
//   * child-visit order and every float expression match the reference
//     (and the CPU oracle) exactly, so hits are bit-identical.
#pragma once

#include <hip/hip_runtime.h>

#include "engine.h"

#pragma clang fp contract(off)

namespace mpenv {

#define MP_LDS __attribute__((address_space(3)))

struct LBVH {
    const MP_LDS BVHNode *nodes;
    const MP_LDS float *verts;
    const MP_LDS float *pre; // sphere-casting kernels only (stageBVHSphere)
    const MP_LDS float *snodes; // sphere-cast node image (stageBVHSphere), else null
    unsigned long long *stats;  // workload counters (DevState::stats), null = off
    int32_t rotStride;          // stageBVHOct: float4s per rotated vertex copy
};

// Workload counter add, one atomic per wave: the active lanes' values
// (each < 16) summed by bit-plane ballots, added by the first active lane.
__device__ __forceinline__ void statAdd(unsigned long long *p, uint32_t v)
{
    const uint64_t act = __ballot(1);
    uint32_t total = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) total += (uint32_t)__popcll(__ballot((v >> b) & 1u)) << b;
    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
    if (below == 0 && total) atomicAdd(p, (unsigned long long)total);
}

__device__ __forceinline__ float expScaleD(int e) { return mp::u2f((uint32_t)(e + 127) << 23); }

constexpr float kSphereR = 15.f;  // consts::agentRadius: the radius of every k_move sphere cast
// Sphere-cast node image: loR[3][4], hiR[3][4], children[4], leaf tri
// count[4] (32 floats) at a stride of kSNodeFloats.  The casts read it with
// ds_read_b32 (bank = dword address mod 32): at a stride of 32 the same field
// of every node sits in one bank, so lanes at different nodes conflict (PMC:
// 44% of k_move's LDS cycles are conflict cycles); an odd stride puts node
// k's field in bank (k + field) mod 32, but k_move does not get faster (it
// waits on its cast chain, not on LDS: stride 33 measured 0.2182 vs 0.2181
// ms, round 3).
constexpr int kSNodeFloats = 32;

// Byte stack: push shifts left by 8 across a 128-bit register pair.
struct ByteStack {
    uint64_t lo, hi;
    int n;
};

__device__ __forceinline__ void bsPush(ByteStack &s, uint32_t v)
{
    s.hi = (s.hi << 8) | (s.lo >> 56);
    s.lo = (s.lo << 8) | (uint64_t)v;
    s.n += 1;
}

__device__ __forceinline__ uint32_t bsPop(ByteStack &s)
{
    uint32_t v = (uint32_t)(s.lo & 0xffu);
    s.lo = (s.lo >> 8) | (s.hi << 56);
    s.hi >>= 8;
    s.n -= 1;
    return v;
}

// Stage nodes + vertices into dynamic LDS (all threads participate).
// LDS image: nodes verbatim (64 B each), then every triangle vertex padded
// to a float4 so a triangle is three ds_read_b128.
// lidar = true: the lidar tree (Scene::lidarNodes, slot order), which k_vis
// walks too (its line-of-sight rays are near-horizontal like the fans; the
// answer does not depend on the tree, geom_dev.h visibleFullD)
__device__ __forceinline__ LBVH stageBVH(char *smem, const SceneDev &sc, bool lidar = false)
{
    const int numNodes = lidar ? sc.numLidarNodes : sc.numNodes;
    const int numVerts = lidar ? sc.numLidarVerts : sc.numVerts;
    const int node_q = numNodes * 4; // uint4 per node
    const uint4 *src_n = reinterpret_cast<const uint4 *>(lidar ? sc.lidarNodes : sc.nodes);
    uint4 *dst_n = reinterpret_cast<uint4 *>(smem);
    for (int k = threadIdx.x; k < node_q; k += blockDim.x) dst_n[k] = src_n[k];
    const float *src_v = lidar ? sc.lidarVerts : sc.verts;
    float4 *dst_v = reinterpret_cast<float4 *>(smem + (size_t)node_q * 16);
    for (int k = threadIdx.x; k < numVerts; k += blockDim.x)
        dst_v[k] = make_float4(src_v[3 * k], src_v[3 * k + 1], src_v[3 * k + 2], 0.f);
    __syncthreads();
    LBVH b;
    b.nodes = (const MP_LDS BVHNode *)(smem);
    b.verts = (const MP_LDS float *)(smem + (size_t)node_q * 16);
    b.pre = nullptr;
    b.snodes = nullptr;
    b.stats = nullptr;
    b.rotStride = 0;
    return b;
}

// stageBVH plus the per-triangle sphere-cast constants (SceneDev::triPre,
// two float4 per triangle) after the vertices.
__device__ __forceinline__ LBVH stageBVHSphere(char *smem, const SceneDev &sc)
{
    const size_t pre_off = (size_t)sc.numNodes * 64 + (size_t)sc.numVerts * 16;
    const int pre_q = (sc.numVerts / 3) * 2;
    const float4 *src_p = reinterpret_cast<const float4 *>(sc.triPre);
    float4 *dst_p = reinterpret_cast<float4 *>(smem + pre_off);
    for (int k = threadIdx.x; k < pre_q; k += blockDim.x) dst_p[k] = src_p[k];
    // Sphere-cast node image (kSNodeFloats per node): per axis a, the
    // children's dequantised slab ends already widened by the cast radius,
    // loR[a][i] = (min_a + 2^e_a * qMin_a[i]) - r and
    // hiR[a][i] = (min_a + 2^e_a * qMax_a[i]) + r -- the very expressions
    // sphereCastNodeCheck evaluates per child (mesh_bvh.inl:817-855) -- then
    // the children and triangle counts.  Built for radius kSphereR (every
    // k_move cast uses the agent radius).
    const size_t sn_off = pre_off + (size_t)(sc.numVerts / 3) * 32;
    float *sn = reinterpret_cast<float *>(smem + sn_off);
    for (int k = threadIdx.x; k < sc.numNodes * 4; k += blockDim.x) {
        const int n = k >> 2, i = k & 3;
        const BVHNode &nd = sc.nodes[n];
        float *o = sn + (size_t)n * kSNodeFloats;
        const float mins[3] = { nd.minX, nd.minY, nd.minZ };
        const int exps[3] = { nd.expX, nd.expY, nd.expZ };
        const uint8_t *qmn[3] = { nd.qMinX, nd.qMinY, nd.qMinZ };
        const uint8_t *qmx[3] = { nd.qMaxX, nd.qMaxY, nd.qMaxZ };
#pragma unroll
        for (int a = 0; a < 3; a++) {
            const float sc_a = expScaleD(exps[a]);
            o[a * 4 + i] = (mins[a] + sc_a * (float)qmn[a][i]) - kSphereR;
            o[12 + a * 4 + i] = (mins[a] + sc_a * (float)qmx[a][i]) + kSphereR;
        }
        o[24 + i] = __int_as_float(nd.children[i]);
        // Triangles sphereCastLeaf tests: always numTrisPerLeaf = 2 in leaf
        // order, whatever triSize says (mesh_bvh.inl:867-880;
        // fetchLeafTriangle never reports a missing triangle, 556-576), so a
        // 1-triangle leaf also tests the next leaf's first triangle.  Only
        // the last triangle's overrun past the vertex array is defined here
        // (not tested).
        int cnt = 0;
        if (nd.children[i] != -1 && (nd.children[i] & 0x80000000)) {
            const int leaf = nd.children[i] & 0x7fffffff;
            cnt = min(2, sc.numVerts / 3 - leaf);
        }
        o[28 + i] = __uint_as_float((uint32_t)cnt);
    }
    LBVH b = stageBVH(smem, sc); // ends with __syncthreads
    b.pre = (const MP_LDS float *)(smem + pre_off);
    b.snodes = (const MP_LDS float *)(smem + sn_off);
    return b;
}

// k_lidar's LDS image: the 8 octant node images of the lidar tree (scene.h
// octantNodeImages, 8 x numLidarNodes nodes) then its vertices as float4
// (three rotated copies).
// The traversal of a ray reads image (d.x < 0) | (d.y < 0) << 1 | (d.z < 0) << 2.  Each node takes
// kOctNodeQ = 4 16-B slots (packed 64-B nodes; a fifth pad slot, which moves
// nodes k != k' (mod 16) to different LDS bank groups, measured no faster in
// round 2).  The vertices follow three times, copy r as (v[r+1], v[r+2],
// v[r]) (mod 3), for rayTriRot (one (x, y, z) copy with per-component
// gathers: k_lidar 0.730 -> 0.744 ms, round 3).
constexpr int kOctNodeQ = 4;

__device__ __forceinline__ LBVH stageBVHOct(char *smem, const SceneDev &sc)
{
    const int node_q = sc.numLidarNodes * kOctNodeQ * 8;
    const uint4 *src_n = reinterpret_cast<const uint4 *>(sc.octNodes);
    uint4 *dst_n = reinterpret_cast<uint4 *>(smem);
    for (int k = threadIdx.x; k < sc.numLidarNodes * 4 * 8; k += blockDim.x)
        dst_n[(k >> 2) * kOctNodeQ + (k & 3)] = src_n[k];
    const float *src_v = sc.lidarVerts;
    float4 *dst_v = reinterpret_cast<float4 *>(smem + (size_t)node_q * 16);
    for (int k = threadIdx.x; k < sc.numLidarVerts * 3; k += blockDim.x) {
        const int r = k / sc.numLidarVerts, v = k - r * sc.numLidarVerts;
        const int r1 = r == 2 ? 0 : r + 1, r2 = r1 == 2 ? 0 : r1 + 1;
        dst_v[k] = make_float4(src_v[3 * v + r1], src_v[3 * v + r2], src_v[3 * v + r], 0.f);
    }
    __syncthreads();
    LBVH b;
    b.nodes = (const MP_LDS BVHNode *)(smem);
    b.verts = (const MP_LDS float *)(smem + (size_t)node_q * 16);
    b.pre = nullptr;
    b.snodes = nullptr;
    b.stats = nullptr;
    b.rotStride = sc.numLidarVerts;
    return b;
}

// sign bits: -0 counts as negative, as in the slab test's copysign'd inverse
__device__ __forceinline__ int rayOctant(mp::Vec3 d)
{
    return (int)((__float_as_uint(d.x) >> 31) | ((__float_as_uint(d.y) >> 31) << 1) |
                 ((__float_as_uint(d.z) >> 31) << 2));
}

typedef float lf4 __attribute__((ext_vector_type(4)));
typedef uint32_t lu4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void loadTri(const LBVH &b, int tri, mp::Vec3 &a, mp::Vec3 &bb, mp::Vec3 &c)
{
    const MP_LDS lf4 *p = reinterpret_cast<const MP_LDS lf4 *>(b.verts) + tri * 3;
    const lf4 x = p[0], y = p[1], z = p[2];
    a = mp::v3(x.x, x.y, x.z);
    bb = mp::v3(y.x, y.y, y.z);
    c = mp::v3(z.x, z.y, z.z);
}

// A node decoded from four ds_read_b128 (mesh_bvh.hpp:61-86 byte layout:
// min xyz | exp xyz, internal | triSize[4] | qMin x,y,z [4] | qMax x,y,z [4]
// | children[4] | parent).  Quantised bounds stay packed 4 per register;
// qb() converts byte i exactly (v_cvt_f32_ubyteN).
struct NodeR {
    float minX, minY, minZ;
    int expX, expY, expZ;
    uint32_t triSize, qMinX, qMinY, qMinZ, qMaxX, qMaxY, qMaxZ;
    int32_t child[4];
};

__device__ __forceinline__ float qb(uint32_t w, int i) { return (float)((w >> (8 * i)) & 0xffu); }

template <int kNodeQ = 4>
__device__ __forceinline__ NodeR loadNode(const LBVH &b, uint32_t idx)
{
    const MP_LDS lu4 *p = reinterpret_cast<const MP_LDS lu4 *>(b.nodes) + idx * kNodeQ;
    const lu4 q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3];
    NodeR n;
    n.minX = __uint_as_float(q0.x);
    n.minY = __uint_as_float(q0.y);
    n.minZ = __uint_as_float(q0.z);
    n.expX = (int)(int8_t)(q0.w & 0xffu);
    n.expY = (int)(int8_t)((q0.w >> 8) & 0xffu);
    n.expZ = (int)(int8_t)((q0.w >> 16) & 0xffu);
    n.triSize = q1.x;
    n.qMinX = q1.y; n.qMinY = q1.z; n.qMinZ = q1.w;
    n.qMaxX = q2.x; n.qMaxY = q2.y; n.qMaxZ = q2.z;
    n.child[0] = (int32_t)q2.w;
    n.child[1] = (int32_t)q3.x;
    n.child[2] = (int32_t)q3.y;
    n.child[3] = (int32_t)q3.z;
    return n;
}

struct RayTxfmD {
    int kx, ky, kz;
    float Sx, Sy, Sz;
};

// mesh_bvh.inl:584-620 (shear constants only; see oracle)
__device__ __forceinline__ RayTxfmD rayTxfm(mp::Vec3 d, mp::Vec3 inv_d)
{
    float abs_x = mp::fabs_(d.x), abs_y = mp::fabs_(d.y), abs_z = mp::fabs_(d.z);
    int kz;
    if (abs_x > abs_y && abs_x > abs_z) kz = 0;
    else if (abs_y > abs_z) kz = 1;
    else kz = 2;
    int kx = kz + 1; if (kx == 3) kx = 0;
    int ky = kx + 1; if (ky == 3) ky = 0;
    if (mp::comp(d, kz) < 0.f) { int t = kx; kx = ky; ky = t; }
    RayTxfmD t;
    t.kx = kx; t.ky = ky; t.kz = kz;
    t.Sx = mp::comp(d, kx) * mp::comp(inv_d, kz);
    t.Sy = mp::comp(d, ky) * mp::comp(inv_d, kz);
    t.Sz = mp::comp(inv_d, kz);
    return t;
}

// mesh_bvh.inl:433-554, backface culling
__device__ __forceinline__ bool rayTri(mp::Vec3 ta, mp::Vec3 tb, mp::Vec3 tc, const RayTxfmD &tx, mp::Vec3 org,
                                       float t_max, float &out_t)
{
    using namespace mp;
    const Vec3 A = ta - org, B = tb - org, C = tc - org;
    const float Az_ = comp(A, tx.kz), Bz_ = comp(B, tx.kz), Cz_ = comp(C, tx.kz);
    const float Ax = fma_(-tx.Sx, Az_, comp(A, tx.kx));
    const float Ay = fma_(-tx.Sy, Az_, comp(A, tx.ky));
    const float Bx = fma_(-tx.Sx, Bz_, comp(B, tx.kx));
    const float By = fma_(-tx.Sy, Bz_, comp(B, tx.ky));
    const float Cx = fma_(-tx.Sx, Cz_, comp(C, tx.kx));
    const float Cy = fma_(-tx.Sy, Cz_, comp(C, tx.ky));
    float U = fma_(Cx, By, -(Cy * Bx));
    float V = fma_(Ax, Cy, -(Ay * Cx));
    float W = fma_(Bx, Ay, -(By * Ax));
    if (U < 0.0f || V < 0.0f || W < 0.0f) return false;
    if (U == 0.0f || V == 0.0f || W == 0.0f) {
        double CxBy = (double)Cx * (double)By;
        double CyBx = (double)Cy * (double)Bx;
        U = (float)(CxBy - CyBx);
        double AxCy = (double)Ax * (double)Cy;
        double AyCx = (double)Ay * (double)Cx;
        V = (float)(AxCy - AyCx);
        double BxAy = (double)Bx * (double)Ay;
        double ByAx = (double)By * (double)Ax;
        W = (float)(BxAy - ByAx);
        if (U < 0.0f || V < 0.0f || W < 0.0f) return false;
    }
    float det = U + V + W;
    if (det == 0.f) return false;
    const float Az = tx.Sz * Az_;
    const float Bz = tx.Sz * Bz_;
    const float Cz = tx.Sz * Cz_;
    const float T = fma_(U, Az, fma_(V, Bz, W * Cz));
    if (T < 0.0f || T > t_max * det) return false;
    const float rcpDet = 1.0f / det;
    out_t = T * rcpDet;
    return true;
}

// rayTri over a rotated vertex copy: the LDS image holds every vertex three
// times, copy kz as (v[kz+1], v[kz+2], v[kz]) (indices mod 3), so the ray's
// copy yields each vertex already in (kx0, ky0, kz) order with kx0 = kz + 1,
// ky0 = kz + 2 -- the shear frame before rayTxfm's swap -- and `sw` (the
// swap: d[kz] < 0) exchanges the first two components.  o0 / o1 / oz are
// the origin's components in the same order.  comp(ta - org, k) ==
// ta[k] - org[k], so every value equals rayTri's bit for bit; per triangle
// 6 selects replace the 18 of the per-component comp() gathers.
__device__ __forceinline__ bool rayTriRot(const MP_LDS lf4 *p, float o0, float o1, float oz, bool sw,
                                          const RayTxfmD &tx, float t_max, float &out_t)
{
    using namespace mp;
    const lf4 a = p[0], b = p[1], c = p[2];
    const float a0 = a.x - o0, a1 = a.y - o1, Az_ = a.z - oz;
    const float b0 = b.x - o0, b1 = b.y - o1, Bz_ = b.z - oz;
    const float c0 = c.x - o0, c1 = c.y - o1, Cz_ = c.z - oz;
    const float Akx = sw ? a1 : a0, Aky = sw ? a0 : a1;
    const float Bkx = sw ? b1 : b0, Bky = sw ? b0 : b1;
    const float Ckx = sw ? c1 : c0, Cky = sw ? c0 : c1;
    const float Ax = fma_(-tx.Sx, Az_, Akx);
    const float Ay = fma_(-tx.Sy, Az_, Aky);
    const float Bx = fma_(-tx.Sx, Bz_, Bkx);
    const float By = fma_(-tx.Sy, Bz_, Bky);
    const float Cx = fma_(-tx.Sx, Cz_, Ckx);
    const float Cy = fma_(-tx.Sy, Cz_, Cky);
    float U = fma_(Cx, By, -(Cy * Bx));
    float V = fma_(Ax, Cy, -(Ay * Cx));
    float W = fma_(Bx, Ay, -(By * Ax));
    if (U < 0.0f || V < 0.0f || W < 0.0f) return false;
    if (U == 0.0f || V == 0.0f || W == 0.0f) {
        double CxBy = (double)Cx * (double)By;
        double CyBx = (double)Cy * (double)Bx;
        U = (float)(CxBy - CyBx);
        double AxCy = (double)Ax * (double)Cy;
        double AyCx = (double)Ay * (double)Cx;
        V = (float)(AxCy - AyCx);
        double BxAy = (double)Bx * (double)Ay;
        double ByAx = (double)By * (double)Ax;
        W = (float)(BxAy - ByAx);
        if (U < 0.0f || V < 0.0f || W < 0.0f) return false;
    }
    float det = U + V + W;
    if (det == 0.f) return false;
    const float Az = tx.Sz * Az_;
    const float Bz = tx.Sz * Bz_;
    const float Cz = tx.Sz * Cz_;
    const float T = fma_(U, Az, fma_(V, Bz, W * Cz));
    if (T < 0.0f || T > t_max * det) return false;
    const float rcpDet = 1.0f / det;
    out_t = T * rcpDet;
    return true;
}

// MeshBVH::traceRay (mesh_bvh.inl:110-208) over the LDS-resident BVH.
// Returns hit flag; *t_out = closest hit t when hit.
// t_max0 < FLT_MAX: only hits up to about t_max0 are sought (boxes entered
// beyond it are pruned from the start); see visibleRayD for when that gives
// the reference's answer.
// kExit: stop as soon as a hit at t <= exit_at is found (t_out is then
// that hit, not necessarily the closest; callers that only compare the
// closest hit with exit_at get the same answer).
template <bool kExit, int kNodeQ = 4, bool kRot = false, bool kOctImage = false>
__device__ __forceinline__ bool bvhTraceRayT(const LBVH &b, mp::Vec3 ray_o, mp::Vec3 ray_d, float &t_out,
                                             float t_max0, float exit_at, int *exit_tri = nullptr)
{
    using namespace mp;
    const float diveps = 0.0000001f;
    Vec3 inv_d = v3(1.f / ray_d.x, 1.f / ray_d.y, 1.f / ray_d.z);
    RayTxfmD tx = rayTxfm(ray_d, inv_d);
    // Loop-invariant in the reference (recomputed per node there; same bits).
    const float rayXInv = copysign_(ray_d.x == 0 ? 1 / diveps : 1 / ray_d.x, ray_d.x);
    const float rayYInv = copysign_(ray_d.y == 0 ? 1 / diveps : 1 / ray_d.y, ray_d.y);
    const float rayZInv = copysign_(ray_d.z == 0 ? 1 / diveps : 1 / ray_d.z, ray_d.z);

    // Slab selection by ray direction sign: fma(q, dq, oq) is monotonic in q
    // and dq != 0, so per axis min(t(qMin), t(qMax)) is t(qMin) when dq > 0
    // and t(qMax) otherwise -- the reference's six fminf/fmaxf give the same
    // values (mesh_bvh.inl:165-183).
    const bool negX = rayXInv < 0.f, negY = rayYInv < 0.f, negZ = rayZInv < 0.f;

    // kRot: the ray's rotated vertex copy and the origin in its order
    const MP_LDS lf4 *vrot = nullptr;
    float ro0 = 0.f, ro1 = 0.f, roz = 0.f;
    bool rsw = false;
    if constexpr (kRot) {
        const int kx0 = tx.kz == 2 ? 0 : tx.kz + 1, ky0 = kx0 == 2 ? 0 : kx0 + 1;
        vrot = reinterpret_cast<const MP_LDS lf4 *>(b.verts) + tx.kz * b.rotStride;
        ro0 = comp(ray_o, kx0);
        ro1 = comp(ray_o, ky0);
        roz = comp(ray_o, tx.kz);
        rsw = tx.kx != kx0;
    }

    float t_max = t_max0;
    bool ray_hit = false;
    ByteStack st;
    st.lo = 0; st.hi = 0; st.n = 0;
    bsPush(st, 0);
    while (st.n > 0) {
        const uint32_t node_idx = bsPop(st);
        const NodeR node = loadNode<kNodeQ>(b, node_idx);
        const float dirQuantX = expScaleD(node.expX) * rayXInv;
        const float dirQuantY = expScaleD(node.expY) * rayYInv;
        const float dirQuantZ = expScaleD(node.expZ) * rayZInv;
        const float originQuantX = (node.minX - ray_o.x) * rayXInv;
        const float originQuantY = (node.minY - ray_o.y) * rayYInv;
        const float originQuantZ = (node.minZ - ray_o.z) * rayZInv;
        // kOctImage: the ray's octant image (rayOctant) holds the near slab
        // in qMin and the far one in qMax already (octantNodeImages)
        const uint32_t nearX = (!kOctImage && negX) ? node.qMaxX : node.qMinX;
        const uint32_t farX = (!kOctImage && negX) ? node.qMinX : node.qMaxX;
        const uint32_t nearY = (!kOctImage && negY) ? node.qMaxY : node.qMinY;
        const uint32_t farY = (!kOctImage && negY) ? node.qMinY : node.qMaxY;
        const uint32_t nearZ = (!kOctImage && negZ) ? node.qMaxZ : node.qMinZ;
        const uint32_t farZ = (!kOctImage && negZ) ? node.qMinZ : node.qMaxZ;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int32_t child = node.child[i];
            if (child == -1) continue;
            // fused like the reference's NVRTC build (--fmad=true)
            const float t_near_x = fma_(qb(nearX, i), dirQuantX, originQuantX);
            const float t_near_y = fma_(qb(nearY, i), dirQuantY, originQuantY);
            const float t_near_z = fma_(qb(nearZ, i), dirQuantZ, originQuantZ);
            const float t_far_x = fma_(qb(farX, i), dirQuantX, originQuantX);
            const float t_far_y = fma_(qb(farY, i), dirQuantY, originQuantY);
            const float t_far_z = fma_(qb(farZ, i), dirQuantZ, originQuantZ);
            const float t_near = fmax_(fmax_(t_near_x, t_near_y), fmax_(t_near_z, 0.f));
            // fmin_ of the four (no operand is NaN; a -0 / +0 choice only
            // meets the `<=` below) without the per-use canonicalisation the
            // compiler inserts for the loop-carried t_max (k_lidar 0.6944 ->
            // 0.6847 ms, round 3)
            float t_far;
            asm("v_min3_f32 %0, %1, %2, %3\n\tv_min_f32 %0, %0, %4"
                : "=&v"(t_far) : "v"(t_far_x), "v"(t_far_y), "v"(t_far_z), "v"(t_max));
            if (t_near <= t_far) {
                if (child & 0x80000000) {
                    const int leaf = child & 0x7fffffff;
                    const int ntri = (int)((node.triSize >> (8 * i)) & 0xffu);
                    bool hit_tri = false;
                    float hit_t = 0.f;
                    float leaf_tmax = t_max;
                    int hit_k = 0;
                    // Leaves hold at most 2 triangles (scene.cpp Builder):
                    // the unrolled pair runs without a loop counter
                    // (k_lidar -3%, k_vis -3%, identical outputs).
#pragma unroll
                    for (int k = 0; k < 2; k++) {
                        if (k >= ntri) break;
                        bool h;
                        if constexpr (kRot) {
                            h = rayTriRot(vrot + (leaf + k) * 3, ro0, ro1, roz, rsw, tx, leaf_tmax, hit_t);
                        } else {
                            Vec3 a, bb, c;
                            loadTri(b, leaf + k, a, bb, c);
                            h = rayTri(a, bb, c, tx, ray_o, leaf_tmax, hit_t);
                        }
                        if (h) {
                            hit_tri = true;
                            leaf_tmax = hit_t;
                            if constexpr (kExit) hit_k = k;
                        }
                    }
                    if (hit_tri) {
                        ray_hit = true;
                        t_max = hit_t;
                        if constexpr (kExit) {
                            if (hit_t <= exit_at) {
                                t_out = hit_t;
                                if (exit_tri) *exit_tri = leaf + hit_k;
                                return true;
                            }
                        }
                    }
                } else {
                    bsPush(st, (uint32_t)child);
                }
            }
        }
    }
    t_out = t_max;
    return ray_hit;
}

__device__ __forceinline__ bool bvhTraceRayD(const LBVH &b, mp::Vec3 ray_o, mp::Vec3 ray_d, float &t_out,
                                             float t_max0 = mp::kFltMax)
{
    return bvhTraceRayT<false>(b, ray_o, ray_d, t_out, t_max0, 0.f);
}

// Orders one wave's LDS writes before other lanes' reads of them (and those
// reads before the next overwrite): a wavefront-scope release/acquire fence
// pair around a wave barrier.  The wave's DS instructions execute in issue
// order, so this constrains the compiler only.
__device__ __forceinline__ void waveSync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Out-of-line traversal for the ray-query test hook.
struct RayHitD {
    float t;
    int hit;
};
__device__ __noinline__ RayHitD bvhTraceRayExactD(const LBVH b, mp::Vec3 ray_o, mp::Vec3 ray_d)
{
    RayHitD r;
    r.hit = bvhTraceRayD(b, ray_o, ray_d, r.t) ? 1 : 0;
    return r;
}

// mesh_bvh.inl:817-855
__device__ __forceinline__ bool sphereNodeCheckD(mp::Vec3 o, mp::Vec3 inv_d, float t_max, float r, mp::AABB aabb)
{
    using namespace mp;
    AABB e = aabb;
    e.pMin.x -= r; e.pMin.y -= r; e.pMin.z -= r;
    e.pMax.x += r; e.pMax.y += r; e.pMax.z += r;
    float t_min = 0.f;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        float inv_d_i = comp(inv_d, i);
        float b_min, b_max;
        if (!__builtin_signbit(inv_d_i)) {
            b_min = comp(e.pMin, i); b_max = comp(e.pMax, i);
        } else {
            b_min = comp(e.pMax, i); b_max = comp(e.pMin, i);
        }
        float i_min = (b_min - comp(o, i)) * inv_d_i;
        float i_max = (b_max - comp(o, i)) * inv_d_i;
        t_min = i_min > t_min ? i_min : t_min;
        t_max = i_max < t_max ? i_max : t_max;
    }
    return t_min < t_max;
}

// mesh_bvh.inl:885-1127 (same quirks as the oracle restatement).  The
// reference marks this swept-sphere / triangle test as heavily based on Jolt
// Physics' (Copyright 2021 Jorrit Rouwe, MIT licence; mesh_bvh.inl:894-915
// carries the licence text); it is followed statement for statement here
// for bit parity, so that credit and licence apply to this function too.
// pre: unit normal, |normal|, squared edge lengths (SceneDev::triPre) --
// the ray-independent subexpressions, same bits as computing them here.
__device__ __forceinline__ float sphereTriD(mp::Vec3 ta, mp::Vec3 tb, mp::Vec3 tc, float4 pre0, float4 pre1,
                                            mp::Vec3 ray_o, mp::Vec3 ray_d, float t_max, float r, mp::Vec3 &out_n)
{
    using namespace mp;
    const Vec3 e01 = tb - ta, e02 = tc - ta, e12 = tc - tb;
    const Vec3 v0 = ta - ray_o, v1 = tb - ray_o, v2 = tc - ray_o;
    const float n_len = pre0.w;
    const Vec3 n = v3(pre0.x, pre0.y, pre0.z);
    const float n_dot_d = dot(n, ray_d);
    const float r2 = r * r;

    if (fabs_(dot(v0, n)) <= r) {
        Vec3 q = triangleClosestPointToOrigin(v0, v1, v2, e01, e02);
        float q_len2 = length2(q);
        if (q_len2 <= r2) {
            float q_len = sqrt_(q_len2);
            out_n = q_len > 0.0f ? q / q_len : kUp;
            return 0.f;
        }
    } else {
        float abs_n_dot_d = fabs_(n_dot_d);
        if (abs_n_dot_d > 1.0e-6f) {
            float sgn = copysign_(1.f, n_dot_d);
            Vec3 extruded_delta = sgn * r * n;
            Vec3 v0e = v0 - extruded_delta;
            float plane_t = dot(v0e, n) / n_dot_d;
            if (plane_t * abs_n_dot_d < -r || plane_t >= t_max) return t_max;
            if (plane_t >= 0.0f) {
                Vec3 e = cross(ray_d, v0e);
                float v = -dot(e02, e) * sgn;
                float w = dot(e01, e) * sgn;
                if (v >= 0.f && w >= 0.f && v + w <= n_len * abs_n_dot_d) {
                    out_n = -sgn * n;
                    return plane_t;
                }
            }
        }
    }

    const float edge_eps = 1e-6f;
    const float d_len2 = length2(ray_d);
    float hit_t = t_max;
    // testEdge x3
    {
        const Vec3 axes[3] = { e01, e02, e12 };
        const Vec3 bases[3] = { v0, v0, v1 };
        const float alen2[3] = { pre1.x, pre1.y, pre1.z };
#pragma unroll
        for (int k = 0; k < 3; k++) {
            Vec3 axis = axes[k];
            Vec3 start = -bases[k];
            const float s_dot_a = dot(start, axis);
            const float d_dot_a = dot(ray_d, axis);
            const float e_dot_a = s_dot_a + d_dot_a;
            if (s_dot_a < 0.0f && e_dot_a < 0.0f) continue;
            const float a_len2 = alen2[k];
            if (s_dot_a > a_len2 && e_dot_a > a_len2) continue;
            float a = a_len2 * d_len2 - d_dot_a * d_dot_a;
            if (fabs_(a) < edge_eps) continue;
            float bq = a_len2 * dot(start, ray_d) - d_dot_a * s_dot_a;
            float c = a_len2 * (length2(start) - r2) - s_dot_a * s_dot_a;
            float det = bq * bq - a * c;
            if (det < 0.0f) continue;
            float t = -(bq + sqrt_(det)) / a;
            if (t < 0.0f || t >= hit_t) continue;
            if (s_dot_a + t * d_dot_a < 0.0f || s_dot_a + t * d_dot_a > a_len2) continue;
            hit_t = t;
        }
    }
    // testVert x3 (mesh_bvh.inl:1073-1104 quirk: ray_o - relative vertex)
    {
        const Vec3 vs[3] = { v0, v1, v2 };
#pragma unroll
        for (int k = 0; k < 3; k++) {
            Vec3 m = ray_o - vs[k];
            float bq = dot(m, ray_d);
            float c = dot(m, m) - r2;
            if (c > 0.0f && bq > 0.0f) continue;
            float discr = bq * bq - c;
            if (discr < 0.0f) continue;
            float t = -bq - sqrt_(discr);
            if (t < 0.f) { hit_t = 0.f; continue; }
            if (t >= hit_t) continue;
            hit_t = t;
        }
    }
    if (hit_t >= t_max) return t_max;
    Vec3 hp = ray_d * hit_t;
    Vec3 ct = triangleClosestPointToOrigin(v0 - hp, v1 - hp, v2 - hp, e01, e02);
    out_n = normalize(ct);
    return hit_t;
}

struct SphereHit {
    float t;
    mp::Vec3 n; // valid only when t < FLT_MAX (the reference writes the normal only on a hit)
};

// MeshBVH::sphereCast (mesh_bvh.inl:743-815).  r must be kSphereR: the
// node image of stageBVHSphere carries slab ends widened by that radius.
// t_max0: MeshBVH::sphereCast's own t_max argument (mesh_bvh.inl:743-747):
// the search starts with hit_t = t_max0 and returns it when nothing is
// nearer.

// One node of the sphere-cast image (stageBVHSphere, kSNodeFloats = 32
// floats: loR x / y / z of the 4 children, hiR x / y / z, the children,
// their triangle counts) in one round of LDS loads: 8 x 16 B instead of ~7
// scalar loads per child, one child after another.  The casts then compute
// every child's slab entry (with 0) and exit without the running hit bound,
// and test t_lo < fminNum(hit_t, t_exit) in child order: the same fminNum
// over the same four values as the reference's running update (a NaN slab
// is ignored either way; a -0 / +0 choice cannot change the < test).
__device__ __forceinline__ void sNodeLoad(const LBVH &b, uint32_t node_idx, lf4 &lx, lf4 &ly, lf4 &lz, lf4 &hx, lf4 &hy,
                                          lf4 &hz, lf4 &cq, lf4 &tq)
{
    const MP_LDS lf4 *q = reinterpret_cast<const MP_LDS lf4 *>(b.snodes + node_idx * kSNodeFloats);
    lx = q[0]; ly = q[1]; lz = q[2]; hx = q[3]; hy = q[4]; hz = q[5]; cq = q[6]; tq = q[7];
}

__device__ __forceinline__ SphereHit bvhSphereCastD(const LBVH b, mp::Vec3 ray_o, mp::Vec3 ray_d, float r,
                                                 float t_max0 = mp::kFltMax)
{
    using namespace mp;
    Vec3 inv_d = v3(1.f / ray_d.x, 1.f / ray_d.y, 1.f / ray_d.z);
    Vec3 closest = v3(0.f, 0.f, 0.f);
    float hit_t = t_max0;
    // sphereCastNodeCheck (mesh_bvh.inl:817-855) with the slab ends chosen
    // once per cast from the sign of inv_d: per axis b_min is the child's
    // (min - r) or (max + r) end, exactly as the per-child selects pick it;
    // the running t_min / t_max updates `i > t ? i : t` are maxNum / minNum
    // (a NaN slab from 0 * inf leaves them unchanged either way, and a -0 / +0
    // tie does not change the final t_min < t_max).
    const bool negX = __builtin_signbit(inv_d.x), negY = __builtin_signbit(inv_d.y),
               negZ = __builtin_signbit(inv_d.z);
    // near / far ends per axis: loR or hiR of the pre-widened node image
    // (stageBVHSphere), picked once per cast from the sign of inv_d
    ByteStack st;
    st.lo = 0; st.hi = 0; st.n = 0;
    bsPush(st, 0);
    while (st.n > 0) {
        const uint32_t node_idx = bsPop(st);
        lf4 lx, ly, lz, hx, hy, hz, cq, tq;
        sNodeLoad(b, node_idx, lx, ly, lz, hx, hy, hz, cq, tq);
        float t_lo4[4], t_ex4[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const float nxv = negX ? hx[i] : lx[i], fxv = negX ? lx[i] : hx[i];
            const float nyv = negY ? hy[i] : ly[i], fyv = negY ? ly[i] : hy[i];
            const float nzv = negZ ? hz[i] : lz[i], fzv = negZ ? lz[i] : hz[i];
            const float i_min_x = (nxv - ray_o.x) * inv_d.x, i_max_x = (fxv - ray_o.x) * inv_d.x;
            const float i_min_y = (nyv - ray_o.y) * inv_d.y, i_max_y = (fyv - ray_o.y) * inv_d.y;
            const float i_min_z = (nzv - ray_o.z) * inv_d.z, i_max_z = (fzv - ray_o.z) * inv_d.z;
            t_lo4[i] = fmax_(fmax_(fmax_(0.f, i_min_x), i_min_y), i_min_z);
            t_ex4[i] = fmin_(fmin_(i_max_x, i_max_y), i_max_z);
        }
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int32_t child = __float_as_int(cq[i]);
            if (child == -1) continue;
            if (t_lo4[i] < fmin_(hit_t, t_ex4[i])) {
                if (child & 0x80000000) {
                    const int leaf = child & 0x7fffffff;
                    const int ntri = (int)__float_as_uint(tq[i]);
                    Vec3 leaf_n = v3(0.f, 0.f, 0.f);
                    float leaf_t = hit_t;
                    for (int k = 0; k < ntri; k++) {
                        Vec3 a, bb, c;
                        loadTri(b, leaf + k, a, bb, c);
                        const MP_LDS lf4 *pp = reinterpret_cast<const MP_LDS lf4 *>(b.pre) + 2 * (leaf + k);
                        const lf4 p0 = pp[0], p1 = pp[1];
                        leaf_t = sphereTriD(a, bb, c, make_float4(p0.x, p0.y, p0.z, p0.w),
                                            make_float4(p1.x, p1.y, p1.z, p1.w), ray_o, ray_d, leaf_t, r, leaf_n);
                    }
                    if (leaf_t < hit_t) {
                        hit_t = leaf_t;
                        closest = leaf_n;
                    }
                } else {
                    bsPush(st, (uint32_t)child);
                }
            }
        }
    }
    if (b.stats) statAdd(b.stats + kStatSphereCasts, 1u);
    SphereHit h;
    h.t = hit_t;
    h.n = closest;
    return h;
}

// Two sphere casts along the same direction from origins that differ in z
// only (applyVelocity's low and high forward casts), in one traversal.  Each
// cast keeps its own hit_t, and each stack entry carries which casts entered
// that node, so a cast tests exactly the children of the nodes it entered,
// in the same depth-first order as bvhSphereCastD (fixed child order; a node
// only the other cast entered changes nothing for it) -- every result is
// bit-identical to two bvhSphereCastD calls.  The x / y slab values are
// shared (same origin xy and direction); z and the running bounds are per
// cast.  act1 = false: cast 1 is not run (h1 untouched).  Inlined into its
// one caller: 164 VGPRs and no scratch, against 168 + 48 B of spills as a
// call (k_move -1.3%, `profiles/r04ap_lab_cast2_inline.jsonl`).
__device__ __forceinline__ void bvhSphereCast2D(const LBVH b, mp::Vec3 o0, float z1, mp::Vec3 ray_d, float r,
                                             float t_max0, bool act1, SphereHit &h0, SphereHit &h1)
{
    using namespace mp;
    Vec3 inv_d = v3(1.f / ray_d.x, 1.f / ray_d.y, 1.f / ray_d.z);
    Vec3 closest0 = v3(0.f, 0.f, 0.f), closest1 = v3(0.f, 0.f, 0.f);
    float hit0 = t_max0, hit1 = t_max0;
    const bool negX = __builtin_signbit(inv_d.x), negY = __builtin_signbit(inv_d.y),
               negZ = __builtin_signbit(inv_d.z);
    const Vec3 o1 = v3(o0.x, o0.y, z1);
    ByteStack st;
    st.lo = 0; st.hi = 0; st.n = 0;
    uint32_t ms = 0; // 2 bits per stack entry: the casts that entered the node
    bsPush(st, 0);
    ms = act1 ? 3u : 1u;
    while (st.n > 0) {
        const uint32_t node_idx = bsPop(st);
        const uint32_t m = ms & 3u;
        ms >>= 2;
        lf4 lx, ly, lz, hx, hy, hz, cq, tq;
        sNodeLoad(b, node_idx, lx, ly, lz, hx, hy, hz, cq, tq);
        float lo0[4], lo1[4], ex0[4], ex1[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const float nxv = negX ? hx[i] : lx[i], fxv = negX ? lx[i] : hx[i];
            const float nyv = negY ? hy[i] : ly[i], fyv = negY ? ly[i] : hy[i];
            const float zn = negZ ? hz[i] : lz[i], zf = negZ ? lz[i] : hz[i];
            const float i_min_x = (nxv - o0.x) * inv_d.x, i_max_x = (fxv - o0.x) * inv_d.x;
            const float i_min_y = (nyv - o0.y) * inv_d.y, i_max_y = (fyv - o0.y) * inv_d.y;
            const float i_min_z0 = (zn - o0.z) * inv_d.z, i_max_z0 = (zf - o0.z) * inv_d.z;
            const float i_min_z1 = (zn - z1) * inv_d.z, i_max_z1 = (zf - z1) * inv_d.z;
            const float lo_xy = fmax_(fmax_(0.f, i_min_x), i_min_y);
            const float ex_xy = fmin_(i_max_x, i_max_y);
            lo0[i] = fmax_(lo_xy, i_min_z0);
            lo1[i] = fmax_(lo_xy, i_min_z1);
            ex0[i] = fmin_(ex_xy, i_max_z0);
            ex1[i] = fmin_(ex_xy, i_max_z1);
        }
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int32_t child = __float_as_int(cq[i]);
            if (child == -1) continue;
            const uint32_t pass = ((m & 1u) && lo0[i] < fmin_(hit0, ex0[i]) ? 1u : 0u) |
                                  ((m & 2u) && lo1[i] < fmin_(hit1, ex1[i]) ? 2u : 0u);
            if (pass == 0u) continue;
            if (child & 0x80000000) {
                const int leaf = child & 0x7fffffff;
                const int ntri = (int)__float_as_uint(tq[i]);
                Vec3 n0 = v3(0.f, 0.f, 0.f), n1 = v3(0.f, 0.f, 0.f);
                float t0 = hit0, t1 = hit1;
                for (int k = 0; k < ntri; k++) {
                    Vec3 a, bb, c;
                    loadTri(b, leaf + k, a, bb, c);
                    const MP_LDS lf4 *pp = reinterpret_cast<const MP_LDS lf4 *>(b.pre) + 2 * (leaf + k);
                    const lf4 p0 = pp[0], p1 = pp[1];
                    const float4 q0 = make_float4(p0.x, p0.y, p0.z, p0.w), q1 = make_float4(p1.x, p1.y, p1.z, p1.w);
                    if (pass & 1u) t0 = sphereTriD(a, bb, c, q0, q1, o0, ray_d, t0, r, n0);
                    if (pass & 2u) t1 = sphereTriD(a, bb, c, q0, q1, o1, ray_d, t1, r, n1);
                }
                if ((pass & 1u) && t0 < hit0) {
                    hit0 = t0;
                    closest0 = n0;
                }
                if ((pass & 2u) && t1 < hit1) {
                    hit1 = t1;
                    closest1 = n1;
                }
            } else {
                bsPush(st, (uint32_t)child);
                ms = (ms << 2) | pass;
            }
        }
    }
    if (b.stats) statAdd(b.stats + kStatSphereCasts, act1 ? 2u : 1u);
    h0.t = hit0;
    h0.n = closest0;
    if (act1) {
        h1.t = hit1;
        h1.n = closest1;
    }
}

constexpr float kCapsuleRadius = 15.f;         // consts::agentRadius
constexpr float kCapsuleSegment = 65.f - 30.f; // standHeight - 2 * agentRadius

struct WorldHit {
    bool hit;
    float t;
    int entity; // agent index within the world, -1 none
};

// traceRayAgainstWorld (utils.cpp:10-72): BVH then the world's N capsules.
// Capsule bases are read from the SoA position columns (cached).
// `self`: the casting agent's index in the world when the ray starts on its
// own capsule's axis (org.xy == its position's xy, so tr.xy is exactly 0,
// and org.z - base.z - r in [0, segment] up to rounding: the lidar and shot
// origins sit r, viewHeight - r... above the feet, 0-35 units up the axis).
// intersectRayZOriginCapsule returns 0 for an origin inside the capsule, so
// that capsule can never be the hit and its test is skipped; -1: test all.
__device__ __forceinline__ WorldHit capsulesD(const float *__restrict__ px, const float *__restrict__ py,
                                              const float *__restrict__ pz, int64_t g0, int N, mp::Vec3 org,
                                              mp::Vec3 d, int self, bool hit, float min_t, uint32_t capMask = ~0u);

__device__ __forceinline__ WorldHit traceWorldD(const LBVH &b, const float *__restrict__ px,
                                                const float *__restrict__ py, const float *__restrict__ pz,
                                                int64_t g0, int N, mp::Vec3 org, mp::Vec3 d, int self = -1,
                                                uint32_t capMask = ~0u)
{
    using namespace mp;
    float min_t = kFltMax;
    float tb;
    const bool hit = bvhTraceRayT<false>(b, org, d, tb, mp::kFltMax, 0.f);
    if (hit) min_t = tb;
    return capsulesD(px, py, pz, g0, N, org, d, self, hit, min_t, capMask);
}

// traceRayAgainstWorld's capsule loop (utils.cpp:40-69) after the BVH hit
// (hit, min_t).
__device__ __forceinline__ WorldHit capsulesD(const float *__restrict__ px, const float *__restrict__ py,
                                              const float *__restrict__ pz, int64_t g0, int N, mp::Vec3 org,
                                              mp::Vec3 d, int self, bool hit, float min_t, uint32_t capMask)
{
    using namespace mp;
    int ent = -1;
    // capMask (wave-uniform): capsules a caller has proven unreachable for
    // every ray of the wave are skipped (k_lidar's forward fans); the rest
    // are visited in the same ascending order, so ties resolve as before.
    if (capMask != ~0u) {
        for (uint32_t m = capMask & ((1u << N) - 1u); m; m &= m - 1u) {
            const int j = __builtin_ctz(m);
            if (j == self) continue;
            Vec3 co = v3(px[g0 + j], py[g0 + j], pz[g0 + j]);
            co.z += kCapsuleRadius;
            Vec3 tr = org - co;
            const float dxy2 = d.x * d.x + d.y * d.y;
            const float cull_r2 = (kCapsuleRadius * 1.01f) * (kCapsuleRadius * 1.01f);
            const float cr = tr.x * d.y - tr.y * d.x;
            if (cr * cr > cull_r2 * dxy2) continue;
            const float along = -(tr.x * d.x + tr.y * d.y + tr.z * d.z);
            const float ahead = along + fmaxD(0.f, kCapsuleSegment * d.z) + kCapsuleRadius * 1.01f;
            if (ahead < 0.f) continue;
            if (along + fminD(0.f, kCapsuleSegment * d.z) - kCapsuleRadius * 1.01f > min_t) continue;
            float t = intersectRayZOriginCapsule(tr, d, kCapsuleRadius, kCapsuleSegment);
            if (t != 0 && t < min_t) {
                min_t = t;
                hit = true;
                ent = j;
            }
        }
        WorldHit h;
        h.hit = hit;
        h.t = min_t;
        h.entity = ent;
        return h;
    }
    // Conservative cull: every point of a Z-capsule lies within r of its
    // vertical axis, so a ray whose xy line passes farther than r from the
    // axis cannot hit it and the exact test would return 0.  The 1% radius
    // margin dwarfs the rounding of the cross product for |org - axis| up to
    // ~60k units (world bounds are ~5.7k), so no hit is ever culled.
    const float dxy2 = d.x * d.x + d.y * d.y;
    const float cull_r2 = (kCapsuleRadius * 1.01f) * (kCapsuleRadius * 1.01f);
    for (int j = 0; j < N; j++) {
        if (j == self) continue;
        Vec3 co = v3(px[g0 + j], py[g0 + j], pz[g0 + j]);
        co.z += kCapsuleRadius;
        Vec3 tr = org - co;
        const float cr = tr.x * d.y - tr.y * d.x;
        if (cr * cr > cull_r2 * dxy2) continue;
        // Behind the origin: the capsule's farthest point along d is at
        // dot(axis base - org, d) + max(0, h d.z) + r (|d| = 1); if that is
        // negative no t > 0 exists.  Same 1% radius margin.
        const float along = -(tr.x * d.x + tr.y * d.y + tr.z * d.z);
        const float ahead = along + fmaxD(0.f, kCapsuleSegment * d.z) + kCapsuleRadius * 1.01f;
        if (ahead < 0.f) continue;
        // Beyond the nearest hit so far: every capsule point lies at least
        // dot(axis base - org, d) + min(0, h d.z) - r along d, so an entering
        // t can be no smaller (same 1% radius margin); the exact test could
        // not pass `t < min_t`.
        if (along + fminD(0.f, kCapsuleSegment * d.z) - kCapsuleRadius * 1.01f > min_t) continue;
        float t = intersectRayZOriginCapsule(tr, d, kCapsuleRadius, kCapsuleSegment);
        if (t != 0 && t < min_t) {
            min_t = t;
            hit = true;
            ent = j;
        }
    }
    WorldHit h;
    h.hit = hit;
    h.t = min_t;
    h.entity = ent;
    return h;
}


// traceRayAgainstWorld(org, d).entity == target (utils.cpp:10-72, as
// isAgentVisible uses it, utils.cpp:218) without the full closest-hit
// search: the answer only depends on hits nearer than the target capsule's
// t_c.  (1) t_c == 0 (missed / inside) -> the target can never be the
// entity.  (2) The BVH search starts with t_max = t_c * 1.001: every
// triangle with t <= 1.001 t_c is still found (its boxes are entered before
// that bound; slab rounding is ~1e-7 relative) so the nearest hit is exact
// whenever it can matter, and any other result is > t_c, which decides the
// capsule loop exactly as the true nearest hit (also > t_c) would.
// (3) The capsule loop then runs as in traceWorldD.
// occ (k_vis, may be null): the ray's occluder hint, a triangle index that
// ended this ray before (DevState::visOcc).  A triangle hit at t <= t_c
// decides "not visible" whatever else lies on the ray: the full search
// would also stop at some hit <= t_c (every triangle with t <= t_c is
// reachable under its 1.001 t_c bound, and a hit strictly nearer than the
// current t_max is always accepted), so testing the hint first returns the
// same answer; on a miss the full search runs and records its occluder.
// numTris bounds the hint (any stale or foreign value is merely a miss).
// visibleRayD's two parts.  visibleQuickD: the decisions that need no
// traversal -- true when the target capsule is missed (t_c == 0) or the
// occluder hint is hit at t <= t_c (both mean "not visible"); otherwise t_c
// is returned for visibleFullD, the BVH search and the capsule loop.  k_vis
// runs the first part on every candidate ray and the second on the
// unresolved ones only, compacted (the answer per ray is the same).
// capsule(j): the base of the world's agent j's capsule (its position).
template <class CapsuleFn>
__device__ __forceinline__ bool visibleQuickD(const LBVH &b, CapsuleFn capsule, mp::Vec3 org, mp::Vec3 d, int target,
                                              const uint16_t *occ, uint32_t numTris, float &t_c)
{
    using namespace mp;
    Vec3 ct = capsule(target);
    ct.z += kCapsuleRadius;
    t_c = intersectRayZOriginCapsule(org - ct, d, kCapsuleRadius, kCapsuleSegment);
    if (t_c == 0) return true;
    if (occ) {
        const uint32_t hint = *occ;
        if (hint < numTris) {
            const Vec3 inv_d = v3(1.f / d.x, 1.f / d.y, 1.f / d.z);
            const RayTxfmD tx = rayTxfm(d, inv_d);
            Vec3 a, bb, c;
            loadTri(b, (int)hint, a, bb, c);
            float th;
            if (rayTri(a, bb, c, tx, org, t_c * 1.001f, th) && th <= t_c) return true;
        }
    }
    return false;
}

template <class CapsuleFn>
__device__ __forceinline__ bool visibleFullD(const LBVH &b, CapsuleFn capsule, int N, mp::Vec3 org, mp::Vec3 d,
                                             int target, float t_c, uint16_t *occ = nullptr)
{
    using namespace mp;
    float min_t = kFltMax;
    float tb;
    int occ_tri = -1;
    // Any triangle hit at t <= t_c already decides the query: the closest
    // hit is then <= t_c, and the target only wins with t_c < closest
    // (utils.cpp:57-69 `t < min_hit_t`), so the search stops there.
    if (bvhTraceRayT<true>(b, org, d, tb, t_c * 1.001f, t_c, occ ? &occ_tri : nullptr)) {
        if (tb <= t_c) {
            if (occ) *occ = (uint16_t)occ_tri;
            return false;
        }
        min_t = tb;
    }
    int ent = -1;
    const float dxy2 = d.x * d.x + d.y * d.y;
    const float cull_r2 = (kCapsuleRadius * 1.01f) * (kCapsuleRadius * 1.01f);
    for (int j = 0; j < N; j++) {
        float t;
        if (j == target) {
            t = t_c;
        } else {
            Vec3 co = capsule(j);
            co.z += kCapsuleRadius;
            const Vec3 tr = org - co;
            // the conservative culls of traceWorldD (skip only exact misses)
            const float cr = tr.x * d.y - tr.y * d.x;
            if (cr * cr > cull_r2 * dxy2) continue;
            const float along = -(tr.x * d.x + tr.y * d.y + tr.z * d.z);
            const float ahead = along + fmaxD(0.f, kCapsuleSegment * d.z) + kCapsuleRadius * 1.01f;
            if (ahead < 0.f) continue;
            if (along + fminD(0.f, kCapsuleSegment * d.z) - kCapsuleRadius * 1.01f > min_t) continue;
            t = intersectRayZOriginCapsule(tr, d, kCapsuleRadius, kCapsuleSegment);
        }
        if (t != 0 && t < min_t) {
            min_t = t;
            ent = j;
        }
    }
    return ent == target;
}

__device__ __forceinline__ bool visibleRayD(const LBVH &b, const float *__restrict__ px,
                                            const float *__restrict__ py, const float *__restrict__ pz, int64_t g0,
                                            int N, mp::Vec3 org, mp::Vec3 d, int target,
                                            uint16_t *occ = nullptr, uint32_t numTris = 0)
{
    float t_c;
    auto capsule = [&](int j) { return mp::v3(px[g0 + j], py[g0 + j], pz[g0 + j]); };
    if (visibleQuickD(b, capsule, org, d, target, occ, numTris, t_c)) return false;
    return visibleFullD(b, capsule, N, org, d, target, t_c, occ);
}

} // namespace mpenv
