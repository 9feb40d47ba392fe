// kernels.hip — the world-batched Zone step as hand-written gfx950 kernels.
//
// The reference runs ~40 ECS systems per step, each a device-wide
// ParallelForNode with a grid barrier in between (sim.cpp:5342-5842;
// NVRTC megakernel).  Every dependency between those systems is *within a
// world* (SURVEY.md §8e), so here a workgroup owns a tile of worlds and the
// system chain becomes LDS/L1-local __syncthreads() barriers.  The step is
// four kernels:
//
//   k_sim    world tile, lane = agent: movement + sphere casts, fire, damage,
//            respawn, heal, zone, breadcrumbs, match info, goals, explore,
//            rewards, done, reset  (sim.cpp:5347-5841 up to resetSystem)
//   k_vis    lane = (agent, opponent): frustum + line-of-sight rays
//            (opponentsWriteVisibilitySystem, sim.cpp:2526-2560)
//   k_obs    lane = agent: opponent masks + all observation tensors
//            (sim.cpp:2562-3052)
//   k_lidar  lane = ray: 80 lidar rays per agent (sim.cpp:3324-3506)
//
// All traversals read an LDS-resident copy of the BVH (geom_dev.h).  Every
// arithmetic expression follows the reference (and the CPU oracle) term by
// term with -ffp-contract=off so that results are bit-identical.
#include <hip/hip_runtime.h>

#include "engine.h"
#include "geom_dev.h"

#pragma clang fp contract(off)

namespace mpenv {

using namespace mp;

// ----------------------------------------------------- consts.hpp:7-72
namespace c {
constexpr int kNumStepsPerZone = 600;
constexpr int kZonePointInterval = 20;
constexpr int kZoneWinPoints = 125;
constexpr int kPoseTransitionSpeed = 10;
constexpr float kAgentRadius = 15.f;
constexpr float kStandHeight = 65.f;
constexpr float kCrouchHeight = 47.f;
constexpr float kProneHeight = 30.f;
constexpr float kMaxRunVelocity = 400.f;
constexpr float kMaxWalkVelocity = 200.f;
constexpr float kMaxCrouchVelocity = 50.f;
constexpr float kMaxProneVelocity = 20.f;
constexpr float kDeaccelerateRate = 1000.f;
constexpr int kRespawnInvincibleSteps = 5;
constexpr int kOutOfCombatSteps = 150;
constexpr float kAutohealPerStep = 5.f;
constexpr int kEpisodeLen = 3000;
constexpr int kNumMoveAmountBuckets = 3;
constexpr int kNumMoveAngleBuckets = 8;
constexpr float kDeltaT = 0.05f;
constexpr int kDiscreteAimYawBuckets = 13;
constexpr int kDiscreteAimPitchBuckets = 7;
constexpr int kGridMax = 40;
// mgr.cpp:1383-1395 weapon stats
constexpr int kMagSize = 30;
constexpr int kReloadTime = 30;
constexpr float kDmgPerBullet = 10.f;
constexpr float kAccuracyScale = 0.005f;
constexpr int kNumWeaponTypes = 1;
} // namespace c

enum { kStand = 0, kCrouch = 1, kProne = 2 };
constexpr uint32_t kFlagNoRespawn = 1u << 3;
constexpr uint32_t kFlagSpawnInMiddle = 1u << 0;
constexpr uint32_t kFlagRandomizeHP = 1u << 1;
constexpr uint32_t kFlagHardcodedSpawns = 1u << 6;
constexpr uint32_t kFlagEnableCurriculum = 1u << 5;
constexpr uint32_t kFlagNavmeshSpawn = 1u << 2;
constexpr uint32_t kFlagSubZones = 1u << 11;

__device__ __forceinline__ float viewHeightD(int pose)
{
    float top = pose == kStand ? c::kStandHeight : (pose == kCrouch ? c::kCrouchHeight : c::kProneHeight);
    return top - c::kAgentRadius;
}

__device__ __forceinline__ int32_t f2iSatD(float f)
{
    if (!(f == f)) return 0;
    if (f >= 2147483520.f) return INT32_MAX;
    if (f <= -2147483648.f) return INT32_MIN;
    return (int32_t)f;
}

// ------------------------------------------------------ SoA accessors
__device__ __forceinline__ Vec3 ldPos(const DevState &S, int64_t g) { return v3(S.px[g], S.py[g], S.pz[g]); }
__device__ __forceinline__ void stPos(const DevState &S, int64_t g, Vec3 p) { S.px[g] = p.x; S.py[g] = p.y; S.pz[g] = p.z; }
__device__ __forceinline__ Vec3 ldVel(const DevState &S, int64_t g) { return v3(S.vx[g], S.vy[g], S.vz[g]); }
__device__ __forceinline__ void stVel(const DevState &S, int64_t g, Vec3 v) { S.vx[g] = v.x; S.vy[g] = v.y; S.vz[g] = v.z; }
__device__ __forceinline__ Quat ldRot(const DevState &S, int64_t g) { return quat(S.rw[g], S.rx[g], S.ry[g], S.rz[g]); }
__device__ __forceinline__ void stRot(const DevState &S, int64_t g, Quat q) { S.rw[g] = q.w; S.rx[g] = q.x; S.ry[g] = q.y; S.rz[g] = q.z; }
__device__ __forceinline__ Quat ldAimRot(const DevState &S, int64_t g) { return quat(S.aw[g], S.ax[g], S.ay[g], S.az[g]); }
__device__ __forceinline__ void stAimRot(const DevState &S, int64_t g, Quat q) { S.aw[g] = q.w; S.ax[g] = q.x; S.ay[g] = q.y; S.az[g] = q.z; }
__device__ __forceinline__ RNG ldRng(const DevState &S, int64_t g)
{
    RNG r; r.key.a = (uint32_t)S.rngA[g]; r.key.b = (uint32_t)S.rngB[g]; r.ctr = (uint32_t)S.rngCtr[g];
    return r;
}
__device__ __forceinline__ void stRng(const DevState &S, int64_t g, const RNG &r)
{
    S.rngA[g] = (int32_t)r.key.a; S.rngB[g] = (int32_t)r.key.b; S.rngCtr[g] = (int32_t)r.ctr;
}
__device__ __forceinline__ RNG ldWRng(const DevState &S, int w)
{
    RNG r; r.key.a = (uint32_t)S.wRngA[w]; r.key.b = (uint32_t)S.wRngB[w]; r.ctr = (uint32_t)S.wRngCtr[w];
    return r;
}
__device__ __forceinline__ void stWRng(const DevState &S, int w, const RNG &r)
{
    S.wRngA[w] = (int32_t)r.key.a; S.wRngB[w] = (int32_t)r.key.b; S.wRngCtr[w] = (int32_t)r.ctr;
}
__device__ __forceinline__ void setFlag(const DevState &S, int64_t g, int32_t bit, bool v)
{
    int32_t f = S.flags[g];
    S.flags[g] = v ? (f | bit) : (f & ~bit);
}

struct AimD {
    float yaw, pitch;
    Quat rot;
};

// utils.cpp:140-167 computeAim
__device__ __forceinline__ AimD computeAimD(float yaw, float pitch)
{
    if (yaw < -kPi) yaw += 2.f * kPi;
    else if (yaw > kPi) yaw -= 2.f * kPi;
    if (pitch < -0.25f * kPi) pitch = -0.25f * kPi;
    if (pitch > 0.25f * kPi) pitch = 0.25f * kPi;
    Quat r = angleAxis(yaw, kUp) * angleAxis(pitch, kRight);
    r = qnormalize(r);
    AimD a;
    a.yaw = yaw; a.pitch = pitch; a.rot = r;
    return a;
}

__device__ __forceinline__ void stAim(const DevState &S, int64_t g, const AimD &a)
{
    S.ayaw[g] = a.yaw; S.apitch[g] = a.pitch; stAimRot(S, g, a.rot);
}

// ====================================================== per-agent systems
// sim.cpp:2057-2091 applyBotActionsSystem
// ---- scripted bots: NavUtils (sim.cpp:4958-5037) + planAStarAISystem
// (sim.cpp:5041-5172).  The triangle loops index the navmesh uniformly
// across the wave, so its vertices come in as scalar loads.
__device__ __forceinline__ Vec3 navVertD(const SceneDev &sc, int tri, int k)
{
    const float *p = sc.navTris + 9 * tri + 3 * k;
    return v3(p[0], p[1], p[2]);
}

__device__ Vec3 navTriCenterD(const SceneDev &sc, int tri)
{
    Vec3 c = v3(0.f, 0.f, 0.f);
    for (int k = 0; k < 3; k++) c = c + navVertD(sc, tri, k) / 3.0f;
    return c;
}

// NearestNavTri (sim.cpp:4975-5010): first containing triangle (xy winding
// test), else the candidate kept by the reference's distance bookkeeping.
__device__ int nearestNavTriD(const SceneDev &sc, Vec3 pos)
{
    float closest = kFltMax;
    int closest_idx = -1;
    for (int tri = 0; tri < sc.numNavTris; tri++) {
        bool contained = true;
        bool gtz = false;
        for (int k = 0; k < 3; k++) {
            const Vec3 v1 = navVertD(sc, tri, k);
            const Vec3 v2 = navVertD(sc, tri, k == 2 ? 0 : k + 1);
            const Vec3 e = v2 - v1;
            const Vec3 vp = pos - v1;
            const Vec3 c = cross(e, vp);
            if ((c.z > 0.0f) != gtz && k > 0) contained = false;
            gtz = c.z > 0.0f;
            float distsq = length2(v1 - pos);
            if (distsq < closest) {
                const float dir = dot(e, vp);
                const Vec3 perp = vp * (-dir / dot(e, e)) + e;
                distsq = dot(perp, perp);
                if (distsq < closest) {
                    closest = fabs_(c.z);
                    closest_idx = tri;
                }
            }
        }
        if (contained) return tri;
    }
    return closest_idx;
}

__device__ __forceinline__ FrameDev makeFrameD(Vec3 pmin, Vec3 pmax, float rot)
{
    FrameDev f;
    f.toFrame = qinv(angleAxis(rot, kUp));
    f.pMin = rotateVec(f.toFrame, pmin);
    f.pMax = rotateVec(f.toFrame, pmax);
    return f;
}

// Zone and goal-region frames, once at scene upload (see FrameDev).
__global__ void k_scene_frames(SceneTables *tab)
{
    const int t = threadIdx.x;
    if (t < kMaxZones) {
        tab->zoneFrame[t] = makeFrameD(tab->zoneAABB[t].pMin, tab->zoneAABB[t].pMax, tab->zoneRot[t]);
    } else if (t >= 16 && t < 16 + 12) {
        const int r = (t - 16) / 3, k = (t - 16) % 3;
        const ZOBBDev &z = tab->goals[r].sub[k];
        tab->goalFrame[r][k] = makeFrameD(z.pMin, z.pMax, z.rotation);
    }
}

// The bots' goal is always a zone centroid: its NearestNavTri is computed
// once per zone at scene upload (same function, same input).
__global__ void k_zone_goals(SceneDev sc, int32_t *out)
{
    const int zi = threadIdx.x;
    if (zi >= sc.numZones) return;
    const AABB z = sc.zoneAABB[zi];
    const Vec3 center = (z.pMin + z.pMax) / 2.f; // as planAStarD forms it
    out[zi] = nearestNavTriD(sc, center);
}

// PathfindToPoint (sim.cpp:5012-5035); goal_tri = NearestNavTri(pos)
__device__ Vec3 pathfindToPointD(const SceneDev &sc, Vec3 start, Vec3 pos, int goal_tri)
{
    const int start_tri = nearestNavTriD(sc, start);
    if (start_tri < 0 || goal_tri < 0) return v3(0.f, 0.f, 0.f); // (asserted in the reference)
    const int next = sc.astar[start_tri * sc.numNavTris + goal_tri];
    if (next == -1) return v3(0.f, 0.f, 0.f);
    if (next == goal_tri) return pos;
    return navTriCenterD(sc, next);
}

__device__ __forceinline__ void planAStarD(const DevState &S, const SceneDev &sc, int64_t g)
{
    if (S.policy[g] != -1) return; // consts::aStarPolicyID
    const int w = (int)(g / S.N);
    RNG rng = ldRng(S, g);
    int move_amount = rngI32(rng, 0, 2);
    int move_angle = rngI32(rng, 0, 2);
    int r_yaw = rngI32(rng, 0, 5);
    const int r_pitch = rngI32(rng, 0, 2);
    const int reload = S.magazine[2 * g] == 0 ? 1 : 0;
    int stand = rngI32(rng, 0, 2);
    stRng(S, g, rng);
    // fire if any opponent is visible (OpponentsVisibility of the last step)
    int fire = (S.visMask[g] & ((1u << S.T) - 1u)) != 0 ? 1 : 0;

    const int zi = S.curZone[w];
    const AABB z = sc.tab->zoneAABB[zi];
    Vec3 center = (z.pMin + z.pMax) / 2.f; // AABB::centroid
    const Vec3 pos = v3(S.px[g], S.py[g], 0.f);
    center = pathfindToPointD(sc, pos, center, sc.tab->zoneGoalTri[zi]);
    center.z = 0.f;
    const float yaw = S.ayaw[g];
    const Vec3 fwd = v3(-sinf_(yaw), cosf_(yaw), 0.f);
    const Vec3 tgt = normalize(center - pos);
    move_amount = dot(fwd, tgt) > 0.6f ? 1 : 0;
    r_yaw = cross(fwd, tgt).z < 0.0f ? 0 + move_amount : 4 - move_amount;
    move_amount *= 2;
    move_angle = 0;
    stand = 0;

    // wall avoidance from last step's forward lidar depths
    float coll_ang = 0.f, coll_norm = 0.f;
    const float *lid = &S.fwdLidar[g * kFwdRays * 4];
    for (int y = 0; y < 2; y++) {
        for (int x = 0; x < 32; x++) {
            if (lid[(y * 32 + x) * 4] < 16.0f) {
                coll_norm++;
                coll_ang += x;
            }
        }
    }
    if (coll_norm > 0.f) {
        coll_ang /= coll_norm;
        move_amount = 1;
        switch ((int)(coll_ang / 32.f * 8.0f)) {
        case 0: move_angle = 2; break;
        case 1:
        case 2: move_angle = 3; break;
        case 3:
        case 4: move_angle = 4; move_amount = 2; break;
        case 5:
        case 6: move_angle = 5; break;
        case 7: move_angle = 6; break;
        }
    }
    if (reload) fire = 0;
    if (fire) r_yaw = 2;
    int32_t *out = &S.botAction[7 * g];
    out[0] = move_amount;
    out[1] = move_angle;
    out[2] = r_yaw;
    out[3] = r_pitch;
    out[4] = fire;
    out[5] = reload;
    out[6] = stand;
}

__device__ __forceinline__ void applyBotActionsD(const DevState &S, int64_t g)
{
    if (S.policy[g] != -1) return;
    const int32_t *hb = &S.botAction[7 * g];
    S.discreteAction[4 * g + 0] = hb[0];
    S.discreteAction[4 * g + 1] = hb[1];
    S.discreteAction[4 * g + 2] = hb[4];
    S.discreteAction[4 * g + 3] = hb[6];
    const float turn_delta = 10.f / (float)(5 / 2);
    S.aimAction[2 * g] = turn_delta * (float)(hb[2] - 5 / 2);
    S.aimAction[2 * g + 1] = turn_delta * (float)(hb[3] - 5 / 2);
}

// sim.cpp:2093-2199 pvpMovementSystem
__device__ __forceinline__ void pvpMovementD(const DevState &S, int64_t g)
{
    if (S.alive[g] == 0.f) return;
    const int32_t a_amount = S.discreteAction[4 * g + 0];
    const int32_t a_angle = S.discreteAction[4 * g + 1];
    const int32_t a_stand = S.discreteAction[4 * g + 3];
    Vec3 vel = ldVel(S, g);
    {
        float v_len = length(vel);
        if (v_len > 0.f) {
            Vec3 norm_v = vel / v_len;
            v_len -= c::kDeaccelerateRate * c::kDeltaT;
            v_len = fmaxD(0.f, v_len);
            vel = norm_v * v_len;
        }
    }
    int cur = S.curPose[g], tgt = S.tgtPose[g], tr = S.transRem[g];
    if (tr > 0) {
        tr -= 1;
        if (tr == 0) cur = tgt;
    }
    if (a_stand != tgt) {
        tgt = a_stand;
        int dst = tgt - cur;
        dst = dst < 0 ? -dst : dst;
        tr = dst * (c::kPoseTransitionSpeed / 2);
    }
    S.curPose[g] = cur; S.tgtPose[g] = tgt; S.transRem[g] = tr;

    float accel_max = 3000;
    if (cur == kCrouch) accel_max = 100;
    else if (cur == kProne) accel_max = 50;
    float move_amount = (float)a_amount * (accel_max / (float)(c::kNumMoveAmountBuckets - 1));
    const float per_bucket = 2.f * kPi / float(c::kNumMoveAngleBuckets);
    float move_angle = float(a_angle) * per_bucket;
    float f_x = move_amount * sinf_(move_angle);
    float f_y = move_amount * cosf_(move_angle);
    vel = vel + rotateVec(ldRot(S, g), v3(f_x, f_y, 0)) * c::kDeltaT;
    if (move_amount != 0) S.respawnSteps[g] = 0;
    float v_len = length(vel);
    if (v_len == 0.f) {
        stVel(S, g, vel);
        return;
    }
    float max_vel = S.maxVel[g];
    {
        const float max_change = 510.f;
        float tgt_v;
        if (cur == kStand) tgt_v = a_amount == 2 ? c::kMaxRunVelocity : c::kMaxWalkVelocity;
        else if (cur == kCrouch) tgt_v = c::kMaxCrouchVelocity;
        else tgt_v = c::kMaxProneVelocity;
        float diff = tgt_v - max_vel;
        float adj = fmaxD(fminD(diff, max_change), -max_change);
        max_vel += adj;
    }
    S.maxVel[g] = max_vel;
    Vec3 v_norm = vel / v_len;
    v_len = fminD(v_len, max_vel);
    stVel(S, g, v_norm * v_len);
}

// sim.cpp:2266-2370 continuous then discrete aim
__device__ __forceinline__ void pvpAimD(const DevState &S, int64_t g)
{
    if (S.alive[g] == 0.f) return;
    float yaw = S.ayaw[g], pitch = S.apitch[g];
    yaw += S.aimAction[2 * g] * c::kDeltaT;
    pitch += S.aimAction[2 * g + 1] * c::kDeltaT;
    AimD a = computeAimD(yaw, pitch);
    yaw = a.yaw; pitch = a.pitch;
    // pvpContinuousAimSystem writes Rotation too; it is overwritten below.
    const float yaw_turn[7] = { 0, 0.00390625f * kPi, 0.0078125f * kPi, 0.015625f * kPi,
                                0.03125f * kPi, 0.0625f * kPi, 0.125f * kPi };
    const float pitch_turn[4] = { 0, 0.0078125f * kPi, 0.015625f * kPi, 0.03125f * kPi };
    int yb = S.discreteAim[2 * g] - c::kDiscreteAimYawBuckets / 2;
    int yba = yb < 0 ? -yb : yb;
    if (yb < 0) yaw -= yaw_turn[yba];
    else yaw += yaw_turn[yba];
    int pb = S.discreteAim[2 * g + 1] - c::kDiscreteAimPitchBuckets / 2;
    int pba = pb < 0 ? -pb : pb;
    if (pb < 0) pitch -= pitch_turn[pba];
    else pitch += pitch_turn[pba];
    a = computeAimD(yaw, pitch);
    stAim(S, g, a);
    stRot(S, g, qnormalize(angleAxis(a.yaw, kUp)));
}

__device__ __forceinline__ Vec3 rotate2DD(Vec3 dir, float radians) // sim.cpp:874-879
{
    float cc = cosf_(radians);
    float s = sinf_(radians);
    return v3(cc * dir.x - s * dir.y, s * dir.x + cc * dir.y, 0);
}

// Distance-bounded sphere casts (k_move).  MeshBVH::sphereCast prunes boxes
// beyond its current hit, so with t_max = B it visits the same boxes in the
// same order as the unbounded cast minus those entered beyond B, and
// returns the same hit and normal whenever the unbounded cast's hit is
// nearer than B -- except through the vertex-test quirk (scene.h
// quirkGrid): testVert tests the ray 2o + t·d against a sphere of radius r
// around each vertex, so a visited triangle with a vertex within r of that
// ray at some t < B returns t (0 when 2o itself is inside) although the
// geometry is far away; a bounded cast may never visit that triangle.  A
// bounded cast is therefore only used when every grid cell under the xy
// path 2o .. 2o + B·d is clear (each clear cell is farther than r + 2 from
// every vertex); otherwise, and where the caller needs more than "hit
// nearer than B or not", the full cast runs.  Vertical casts have a
// one-cell path.  DESIGN.md §2.
// Bound = the largest distance the caller compares a hit with + this slack
// (a bounded miss then reads as a hit that far away, well past every
// comparison, whatever the rounding).
constexpr float kCastSlack = 4.f;

__device__ __forceinline__ bool castQuirkFreeD(const SceneDev &sc, Vec3 o)
{
    const float fx = ((o.x + o.x) - sc.qgMinX) * sc.qgInvCell;
    const float fy = ((o.y + o.y) - sc.qgMinY) * sc.qgInvCell;
    if (!(fx >= 0.f && fx < (float)sc.qgW && fy >= 0.f && fy < (float)sc.qgH)) return true;
    const uint32_t bit = (uint32_t)(int)fy * (uint32_t)sc.qgW + (uint32_t)(int)fx;
    return !((sc.quirkGrid[bit >> 5] >> (bit & 31)) & 1u);
}

// Every cell of the xy bounding box of the segment 2o .. 2o + B·d is clear
// (cells outside the grid are clear by construction: the grid reaches
// r + margin + one cell beyond every vertex).
__device__ __forceinline__ bool castPathQuirkFreeD(const SceneDev &sc, Vec3 o, Vec3 d, float B)
{
    const float px = o.x + o.x, py = o.y + o.y;
    const float qx = px + d.x * B, qy = py + d.y * B;
    const int x0 = max((int)floorf((fminf(px, qx) - sc.qgMinX) * sc.qgInvCell), 0);
    const int x1 = min((int)floorf((fmaxf(px, qx) - sc.qgMinX) * sc.qgInvCell), sc.qgW - 1);
    const int y0 = max((int)floorf((fminf(py, qy) - sc.qgMinY) * sc.qgInvCell), 0);
    const int y1 = min((int)floorf((fmaxf(py, qy) - sc.qgMinY) * sc.qgInvCell), sc.qgH - 1);
    for (int y = y0; y <= y1; y++)
        for (int x = x0; x <= x1; x++) {
            const uint32_t bit = (uint32_t)y * (uint32_t)sc.qgW + (uint32_t)x;
            if ((sc.quirkGrid[bit >> 5] >> (bit & 31)) & 1u) return false;
        }
    return true;
}

// The cast's hit if nearer than `near_b`, else t = kFltMax: for callers to
// which every hit at or beyond near_b acts like no hit.  Horizontal d.
__device__ __forceinline__ SphereHit castNearD(const LBVH &bvh, const SceneDev &sc, Vec3 o, Vec3 d, float near_b)
{
    if (!castPathQuirkFreeD(sc, o, d, near_b)) return bvhSphereCastD(bvh, o, d, kSphereR);
    SphereHit h = bvhSphereCastD(bvh, o, d, kSphereR, near_b);
    if (!(h.t < near_b)) h.t = kFltMax;
    return h;
}

// castNearD for the low cast from o and, when act1, the high cast from
// (o.x, o.y, z1): one traversal (bvhSphereCast2D), the same results.  The
// path guard depends on o.xy, d and near_b only, so both casts take the
// same branch.
__device__ __forceinline__ void castNear2D(const LBVH &bvh, const SceneDev &sc, Vec3 o, float z1, Vec3 d,
                                           float near_b, bool act1, SphereHit &h0, SphereHit &h1)
{
    if (!castPathQuirkFreeD(sc, o, d, near_b)) {
        bvhSphereCast2D(bvh, o, z1, d, kSphereR, kFltMax, act1, h0, h1);
        return;
    }
    bvhSphereCast2D(bvh, o, z1, d, kSphereR, near_b, act1, h0, h1);
    if (!(h0.t < near_b)) h0.t = kFltMax;
    if (act1 && !(h1.t < near_b)) h1.t = kFltMax;
}

// The full cast's t, searched within near_b first.  Vertical d only (the
// path guard is the cell of 2o).
__device__ __forceinline__ float castFirstNearD(const LBVH &bvh, const SceneDev &sc, Vec3 o, Vec3 d, float near_b)
{
    if (castQuirkFreeD(sc, o)) {
        const float t = bvhSphereCastD(bvh, o, d, kSphereR, near_b).t;
        if (t < near_b) return t;
    }
    return bvhSphereCastD(bvh, o, d, kSphereR).t;
}

// Index of the n-th set bit (0-based) of m; m has more than n set bits.
__device__ __forceinline__ int nthSetBitD(uint64_t m, int n)
{
    int pos = 0;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
        const uint64_t low = m & ((1ull << w) - 1ull);
        const int c = __popcll(low);
        if (n >= c) {
            n -= c;
            m >>= w;
            pos += w;
        } else {
            m = low;
        }
    }
    return pos;
}

// The "stuck" fallback's four horizontal casts (sim.cpp:962-984), for the
// lanes of the wave with `need` set: their 4·k casts are dealt one per
// active lane across the wave (rounds of as many casts as the wave has
// active lanes) instead of four in a row on the owning lane -- a wave holding
// one stuck agent runs one cast's time, not four.  Each cast is the same
// function of the same owner inputs (x, v_norm, low_check shuffled from the
// owner), so hd4 is bit-identical to the serial loop's.  Called by every
// active lane of the wave; on small batches k_move runs 8-32 agents per
// wave (launchMove), and round 6 deals over those lanes too (rounds 4-5 fell
// back to the serial loop on any partial wave, i.e. always below C3).
__device__ __forceinline__ void stuckCastsD(const LBVH &bvh, bool need, Vec3 x, Vec3 v_norm, float low_check,
                                            float hd4[4])
{
    const float r = c::kAgentRadius;
    const uint64_t act = __ballot(1);
    const uint64_t m = __ballot(need);
    if (m == 0ull) return;
    const int na = __popcll(act);
    const int lane = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    const int arank = __popcll(act & ((1ull << lane) - 1ull)); // this lane's index among the active lanes
    const int rank = __popcll(m & ((1ull << lane) - 1ull));    // owner's index among the stuck lanes
    const int tasks = 4 * __popcll(m);
    for (int base = 0; base < tasks; base += na) {
        const int t = base + arank;
        const int owner = nthSetBitD(m, min(t, tasks - 1) >> 2);
        const float ox = __shfl(x.x, owner), oy = __shfl(x.y, owner), oz = __shfl(x.z, owner);
        const float vx = __shfl(v_norm.x, owner), vy = __shfl(v_norm.y, owner), vz = __shfl(v_norm.z, owner);
        const float lc = __shfl(low_check, owner);
        float hd = 0.f;
        if (t < tasks) {
            const Vec3 dv = rotate2DD(v3(vx, vy, vz), (float)(t & 3) * 3.14159f * 0.5f);
            Vec3 ray_o = v3(ox, oy, oz) - dv * r * 2.0f;
            ray_o.z += lc;
            hd = bvhSphereCastD(bvh, ray_o, dv, r).t;
        }
#pragma unroll
        for (int dir = 0; dir < 4; dir++) {
            const int tt = 4 * rank + dir;
            // the active lane that ran task tt this round (any lane when none did)
            const int src = nthSetBitD(act, min(max(tt - base, 0), na - 1));
            const float got = __shfl(hd, src);
            if (need && tt >= base && tt < base + na) hd4[dir] = got;
        }
    }
}

// sim.cpp:889-1039 applyVelocitySystem + updateMoveStateSystem.  Split at
// the stuck fallback so the wave can share its casts (stuckCastsD): part 1
// up to the ground check, the fallback's casts, part 2 to the end.
__device__ __forceinline__ void applyVelocityD(const DevState &S, const SceneDev &sc, const LBVH &bvh, int64_t g)
{
    const Vec3 x = ldPos(S, g);
    Vec3 v = ldVel(S, g);
    v.z = 0;
    Vec3 new_pos = x;
    Vec3 new_vel = v3(0.f, 0.f, 0.f);
    const int pose = S.curPose[g];
    float v_len = length(v);
    const float buffer = 0.05f * c::kAgentRadius;
    const float r = c::kAgentRadius;
    float top = c::kStandHeight - r;
    float low_check = c::kProneHeight;
    if (pose == kCrouch) {
        top = c::kCrouchHeight - r;
    } else if (pose == kProne) {
        top = low_check;
        low_check = c::kProneHeight - r + buffer;
    }
    Vec3 v_norm = v3(0.f, 0.f, 0.f);
    Vec3 hit_pos = x, ground_check = x;
    float ground_dist = 0.f;
    bool cont = false, stuck_path = false;
    do {
        if (v_len == 0.f) break;
        v_norm = v / v_len;
        float move_dist = v_len * c::kDeltaT;

        Vec3 ray_o = x;
        ray_o.z += top;
        Vec3 normal = v3(0.f, 0.f, 0.f);
        {
            // the ground below, wherever it is (a bounded first try gains
            // nothing here: the downward cast prunes at the floor anyway)
            SphereHit h = bvhSphereCastD(bvh, ray_o, -kUp, r);
            if (h.t < kFltMax) normal = h.n;
        }
        if (normal.z > 0.0f && (double)normal.z < 0.7 && dot(normal, v_norm) < 0.0f) break;

        // The forward casts only matter nearer than move_dist + buffer: a
        // farther hit leaves hit_pos at move_dist, takes no slide and the
        // normal / high_hit it sets are read only by the slide (bound with a
        // margin of kCastSlack so no value near a decision is ever cut).
        const float fwd_b = (move_dist + buffer) + kCastSlack;
        ray_o = x + v_norm * buffer * 0.5f;
        ray_o.z += low_check;
        // the low cast and (standing / crouching) the high cast from
        // (ray_o.xy, x.z + top), traversed together
        SphereHit hl, hh;
        hh.t = kFltMax;
        castNear2D(bvh, sc, ray_o, x.z + top, v_norm, fwd_b, pose != kProne, hl, hh);
        float low_dist = hl.t;
        if (hl.t < kFltMax) normal = hl.n;
        float high_dist = low_dist;
        bool high_hit = false;
        if (pose != kProne) {
            high_dist = hh.t;
            if (high_dist < low_dist) {
                low_dist = high_dist;
                normal = hh.n;
                high_hit = true;
            }
        }
        bool stuck = low_dist == 0.0f || high_dist == 0.0f;
        low_dist = fmaxD(0.0f, low_dist - buffer);
        high_dist = fmaxD(0.0f, high_dist - buffer);
        hit_pos = x + v_norm * fminD(low_dist, move_dist);

        if (move_dist > low_dist) {
            Vec3 slide_dir = normalize(cross(kUp, normal));
            if (dot(slide_dir, v_norm) < 0) slide_dir = -slide_dir;
            ray_o = x + v_norm * low_dist;
            ray_o.z += high_hit ? top : low_check;
            float max_move = move_dist - low_dist;
            // only min(slide - buffer, max_move) is used
            float slide = castNearD(bvh, sc, ray_o, slide_dir, (max_move + buffer) + kCastSlack).t;
            slide = fmaxD(0.0f, slide - buffer);
            slide = fminD(slide, max_move);
            if (slide > 0.0f) hit_pos = hit_pos + slide_dir * slide;
        }

        ground_check = hit_pos;
        ground_check.z += top;
        // min(ground_dist, top) is used, and whether there is ground at all
        ground_dist = castFirstNearD(bvh, sc, ground_check, -kUp, 2.f * top + 10.f);
        if (ground_dist == kFltMax) break;
        stuck_path = (ground_dist <= 0.0f || stuck);
        cont = true;
    } while (false);

    float hd4[4] = { 0.f, 0.f, 0.f, 0.f };
    stuckCastsD(bvh, stuck_path, x, v_norm, low_check, hd4);

    while (cont) {
        if (stuck_path) {
            float furthest = 0.0f;
            int best_dir = -1;
            for (int dir = 0; dir < 4; dir++) {
                if (hd4[dir] > furthest) {
                    furthest = hd4[dir];
                    best_dir = dir;
                }
            }
            if (best_dir != -1) {
                Vec3 dv = rotate2DD(v_norm, (float)best_dir * 3.14159f * 0.5f);
                hit_pos = x + dv * (fminD(furthest - r * 2.0f, -buffer));
                ground_check = hit_pos;
                ground_check.z += top;
                ground_dist = bvhSphereCastD(bvh, ground_check, -kUp, r).t;
                if (ground_dist == kFltMax) break;
            }
        }

        float fall_dist = fminD(ground_dist, top) + r;
        Vec3 np = ground_check;
        np.z -= fall_dist;
        Vec3 to_new = np - x;
        float to_new_dist = length(to_new);
        if (to_new_dist == 0.f) break;
        new_pos = np;
        new_vel = to_new / c::kDeltaT;
        break;
    }
    // updateMoveStateSystem (sim.cpp:1030-1039)
    stPos(S, g, new_pos);
    stVel(S, g, new_vel);
}

// sim.cpp:1041-1104 fallSystem + updateMoveStatePostFallSystem
__device__ __forceinline__ void fallD(const DevState &S, const SceneDev &sc, const LBVH &bvh, int64_t g)
{
    if (S.alive[g] == 0.f) return;
    const float fall_rate = 386.08858267717f;
    const float cast_offset = c::kAgentRadius;
    Vec3 pos = ldPos(S, g);
    Vec3 ray_o = pos;
    ray_o.z += c::kAgentRadius + cast_offset;
    // min(ground - cast_offset, fall_rate * dt) is used, and whether there
    // is ground at all
    float ground = castFirstNearD(bvh, sc, ray_o, -kUp, 2.f * (cast_offset + fall_rate * c::kDeltaT) + 10.f);
    if (ground == kFltMax || ground < cast_offset) return;
    float fall = fminD(ground - cast_offset, fall_rate * c::kDeltaT);
    pos.z -= fall;
    S.pz[g] = pos.z;
}

// sim.cpp:1443-1615 fireSystem
// ---- event log (sim.cpp:23-39 logEvent; GameEvent types.hpp:729-760)
__device__ __forceinline__ uint64_t matchIdD(const DevState &S, const SceneDev &sc, int w)
{
    return ((uint64_t)(sc.worldOffset + (uint32_t)w) << 32) | (uint64_t)(uint32_t)S.episode[w];
}

__device__ __forceinline__ void putEventD(const DevState &S, const SceneDev &sc, int w, int slot, uint32_t type,
                                          int a, int b, int c16)
{
    mpenv_game_event ev;
    ev.type = type;
    ev.pad_ = 0;
    ev.match_id = matchIdD(S, sc, w);
    ev.step = (uint32_t)S.curStep[w];
    ev.a = (uint8_t)a;
    ev.b = (uint8_t)b;
    ev.c16 = (uint16_t)c16;
    S.events[(int64_t)w * S.evStride + slot] = ev;
}

__device__ __forceinline__ int playerIdD(const DevState &S, int i) { return (i / S.T) * kMaxTeamSize + i % S.T; }

// What fireD reads about its own agent, loaded before any of its stores.
struct FireIn {
    int32_t flags, mag0, mag1, fire, pose, respawn;
    float alive, hp, ayaw, apitch;
    Vec3 pos;
    RNG rng;
};

__device__ __forceinline__ FireIn fireLoadD(const DevState &S, int64_t g)
{
    FireIn f;
    f.flags = S.flags[g];
    f.alive = S.alive[g];
    f.mag0 = S.magazine[2 * g];
    f.mag1 = S.magazine[2 * g + 1];
    f.fire = S.discreteAction[4 * g + 2];
    f.pose = S.curPose[g];
    f.respawn = S.respawnSteps[g];
    f.hp = S.hp[g];
    f.ayaw = S.ayaw[g];
    f.apitch = S.apitch[g];
    f.pos = ldPos(S, g);
    f.rng = ldRng(S, g);
    return f;
}

// sim.cpp:1443-1615 fireSystem.  in: the agent's own inputs (fireLoadD);
// lpx / lpy / lpz, lhp, lrs: the world's agents' positions, hp and respawn
// counters in LDS (k_sim stages them), indexed from lb (the world's first
// lane).
__device__ __forceinline__ void fireD(const DevState &S, const SceneDev &sc, const LBVH &bvh, int w, int i, const FireIn &in,
                                      const float *lpx, const float *lpy, const float *lpz, const float *lhp,
                                      const float *lrs, int lb)
{
    const int N = S.N;
    const int64_t g0 = (int64_t)w * N;
    const int64_t g = g0 + i;
    S.landedOn[g] = -1;
    S.firedT[g] = -kFltMax;
    int32_t flags = in.flags & ~(kFlagSuccessfulKill | kFlagReloadedFullMag);
    if (in.alive == 0.f) {
        S.flags[g] = flags;
        return;
    }
    int32_t mag0 = in.mag0, mag1 = in.mag1;
    const int fire = in.fire;
    if (fire == 2) {
        if (sc.eventsOn) putEventD(S, sc, w, 2 * i, MPENV_EVENT_RELOAD, playerIdD(S, i), mag0, 0);
        if (mag0 == c::kMagSize) flags |= kFlagReloadedFullMag;
        mag0 = c::kMagSize;
        mag1 = c::kReloadTime;
    }
    bool reloading = mag1 > 0;
    if (reloading) mag1 -= 1;
    bool should_fire = false;
    if (!reloading && mag0 > 0) should_fire = fire == 1;
    if (!should_fire) {
        S.magazine[2 * g] = mag0;
        S.magazine[2 * g + 1] = mag1;
        S.flags[g] = flags;
        return;
    }
    mag0 -= 1;
    S.magazine[2 * g] = mag0;
    S.magazine[2 * g + 1] = mag1;

    Vec3 fire_from = in.pos;
    fire_from.z += viewHeightD(in.pose);
    RNG rng = in.rng;
    float u1 = rngUniform(rng);
    float u2 = rngUniform(rng);
    stRng(S, g, rng);
    float z1 = sqrt_(-2.f * logf_(u1)) * cosf_(2.f * kPi * u2);
    float z2 = sqrt_(-2.f * logf_(u1)) * sinf_(2.f * kPi * u2);
    const float acc = c::kAccuracyScale;
    const float bias = 1.5f;
    float up_delta = fminD(fmaxD((z1 + bias) * acc, 0.f), 4.f * acc);
    float right_delta = fminD(fmaxD(z2 * acc, -4.f * acc), 4.f * acc);
    AimD a = computeAimD(in.ayaw + right_delta, in.apitch + up_delta);
    stAim(S, g, a);
    Vec3 fire_dir = rotateVec(a.rot, kFwd);

    WorldHit h = traceWorldD(bvh, lpx, lpy, lpz, lb, N, fire_from, fire_dir, i); // from its own axis
    if (S.stats) statAdd(S.stats + kStatShots, 1u);
    S.firedT[g] = h.hit ? h.t : kFltMax;
    bool success = h.hit;
    const int team = i / S.T, offset = i - team * S.T;
    if (h.entity == -1) {
        success = false;
    } else {
        const int tteam = h.entity / S.T;
        if (success && tteam == team) success = false;
        if (success && __float_as_int(lrs[lb + h.entity]) > 0) success = false;
    }
    if (success) {
        if (sc.eventsOn) putEventD(S, sc, w, 2 * i, MPENV_EVENT_PLAYER_SHOT, playerIdD(S, i), playerIdD(S, h.entity), 0);
        S.landedOn[g] = h.entity;
        if (lhp[lb + h.entity] <= c::kDmgPerBullet) {
            flags |= kFlagSuccessfulKill;
            if (sc.eventsOn) putEventD(S, sc, w, 2 * i + 1, MPENV_EVENT_KILL, playerIdD(S, i), playerIdD(S, h.entity), 0);
        }
        S.dmg[(int64_t)offset * S.dmgStride + g0 + h.entity] = c::kDmgPerBullet;
    }
    S.flags[g] = flags;
}

// sim.cpp:1794-1836 applyDmgSystem
// What the world lane's respawn reads about an agent after applyDmgD (k_sim
// hands it over in LDS).
struct DmgOut {
    bool alive;
    int32_t flags;
    Vec3 pos;
};

__device__ DmgOut applyDmgD(const DevState &S, int64_t g)
{
    // every input read before the first store (the damage slots are floats
    // like the stores between them, which would serialise the loads)
    int32_t flags = S.flags[g] & ~kFlagWasKilled;
    Vec3 pos = ldPos(S, g);
    const int rs = S.respawnSteps[g];
    float hp = S.hp[g];
    const bool was_alive = S.alive[g] == 1.f;
    int ah = S.autohealSteps[g];
    const int T = S.T;
    float dm[kMaxTeamSize];
    #pragma unroll
    for (int k = 0; k < kMaxTeamSize; k++) dm[k] = k < T ? S.dmg[(int64_t)k * S.dmgStride + g] : 0.f;
    if (rs > 0) S.respawnSteps[g] = rs - 1;
    int was_shot = 0;
    #pragma unroll
    for (int k = 0; k < kMaxTeamSize; k++) {
        if (k >= T) break;
        if (dm[k] > 0.f) was_shot += 1;
        hp -= dm[k];
        S.dmg[(int64_t)k * S.dmgStride + g] = 0.f;
    }
    if (was_shot > 0) ah = c::kOutOfCombatSteps;
    S.wasShot[g] = was_shot;
    if (was_alive && hp <= 0.f) flags |= kFlagWasKilled | kFlagHasDied;
    if (S.stats) {
        statAdd(S.stats + kStatHits, was_shot > 0 ? 1u : 0u);
        statAdd(S.stats + kStatKills, (was_alive && hp <= 0.f) ? 1u : 0u);
    }
    const bool dead = hp <= 0.f;
    if (dead) {
        hp = 0.f;
        S.alive[g] = 0.f;
        pos = v3(0, 0, 10000.f);
        stPos(S, g, pos);
        stVel(S, g, v3(0, 0, 0));
    } else {
        S.alive[g] = 1.f;
        // sim.cpp:1875-1890 autoHealSystem for the agents alive after the
        // damage (nothing between the two systems changes them; a
        // respawned agent's autoheal is spawnApplyD's)
        if (ah == 0 && hp < 100.f) hp = fminD(100.f, hp + c::kAutohealPerStep);
        else if (ah > 0) ah -= 1;
    }
    if (was_shot > 0 || !dead) S.autohealSteps[g] = ah;
    S.hp[g] = hp;
    S.flags[g] = flags;
    DmgOut o;
    o.alive = !dead;
    o.flags = flags;
    o.pos = pos;
    return o;
}

// ====================================================== spawning / reset
// utils.cpp:273-479 standardSpawnPoint (Zone task)
// Draw keys of an agent's fresh combat RNG (counters 0 .. kPreDraws-1),
// computed by the agent's own lane before a world reset so the world lane
// does not evaluate them one after another (k_sim, resetPreD).
constexpr int kPreDraws = 10;

// What the world lane's spawn loop reads about its world's agents, kept in
// LDS by k_sim (null members: read memory): positions [N][3] and alive
// bytes, both updated as agents spawn (the respawn scoring sees earlier
// spawns), and each agent's flags before the spawn (as float bits).
// tabA / tabB / tabC: LDS copies of the scene's spawn lists (aSpawns,
// bSpawns, commonRespawns), or null.
struct SpawnLds {
    float *pos;
    uint8_t *alive;
    const float *flags;
    const Spawn *tabA, *tabB, *tabC;
};

// World values the spawn loop reads once (not per agent).
struct SpawnWorld {
    int teamA, cz, episodeCurr;
    uint32_t curStep;
};

// Spawn indices taken so far in a world reset's loop, per team list (bits
// 0..127).  The reset cleared both lists just before (resetPreD), so
// "tracker[idx] == curStep" holds exactly for the indices taken here.
struct SpawnTaken {
    uint64_t a0, a1, b0, b1;
};

// One common respawn point's score for agent ai (utils.cpp:410-475 inside
// standardSpawnPoint's respawn branch): recently used points, points near
// any live agent, near live opponents, and near the zone score higher.
__device__ __forceinline__ float respawnScoreD(const DevState &S, const Spawn *options, int s, int ai, int team,
                                               uint32_t last_used, uint32_t cur_step, Vec3 zone_center,
                                               const SpawnLds &L, int64_t g0)
{
    const int N = S.N;
    float score = 0.f;
    uint32_t elapsed = (uint32_t)(c::kDeltaT * float(cur_step - last_used));
    const float elapsed_weight = 0.1f, dist_weight = 0.01f;
    if (elapsed < 3.f) score += elapsed_weight * (3.f - elapsed);
    Spawn sp = options[s];
    Vec3 spawn_pt = 0.5f * (sp.region.pMin + sp.region.pMax);
    #pragma unroll 1
    for (int j = 0; j < N; j++) {
        if (j == ai) continue;
        if (L.alive ? L.alive[j] == 0 : S.alive[g0 + j] == 0.f) continue;
        const Vec3 pj = L.pos ? v3(L.pos[3 * j], L.pos[3 * j + 1], L.pos[3 * j + 2]) : ldPos(S, g0 + j);
        float dist = distance(spawn_pt, pj);
        if (dist < 4.f * c::kAgentRadius) {
            score += 100000.f;
        } else {
            if (j / S.T == team) continue;
            score += dist_weight * (1.f / dist);
        }
    }
    float dz = distance(spawn_pt, zone_center);
    if (dz < 100.f) score += 1000000.f;
    return score;
}

__device__ __forceinline__ void standardSpawnPointD(const DevState &S, const SceneDev &sc, int w, int ai, bool is_respawn,
                                    bool use_middle, RNG &rng, Vec3 &out_pt, float &out_yaw,
                                    const RandKey *pre, const SpawnWorld &sw, const SpawnLds &L, SpawnTaken &tk)
{
    // rng's draws, from `pre` while the counter is inside it (same keys
    // splitI(rng.key, ctr) the RNG would produce)
    auto adv = [&]() {
        const RandKey k = (pre && rng.ctr < (uint32_t)kPreDraws) ? pre[rng.ctr] : splitI(rng.key, rng.ctr);
        rng.ctr += 1;
        return k;
    };
    const int N = S.N;
    const int64_t g0 = (int64_t)w * N;
    const int team = ai / S.T;
    const uint32_t cur_step = sw.curStep;
    uint32_t *track = &S.spawnTrack[(int64_t)w * 3 * sc.spawnTrackLen];

    const Spawn *options;
    auto spawnAgent = [&](int idx) {
        Spawn s = options[idx];
        float x_rnd = keyUniform(adv());
        float y_rnd = keyUniform(adv());
        float z_rnd = keyUniform(adv());
        float yaw_rnd = keyUniform(adv());
        float x_min = s.region.pMin.x, x_diff = s.region.pMax.x - x_min;
        float y_min = s.region.pMin.y, y_diff = s.region.pMax.y - y_min;
        float z_min = s.region.pMin.z, z_diff = s.region.pMax.z - z_min;
        out_pt = v3(x_min + x_rnd * x_diff, y_min + y_rnd * y_diff, z_min + z_rnd * z_diff);
        out_yaw = s.yawMin + yaw_rnd * (s.yawMax - s.yawMin);
    };

    if (!is_respawn || sc.numCommon == 0) {
        uint32_t *tracker;
        int num_default, num_extra, num_spawns;
        const bool list_a = team == sw.teamA;
        if (list_a) {
            options = L.tabA ? L.tabA : sc.aSpawns;
            num_default = sc.numDefaultA;
            num_extra = sc.numA - sc.numDefaultA;
            tracker = track;
        } else {
            options = L.tabB ? L.tabB : sc.bSpawns;
            num_default = sc.numDefaultB;
            num_extra = sc.numB - sc.numDefaultB;
            tracker = track + sc.spawnTrackLen;
        }
        if (use_middle) {
            options += num_default;
            num_spawns = num_extra;
        } else {
            num_spawns = num_default;
        }
        if (pre && !is_respawn && rng.ctr == 0 && num_spawns <= 128) {
            // world reset: the agent's draw keys in one round of loads, the
            // taken indices from tk instead of the tracker
            RandKey k[kPreDraws];
            #pragma unroll
            for (int c = 0; c < kPreDraws; c++) k[c] = pre[c];
            uint64_t &t0 = list_a ? tk.a0 : tk.b0, &t1 = list_a ? tk.a1 : tk.b1;
            auto taken = [&](int idx) { return (((idx < 64 ? t0 : t1) >> (idx & 63)) & 1ull) != 0; };
            int init_idx = keyI32(k[5], 0, num_spawns), used = 6;
            #pragma unroll
            for (int t = 4; t >= 0; t--) {
                const int idx = keyI32(k[t], 0, num_spawns);
                if (!taken(idx)) { init_idx = idx; used = t + 1; }
            }
            // draws used .. used + 3 position the agent (spawnAgent)
            RandKey kk[4];
            #pragma unroll
            for (int j = 0; j < 4; j++) {
                kk[j] = k[6 + j];
                #pragma unroll
                for (int t = 5; t >= 1; t--)
                    if (used == t) kk[j] = k[t + j];
            }
            rng.ctr = (uint32_t)(used + 4);
            const Spawn sp = options[init_idx];
            const float x_min = sp.region.pMin.x, x_diff = sp.region.pMax.x - x_min;
            const float y_min = sp.region.pMin.y, y_diff = sp.region.pMax.y - y_min;
            const float z_min = sp.region.pMin.z, z_diff = sp.region.pMax.z - z_min;
            out_pt = v3(x_min + keyUniform(kk[0]) * x_diff, y_min + keyUniform(kk[1]) * y_diff,
                        z_min + keyUniform(kk[2]) * z_diff);
            out_yaw = sp.yawMin + keyUniform(kk[3]) * (sp.yawMax - sp.yawMin);
            (init_idx < 64 ? t0 : t1) |= 1ull << (init_idx & 63);
            tracker[init_idx] = cur_step;
            return;
        }
        int init_idx = -1;
        for (int k = 0; k < 5; k++) {
            int idx = keyI32(adv(), 0, num_spawns);
            if (tracker[idx] == cur_step) continue;
            init_idx = idx;
            break;
        }
        if (init_idx == -1) init_idx = keyI32(adv(), 0, num_spawns);
        spawnAgent(init_idx);
        tracker[init_idx] = cur_step;
        return;
    }

    options = L.tabC ? L.tabC : sc.commonRespawns;
    uint32_t *rtrack = track + 2 * sc.spawnTrackLen;
    const int cz = sw.cz;
    AABB za = sc.tab->zoneAABB[cz];
    Vec3 zone_center = 0.5f * (za.pMin + za.pMax);
    float best_score = kFltMax;
    int best_idx = -1;
    // the next entry's tracker load is in flight during this one's scoring
    uint32_t next_used = sc.numCommon > 0 ? rtrack[0] : 0u;
    for (int s = 0; s < sc.numCommon; s++) {
        const uint32_t last_used = next_used;
        if (s + 1 < sc.numCommon) next_used = rtrack[s + 1];
        if (last_used == cur_step) continue;
        const float score = respawnScoreD(S, options, s, ai, team, last_used, cur_step, zone_center, L, g0);
        if (score < best_score) {
            best_idx = s;
            best_score = score;
        }
    }
    if (best_idx < 0) best_idx = 0;
    spawnAgent(best_idx);
    rtrack[best_idx] = cur_step;
}

// AgentPolicy idx clamped to the 8 sub-zones (sim.cpp:1996-1997)
__device__ __forceinline__ int subZoneIndexD(const DevState &S, int64_t g)
{
    const int p = S.policy[g];
    return p < 0 ? 0 : (p > 7 ? 7 : p);
}

// The zone box of zone cz in its own frame (spawnAgents' in-zone test).
struct ZoneBox {
    AABB box;
    Vec3 center;
    Quat toZone;
};

__device__ __forceinline__ ZoneBox zoneBoxD(const SceneDev &sc, int cz)
{
    ZoneBox z;
    z.box = sc.tab->zoneAABB[cz];
    z.center = (z.box.pMax + z.box.pMin) / 2.f;
    z.toZone = qinv(angleAxis(sc.tab->zoneRot[cz], kUp));
    z.box.pMin = rotateVec(z.toZone, z.box.pMin);
    z.box.pMax = rotateVec(z.toZone, z.box.pMax);
    return z;
}

// A spawned agent's own stores once its spawn point is chosen (the rest of
// utils.cpp:734-948's loop body).  rng_ctr >= 0: the agent's RNG counter
// after its spawn draws (its key is unchanged); flags: the agent's flags
// before the spawn.  Run by the world lane, or (k_sim) by the agent's own
// lane from the world lane's record.
__device__ __forceinline__ void spawnApplyD(const DevState &S, const SceneDev &sc, int64_t g, bool is_respawn,
                                            Vec3 spawn_pt, float spawn_yaw, int32_t rng_ctr, float hp, int32_t mag,
                                            int32_t flags, const ZoneBox &zb)
{
    stPos(S, g, spawn_pt);
    if (!is_respawn) { S.sx[g] = spawn_pt.x; S.sy[g] = spawn_pt.y; S.sz[g] = spawn_pt.z; }
    if (rng_ctr >= 0) S.rngCtr[g] = rng_ctr;
    stRot(S, g, qnormalize(angleAxis(spawn_yaw, kUp)));
    stAim(S, g, computeAimD(spawn_yaw, 0.f));
    stVel(S, g, v3(0.f, 0.f, 0.f));
    S.weapon[g] = 0;
    // a respawn is followed by autoHealSystem (sim.cpp:1875-1890; alive, no
    // autoheal countdown)
    if (is_respawn && hp < 100.f) hp = fminD(100.f, hp + c::kAutohealPerStep);
    S.hp[g] = hp;
    S.magazine[2 * g] = mag;
    S.magazine[2 * g + 1] = 0;
    S.respawnSteps[g] = is_respawn ? 0 : c::kRespawnInvincibleSteps;
    S.autohealSteps[g] = 0;
    {
        Vec3 pz = rotateVec(zb.toZone, spawn_pt);
        spawn_pt.z += c::kStandHeight / 2.f;
        flags = aabbContains(zb.box, pz) ? (flags | kFlagInZone) : (flags & ~kFlagInZone);
        S.minDistZone[g] = distance(spawn_pt, zb.center);
    }
    if (sc.simFlags & kFlagSubZones) {
        // utils.cpp:906-926: spawn_pt already carries the +standHeight/2
        // of the zone block and receives it a second time
        const ZOBBDev &sz = sc.tab->subZones[subZoneIndexD(S, g)];
        AABB za = { sz.pMin, sz.pMax };
        Vec3 sub_center = (za.pMax + za.pMin) / 2.f;
        Quat to_sub = qinv(angleAxis(sz.rotation, kUp));
        za.pMin = rotateVec(to_sub, za.pMin);
        za.pMax = rotateVec(to_sub, za.pMax);
        Vec3 pz = rotateVec(to_sub, spawn_pt);
        spawn_pt.z += c::kStandHeight / 2.f;
        flags = aabbContains(za, pz) ? (flags | kFlagInSubZone) : (flags & ~kFlagInSubZone);
        S.minDistSub[g] = distance(spawn_pt, sub_center);
    }
    S.flags[g] = flags;
    S.curPose[g] = kStand; S.tgtPose[g] = kStand; S.transRem[g] = 0;
    S.maxVel[g] = c::kMaxWalkVelocity;
    S.dyv[g] = 0.f; S.dpv[g] = 0.f;
    S.alive[g] = 1.f;
}

// The world lane's spawn record of one agent for spawnApplyD on the agent's
// lane (k_sim, LDS): position, yaw, hp, then magazine and RNG counter as
// float bits.
constexpr int kSpawnRec = 8;

__device__ __forceinline__ void spawnApplyRecD(const DevState &S, const SceneDev &sc, int64_t g, bool is_respawn,
                                               const float *rec, int32_t flags, const ZoneBox &zb)
{
    spawnApplyD(S, sc, g, is_respawn, v3(rec[0], rec[1], rec[2]), rec[3], __float_as_int(rec[6]), rec[4],
                __float_as_int(rec[5]), flags, zb);
}

// utils.cpp:734-948 spawnAgents
// dead: the world's dead agents as a bit mask when the caller knows them
// (k_sim: from applyDmgD's results in LDS; a reset: all), else -1 and read
// from alive.  L: the caller's LDS copies of the world's agents (k_sim), or
// null members.  A reset (!is_respawn) also stores each agent's start
// position (sx, sy, sz: resetPersistentEntities sets them from the spawn).
__device__ __forceinline__ void spawnAgentsD(const DevState &S, const SceneDev &sc, int w, bool is_respawn,
                                             const RandKey *pre = nullptr, int64_t dead = -1,
                                             SpawnLds L = SpawnLds{ nullptr, nullptr, nullptr, nullptr, nullptr, nullptr },
                                             float *rec = nullptr, RNG *base_out = nullptr,
                                             const SpawnWorld *sw_in = nullptr, const RNG *base_in = nullptr)
{
    const int N = S.N;
    const int64_t g0 = (int64_t)w * N;
    // Dead set fixed before the loop (utils.cpp:767-780).
    uint32_t dead_mask = 0;
    if (dead >= 0) {
        dead_mask = (uint32_t)dead;
    } else {
        #pragma unroll 1
        for (int i = 0; i < N; i++)
            if (S.alive[g0 + i] == 0.f) dead_mask |= 1u << i;
    }
    if (dead_mask == 0) {
        if (base_out) *base_out = base_in ? *base_in : ldWRng(S, w);
        return;
    }
    // (a reset hands over the world values and RNG it has just stored)
    RNG base = base_in ? *base_in : ldWRng(S, w);
    SpawnWorld sw;
    if (sw_in) {
        sw = *sw_in;
    } else {
        sw.teamA = S.teamA[w];
        sw.cz = S.curZone[w];
        sw.curStep = (uint32_t)S.curStep[w];
        sw.episodeCurr = S.episodeCurr[w];
    }
    // episodes[sampleI32(0, numEpisodes = 0)]: an empty range, the value is
    // 0 whatever the key -- only the counter advances
    base.ctr += 1;
    bool use_middle = false;
    if (sc.simFlags & kFlagSpawnInMiddle) use_middle = rngUniform(base) < 0.5f;
    const bool randomize_hp = (sc.simFlags & kFlagRandomizeHP) != 0;
    const int cz = sw.cz;
    // the zone box in its own frame, once for every agent (record mode: the
    // agents' lanes compute it)
    ZoneBox zb;
    if (!rec) zb = zoneBoxD(sc, cz);
    SpawnTaken tk = { 0ull, 0ull, 0ull, 0ull };

    #pragma unroll 1
    for (int ai = 0; ai < N; ai++) {
        if (!(dead_mask & (1u << ai))) continue;
        const int64_t g = g0 + ai;
        Vec3 spawn_pt;
        float spawn_yaw;
        int32_t rng_ctr = -1;
        if ((sc.simFlags & kFlagHardcodedSpawns) && !is_respawn) {
            // utils.cpp:480-650 hardcodedSpawnPoint
            const int team = ai / S.T;
            hardcodedSpawn((team == sw.teamA ? 0 : 3) + (ai - team * S.T), spawn_pt, spawn_yaw);
        } else if (sc.simFlags & kFlagNavmeshSpawn) {
            // utils.cpp:807-809
            spawn_pt = navSamplePoint(sc.navTris, sc.navCdf, sc.numNavTris, rngAdvance(base));
            spawn_yaw = rngUniform(base) * 2.f * kPi;
        } else {
            const RandKey *apre = pre ? pre + ai * (kPreDraws + 1) : nullptr;
            // a reset's agent RNG is the fresh key resetPreD stored (apre[0])
            RNG rng = apre ? makeRNG(apre[0]) : ldRng(S, g);
            standardSpawnPointD(S, sc, w, ai, is_respawn, use_middle, rng, spawn_pt, spawn_yaw,
                                apre ? apre + 1 : nullptr, sw, L, tk);
            rng_ctr = (int32_t)rng.ctr; // (the key is unchanged)
            if ((sc.simFlags & kFlagEnableCurriculum) && sw.episodeCurr == 0) {
                // utils.cpp:819-837 LearnShooting
                const bool north = spawn_pt.y > 0.f;
                const float x = -700.f + rngUniform(base) * 1400.f;
                const float y = rngUniform(base) * 350.f;
                spawn_pt = v3(x, north ? y : -y, 0.f);
            }
        }
        if (L.pos) { L.pos[3 * ai] = spawn_pt.x; L.pos[3 * ai + 1] = spawn_pt.y; L.pos[3 * ai + 2] = spawn_pt.z; }
        if (L.alive) L.alive[ai] = 1;
        // sampleI32(0, numWeaponTypes = 1) is 0 whatever the key: advance only
        static_assert(c::kNumWeaponTypes == 1, "weapon draw shortcut assumes one weapon type");
        base.ctr += 1;
        float hp = 100.f;
        int32_t mag = c::kMagSize;
        if (randomize_hp) {
            int tenth = rngI32(base, 1, 11);
            hp = float(tenth * 10);
            mag = rngI32(base, 0, c::kMagSize);
        }
        if (rec) {
            float *r = rec + ai * kSpawnRec;
            r[0] = spawn_pt.x; r[1] = spawn_pt.y; r[2] = spawn_pt.z; r[3] = spawn_yaw;
            r[4] = hp; r[5] = __int_as_float(mag); r[6] = __int_as_float(rng_ctr);
        } else {
            const int32_t flags = L.flags ? __float_as_int(L.flags[ai]) : S.flags[g];
            spawnApplyD(S, sc, g, is_respawn, spawn_pt, spawn_yaw, rng_ctr, hp, mag, flags, zb);
        }
    }
    // (the caller that continues drawing takes the RNG back instead of
    // reloading it behind every store above)
    if (base_out) *base_out = base;
    else stWRng(S, w, base);
}

// k_sim's respawn (spawnAgents with is_respawn, common respawn points, no
// navmesh spawns) with each dead agent's candidate scoring spread over its
// world's N lanes: one dead agent per world per round, in agent order; every
// lane scores candidates i, i + N, ... exactly as respawnScoreD (same
// summation order), the world lane takes the lowest score (lowest index on
// ties, as the sequential strict-< scan does), draws the spawn point and
// writes the agent's record (spawnApplyRecD on the agent's lane applies it).
// Points taken earlier this step are tracked in LDS (usedL) next to the
// tracker loads, so no lane reads back a tracker entry another lane stored.
// Called by every thread of the block (block barriers).  coop: LDS scratch,
// 4 floats per thread.
__device__ __forceinline__ void respawnCoopD(const DevState &S, const SceneDev &sc, int w, int i, int wl, bool act,
                                             const SpawnLds &L, float *rec, float *coop)
{
    const int N = S.N, T = S.T;
    const int64_t g0 = (int64_t)w * N;
    const int B = (int)blockDim.x;
    float *const bestS = coop;          // per lane: best score
    float *const bestI = coop + B;      // per lane: its index (float bits)
    float *const curA = coop + 2 * B;   // per world: the agent this round (float bits)
    float *const usedL = coop + 3 * B;  // per world: 2 x 32 bits of points taken this step
    const bool wl0 = act && i == 0;
    uint32_t rem = 0;
    RNG base;
    int episode_curr = 0;
    const bool randomize_hp = (sc.simFlags & kFlagRandomizeHP) != 0;
    if (wl0) {
        for (int k = 0; k < N; k++)
            if (!L.alive[k]) rem |= 1u << k;
        if (rem) {
            base = ldWRng(S, w);
            episode_curr = S.episodeCurr[w];
            base.ctr += 1; // episodes[sampleI32(0, 0)] (spawnAgentsD)
            if (sc.simFlags & kFlagSpawnInMiddle) (void)rngUniform(base);
        }
        usedL[2 * wl] = 0.f;
        usedL[2 * wl + 1] = 0.f;
    }
    const uint32_t *rtrack = act ? &S.spawnTrack[(int64_t)w * 3 * sc.spawnTrackLen + 2 * sc.spawnTrackLen] : nullptr;
    uint32_t cur_step = 0u;
    const Spawn *options = L.tabC;
    #pragma unroll 1
    for (;;) {
        int ai = -1;
        if (wl0) {
            ai = rem ? __builtin_ctz(rem) : -1;
            curA[wl] = __int_as_float(ai);
        }
        if (!__syncthreads_or(ai >= 0)) break;
        const int a = act ? __float_as_int(curA[wl]) : -1;
        if (a >= 0) {
            // (read only in blocks with a respawn: most launches have none)
            cur_step = (uint32_t)S.curStep[w];
            const AABB za = sc.tab->zoneAABB[S.curZone[w]];
            const Vec3 zone_center = 0.5f * (za.pMin + za.pMax);
            const uint32_t used0 = (uint32_t)__float_as_int(usedL[2 * wl]), used1 = (uint32_t)__float_as_int(usedL[2 * wl + 1]);
            const int team = a / T;
            float bs = kFltMax;
            int bi = -1;
            #pragma unroll 1
            for (int sp = i; sp < sc.numCommon; sp += N) {
                const bool taken = ((sp < 32 ? used0 : used1) >> (sp & 31)) & 1u;
                const uint32_t last_used = taken ? cur_step : rtrack[sp];
                if (last_used == cur_step) continue;
                const float score = respawnScoreD(S, options, sp, a, team, last_used, cur_step, zone_center, L, g0);
                if (score < bs) {
                    bs = score;
                    bi = sp;
                }
            }
            bestS[threadIdx.x] = bs;
            bestI[threadIdx.x] = __int_as_float(bi);
        }
        __syncthreads();
        if (wl0 && ai >= 0) {
            float best = kFltMax;
            int best_idx = -1;
            for (int k = 0; k < N; k++) {
                const int s_k = __float_as_int(bestI[wl * N + k]);
                if (s_k < 0) continue;
                const float sc_k = bestS[wl * N + k];
                if (sc_k < best || (sc_k == best && s_k < best_idx)) {
                    best = sc_k;
                    best_idx = s_k;
                }
            }
            if (best_idx < 0) best_idx = 0;
            const int64_t g = g0 + ai;
            // standardSpawnPoint's spawnAgent(best_idx), the agent's RNG
            RNG rng = ldRng(S, g);
            const Spawn sp = options[best_idx];
            const float x_rnd = rngUniform(rng), y_rnd = rngUniform(rng), z_rnd = rngUniform(rng);
            const float yaw_rnd = rngUniform(rng);
            const float x_min = sp.region.pMin.x, x_diff = sp.region.pMax.x - x_min;
            const float y_min = sp.region.pMin.y, y_diff = sp.region.pMax.y - y_min;
            const float z_min = sp.region.pMin.z, z_diff = sp.region.pMax.z - z_min;
            Vec3 spawn_pt = v3(x_min + x_rnd * x_diff, y_min + y_rnd * y_diff, z_min + z_rnd * z_diff);
            const float spawn_yaw = sp.yawMin + yaw_rnd * (sp.yawMax - sp.yawMin);
            S.spawnTrack[(int64_t)w * 3 * sc.spawnTrackLen + 2 * sc.spawnTrackLen + best_idx] = cur_step;
            if (best_idx < 32) usedL[2 * wl] = __int_as_float(__float_as_int(usedL[2 * wl]) | (int)(1u << best_idx));
            else usedL[2 * wl + 1] = __int_as_float(__float_as_int(usedL[2 * wl + 1]) | (int)(1u << (best_idx & 31)));
            if ((sc.simFlags & kFlagEnableCurriculum) && episode_curr == 0) {
                // utils.cpp:819-837 LearnShooting
                const bool north = spawn_pt.y > 0.f;
                const float x = -700.f + rngUniform(base) * 1400.f;
                const float y = rngUniform(base) * 350.f;
                spawn_pt = v3(x, north ? y : -y, 0.f);
            }
            L.pos[3 * ai] = spawn_pt.x; L.pos[3 * ai + 1] = spawn_pt.y; L.pos[3 * ai + 2] = spawn_pt.z;
            L.alive[ai] = 1;
            base.ctr += 1; // the weapon draw (spawnAgentsD)
            float hp = 100.f;
            int32_t mag = c::kMagSize;
            if (randomize_hp) {
                int tenth = rngI32(base, 1, 11);
                hp = float(tenth * 10);
                mag = rngI32(base, 0, c::kMagSize);
            }
            float *r = rec + ai * kSpawnRec;
            r[0] = spawn_pt.x; r[1] = spawn_pt.y; r[2] = spawn_pt.z; r[3] = spawn_yaw;
            r[4] = hp; r[5] = __int_as_float(mag); r[6] = __int_as_float((int32_t)rng.ctr);
            rem &= rem - 1u;
            if (rem == 0) stWRng(S, w, base);
        }
        __syncthreads();
    }
}

// level_gen.cpp:330-582 resetPersistentEntities
// resetPersistentEntities, agent i's own part (level_gen.cpp:330-370):
// position, combat RNG split_i(episodeKey, i + 1), combat flags, last-known
// observations, breadcrumb state.
// Returns the agent's flags after the reset.
__device__ __forceinline__ int32_t resetAgentD(const DevState &S, int64_t g, RandKey agent_key)
{
    stPos(S, g, v3(kFltMax, kFltMax, kFltMax));
    stRng(S, g, makeRNG(agent_key));
    S.landedOn[g] = -1;
    S.respawnSteps[g] = 0;
    S.autohealSteps[g] = 0;
    S.wasShot[g] = 0;
    S.firedT[g] = -kFltMax;
    const int32_t flags = S.flags[g] & (kFlagInZone | kFlagInSubZone);
    S.flags[g] = flags;
    S.alive[g] = 0.f;
    float4 *lk = reinterpret_cast<float4 *>(&S.lkObs[g * 6 * kOtherObs]);
    for (int k = 0; k < 6 * kOtherObs / 4; k++) lk[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k = 0; k < 18; k++) S.lkPos[g * 18 + k] = -1000.f;
    S.bcPenalty[g] = 0.f;
    S.bcLast[g] = -1;
    S.bcSteps[g] = 0;
    return flags;
}

// pre != nullptr: every agent's resetAgentD already ran on its own lane and
// pre holds, per agent, its RNG key then kPreDraws draw keys (resetPreD);
// L (k_sim, LDS): the flags resetAgentD left and the spawn lists.
// rec (k_sim, LDS, only without curriculum snapshots): spawn records for
// the agents' lanes, which also do resetAgentTailD.
__device__ __forceinline__ void resetAgentTailD(const DevState &S, int64_t g)
{
    for (int k = 0; k < 4; k++) S.discreteAction[4 * g + k] = 0;
    S.aimAction[2 * g] = 0.f; S.aimAction[2 * g + 1] = 0.f;
    S.newCells[g] = 0;
    float *rc = &S.rewardCoefs[9 * g];
    rc[0] = 0.f; rc[1] = 0.5f; rc[2] = 0.005f; rc[3] = 0.05f; rc[4] = 0.01f;
    rc[5] = 0.1f; rc[6] = 0.0005f; rc[7] = 1.f; rc[8] = 0.1f;
}

__device__ __forceinline__ void resetPersistentEntitiesD(const DevState &S, const SceneDev &sc, int w, RandKey episode_key,
                                         const RandKey *pre = nullptr,
                                         SpawnLds L = SpawnLds{ nullptr, nullptr, nullptr, nullptr, nullptr, nullptr },
                                         float *rec = nullptr, const SpawnWorld *sw_in = nullptr,
                                         const RNG *base_in = nullptr)
{
    const int N = S.N;
    const int64_t g0 = (int64_t)w * N;
    #pragma unroll 1
    for (int i = 0; i < N && !pre; i++) {
        const int64_t g = g0 + i;
        stPos(S, g, v3(kFltMax, kFltMax, kFltMax));
        RNG r = makeRNG(splitI(episode_key, (uint32_t)(i + 1)));
        stRng(S, g, r);
        S.landedOn[g] = -1;
        S.respawnSteps[g] = 0;
        S.autohealSteps[g] = 0;
        S.wasShot[g] = 0;
        S.firedT[g] = -kFltMax;
        S.flags[g] = S.flags[g] & (kFlagInZone | kFlagInSubZone); // successfulKill/wasKilled/hasDied/reloadedFullMag = false
        S.alive[g] = 0.f;
        float4 *lk = reinterpret_cast<float4 *>(&S.lkObs[g * 6 * kOtherObs]);
        for (int k = 0; k < 6 * kOtherObs / 4; k++) lk[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int k = 0; k < 18; k++) S.lkPos[g * 18 + k] = -1000.f;
        S.bcPenalty[g] = 0.f;
        S.bcLast[g] = -1;
        S.bcSteps[g] = 0;
    }
    if (!pre) {
        uint32_t *track = &S.spawnTrack[(int64_t)w * 3 * sc.spawnTrackLen];
        for (int k = 0; k < 3 * sc.spawnTrackLen; k++) track[k] = 0xFFFFFFFFu;
    }
    // every agent is dead here (resetAgentD); spawnAgentsD also stores the
    // start positions sx, sy, sz (= the spawn positions)
    RNG base;
    spawnAgentsD(S, sc, w, false, pre, pre ? (int64_t)((1u << N) - 1u) : -1, L, rec, &base, sw_in, base_in);

    #pragma unroll 1
    for (int i = 0; i < N; i++) {
        if (!rec) resetAgentTailD(S, g0 + i);
        // level_gen.cpp:427-446: nine discarded coefficient draws.
        base.ctr += 9;
    }
    // GoalRegionsState (level_gen.cpp:472-485)
    S.goalMin0[w] = kFltMax;
    S.goalMin1[w] = kFltMax;
    S.goalTeam0[w] = 0.f;
    S.goalTeam1[w] = 0.f;

    // level_gen.cpp:498-580: start from a recorded match state half the time
    // (not in eval mode); the uniform is drawn whenever snapshots exist
    if (sc.numSnapshots > 0 && rngUniform(base) < 0.5f && !S.trainCtrl[0]) {
        const mpenv_curriculum_snapshot &sn = sc.curriculum[rngI32(base, 0, sc.numSnapshots)];
        S.curZone[w] = sn.cur_zone;
        if (sn.cur_zone_controller == -1) {
            S.controlling[w] = -1;
            S.captured[w] = 0;
        } else {
            S.captured[w] = 1;
            S.controlling[w] = sn.cur_zone_controller;
            S.stepsUntilPoint[w] = sn.steps_until_point;
            S.zoneSteps[w] = sn.zone_steps_remaining;
        }
        S.curStep[w] = sn.step;
        const int half = N / 2;
        const int team_a = S.teamA[w];
        #pragma unroll 1
        for (int i = 0; i < N; i++) {
            const int j = team_a == 0 ? i : (i < half ? half + i : i - half);
            const int64_t g = g0 + j;
            const mpenv_packed_player &p = sn.players[i];
            stPos(S, g, v3((float)p.pos[0], (float)p.pos[1], (float)p.pos[2]));
            const AimD aim = computeAimD((float)p.yaw * kPi / 32768.f, (float)p.pitch * kPi / 32768.f);
            stAim(S, g, aim);
            stRot(S, g, qnormalize(angleAxis(aim.yaw, kUp)));
            S.hp[g] = (float)p.hp;
            S.magazine[2 * g] = p.mag_num_bullets;
            S.magazine[2 * g + 1] = p.is_reloading;
            if (p.flags & 4) { S.curPose[g] = kCrouch; S.tgtPose[g] = kCrouch; S.transRem[g] = 0; }
            if (p.flags & 8) { S.curPose[g] = kProne; S.tgtPose[g] = kProne; S.transRem[g] = 0; }
        }
    }
    stWRng(S, w, base);
}

// sim.cpp:732-833 initWorld
__device__ __forceinline__ void initWorldD(const DevState &S, const SceneDev &sc, int w, bool triggered_reset, const int32_t *tc,
                           const RandKey *pre = nullptr,
                           SpawnLds L = SpawnLds{ nullptr, nullptr, nullptr, nullptr, nullptr, nullptr },
                           float *rec = nullptr)
{
    const uint32_t world_id = sc.worldOffset + (uint32_t)w;
    S.matchValid[w] = 1; // matchID = worldID << 32 | curEpisodeIdx (sim.cpp:736-738)
    SpawnWorld sw;
    sw.episodeCurr = S.worldCurr[w];
    S.episodeCurr[w] = sw.episodeCurr;
    const uint32_t ep = (uint32_t)S.episode[w];
    RandKey episode_key = splitI(sc.initRandKey, ep, world_id);
    RNG base = makeRNG(splitI(episode_key, 0));
    bool flip = false;
    if (tc[2]) flip = rngUniform(base) < 0.5f;
    sw.teamA = flip ? 1 : 0;
    S.teamA[w] = sw.teamA;
    const int32_t cur_step = (triggered_reset && tc[1]) ? rngI32(base, 0, c::kEpisodeLen - 1) : 0;
    S.curStep[w] = cur_step;
    sw.curStep = (uint32_t)cur_step;
    S.finished[w] = 0;
    const float use_prob = 1.0f;
    const float tier_probs[5] = { 0.f, 0.f, 0.3f, 0.3f, 0.4f };
    S.spawnCurriculum[w] = rngUniform(base) < use_prob ? 1 : 0;
    float cdf[5];
    float running = 0.f;
    for (int i = 0; i < 5; i++) { running += tier_probs[i]; cdf[i] = running; }
    float sel = running * rngUniform(base);
    for (int i = 0; i < 5; i++) {
        if (sel < cdf[i]) { S.curTier[w] = i; break; }
    }
    S.curSpawnIdx[w] = rngI32(base, 0, 0);
    if (sc.simFlags & kFlagHardcodedSpawns) (void)rngI32(base, 0, 4);
    sw.cz = rngI32(base, 0, sc.numZones);
    if (sc.task == MPENV_TASK_ZONE_CAPTURE_DEFEND) sw.cz = 3; // sim.cpp:822-825
    S.curZone[w] = sw.cz;
    S.controlling[w] = -1;
    S.contested[w] = 0;
    S.captured[w] = 0;
    S.earned[w] = 0;
    S.zoneSteps[w] = c::kNumStepsPerZone;
    S.stepsUntilPoint[w] = c::kZonePointInterval;
    S.subState[w] = 0; // every sub-zone: controlling -1, not contested / captured (sim.cpp:815-820)
    stWRng(S, w, base);
    resetPersistentEntitiesD(S, sc, w, episode_key, pre, L, rec, &sw, &base);
    S.filtAct0[w] = 0; S.filtAct1[w] = 0;
    S.filtMatched0[w] = 0; S.filtMatched1[w] = 0;
}

// sim.cpp:835-872 resetSystem
__device__ __forceinline__ bool resetDueD(const DevState &S, const SceneDev &sc, int w)
{
    return S.reset[w] != 0 || (sc.autoReset && S.finished[w]);
}

// The per-agent half of a coming world reset, on the agent's own lane
// (k_sim, before resetSystemD): the episode key initWorld will derive, the
// agent's combat RNG key split_i(episodeKey, i + 1) and its first kPreDraws
// draw keys into pre[0], pre[1..], the agent's resetPersistentEntities
// stores, and its share of the spawn-usage tracker reset.
// Returns the agent's flags after its reset.
__device__ __forceinline__ int32_t resetPreD(const DevState &S, const SceneDev &sc, int w, int i, RandKey *pre)
{
    const uint32_t world_id = sc.worldOffset + (uint32_t)w;
    const uint32_t ep = (uint32_t)S.episodeCounter[w]; // the episode resetSystemD is about to start
    const RandKey episode_key = splitI(sc.initRandKey, ep, world_id);
    const RandKey key = splitI(episode_key, (uint32_t)(i + 1));
    pre[0] = key;
    for (int c = 0; c < kPreDraws; c++) pre[1 + c] = splitI(key, (uint32_t)c);
    const int32_t flags = resetAgentD(S, (int64_t)w * S.N + i, key);
    uint32_t *track = &S.spawnTrack[(int64_t)w * 3 * sc.spawnTrackLen];
    for (int k = i; k < 3 * sc.spawnTrackLen; k += S.N) track[k] = 0xFFFFFFFFu;
    return flags;
}

__device__ __forceinline__ void resetSystemD(const DevState &S, const SceneDev &sc, int w, const RandKey *pre = nullptr,
                                             SpawnLds L = SpawnLds{ nullptr, nullptr, nullptr, nullptr, nullptr, nullptr },
                                             float *rec = nullptr)
{
    const int32_t force = S.reset[w];
    if (!resetDueD(S, sc, w)) return;
    S.reset[w] = 0;
    const int32_t ep = S.episodeCounter[w];
    S.episode[w] = ep;
    S.episodeCounter[w] = ep + 1;
    if (sc.simFlags & kFlagEnableCurriculum) {
        if ((uint32_t)ep < 50) {
            RNG base = ldWRng(S, w);
            if (rngUniform(base) < ((uint32_t)ep + 1) / (float)50) S.worldCurr[w] = 1;
            else S.worldCurr[w] = 0;
            stWRng(S, w, base);
        } else {
            S.worldCurr[w] = 1;
        }
    }
    initWorldD(S, sc, w, force == 1, S.trainCtrl, pre, L, rec);
}

// ====================================================== per-world systems
// sim.cpp:1892-1976 zoneSystem
__device__ void zoneSystemD(const DevState &S, const SceneDev &sc, int w)
{
    const int N = S.N;
    const int64_t g0 = (int64_t)w * N;
    int cz = S.curZone[w];
    int ctrl = S.controlling[w];
    int zsr = S.zoneSteps[w];
    int sup = S.stepsUntilPoint[w];
    bool captured = S.captured[w] != 0;
    if (ctrl != -1) zsr -= 1;
    if (zsr == 0) {
        cz += 1;
        if (cz == sc.numZones) cz = 0;
        captured = false;
        zsr = c::kNumStepsPerZone;
        sup = c::kZonePointInterval;
        AABB za = sc.tab->zoneAABB[cz];
        Vec3 center = (za.pMax + za.pMin) / 2.f;
#pragma unroll 1
        for (int i = 0; i < N; i++) S.minDistZone[g0 + i] = distance(ldPos(S, g0 + i), center);
    }
    AABB za = sc.tab->zoneAABB[cz];
    Quat to_zone = qinv(angleAxis(sc.tab->zoneRot[cz], kUp));
    za.pMin = rotateVec(to_zone, za.pMin);
    za.pMax = rotateVec(to_zone, za.pMax);
    int na = 0, nb = 0;
#pragma unroll 1
    for (int i = 0; i < N; i++) {
        Vec3 p = ldPos(S, g0 + i);
        p.z += c::kStandHeight / 2.f;
        Vec3 pz = rotateVec(to_zone, p);
        bool in = aabbContains(za, pz);
        setFlag(S, g0 + i, kFlagInZone, in);
        if (!in) continue;
        if (i / S.T == 0) na += 1;
        else nb += 1;
    }
    sup -= 1;
    bool contested = na > 0 && nb > 0;
    if (contested || (na == 0 && nb == 0)) {
        ctrl = -1;
        captured = false;
        sup = c::kZonePointInterval;
    } else if (na > 0 && nb == 0) {
        if (ctrl != 0) { ctrl = 0; captured = false; sup = c::kZonePointInterval; }
    } else if (na == 0 && nb > 0) {
        if (ctrl != 1) { ctrl = 1; captured = false; sup = c::kZonePointInterval; }
    }
    S.curZone[w] = cz;
    S.controlling[w] = ctrl;
    S.zoneSteps[w] = zsr;
    S.stepsUntilPoint[w] = sup;
    S.captured[w] = captured ? 1 : 0;
    S.contested[w] = contested ? 1 : 0;
}

// zoneSystem split for the step kernel: the world lane rotates the zone
// (zonePreD), every agent lane tests itself against the zone box in
// parallel (zoneInD; the world lane walked the N agents one load round trip
// at a time), and the world lane counts the teams and stores (zonePostD).
// Same arithmetic and stores as zoneSystemD, which the replay path keeps.
struct ZonePre {
    int cz, ctrl, zsr, sup;
    bool captured;
};

__device__ __forceinline__ ZonePre zonePreD(const DevState &S, const SceneDev &sc, int w)
{
    const int N = S.N;
    const int64_t g0 = (int64_t)w * N;
    ZonePre z;
    z.cz = S.curZone[w];
    z.ctrl = S.controlling[w];
    z.zsr = S.zoneSteps[w];
    z.sup = S.stepsUntilPoint[w];
    z.captured = S.captured[w] != 0;
    if (z.ctrl != -1) z.zsr -= 1;
    if (z.zsr == 0) {
        z.cz += 1;
        if (z.cz == sc.numZones) z.cz = 0;
        z.captured = false;
        z.zsr = c::kNumStepsPerZone;
        z.sup = c::kZonePointInterval;
        AABB za = sc.tab->zoneAABB[z.cz];
        Vec3 center = (za.pMax + za.pMin) / 2.f;
#pragma unroll 1
        for (int i = 0; i < N; i++) S.minDistZone[g0 + i] = distance(ldPos(S, g0 + i), center);
    }
    return z;
}

__device__ __forceinline__ bool zoneInD(const DevState &S, const SceneDev &sc, int cz, int64_t g)
{
    const FrameDev &f = sc.tab->zoneFrame[cz];
    AABB za;
    za.pMin = f.pMin;
    za.pMax = f.pMax;
    Vec3 p = ldPos(S, g);
    p.z += c::kStandHeight / 2.f;
    const bool in = aabbContains(za, rotateVec(f.toFrame, p));
    setFlag(S, g, kFlagInZone, in);
    return in;
}

__device__ __forceinline__ void zonePostD(const DevState &S, int w, ZonePre z, int na, int nb)
{
    z.sup -= 1;
    bool contested = na > 0 && nb > 0;
    if (contested || (na == 0 && nb == 0)) {
        z.ctrl = -1;
        z.captured = false;
        z.sup = c::kZonePointInterval;
    } else if (na > 0 && nb == 0) {
        if (z.ctrl != 0) { z.ctrl = 0; z.captured = false; z.sup = c::kZonePointInterval; }
    } else if (na == 0 && nb > 0) {
        if (z.ctrl != 1) { z.ctrl = 1; z.captured = false; z.sup = c::kZonePointInterval; }
    }
    S.curZone[w] = z.cz;
    S.controlling[w] = z.ctrl;
    S.zoneSteps[w] = z.zsr;
    S.stepsUntilPoint[w] = z.sup;
    S.captured[w] = z.captured ? 1 : 0;
    S.contested[w] = contested ? 1 : 0;
}

// SubZone state packed 4 bits per sub-zone k at bit 4k: controlling team + 1,
// contested << 2, captured << 3 (the DEBUG_WORLD_I32 layout).
__device__ __forceinline__ int subCtrlD(uint32_t st, int k) { return (int)((st >> (4 * k)) & 3u) - 1; }

// sim.cpp:1978-2041 subzoneSystem over sub-zones 0..7
__device__ void subzoneSystemD(const DevState &S, const SceneDev &sc, int w)
{
    const int N = S.N;
    const int64_t g0 = (int64_t)w * N;
    uint32_t st = (uint32_t)S.subState[w];
    for (int k = 0; k < 8; k++) {
        const ZOBBDev &sz = sc.tab->subZones[k];
        AABB za = { sz.pMin, sz.pMax };
        Quat to_zone = qinv(angleAxis(sz.rotation, kUp));
        za.pMin = rotateVec(to_zone, za.pMin);
        za.pMax = rotateVec(to_zone, za.pMax);
        int na = 0, nb = 0;
        #pragma unroll 1
        for (int i = 0; i < N; i++) {
            const int64_t g = g0 + i;
            if (subZoneIndexD(S, g) != k) continue;
            Vec3 p = ldPos(S, g);
            p.z += c::kStandHeight / 2.f;
            const bool in = aabbContains(za, rotateVec(to_zone, p));
            setFlag(S, g, kFlagInSubZone, in);
            if (!in) continue;
            S.minDistSub[g] = 0.f;
            if (i / S.T == 0) na += 1;
            else nb += 1;
        }
        int ctrl = subCtrlD(st, k);
        bool captured = (st >> (4 * k + 3)) & 1u;
        const bool contested = na > 0 && nb > 0;
        if (contested || (na == 0 && nb == 0)) {
            ctrl = -1;
            captured = false;
        } else if (na > 0 && nb == 0) {
            if (ctrl != 0) { ctrl = 0; captured = false; }
        } else if (na == 0 && nb > 0) {
            if (ctrl != 1) { ctrl = 1; captured = false; }
        }
        const uint32_t nib = (uint32_t)(ctrl + 1) | (contested ? 4u : 0u) | (captured ? 8u : 0u);
        st = (st & ~(0xFu << (4 * k))) | (nib << (4 * k));
    }
    S.subState[w] = (int32_t)st;
}

__device__ __forceinline__ float4 *crumbPtr(const DevState &S, int w) { return &S.crumbs[(int64_t)w * kMaxCrumbs * 2]; }

// sim.cpp:4845-4889 leaveBreadcrumbsSystem, agent part: refresh own last
// crumb or request a new one (returns true; appended in agent order by the
// world lane, the requests handed over in LDS).  The penalty's reset to 0
// is crumbRoundsD's starting value (the two always run together).
__device__ bool leaveBreadcrumbAgentD(const DevState &S, int w, int64_t g)
{
    const Vec3 pos = ldPos(S, g);
    const int32_t last = S.bcLast[g];
    bool updated = false;
    if (last != -1) {
        float4 *cr = crumbPtr(S, w);
        const int n = S.numCrumbs[w];
        // the first crumb with id `last`, its ids read 8 at a time (one
        // round of loads per 8 crumbs; past the end re-reads the last)
        constexpr int kIds = 8;
        int hit = -1;
        #pragma unroll 1
        for (int k0 = 0; k0 < n && hit < 0; k0 += kIds) {
            int id[kIds];
            #pragma unroll
            for (int j = 0; j < kIds; j++) id[j] = __float_as_int(cr[2 * min(k0 + j, n - 1) + 1].z);
            #pragma unroll
            for (int j = kIds - 1; j >= 0; j--)
                if (k0 + j < n && id[j] == last) hit = k0 + j;
        }
        if (hit >= 0) {
            const float4 p = cr[2 * hit];
            if (distance(pos, v3(p.x, p.y, p.z)) < c::kAgentRadius * 4) {
                cr[2 * hit].w = 1.f;
                updated = true;
                S.bcSteps[g] = 0;
            }
        }
    }
    bool request = false;
    if (!updated) {
        int steps = S.bcSteps[g] + 1;
        if (steps > 10) {
            request = true;
            steps = 0;
        }
        S.bcSteps[g] = steps;
    }
    return request;
}

// World part of leaveBreadcrumbsSystem: append requested crumbs in agent
// order (req: bit i = agent i asked, from leaveBreadcrumbAgentD; lpos: the
// world's agents' positions [N][3] in LDS).
__device__ void appendCrumbsD(const DevState &S, int w, uint32_t req, const float *lpos)
{
    if (req == 0) return;
    const int N = S.N;
    const int64_t g0 = (int64_t)w * N;
    float4 *cr = crumbPtr(S, w);
    int n = S.numCrumbs[w];
    int next_id = S.nextCrumbId[w];
    #pragma unroll 1
    for (int i = 0; i < N; i++) {
        const int64_t g = g0 + i;
        if (!(req & (1u << i))) continue;
        if (n < kMaxCrumbs) {
            const int team = i / S.T, off = i - team * S.T;
            cr[2 * n] = make_float4(lpos[3 * i], lpos[3 * i + 1], lpos[3 * i + 2], 1.f);
            cr[2 * n + 1] = make_float4((float)team, (float)off, __int_as_float(next_id), 0.f);
            S.bcLast[g] = next_id;
            next_id += 1;
            n += 1;
        } else {
            S.crumbOverflow[w] += 1;
            S.bcLast[g] = -1;
        }
    }
    S.numCrumbs[w] = n;
    S.nextCrumbId[w] = next_id;
}

// sim.cpp:4892-4926 accumulateBreadcrumbPenaltiesSystem, with its decay and
// compaction of the world's crumbs, by the world's N agent lanes together
// (called by every thread of the block: it has block barriers).  Each round
// the lanes load N consecutive crumbs into LDS (buf: 2 float4 per lane);
// every agent adds the round's crumbs to its penalty in creation order, and
// each lane decays its own crumb and, if it survives, stores it at its
// compacted slot (the survivors before it: earlier rounds' plus this
// round's lower lanes).  Stores only go to slots at or below the round being
// read, whose crumbs are already in LDS.
__device__ __forceinline__ void crumbRoundsD(const DevState &S, int w, int i, bool act, int wl, float4 *buf)
{
    const int N = S.N;
    const int64_t g = (int64_t)w * N + i;
    const int team = i / S.T, off = i - team * S.T;
    float4 *cr = act ? crumbPtr(S, w) : nullptr;
    const int n = act ? S.numCrumbs[w] : 0;
    const Vec3 pos = act ? ldPos(S, g) : v3(0.f, 0.f, 0.f);
    float total = 0.f; // leaveBreadcrumbsSystem's reset (sim.cpp:4845-4889)
    int kept = 0;      // survivors of the earlier rounds
    const float4 *wb = buf + 2 * wl * N;
    // the next round's crumb is loaded while this round runs: it sits at a
    // slot >= r0 + N, which no store of this round (slots < r0 + N) touches
    float4 pn = make_float4(0.f, 0.f, 0.f, 0.f), mn = pn;
    if (i < n) {
        pn = cr[2 * i];
        mn = cr[2 * i + 1];
    }
    #pragma unroll 1
    for (int r0 = 0; __syncthreads_or(r0 < n); r0 += N) {
        const int k = r0 + i;
        float4 p = make_float4(0.f, 0.f, 0.f, 0.f), meta = p;
        if (k < n) {
            p = pn;
            meta = mn;
            buf[2 * threadIdx.x] = p;
            buf[2 * threadIdx.x + 1] = meta;
        }
        if (k + N < n) {
            pn = cr[2 * (k + N)];
            mn = cr[2 * (k + N) + 1];
        }
        __syncthreads();
        if (r0 < n) {
            const int cnt = min(N, n - r0);
            int before = 0, round_kept = 0;
            #pragma unroll 1
            for (int j = 0; j < cnt; j++) {
                const float4 pj = wb[2 * j], mj = wb[2 * j + 1];
                if (!((int)mj.x != team || (int)mj.y == off))
                    if (distance(pos, v3(pj.x, pj.y, pj.z)) <= c::kAgentRadius * 4.f) total += pj.w;
                const bool keep = !(pj.w - 0.025f <= 0.f);
                round_kept += keep ? 1 : 0;
                if (j < i && keep) before += 1;
            }
            if (k < n) {
                p.w -= 0.025f;
                if (!(p.w <= 0.f)) {
                    const int m = kept + before;
                    cr[2 * m] = p;
                    cr[2 * m + 1] = meta;
                }
            }
            kept += round_kept;
        }
    }
    if (act) {
        S.bcPenalty[g] = total;
        if (i == 0) S.numCrumbs[w] = kept;
    }
}

// Filter boxes of updateFiltersState (sim.cpp:128-291): x/y ranges of the
// three hard-coded analytics filters.
__constant__ const int16_t kFiltMinX[3] = { -1272, 852, -32768 }, kFiltMinY[3] = { -866, -851, -32768 };
__constant__ const int16_t kFiltMaxX[3] = { -825, 1280, 32767 }, kFiltMaxY[3] = { 696, 593, 32767 };

__device__ __forceinline__ bool inFilterBoxD(Vec3 p, int fi)
{
    return !(p.x < kFiltMinX[fi] || p.y < kFiltMinY[fi] || p.x > kFiltMaxX[fi] || p.y > kFiltMaxY[fi]);
}

// What zoneMatchInfoSystem + updateFiltersState read per agent, computed by
// the agent's own lane (all in parallel) and handed to the world lane
// through LDS: bit 0 wasKilled, 1 hasDiedDuringEpisode, 2 / 3 inside filter
// box 0 / 1, 4 a landed shot with shooter and target inside filter box 2.
enum : uint32_t { kMbKilled = 1, kMbDied = 2, kMbF0 = 4, kMbF1 = 8, kMbF2 = 16 };

__device__ __forceinline__ uint32_t matchAgentBitsD(const DevState &S, int w, int i)
{
    const int64_t g0 = (int64_t)w * S.N, g = g0 + i;
    const int32_t f = S.flags[g];
    uint32_t b = 0;
    if (f & kFlagWasKilled) b |= kMbKilled;
    if (f & kFlagHasDied) b |= kMbDied;
    const Vec3 p = ldPos(S, g);
    if (inFilterBoxD(p, 0)) b |= kMbF0;
    if (inFilterBoxD(p, 1)) b |= kMbF1;
    const int lo = S.landedOn[g];
    if (lo != -1 && inFilterBoxD(p, 2) && inFilterBoxD(ldPos(S, g0 + lo), 2)) b |= kMbF2;
    return b;
}

// Agent bit masks (bit i = agent i of the world) from the LDS bytes.
struct MatchMasks {
    uint32_t killed, died, f0, f1, f2;
};

__device__ __forceinline__ MatchMasks matchMasksD(const uint8_t *mb, int N)
{
    MatchMasks m = { 0u, 0u, 0u, 0u, 0u };
    #pragma unroll 1
    for (int i = 0; i < N; i++) {
        const uint32_t b = mb[i];
        m.killed |= ((b & kMbKilled) ? 1u : 0u) << i;
        m.died |= ((b & kMbDied) ? 1u : 0u) << i;
        m.f0 |= ((b & kMbF0) ? 1u : 0u) << i;
        m.f1 |= ((b & kMbF1) ? 1u : 0u) << i;
        m.f2 |= ((b & kMbF2) ? 1u : 0u) << i;
    }
    return m;
}

// sim.cpp:128-291 updateFiltersState from the world's agent bits.  The
// filter state is read once (by the caller, with its other loads: last[6]
// [team][filter], act[2]) and written once.
struct FilterState {
    int32_t last[6];
    uint32_t act[2];
};

__device__ __forceinline__ FilterState loadFiltersD(const DevState &S, int w)
{
    FilterState f;
    const int32_t *lastp = &S.filtLast[(int64_t)w * 6];
    for (int k = 0; k < 6; k++) f.last[k] = lastp[k];
    f.act[0] = (uint32_t)S.filtAct0[w];
    f.act[1] = (uint32_t)S.filtAct1[w];
    return f;
}

__device__ __forceinline__ void updateFiltersBitsD(const DevState &S, int w, int cur_step, const MatchMasks &mm,
                                                   FilterState fs)
{
    const int T = S.T;
    int32_t *lastp = &S.filtLast[(int64_t)w * 6]; // [team][filter]
    int32_t *last = fs.last;
    uint32_t *act = fs.act;
    const uint32_t team0 = (1u << T) - 1u, team1 = team0 << T;
    const int min_num[2] = { 5, 1 };
    for (int fi = 0; fi < 3; fi++) {
        for (int t = 0; t < 2; t++) {
            if (act[t] & (1u << fi)) {
                if (cur_step - last[t * 3 + fi] > 0) act[t] &= ~(1u << fi);
            }
        }
        if (fi == 2) {
            // any landed shot inside box 2 activates the shooter's team
            for (int t = 0; t < 2; t++) {
                if (mm.f2 & (t == 0 ? team0 : team1)) {
                    act[t] |= 1u << fi;
                    last[t * 3 + fi] = cur_step;
                }
            }
        } else {
            const uint32_t in = fi == 0 ? mm.f0 : mm.f1;
            const int cnt[2] = { __builtin_popcount(in & team0), __builtin_popcount(in & team1) };
            for (int t = 0; t < 2; t++) {
                if (cnt[t] >= min_num[fi]) {
                    act[t] |= 1u << fi;
                    last[t * 3 + fi] = cur_step;
                }
            }
        }
    }
    for (int k = 0; k < 6; k++) lastp[k] = last[k];
    S.filtAct0[w] = (int32_t)act[0];
    S.filtAct1[w] = (int32_t)act[1];
    if (__builtin_popcount(act[0]) == 3) S.filtMatched0[w] = cur_step;
    if (__builtin_popcount(act[1]) == 3) S.filtMatched1[w] = cur_step;
}

// sim.cpp:4470-4673 zoneMatchInfoSystem
__device__ void writeSnapshotD(const DevState &S, const SceneDev &sc, int w, bool new_captured);

// Run by one lane per world: every world value it reads is loaded up front
// and the results are stored once at the end, so its global accesses are a
// couple of round trips (the agent bytes come from LDS as a char pointer,
// which may alias anything: read-modify-writes through memory next to them
// were reloaded after every LDS read).  The snapshot (events mode) reads
// captured / stepsUntilPoint after this step's update, curStep before it.
__device__ __forceinline__ void zoneMatchInfoD(const DevState &S, const SceneDev &sc, int w, const uint8_t *mb)
{
    const int N = S.N, T = S.T;
    int32_t *mr = &S.matchResult[(int64_t)w * 30];
    int32_t *zs_all = &S.zoneStats[(int64_t)w * 25];
    const MatchMasks mm = matchMasksD(mb, N);
    const int cur_step = S.curStep[w] + 1;
    const int reset_w = S.reset[w];
    int m[5] = { mr[0], mr[1], mr[2], mr[3], mr[4] };
    const int ctrl = S.controlling[w];
    int sup = S.stepsUntilPoint[w];
    bool captured = S.captured[w] != 0;
    const int cz = S.curZone[w];
    const bool contested = S.contested[w] != 0;
    const int team_a = S.teamA[w];
    int32_t *zs = &zs_all[cz * 5];
    int z[5] = { zs[0], zs[1], zs[2], zs[3], zs[4] };
    const FilterState fs = loadFiltersD(S, w); // before this function's stores

    bool finished = cur_step >= c::kEpisodeLen || reset_w == 1;
    if (cur_step == 1) {
        m[0] = -1; m[1] = 0; m[2] = 0; m[3] = 0; m[4] = 0;
    }
    const uint32_t team0 = (1u << T) - 1u, team1 = team0 << T;
    // a killed agent of team t scores for team t ^ 1 (mr[1 + (t ^ 1)])
    m[2] += __builtin_popcount(mm.killed & team0);
    m[1] += __builtin_popcount(mm.killed & team1);
    bool earned = false;
    bool new_captured = false;
    if (sup == 0) {
        sup = c::kZonePointInterval;
        if (!captured) {
            captured = true;
            new_captured = true;
        }
        if (ctrl >= 0) m[3 + ctrl] += 1;
        earned = true;
    }
    if (m[3] >= c::kZoneWinPoints || m[4] >= c::kZoneWinPoints) finished = true;
    // sim.cpp:4534-4575: ZoneCaptureDefend ends on the attacker's first
    // point, the defender's 8th, or when every attacker has died once
    const bool zcd = sc.task == MPENV_TASK_ZONE_CAPTURE_DEFEND;
    const int attacker = team_a == 1 ? 1 : 0, defender = attacker ^ 1;
    bool attackers_all_died = true;
    if (zcd) {
        if (m[3 + attacker] == 1) finished = true;
        if (m[3 + defender] == 8) finished = true;
        const uint32_t am = attacker == 0 ? team0 : team1;
        attackers_all_died = (mm.died & am) == am;
        if (attackers_all_died) finished = true;
    }
    z[4] += 1;
    if (captured && ctrl >= 0) z[1 + ctrl] += 1;
    if (contested) z[3] += 1;
    if (new_captured) z[0] += 1;

    S.stepsUntilPoint[w] = sup;
    S.captured[w] = captured ? 1 : 0;
    S.earned[w] = earned ? 1 : 0;
    for (int k = 0; k < 5; k++) zs[k] = z[k];
    updateFiltersBitsD(S, w, cur_step, mm, fs);
    if (sc.eventsOn) writeSnapshotD(S, sc, w, new_captured);
    if (finished) {
        if (zcd) {
            if (m[3 + attacker] == 1) m[0] = attacker;
            else if (m[3 + defender] == 8 || attackers_all_died) m[0] = defender;
            else m[0] = 2;
        } else if (m[3] > m[4]) m[0] = 0;
        else if (m[4] > m[3]) m[0] = 1;
        else m[0] = 2;
        // every zone's stats in one round of loads, then the stores (one
        // load-store pair per entry waited for each store before the next load)
        int32_t zv[25];
        #pragma unroll
        for (int k = 0; k < 25; k++) zv[k] = zs_all[k];
        #pragma unroll
        for (int k = 0; k < 25; k++) mr[5 + k] = zv[k];
        #pragma unroll
        for (int k = 0; k < 25; k++) zs_all[k] = 0;
    }
    for (int k = 0; k < 5; k++) mr[k] = m[k];
    S.curStep[w] = cur_step;
    S.finished[w] = finished ? 1 : 0;
}

// Capture event + writePackedStepSnapshot (sim.cpp:4592-4634, 41-106).  The
// reference's per-world eventLoggedInStep / eventMask accumulate from every
// logEvent since the last snapshot; here they are folded in from this
// step's event slots, and reset when a snapshot is written (only for a
// valid matchID, i.e. after the first triggered reset).
__device__ void writeSnapshotD(const DevState &S, const SceneDev &sc, int w, bool new_captured)
{
    const int N = S.N;
    const int64_t g0 = (int64_t)w * N;
    const bool valid = S.matchValid[w] != 0;
    if (valid && new_captured) {
        const int cz = S.curZone[w];
        AABB za = sc.tab->zoneAABB[cz];
        Quat to_zone = qinv(angleAxis(sc.tab->zoneRot[cz], kUp));
        za.pMin = rotateVec(to_zone, za.pMin);
        za.pMax = rotateVec(to_zone, za.pMax);
        uint32_t mask = 0;
        const int ctrl = S.controlling[w];
        #pragma unroll 1
        for (int i = 0; i < N; i++) {
            if (i / S.T != ctrl) continue;
            Vec3 p = ldPos(S, g0 + i);
            p.z += c::kStandHeight / 2.f;
            if (aabbContains(za, rotateVec(to_zone, p))) mask |= 1u << i;
        }
        putEventD(S, sc, w, 2 * N, MPENV_EVENT_CAPTURE, cz, ctrl, (int)mask);
    }
    int32_t logged = S.evLogged[w], emask = S.evMask[w];
    const mpenv_game_event *ev = &S.events[(int64_t)w * S.evStride];
    for (int k = 0; k < S.evStride; k++) {
        if (ev[k].type != 0) {
            logged = 1;
            emask |= (int32_t)ev[k].type;
        }
    }
    if (!valid) {
        S.evLogged[w] = logged;
        S.evMask[w] = emask;
        S.snapWritten[w] = 0;
        return;
    }
    mpenv_packed_step_snapshot sn;
    sn.num_events = (uint32_t)logged;
    sn.event_mask = (uint32_t)emask;
    sn.match_id = matchIdD(S, sc, w);
    sn.step = (uint16_t)S.curStep[w];
    sn.cur_zone = (uint8_t)S.curZone[w];
    sn.cur_zone_controller = (int8_t)(S.captured[w] ? S.controlling[w] : -1);
    sn.zone_steps_remaining = (uint16_t)S.zoneSteps[w];
    sn.steps_until_point = (uint16_t)S.stepsUntilPoint[w];
    for (int i = 0; i < kMaxAgents; i++) {
        mpenv_packed_player &pl = sn.players[i];
        if (i >= N) {
            pl = mpenv_packed_player {};
            continue;
        }
        const int64_t g = g0 + i;
        // float -> i16 through i32 (in range except yaw == +pi, which wraps)
        pl.pos[0] = (int16_t)(int32_t)S.px[g];
        pl.pos[1] = (int16_t)(int32_t)S.py[g];
        pl.pos[2] = (int16_t)(int32_t)S.pz[g];
        pl.yaw = (int16_t)(int32_t)(S.ayaw[g] * 32768 / kPi);
        pl.pitch = (int16_t)(int32_t)(S.apitch[g] * 32768 / kPi);
        pl.mag_num_bullets = (uint8_t)(uint16_t)S.magazine[2 * g];
        pl.is_reloading = (uint8_t)S.magazine[2 * g + 1];
        pl.hp = (uint8_t)S.hp[g];
        uint8_t fl = 0;
        if (S.landedOn[g] != -1) fl |= 2;
        if (S.curPose[g] == kCrouch) fl |= 4;
        else if (S.curPose[g] == kProne) fl |= 8;
        pl.flags = fl;
    }
    S.snapshots[w] = sn;
    S.evLogged[w] = 0;
    S.evMask[w] = 0;
    S.snapWritten[w] = 1;
}

// pvpRecordSystem (sim.cpp:4750-4792): per agent lane + curStep by the world lane
__device__ void recordAgentD(const DevState &S, int w, int i)
{
    const int64_t g = (int64_t)w * S.N + i;
    mpenv_agent_log &a = S.recordLog[w].agents[i];
    a.position[0] = S.px[g]; a.position[1] = S.py[g]; a.position[2] = S.pz[g];
    a.aim_yaw = S.ayaw[g];
    a.aim_pitch = S.apitch[g];
    a.aim_rot[0] = S.aw[g]; a.aim_rot[1] = S.ax[g]; a.aim_rot[2] = S.ay[g]; a.aim_rot[3] = S.az[g];
    a.hp = S.hp[g];
    a.mag_num_bullets = S.magazine[2 * g];
    a.mag_is_reloading = S.magazine[2 * g + 1];
    a.cur_pose = S.curPose[g];
    a.tgt_pose = S.tgtPose[g];
    a.transition_remaining = S.transRem[g];
    a.shot_agent_idx = S.landedOn[g];
    a.fired_shot_t = S.firedT[g];
    a.was_killed = (S.flags[g] & kFlagWasKilled) ? 1 : 0;
    a.successful_kill = (S.flags[g] & kFlagSuccessfulKill) ? 1 : 0;
    a.pad_[0] = 0;
    a.pad_[1] = 0;
}

// pvpReplaySystem (sim.cpp:4794-4843) for one agent (shot visualisation,
// viewer-only, is skipped)
__device__ void replayAgentD(const DevState &S, int w, int i)
{
    const int64_t g = (int64_t)w * S.N + i;
    const mpenv_agent_log &a = S.replayLog[w].agents[i];
    S.px[g] = a.position[0]; S.py[g] = a.position[1]; S.pz[g] = a.position[2];
    S.ayaw[g] = a.aim_yaw;
    S.apitch[g] = a.aim_pitch;
    S.aw[g] = a.aim_rot[0]; S.ax[g] = a.aim_rot[1]; S.ay[g] = a.aim_rot[2]; S.az[g] = a.aim_rot[3];
    stRot(S, g, qnormalize(angleAxis(a.aim_yaw, kUp)));
    S.hp[g] = a.hp;
    S.magazine[2 * g] = a.mag_num_bullets;
    S.magazine[2 * g + 1] = a.mag_is_reloading;
    S.curPose[g] = a.cur_pose;
    S.tgtPose[g] = a.tgt_pose;
    S.transRem[g] = a.transition_remaining;
    S.landedOn[g] = a.shot_agent_idx;
    S.firedT[g] = a.fired_shot_t;
    int32_t fl = S.flags[g] & ~(kFlagWasKilled | kFlagSuccessfulKill);
    if (a.was_killed) fl |= kFlagWasKilled | kFlagHasDied;
    if (a.successful_kill) fl |= kFlagSuccessfulKill;
    S.flags[g] = fl;
}

// sim.cpp:3998-4087 distToZOBB + evaluateGoalRegionsSystem
// distToZOBB (sim.cpp:3998-4020) with the frame precomputed (k_scene_frames)
__device__ __forceinline__ float distToFrameD(const FrameDev &f, Vec3 pos)
{
    const Vec3 p = rotateVec(f.toFrame, pos);
    float sq = 0.f;
    for (int i = 0; i < 3; i++) {
        float v = comp(p, i);
        if (v < comp(f.pMin, i)) { float d = comp(f.pMin, i) - v; sq += d * d; }
        if (v > comp(f.pMax, i)) { float d = v - comp(f.pMax, i); sq += d * d; }
    }
    return sqrt_(sq);
}

// Agent lanes: the agent's distance to each sub-region of the goals its team
// is scored on (the world lane's inner loop, spread over the agents);
// d[r * 3 + s], unused entries left alone.
__device__ __forceinline__ void goalDistAgentD(const DevState &S, const SceneDev &sc, int w, int i, Vec3 pos, float *d)
{
    const int attacker = S.teamA[w];
    const int team = i / S.T;
    for (int r = 0; r < sc.numGoals && r < 2; r++) {
        const GoalRegionDev &gr = sc.tab->goals[r];
        const int region_team = gr.attackerTeam ? attacker : (attacker ^ 1);
        if (team != region_team) continue;
        for (int s = 0; s < gr.numSub; s++) d[r * 3 + s] = distToFrameD(sc.tab->goalFrame[r][s], pos);
    }
}

// gd: the world's agents' goalDistAgentD rows in LDS (stride 6).
__device__ __forceinline__ void goalRegionsD(const DevState &S, const SceneDev &sc, int w, const float *gd)
{
    const int N = S.N;
    float team_step[2] = { 0.f, 0.f };
    float mins[2] = { S.goalMin0[w], S.goalMin1[w] };
    const int attacker = S.teamA[w];
    for (int r = 0; r < sc.numGoals && r < 2; r++) {
        const GoalRegionDev &gr = sc.tab->goals[r];
        const int region_team = gr.attackerTeam ? attacker : (attacker ^ 1);
        float max_min = -kFltMax;
        for (int s = 0; s < gr.numSub; s++) {
            float min_d = kFltMax;
            #pragma unroll 1
            for (int i = 0; i < N; i++) {
                if (i / S.T != region_team) continue;
                float d = gd[i * 6 + r * 3 + s];
                if (d < min_d) min_d = d;
            }
            if (min_d > max_min) max_min = min_d;
        }
        float prev = mins[r];
        if (prev == kFltMax) {
            mins[r] = max_min;
        } else {
            float diff = prev - max_min;
            if (diff > 0.f) {
                mins[r] = max_min;
                team_step[region_team] += diff * gr.rewardStrength;
            }
        }
    }
    S.goalMin0[w] = mins[0];
    S.goalMin1[w] = mins[1];
    S.goalTeam0[w] = team_step[0];
    S.goalTeam1[w] = team_step[1];
}

// sim.cpp:3508-3536 exploreVisitedSystem.  The reference keeps a u32
// episode tag per cell and counts a cell when its tag differs from the
// current episode index, then stores the index.  Tags only ever take the
// current, increasing index (curEpisodeIdx = worldEpisodeCounter++), so
// "tag == current episode" is all the state that matters: one bit per cell
// for the agent's episode exploreEp, cleared when the episode moves on
// (lazily, here).  Episode 0 starts from level_gen.cpp:166-171's tags: 0 on
// cells outside the y<40, x<40 quadrant, i.e. already set (k_init_explore).
// Bits live in 8 x 8-cell u64 tiles; the current tile is cached in SoA
// columns and written back to the row when the agent leaves it.
__device__ __forceinline__ int exploreBitD(int cx, int cy) { return (cy & 7) * 8 + (cx & 7); }
__device__ __forceinline__ int exploreTileD(int cx, int cy) { return (cy >> 3) * kExploreTilesX + (cx >> 3); }

__device__ void exploreVisitedD(const DevState &S, int w, int64_t g)
{
    Vec3 delta = ldPos(S, g) - v3(S.sx[g], S.sy[g], S.sz[g]);
    int32_t x = f2iSatD((delta.x + 0.5f) / (c::kAgentRadius * 2.f));
    int32_t y = f2iSatD((delta.y + 0.5f) / (c::kAgentRadius * 2.f));
    int64_t cx = (int64_t)x + c::kGridMax, cy = (int64_t)y + c::kGridMax;
    if (cx < 0 || cx >= kGridW || cy < 0 || cy >= kGridW) return;
    uint64_t *row = &S.exploreBits[g * kExploreTiles];
    const int32_t cur = S.episode[w];
    int32_t tile = S.exploreTile[g];
    uint64_t word = (uint64_t)(uint32_t)S.exploreLo[g] | ((uint64_t)(uint32_t)S.exploreHi[g] << 32);
    if (S.exploreEp[g] != cur) {
        for (int k = 0; k < kExploreTiles; k++) row[k] = 0ull;
        S.exploreEp[g] = cur;
        tile = -1;
    }
    const int t = exploreTileD((int)cx, (int)cy);
    if (t != tile) {
        if (tile >= 0) row[tile] = word;
        word = row[t];
        tile = t;
        S.exploreTile[g] = t;
    }
    const uint64_t bit = 1ull << exploreBitD((int)cx, (int)cy);
    if (!(word & bit)) {
        word |= bit;
        if (length2(delta) > 2.f) S.newCells[g] += 1;
    }
    S.exploreLo[g] = (int32_t)(uint32_t)word;
    S.exploreHi[g] = (int32_t)(uint32_t)(word >> 32);
}

// sim.cpp:4089-4200 zoneCaptureDefendRewardSystem: goal-region progress,
// kills and control of the zone by the agent's own team, +-20 / -5 at the
// end of the match; no curriculum, breadcrumb or area terms.
__device__ float zoneCaptureDefendRewardD(const DevState &S, const SceneDev &sc, int w, int i)
{
    const int64_t g = (int64_t)w * S.N + i;
    const int team = i / S.T;
    int32_t flags = S.flags[g];
    const float *rc = &S.rewardCoefs[9 * g];
    const float shot = rc[1], explore = rc[2], ctrl_s = rc[5], earned_s = rc[7];
    float r = 0.f;
    r += 0.02f * (team == 0 ? S.goalTeam0[w] : S.goalTeam1[w]);
    if (flags & kFlagReloadedFullMag) r -= 0.01f;
    if (flags & kFlagSuccessfulKill) r += 1.f;
    if (S.landedOn[g] != -1) r += shot * 1.f;
    if (flags & kFlagWasKilled) r -= 1.f;
    if (S.wasShot[g] > 0) r -= shot * 1.f;
    uint32_t nn = (uint32_t)S.newCells[g];
    S.newCells[g] = 0;
    if (nn > 0) r += float(nn) * explore;
    if (!(flags & kFlagInZone)) {
        AABB za = sc.tab->zoneAABB[S.curZone[w]];
        Vec3 center = (za.pMax + za.pMin) / 2.f;
        float dist = distance(center, ldPos(S, g));
        if (dist < S.minDistZone[g]) S.minDistZone[g] = dist;
    }
    const int ctrl = S.controlling[w];
    if (ctrl != -1 && ctrl == team) {
        r += ctrl_s;
        if (S.earned[w]) r += earned_s;
    }
    if (S.finished[w]) {
        const int win = S.matchResult[(int64_t)w * 30];
        if (win == 2) r -= 5.f;
        else if (win == team) r += 20.f;
        else r -= 20.f;
    }
    if (S.alive[g] == 0.f) {
        S.flags[g] = flags & ~(kFlagSuccessfulKill | kFlagWasKilled);
        S.landedOn[g] = -1;
        S.wasShot[g] = 0;
        S.firedT[g] = -kFltMax;
    }
    S.reward[g] = r;
    return r;
}

// sim.cpp:3734-3847 subzoneRewardSystem (after the LearnShooting branch,
// which zoneRewardD handles for both): kills pay 3, the agent's own
// sub-zone drives the in-zone / approach / control terms, no earned-point
// or area terms.
__device__ float subzoneRewardD(const DevState &S, const SceneDev &sc, int w, int i)
{
    const int64_t g = (int64_t)w * S.N + i;
    int32_t flags = S.flags[g];
    const int landed = S.landedOn[g];
    const float *rc = &S.rewardCoefs[9 * g];
    const float shot = rc[1], explore = rc[2], in_zone = rc[3], ctrl_s = rc[5], zdist = rc[6], crumb = rc[8];
    float r = 0.f;
    r -= crumb * S.bcPenalty[g];
    if (flags & kFlagReloadedFullMag) r -= 0.5f;
    if (flags & kFlagSuccessfulKill) r += 3.f;
    if (landed != -1) r += shot * 1.f;
    if (flags & kFlagWasKilled) r -= 1.5f;
    if (S.wasShot[g] > 0) r -= shot * 1.f;
    uint32_t nn = (uint32_t)S.newCells[g];
    S.newCells[g] = 0;
    if (nn > 0) r += float(nn) * explore;
    const int k = subZoneIndexD(S, g);
    if (flags & kFlagInSubZone) {
        r += in_zone;
    } else {
        const ZOBBDev &sz = sc.tab->subZones[k];
        Vec3 center = (sz.pMax + sz.pMin) / 2.f;
        float dist = distance(center, ldPos(S, g));
        float md = S.minDistSub[g];
        if (dist < md) {
            float scale = zdist;
            if (!(flags & kFlagHasDied)) scale *= 10.f;
            r += scale * (md - dist);
            S.minDistSub[g] = dist;
        }
    }
    const int ctrl = subCtrlD((uint32_t)S.subState[w], k);
    if (ctrl != -1) {
        if (ctrl == i / S.T) r += ctrl_s;
        else r -= ctrl_s;
    }
    if (S.alive[g] == 0.f) {
        S.flags[g] = flags & ~(kFlagSuccessfulKill | kFlagWasKilled);
        S.landedOn[g] = -1;
        S.wasShot[g] = 0;
        S.firedT[g] = -kFltMax;
    }
    S.reward[g] = r;
    return r;
}

// sim.cpp:3849-3996 zoneRewardSystem (+ learnShootingRewardSystem 3707-3732)
// Every reward system returns the reward it stored (k_sim hands it to the
// team reward through LDS).
__device__ __forceinline__ float zoneRewardD(const DevState &S, const SceneDev &sc, int w, int i)
{
    const int64_t g0 = (int64_t)w * S.N;
    const int64_t g = g0 + i;
    int32_t flags = S.flags[g];
    const int landed = S.landedOn[g];
    float r = 0.f;
    if (sc.task == MPENV_TASK_ZONE_CAPTURE_DEFEND) {
        return zoneCaptureDefendRewardD(S, sc, w, i);
    }
    if (S.worldCurr[w] == 0) {
        if (landed != -1) r += 0.5f;
        else if (S.firedT[g] >= 0.f) r -= 0.05f;
        if (flags & kFlagReloadedFullMag) r -= 0.5f;
        S.reward[g] = r;
        return r;
    }
    if (sc.simFlags & kFlagSubZones) {
        return subzoneRewardD(S, sc, w, i);
    }
    const float *rc = &S.rewardCoefs[9 * g];
    const float shot = rc[1], explore = rc[2], in_zone = rc[3], ctrl_s = rc[5], zdist = rc[6], earned_s = rc[7],
                crumb = rc[8];
    const int team = i / S.T, off = i - team * S.T;
    const Vec3 pos = ldPos(S, g);
    r -= crumb * S.bcPenalty[g];
    if (flags & kFlagReloadedFullMag) r -= 0.5f;
    if (flags & kFlagSuccessfulKill) r += 1.f;
    if (landed != -1) r += shot * 1.f;
    if (flags & kFlagWasKilled) r -= 1.5f;
    if (S.wasShot[g] > 0) r -= shot * 1.f;
    uint32_t nn = (uint32_t)S.newCells[g];
    S.newCells[g] = 0;
    if (nn > 0) r += float(nn) * explore;
    if (flags & kFlagInZone) {
        r += in_zone;
    } else {
        AABB za = sc.tab->zoneAABB[S.curZone[w]];
        Vec3 center = (za.pMax + za.pMin) / 2.f;
        float dist = distance(center, pos);
        float md = S.minDistZone[g];
        if (dist < md) {
            float scale = zdist;
            if (!(flags & kFlagHasDied)) scale *= 10.f;
            r += scale * (md - dist);
            S.minDistZone[g] = dist;
        }
    }
    const int ctrl = S.controlling[w];
    const bool earned = S.earned[w] != 0;
    if (ctrl != -1) {
        if (ctrl == team) {
            r += ctrl_s;
            if (earned) r += earned_s;
        } else {
            r -= ctrl_s;
            if (earned) r -= earned_s;
        }
    }
    if (S.alive[g] == 0.f) {
        S.flags[g] = flags & ~(kFlagSuccessfulKill | kFlagWasKilled);
        S.landedOn[g] = -1;
        S.wasShot[g] = 0;
        S.firedT[g] = -kFltMax;
        S.reward[g] = r;
        return r;
    }
    {
        float poly = 0.f;
        const int num_teammates = S.T - 1;
        for (int k = 0; k < num_teammates - 1; k++) {
            const int64_t t1 = g0 + team * S.T + (k < off ? k : k + 1);
            const int64_t t2 = g0 + team * S.T + (k + 1 < off ? k + 1 : k + 2);
            float e1x = S.px[t1] - pos.x, e1y = S.py[t1] - pos.y;
            float e2x = S.px[t2] - pos.x, e2y = S.py[t2] - pos.y;
            float tri = e1x * e2y - e1y * e2x;
            poly += fabs_(tri);
        }
        float dx = sc.worldBounds.pMax.x - sc.worldBounds.pMin.x;
        float dy = sc.worldBounds.pMax.y - sc.worldBounds.pMin.y;
        float area = dx * dy;
        float frac = poly / (2.f * area);
        r += frac * 1e-2f;
    }
    S.reward[g] = r;
    return r;
}

// ====================================================== kernels
constexpr int kBlock = 256;

// XCD-aware block order (cdna_hip_programming.md T1): the dispatcher deals
// consecutive blocks round-robin to the 8 XCDs, each with its own L2; the
// step kernels index worlds / agents by block, so neighbouring blocks share
// cache lines of the per-world and per-agent columns.  Renumbered, each XCD
// runs one contiguous range of blocks (bijective for any grid size).
__device__ __forceinline__ uint32_t xcdBlockId()
{
    const uint32_t nwg = gridDim.x, orig = blockIdx.x;
    const uint32_t xcd = orig % 8u, q = nwg / 8u, r = nwg % 8u;
    return (xcd < r ? xcd * (q + 1u) : r * (q + 1u) + (xcd - r) * q) + orig / 8u;
}

// Persistent-entity setup + the Sim constructor's initWorld(ctx, true)
// (sim.cpp:5850-5980, level_gen.cpp:19-328).  One thread per world.
__global__ void __launch_bounds__(64) k_construct(DevState S, SceneDev sc, int32_t tc0, int32_t tc1, int32_t tc2)
{
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= S.W) return;
    const int N = S.N;
    const int64_t g0 = (int64_t)w * N;
    #pragma unroll 1
    for (int i = 0; i < N; i++) {
        const int64_t g = g0 + i;
        S.policy[g] = 0;
        S.aimAction[2 * g] = 0.f; S.aimAction[2 * g + 1] = 0.f;
        S.discreteAim[2 * g] = c::kDiscreteAimYawBuckets / 2;
        S.discreteAim[2 * g + 1] = c::kDiscreteAimPitchBuckets / 2;
        S.dyv[g] = 0.f; S.dpv[g] = 0.f;
        for (int k = 0; k < kMaxTeamSize; k++) S.dmg[(int64_t)k * S.dmgStride + g] = 0.f;
        stRot(S, g, quat(1, 0, 0, 0));
        stAimRot(S, g, quat(1, 0, 0, 0));
        S.landedOn[g] = -1;
        S.bcLast[g] = -1;
        S.flags[g] = 0;
    }
    S.episode[w] = 0;
    S.episodeCounter[w] = 0;
    S.curTier[w] = 0;
    S.curSpawnIdx[w] = 0;
    S.numCrumbs[w] = 0;
    S.nextCrumbId[w] = 0;
    S.crumbOverflow[w] = 0;
    S.reset[w] = 0;
    for (int k = 0; k < 6; k++) S.filtLast[(int64_t)w * 6 + k] = 0;
    S.worldCurr[w] = 1; // WorldCurriculum::FullMatch (sim.cpp:5959)
    const int32_t tc[3] = { tc0, tc1, tc2 };
    initWorldD(S, sc, w, true, tc);
    S.matchValid[w] = 0; // matchID = ~0 after construction (sim.cpp:5971)
    S.evLogged[w] = 0;
    S.evMask[w] = 0;
    S.snapWritten[w] = 0;
    for (int k = 0; k < 25; k++) S.zoneStats[(int64_t)w * 25 + k] = 0;
    S.filtAct0[w] = 0; S.filtAct1[w] = 0;
    S.filtMatched0[w] = -1; S.filtMatched1[w] = -1;
}

// ExploreTracker initial contents (level_gen.cpp:166-171: 0xFFFFFFFF on the
// y<40, x<40 quadrant; the other cells start at 0) as the
// bitset of episode 0: the cells whose tag is 0 are set; no tile cached.
__global__ void __launch_bounds__(256) k_init_explore(DevState S, int64_t total)
{
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < total; k += (int64_t)gridDim.x * blockDim.x) {
        const int t = (int)(k % kExploreTiles);
        const int tx = t % kExploreTilesX, ty = t / kExploreTilesX;
        uint64_t v = 0ull;
        for (int b = 0; b < 64; b++) {
            const int x = tx * 8 + (b & 7), y = ty * 8 + (b >> 3);
            if (x >= kGridW || y >= kGridW) continue;
            if (!(y < c::kGridMax && x < c::kGridMax)) v |= 1ull << b;
        }
        S.exploreBits[k] = v;
        if (t == 0) {
            const int64_t g = k / kExploreTiles;
            S.exploreEp[g] = 0;
            S.exploreTile[g] = -1;
            S.exploreLo[g] = 0;
            S.exploreHi[g] = 0;
        }
    }
}

__global__ void __launch_bounds__(64) k_reset_only(DevState S, SceneDev sc)
{
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= S.W) return;
    resetSystemD(S, sc, w);
}

// The Step graph up to and including resetSystem, one workgroup per tile of
// floor(256 / N) worlds, one lane per agent.
// Step graph part 1 (sim.cpp:5299-5320 up to updateMoveStatePostFall): the
// per-agent systems, which read no other agent's state.  Lane = agent, no
// barriers, so sphere-cast latency overlaps across the whole grid.
// apw: agents per wave (64, or fewer on small batches: a wave runs the
// longest of its lanes' sphere-cast chains, so when the batch leaves SIMDs
// idle, fewer agents per wave shorten every wave; launchMove picks it).
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3))) k_move(DevState S, SceneDev sc, int apw)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    LBVH bvh = stageBVHSphere(smem, sc);
    bvh.stats = S.stats;
    [&]() {
        const int lane = threadIdx.x & 63;
        if (lane >= apw) return;
        const int64_t wave = ((int64_t)xcdBlockId() * blockDim.x + threadIdx.x) >> 6;
        const int64_t g = wave * apw + lane;
        if (g >= S.A) return;
        if (S.stats) statAdd(S.stats + kStatAliveAgents, S.alive[g] != 0.f ? 1u : 0u);
        planAStarD(S, sc, g);
        if (sc.replayOn) return; // pvpReplayLogic replaces the gameplay systems (sim.cpp:5587-5605)
        applyBotActionsD(S, g);
        pvpMovementD(S, g);
        pvpAimD(S, g);
        applyVelocityD(S, sc, bvh, g);
        fallD(S, sc, bvh, g);
    }();
}

// Step graph part 2 (fireSystem onward): per-world phases.  A workgroup
// holds floor(kSimBlock / N) whole worlds, lane = agent, phases separated
// by workgroup barriers.
constexpr int kSimBlock = 128;
// k_sim's dynamic LDS: the BVH image, which the phases after the last BVH
// use reuse (the reset's draw keys, kPreDraws + 1 per lane, then the spawn
// records, kSpawnRec floats per lane), then the spawn lists.
constexpr size_t kSimKeyBytes = (size_t)kSimBlock * (kPreDraws + 1) * sizeof(RandKey);
__host__ __device__ size_t simSpawnOffset(const SceneDev &sc)
{
    const size_t bvh = (size_t)sc.numNodes * 64 + (size_t)sc.numVerts * 16;
    const size_t reuse = kSimKeyBytes + (size_t)kSimBlock * kSpawnRec * 4;
    return ((bvh > reuse ? bvh : reuse) + 15) & ~(size_t)15;
}

__device__ __forceinline__ float flankRewardD(const DevState &S, const SceneDev &sc, const LBVH &bvh, int w, int i);

// 4 waves/SIMD (128 VGPRs, at the price of ~420 B/lane of scratch spills):
// k_sim alone 0.196 -> 0.139 ms -- every wave of a C3 launch resident,
// which hides the per-world phases' latency better than the spills cost.
#define MP_SIM_ATTR __attribute__((amdgpu_waves_per_eu(4)))
// flatten: every phase inlined (an outlined call needs a stack frame in
// scratch for the whole kernel and spills around the call).
__global__ void __launch_bounds__(kSimBlock) MP_SIM_ATTR __attribute__((flatten)) k_sim(DevState S, SceneDev sc)
{

    extern __shared__ __attribute__((aligned(16))) char smem[];
    // dynamic LDS (simLdsBytes): the BVH image, which the reset phase reuses
    // for its draw keys, then the scene's spawn lists
    Spawn *const tabA = reinterpret_cast<Spawn *>(smem + simSpawnOffset(sc));
    Spawn *const tabB = tabA + sc.numA, *const tabC = tabB + sc.numB;
    {
        const int nq = (sc.numA + sc.numB + sc.numCommon) * (int)(sizeof(Spawn) / 16);
        const int na = sc.numA * (int)(sizeof(Spawn) / 16), nb = sc.numB * (int)(sizeof(Spawn) / 16);
        uint4 *dst = reinterpret_cast<uint4 *>(tabA);
        for (int k = threadIdx.x; k < nq; k += blockDim.x) {
            const uint4 *src = k < na ? reinterpret_cast<const uint4 *>(sc.aSpawns) + k
                             : k < na + nb ? reinterpret_cast<const uint4 *>(sc.bSpawns) + (k - na)
                                           : reinterpret_cast<const uint4 *>(sc.commonRespawns) + (k - na - nb);
            dst[k] = *src;
        }
    }
    const LBVH bvh = stageBVH(smem, sc); // (its barrier also covers the spawn lists)
    // spawn records in the BVH's LDS once nothing reads the BVH any more:
    // the respawn (after fireD) unless the flank reward traces rays later,
    // the reset (last phase) unless curriculum snapshots rewrite agents after
    // the spawn (then the world lane stores everything itself)
    float *const spawnRec = reinterpret_cast<float *>(smem + kSimKeyBytes);
    const bool recRespawn = !sc.flank && !(sc.simFlags & kFlagNoRespawn);
    const bool recReset = sc.numSnapshots == 0;
    const int N = S.N;
    const int wpb = kSimBlock / N;
    const int wl = threadIdx.x / N;
    const int i = threadIdx.x - wl * N;
    const int w = (int)xcdBlockId() * wpb + wl;
    const bool act = (wl < wpb) && (w < S.W);
    const bool wlane = act && i == 0;
    const int64_t g = (int64_t)w * N + i;

    __shared__ uint8_t agentB[kSimBlock]; // per-agent bytes for the world lane (alive, done)
    // per-agent floats for the world lane, reused by phase: respawn
    // (positions [3 * kSimBlock], flags), crumb rounds (2 float4 per lane),
    // goal distances (stride 6), rewards, reset (flags)
    __shared__ __attribute__((aligned(16))) float goalDist[kSimBlock * 8];
    float *const sposL = goalDist;
    float *const sflagL = goalDist + 3 * kSimBlock;
    if (act && sc.eventsOn) { // ClearTmpNode<GameEventEntity> at step start (sim.cpp:5344)
        mpenv_game_event *ev = &S.events[(int64_t)w * S.evStride];
        ev[2 * i].type = 0;
        ev[2 * i + 1].type = 0;
        if (wlane) ev[2 * N].type = 0;
    }
    if (sc.replayOn) {
        // pvpReplayLogic: pvpReplaySystem then zoneSystem
        if (act) replayAgentD(S, w, i);
        if (wlane) S.curStep[w] = S.replayLog[w].cur_step;
        __syncthreads();
        if (wlane) zoneSystemD(S, sc, w);
        __syncthreads();
    } else {
        {
            // every agent's own fire inputs in one round of loads; the
            // world's positions, hp and respawn counters (the shots' capsule
            // tests and targets) through LDS (goalDist's, free until the
            // respawn below)
            float *const fpx = goalDist, *const fpy = goalDist + kSimBlock, *const fpz = goalDist + 2 * kSimBlock;
            float *const fhp = goalDist + 3 * kSimBlock, *const frs = goalDist + 4 * kSimBlock;
            FireIn fin;
            if (act) {
                fin = fireLoadD(S, g);
                fpx[threadIdx.x] = fin.pos.x;
                fpy[threadIdx.x] = fin.pos.y;
                fpz[threadIdx.x] = fin.pos.z;
                fhp[threadIdx.x] = fin.hp;
                frs[threadIdx.x] = __int_as_float(fin.respawn);
            }
            __syncthreads();
            if (act) fireD(S, sc, bvh, w, i, fin, fpx, fpy, fpz, fhp, frs, wl * N);
        }
        __syncthreads();
        // the agents' alive states, positions and flags go to the world
        // lane's respawn through LDS (it read them back from memory one
        // agent at a time)
        bool dead_now = false;
        if (act) {
            const DmgOut d = applyDmgD(S, g);
            dead_now = !d.alive;
            agentB[threadIdx.x] = d.alive ? 1 : 0;
            sposL[3 * threadIdx.x] = d.pos.x;
            sposL[3 * threadIdx.x + 1] = d.pos.y;
            sposL[3 * threadIdx.x + 2] = d.pos.z;
            sflagL[threadIdx.x] = __int_as_float(d.flags);
        }
        __syncthreads();
        const bool coopRespawn = recRespawn && sc.numCommon > 0 && sc.numCommon <= 64 &&
                                 !(sc.simFlags & kFlagNavmeshSpawn);
        if (coopRespawn)
            respawnCoopD(S, sc, w, i, wl, act,
                         SpawnLds{ &sposL[3 * wl * N], &agentB[wl * N], &sflagL[wl * N], tabA, tabB, tabC },
                         spawnRec + wl * N * kSpawnRec, reinterpret_cast<float *>(smem));
        else if (wlane && !(sc.simFlags & kFlagNoRespawn)) {
            uint32_t dead = 0;
            #pragma unroll 1
            for (int k = 0; k < N; k++)
                if (!agentB[wl * N + k]) dead |= 1u << k;
            spawnAgentsD(S, sc, w, true, nullptr, dead,
                         SpawnLds{ &sposL[3 * wl * N], &agentB[wl * N], &sflagL[wl * N], tabA, tabB, tabC },
                         recRespawn ? spawnRec + wl * N * kSpawnRec : nullptr);
        }
        if (recRespawn) {
            // the respawned agents' own stores, from the world lane's records
            __syncthreads();
            if (dead_now) {
                const ZoneBox zb = zoneBoxD(sc, S.curZone[w]);
                spawnApplyRecD(S, sc, g, true, spawnRec + threadIdx.x * kSpawnRec, __float_as_int(sflagL[threadIdx.x]), zb);
            }
        }
        __syncthreads();
        {
            __shared__ int zoneCz[kSimBlock];
            __shared__ uint8_t zoneIn[kSimBlock];
            ZonePre zp;
            if (wlane) {
                zp = zonePreD(S, sc, w);
                zoneCz[wl] = zp.cz;
            }
            __syncthreads();
            // Agent phase shared by the zone test, the recorder and
            // leaveBreadcrumbs: none reads what another writes (InZone and
            // CrumbRequest are different flag bits of the lane's own agent;
            // the recorder reads neither), so they run between one pair of
            // barriers instead of three.
            if (act) {
                // bit 0 in the zone, bit 1 a new breadcrumb requested
                const bool zin = zoneInD(S, sc, zoneCz[wl], g);
                if (sc.recordOn) recordAgentD(S, w, i);
                const bool req = leaveBreadcrumbAgentD(S, w, g);
                zoneIn[threadIdx.x] = (zin ? 1 : 0) | (req ? 2 : 0);
                // the position a requested crumb takes (sposL's LDS, free here)
                const Vec3 p = ldPos(S, g);
                sposL[3 * threadIdx.x] = p.x;
                sposL[3 * threadIdx.x + 1] = p.y;
                sposL[3 * threadIdx.x + 2] = p.z;
            }
            if (wlane && sc.recordOn) S.recordLog[w].cur_step = S.curStep[w];
            __syncthreads();
            if (wlane) {
                int na = 0, nb = 0;
                uint32_t req = 0;
                #pragma unroll 1
                for (int k = 0; k < N; k++) {
                    const int b = zoneIn[wl * N + k];
                    if (b & 2) req |= 1u << k;
                    if (!(b & 1)) continue;
                    if (k / S.T == 0) na += 1;
                    else nb += 1;
                }
                zonePostD(S, w, zp, na, nb);
                if (sc.simFlags & kFlagSubZones) subzoneSystemD(S, sc, w);
                appendCrumbsD(S, w, req, &sposL[3 * wl * N]);
            }
        }
        __syncthreads();
        // accumulateBreadcrumbPenalties and the crumbs' decay (the end of
        // that system), in rounds over LDS (goalDist's, free until below)
        crumbRoundsD(S, w, i, act, wl, reinterpret_cast<float4 *>(goalDist));
    }
    // zoneMatchInfoSystem's per-agent reads, one lane per agent (the world
    // lane would otherwise walk them serially)
    __shared__ uint8_t matchBits[kSimBlock];
    if (act) {
        matchBits[threadIdx.x] = (uint8_t)matchAgentBitsD(S, w, i);
        goalDistAgentD(S, sc, w, i, ldPos(S, g), &goalDist[threadIdx.x * 6]);
    }
    __syncthreads();
    if (wlane) {
        zoneMatchInfoD(S, sc, w, &matchBits[wl * N]);
        goalRegionsD(S, sc, w, &goalDist[wl * N * 6]);
    }
    __syncthreads();
    // rewards and done flags go to the world lane through LDS (rewL, agentB)
    // instead of being read back from memory one agent at a time
    // (in goalDist's LDS, whose last reader finished before the barrier above;
    // teamL: 2 per world, at most kSimBlock / 2 worlds as N >= 2)
    float *const rewL = goalDist;
    float *const teamL = goalDist + kSimBlock;
    if (act) {
        exploreVisitedD(S, w, g);
        if (sc.flank && sc.task == MPENV_TASK_ZONE) rewL[threadIdx.x] = flankRewardD(S, sc, bvh, w, i);
        else rewL[threadIdx.x] = zoneRewardD(S, sc, w, i);
    }
    __syncthreads();
    if (wlane) {
        // pvpTeamRewardSystem (sim.cpp:4292-4313)
        float tr[2] = { 0.f, 0.f };
        int ts[2] = { 0, 0 };
        #pragma unroll 1
        for (int j = 0; j < N; j++) {
            int t = j / S.T;
            tr[t] += rewL[wl * N + j];
            ts[t] += 1;
        }
        tr[0] /= float(ts[0]);
        tr[1] /= float(ts[1]);
        S.teamRew0[w] = tr[0];
        S.teamRew1[w] = tr[1];
        teamL[2 * wl] = tr[0];
        teamL[2 * wl + 1] = tr[1];
    }
    __syncthreads();
    if (act) {
        // pvpFinalRewardSystem (sim.cpp:4315-4339) + doneSystem (4712-4717)
        const int team = i / S.T;
        const float spirit = S.rewardCoefs[9 * g];
        const bool done = S.finished[w] != 0;
        const float my = rewL[threadIdx.x];
        const float team_r = teamL[2 * wl + team];
        const float fr = my * (1.f - spirit) + team_r * spirit;
        S.reward[g] = fr;
        S.done[g] = done ? 1 : 0;
        rewL[threadIdx.x] = fr;
        agentB[threadIdx.x] = done ? 1 : 0;
    }
    // resets: the agents' own parts in parallel, then the world lane
    // (the BVH image is dead from here on: the reset's draw keys go there)
    RandKey *pre = reinterpret_cast<RandKey *>(smem) + (int64_t)wl * N * (kPreDraws + 1);
    const bool resetting = act && resetDueD(S, sc, w);
    if (resetting) sflagL[threadIdx.x] = __int_as_float(resetPreD(S, sc, w, i, pre + i * (kPreDraws + 1)));
    __syncthreads();
    if (wlane) {
        // fullTeamDoneRewardSystem (sim.cpp:4720-4747)
        for (int t = 0; t < 2; t++) {
            float r = 0.f;
            bool done = true;
            for (int j = t * S.T; j < (t + 1) * S.T; j++) {
                r += rewL[wl * N + j];
                if (!agentB[wl * N + j]) done = false;
            }
            S.ftReward[(int64_t)w * 2 + t] = r;
            S.ftDone[(int64_t)w * 2 + t] = done ? 1 : 0;
        }
        resetSystemD(S, sc, w, pre, SpawnLds{ nullptr, nullptr, &sflagL[wl * N], tabA, tabB, tabC },
                     recReset ? spawnRec + wl * N * kSpawnRec : nullptr);
    }
    if (recReset) {
        // the reset agents' own stores, from the world lane's records
        __syncthreads();
        if (resetting) {
            const ZoneBox zb = zoneBoxD(sc, S.curZone[w]);
            spawnApplyRecD(S, sc, g, false, spawnRec + threadIdx.x * kSpawnRec, __float_as_int(sflagL[threadIdx.x]), zb);
            resetAgentTailD(S, g);
        }
    }
}

// utils.cpp:169-184 inFrustum
__device__ __forceinline__ bool inFrustumD(const SceneDev &sc, Vec3 vp)
{
    bool in = true;
    in = in && vp.y * sc.frustum[1] - fabs_(vp.x) * sc.frustum[0] > -c::kAgentRadius;
    in = in && vp.y * sc.frustum[3] - fabs_(vp.z) * sc.frustum[2] > -c::kAgentRadius;
    return in;
}

// opponentsWriteVisibilitySystem (sim.cpp:2526-2560) + isAgentVisible
// (utils.cpp:169-271): agent i sees opponent k if any of 4 sample points on
// k (bottom, top, left, right) passes the view tests and the closest hit of
// the ray toward it is k's capsule.
//
// Ray compaction: lane = (agent, opponent); each 64-lane wave holds whole
// agents (floor(64/T) of them).  Phase A tests the sample points (cheap) and
// reserves LDS slots for the candidate rays; phase B traces the compacted
// ray list with every lane of the workgroup, OR-ing hits into per-agent LDS
// masks; phase C writes one mask byte per agent.  Only ~1.5 of the 4 points
// survive the view tests on average, so the dense pass replaces a per-lane
// loop that ran at roughly a third of the wave's lanes.
constexpr int kVisMaxRays = kBlock * 4;

// k_vis stages its block's agents with their worlds' whole rosters (the
// opponents the block's lanes test and every capsule a ray may meet) in LDS
// after the BVH image: 4 waves x floor(64/T) agents plus up to N-1 agents of
// the partial first and last worlds.  Columns: px, py, pz, view height,
// aim quaternion (w, x, y, z), alive.
constexpr int kVisStageCols = 9;
__host__ __device__ __forceinline__ int visStageAgents(int T, int N) { return (kBlock / 64) * (64 / T) + 2 * (N - 1); }

__device__ __forceinline__ Vec3 visSamplePointD(const DevState &S, int64_t gt, Vec3 delta_right, int p)
{
    Vec3 pt = ldPos(S, gt);
    pt.z += p == 0 ? c::kAgentRadius : viewHeightD(S.curPose[gt]);
    if (p == 2) pt = pt - delta_right;
    if (p == 3) pt = pt + delta_right;
    return pt;
}

// utils.cpp:169-271 isAgentVisible for one (viewer, target) pair, lane-wise
// (the flank reward's checks; k_vis batches the opponent checks instead).
__device__ __forceinline__ bool isAgentVisibleD(const DevState &S, const SceneDev &sc, const LBVH &bvh, int w, Vec3 org,
                                Quat aim_rot, int target)
{
    const int N = S.N;
    const int64_t g0 = (int64_t)w * N;
    const Quat inv_rot = qinv(aim_rot);
    const Vec3 delta_right = rotateVec(aim_rot, kRight) * 0.9f * c::kAgentRadius;
    for (int p = 0; p < 4; p++) {
        Vec3 to_test = visSamplePointD(S, g0 + target, delta_right, p) - org;
        Vec3 view = rotateVec(inv_rot, to_test);
        if (view.y <= 0.f) continue;
        if (!inFrustumD(sc, view)) continue;
        const float len = length(to_test);
        if (len < c::kAgentRadius) continue;
        to_test = to_test / len;
        if (visibleRayD(bvh, S.px, S.py, S.pz, g0, N, org, to_test, target)) return true;
    }
    return false;
}

// sim.cpp:4202-4278 flankRewardSystem (Task.Zone with train_flank): small
// bonuses for teammates out of sight or >= 100 units away and for each
// opponent that cannot see the agent (judged with the agent's own aim),
// hits / kills from behind the target, exploration.  CombatState is taken
// by value there, so nothing is cleared.
__device__ __forceinline__ float flankRewardD(const DevState &S, const SceneDev &sc, const LBVH &bvh, int w, int i)
{
    const int T = S.T, N = S.N;
    const int64_t g0 = (int64_t)w * N;
    const int64_t g = g0 + i;
    const int team = i / T, off = i - team * T;
    const Vec3 pos = ldPos(S, g);
    const Quat aim_rot = ldAimRot(S, g);
    float r = 0.f;
    Vec3 vis = pos;
    vis.z += viewHeightD(S.curPose[g]);
    const float flank_dist = 100.f;
    float mates = 0.f;
    for (int k = 0; k < T - 1; k++) {
        const int j = team * T + (k < off ? k : k + 1);
        const Vec3 dir = ldPos(S, g0 + j) - pos;
        const bool seen = isAgentVisibleD(S, sc, bvh, w, vis, aim_rot, j);
        if (length2(dir) >= flank_dist * flank_dist || !seen) mates += 0.001f;
    }
    r += mates;
    float opps = 0.f;
    for (int k = 0; k < T; k++) {
        const int64_t go = g0 + (team ^ 1) * T + k;
        Vec3 op_pos = ldPos(S, go);
        op_pos.z += viewHeightD(S.curPose[go]);
        if (!isAgentVisibleD(S, sc, bvh, w, op_pos, aim_rot, i)) opps += 0.001f;
    }
    r += opps;
    const int landed = S.landedOn[g];
    if (landed != -1) {
        const float yaw_diff = fabs_(S.ayaw[g0 + landed] - S.ayaw[g]);
        if (yaw_diff > kPi) r += (S.flags[g] & kFlagSuccessfulKill) ? 1.f : 0.2f;
    }
    uint32_t nn = (uint32_t)S.newCells[g];
    S.newCells[g] = 0;
    if (nn > 0) r += float(nn) * S.rewardCoefs[9 * g + 2];
    S.reward[g] = r;
    return r;
}

__global__ void __launch_bounds__(kBlock) k_vis(DevState S, SceneDev sc)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ uint16_t rays[kVisMaxRays];  // (lane << 2) | point
    __shared__ uint16_t rays2[kVisMaxRays]; // phase B2: indices into rays
    __shared__ uint32_t masks[kBlock]; // per agent of the block (<= 4 waves x 64/T)
    __shared__ uint32_t nrays, nrays2;
    if (threadIdx.x == 0) {
        nrays = 0;
        nrays2 = 0;
    }
    masks[threadIdx.x] = 0;
    const int T = S.T, N = S.N;
    const int apw = 64 / T;
    const int wl = threadIdx.x & 63;
    const int64_t wave = ((int64_t)xcdBlockId() * blockDim.x + threadIdx.x) >> 6;
    const int64_t agent0 = (((int64_t)xcdBlockId() * blockDim.x) >> 6) * apw; // first agent of the block
    const int nsMax = visStageAgents(T, N);
    float *st = (float *)(smem + (size_t)sc.numLidarNodes * 64 + (size_t)sc.numLidarVerts * 16);
    const int64_t s0 = (agent0 / N) * N;
    {
        const int64_t a_hi = min(S.A, agent0 + (int64_t)(kBlock / 64) * apw);
        const int ns = agent0 < a_hi ? (int)(((a_hi - 1) / N + 1) * N - s0) : 0;
        for (int k = threadIdx.x; k < ns; k += kBlock) {
            const int64_t g = s0 + k;
            st[0 * nsMax + k] = S.px[g];
            st[1 * nsMax + k] = S.py[g];
            st[2 * nsMax + k] = S.pz[g];
            st[3 * nsMax + k] = viewHeightD(S.curPose[g]);
            st[4 * nsMax + k] = S.aw[g];
            st[5 * nsMax + k] = S.ax[g];
            st[6 * nsMax + k] = S.ay[g];
            st[7 * nsMax + k] = S.az[g];
            st[8 * nsMax + k] = S.alive[g];
        }
    }
    const LBVH bvh = stageBVH(smem, sc, true); // the lidar tree; barrier
    auto sPos = [&](int64_t g) {
        const int l = (int)(g - s0);
        return v3(st[0 * nsMax + l], st[1 * nsMax + l], st[2 * nsMax + l]);
    };
    auto sAim = [&](int64_t g) {
        const int l = (int)(g - s0);
        return quat(st[4 * nsMax + l], st[5 * nsMax + l], st[6 * nsMax + l], st[7 * nsMax + l]);
    };
    auto sView = [&](int64_t g) { return st[3 * nsMax + (int)(g - s0)]; };
    auto sAlive = [&](int64_t g) { return st[8 * nsMax + (int)(g - s0)]; };
    // visSamplePointD from the stage
    auto sSample = [&](int64_t gt, Vec3 delta_right, int p) {
        Vec3 pt = sPos(gt);
        pt.z += p == 0 ? c::kAgentRadius : sView(gt);
        if (p == 2) pt = pt - delta_right;
        if (p == 3) pt = pt + delta_right;
        return pt;
    };

    // ---- phase A: view tests, reserve ray slots
    {
        const int64_t g = wave * apw + wl / T;
        const int k = wl % T;
        const bool valid = wl < apw * T && g < S.A;
        uint32_t cand = 0;
        if (valid) {
            const int w = (int)(g / N);
            const int i = (int)(g - (int64_t)w * N);
            const int64_t gt = (int64_t)w * N + ((i / T) ^ 1) * T + k;
            if (sAlive(g) != 0.f && sAlive(gt) != 0.f) {
                Vec3 org = sPos(g);
                org.z += sView(g);
                const Quat aim_rot = sAim(g);
                const Quat inv_rot = qinv(aim_rot);
                const Vec3 delta_right = rotateVec(aim_rot, kRight) * 0.9f * c::kAgentRadius;
#pragma unroll
                for (int p = 0; p < 4; p++) {
                    Vec3 to_test = sSample(gt, delta_right, p) - org;
                    Vec3 view = rotateVec(inv_rot, to_test);
                    if (view.y <= 0.f) continue;
                    if (!inFrustumD(sc, view)) continue;
                    if (length(to_test) < c::kAgentRadius) continue;
                    cand |= 1u << p;
                }
            }
        }
        const int nc = __popc(cand);
        if (S.stats) {
            uint32_t pair = 0;
            if (valid && sAlive(g) != 0.f) {
                const int64_t gt2 = (g / N) * N + (((int)(g % N) / T) ^ 1) * T + k;
                pair = sAlive(gt2) != 0.f ? 1u : 0u;
            }
            statAdd(S.stats + kStatLosPairs, pair);
            statAdd(S.stats + kStatLosRays, (uint32_t)nc);
        }
        // Ray-slot reservation: the wave's exclusive prefix sum of its
        // lanes' candidate counts (4 ballots of one bit each, mbcnt), one
        // LDS atomic per wave for the base.
        uint32_t before = 0, wtotal = 0;
#pragma unroll
        for (int bit = 0; bit < 3; bit++) {
            const uint64_t m = __ballot((nc >> bit) & 1);
            before += (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) << bit;
            wtotal += (uint32_t)__popcll(m) << bit;
        }
        uint32_t base = 0;
        if (wl == 0 && wtotal) base = atomicAdd(&nrays, wtotal);
        base = __shfl(base, 0);
        if (nc) {
            uint32_t slot = base + before;
            const uint16_t lane_id = (uint16_t)(threadIdx.x << 2);
            for (int p = 0; p < 4; p++)
                if (cand & (1u << p)) rays[slot++] = (uint16_t)(lane_id | p);
        }
    }
    __syncthreads();

    // ---- phase B: the compacted rays.  B1 decides what needs no traversal
    // (target capsule missed, occluder hint hit); the rest are compacted
    // again so B2's traversals run in dense waves (a wave of mixed rays
    // otherwise idles all but its few traversing lanes).
    const uint32_t total = nrays;
    const uint32_t numTris = (uint32_t)(sc.numLidarVerts / 3);
    // the occluder hint stores triangle ids as u16 with 0xffff = none: off
    // for scenes of 65,535 triangles or more
    const bool hints = numTris < 0xffffu;
    auto rayOf = [&](uint32_t r, int64_t &g, int &k, int &p, int64_t &g0, int &target, Vec3 &org, Vec3 &dir) {
        const uint32_t d = rays[r];
        const int lane = (int)(d >> 2);
        p = (int)(d & 3);
        const int lwl = lane & 63;
        g = ((((int64_t)xcdBlockId() * blockDim.x + lane) >> 6) * apw) + lwl / T;
        k = lwl % T;
        const int w = (int)(g / N);
        const int i = (int)(g - (int64_t)w * N);
        g0 = (int64_t)w * N;
        target = ((i / T) ^ 1) * T + k;
        org = sPos(g);
        org.z += sView(g);
        const Quat aim_rot = sAim(g);
        const Vec3 delta_right = rotateVec(aim_rot, kRight) * 0.9f * c::kAgentRadius;
        Vec3 to_test = sSample(g0 + target, delta_right, p) - org;
        const float len = length(to_test);
        dir = to_test / len;
    };
    for (uint32_t r = threadIdx.x; r < total; r += kBlock) {
        int64_t g, g0;
        int k, p, target;
        Vec3 org, dir;
        rayOf(r, g, k, p, g0, target, org, dir);
        float t_c;
        const int l0 = (int)(g0 - s0);
        auto capsule = [&](int j) { return v3(st[0 * nsMax + l0 + j], st[1 * nsMax + l0 + j], st[2 * nsMax + l0 + j]); };
        if (!visibleQuickD(bvh, capsule, org, dir, target,
                           hints ? S.visOcc + (g * T + k) * 4 + p : nullptr, numTris, t_c))
            rays2[atomicAdd(&nrays2, 1u)] = (uint16_t)r;
    }
    __syncthreads();
    const uint32_t total2 = nrays2;
    if (S.stats && threadIdx.x == 0) atomicAdd(S.stats + kStatLosTraced, (unsigned long long)total2);
    for (uint32_t q = threadIdx.x; q < total2; q += kBlock) {
        int64_t g, g0;
        int k, p, target;
        Vec3 org, dir;
        rayOf(rays2[q], g, k, p, g0, target, org, dir);
        // t_c again (the same bits as in B1)
        const int l0 = (int)(g0 - s0);
        auto capsule = [&](int j) { return v3(st[0 * nsMax + l0 + j], st[1 * nsMax + l0 + j], st[2 * nsMax + l0 + j]); };
        Vec3 ct = capsule(target);
        ct.z += kCapsuleRadius;
        const float t_c = intersectRayZOriginCapsule(org - ct, dir, kCapsuleRadius, kCapsuleSegment);
        const bool seen = visibleFullD(bvh, capsule, N, org, dir, target, t_c,
                                       hints ? S.visOcc + (g * T + k) * 4 + p : nullptr);
        if (seen) atomicOr(&masks[(int)(g - agent0)], 1u << k);
        if (S.stats) statAdd(S.stats + kStatLosSeen, seen ? 1u : 0u);
    }
    __syncthreads();

    // ---- phase C: one byte per agent
    {
        const int64_t g = wave * apw + wl / T;
        const bool valid = wl < apw * T && g < S.A;
        if (valid && wl % T == 0) S.visMask[g] = (uint8_t)masks[(int)(g - agent0)];
    }
}

__device__ __forceinline__ Vec3 normalizedPosD(const SceneDev &sc, Vec3 p) // sim.cpp:2693-2718
{
    float min_x = sc.worldBounds.pMin.x, min_y = sc.worldBounds.pMin.y, min_z = sc.worldBounds.pMin.z;
    float max_x = sc.worldBounds.pMax.x, max_y = sc.worldBounds.pMax.y, max_z = sc.worldBounds.pMax.z;
    float xr = max_x - min_x, yr = max_y - min_y, zr = max_z - min_z;
    float x = (p.x - min_x) / xr, y = (p.y - min_y) / yr, z = (p.z - min_z) / zr;
    return v3(clampf(x, 0.f, 1.f), clampf(y, 0.f, 1.f), clampf(z, 0.f, 1.f));
}

struct SelfFrame {
    Vec3 pos;
    Quat invRot;
    float yaw, pitch;
};

__device__ __forceinline__ void relAnglesD(const SelfFrame &sf, Vec3 to, float &dist_out, float &yaw_out,
                                           float &pitch_out)
{
    float d = length(to);
    if (d < 1e-2f) {
        dist_out = 0.f; yaw_out = 0.f; pitch_out = 0.f;
        return;
    }
    to = to / d;
    float new_yaw = -atan2f_(to.x, to.y);
    float new_pitch = asinf_(clampf(to.z, -1.f, 1.f));
    float yaw_delta = new_yaw - sf.yaw;
    float pitch_delta = new_pitch - sf.pitch;
    if (yaw_delta > kPi) yaw_delta -= 2.f * kPi;
    else if (yaw_delta < -kPi) yaw_delta += 2.f * kPi;
    dist_out = d; yaw_out = yaw_delta; pitch_out = pitch_delta;
}

__device__ __forceinline__ Vec3 normalizedPosUnclampedD(const SceneDev &sc, Vec3 p)
{
    float min_x = sc.worldBounds.pMin.x, min_y = sc.worldBounds.pMin.y, min_z = sc.worldBounds.pMin.z;
    float max_x = sc.worldBounds.pMax.x, max_y = sc.worldBounds.pMax.y, max_z = sc.worldBounds.pMax.z;
    float xr = max_x - min_x, yr = max_y - min_y, zr = max_z - min_z;
    return v3((p.x - min_x) / xr, (p.y - min_y) / yr, (p.z - min_z) / zr);
}

// ---- k_obs: pvpOpponentMasksSystem (sim.cpp:2562-2614), pvpObservationsSystem
// (sim.cpp:2645-3052) and fullTeamObservationsSystem (sim.cpp:3054-3301).
//
// Load first, then store.  gfx9's vector-memory counter retires loads and
// stores in issue order, so a load issued after a burst of stores cannot be
// waited for without waiting for those stores' write acknowledgements too.
// The round-1..4 k_obs gathered each world-mate's fields from HBM/L2 inside
// its slot loop, between the previous slot's row stores: every slot paid a
// full store round trip (55 `s_waitcnt vmcnt(0)` in its ISA; ~95 us per wave
// for ~141 KB of rows, 3.4 TB/s).  Now every input is read before the first
// store: a block (256 consecutive agents) stages the columns of every agent
// of its worlds in LDS (<= 256 + 2 (N - 1) agents, coalesced column loads),
// each lane loads its own rotation and world fields, and from then on the
// kernel only reads LDS and stores.
//
// Rows leave through a per-wave LDS transpose, half a wave (32 rows) at a
// time so the stage fits next to the agent columns (3 blocks per CU): a
// lane computes its row in registers, its half writes the rows to LDS, and
// every lane of the wave stores whole row pieces (float4 where the rows are
// 16-B aligned), so a store instruction writes a few whole 128-B lines
// instead of one 4-16 B piece of 64 different rows.
constexpr int kObsBlock = 256;
constexpr int kObsStageMax = kObsBlock + 2 * (kMaxAgents - 1); // the block's agents plus a partial world at each end
enum : int {
    kOsPX, kOsPY, kOsPZ, kOsVX, kOsVY, kOsVZ, kOsYaw, kOsPitch, kOsDYV, kOsDPV, kOsHP, kOsFired, kOsAlive, // f32
    kOsCurPose, kOsTgtPose, kOsWeapon, kOsVis, kOsTrans, kOsFlags, kOsShot, kOsHeal, kOsMag0, kOsMag1,      // i32
    kObsCols
};
constexpr int kObsRowPad = kOtherObs + 4; // LDS row stride (floats) of the 32-float rows: 16-B aligned
constexpr int kObsSpanPad = 44;           // floats per staged row: >= kObsRowPad and the 43-float self obs

// The block's agent columns in LDS (index = global agent id - s0).
struct ObsStage {
    const float (*c)[kObsStageMax];
    __device__ __forceinline__ float f(int col, int k) const { return c[col][k]; }
    __device__ __forceinline__ int32_t i(int col, int k) const { return __float_as_int(c[col][k]); }
    __device__ __forceinline__ Vec3 pos(int k) const { return v3(c[kOsPX][k], c[kOsPY][k], c[kOsPZ][k]); }
    __device__ __forceinline__ Vec3 vel(int k) const { return v3(c[kOsVX][k], c[kOsVY][k], c[kOsVZ][k]); }
    __device__ __forceinline__ bool alive(int k) const { return c[kOsAlive][k] != 0.f; }
};

// fillCommonOb (sim.cpp:2720-2774) of stage agent j into a register array;
// returns alive.
__device__ __forceinline__ bool fillCommonS(const ObsStage &st, const SceneDev &sc, const SelfFrame &sf, int j,
                                            float *ob, float *pos_ob)
{
    ob[0] = 1.f;
    if (!st.alive(j)) return false;
    ob[1] = 1.f;
    Vec3 np = normalizedPosD(sc, st.pos(j));
    ob[2] = np.x; ob[3] = np.y; ob[4] = np.z;
    pos_ob[0] = np.x; pos_ob[1] = np.y; pos_ob[2] = np.z;
    ob[5] = 0.5f * ((st.f(kOsYaw, j) / kPi) + 1.f);
    ob[6] = 0.5f * (st.f(kOsPitch, j) / (0.25f * kPi) + 1.f);
    Vec3 rv = rotateVec(sf.invRot, st.vel(j));
    ob[7] = rv.x; ob[8] = rv.y; ob[9] = rv.z;
    ob[10] = st.f(kOsDYV, j); ob[11] = st.f(kOsDPV, j);
    const int cp = st.i(kOsCurPose, j), tp = st.i(kOsTgtPose, j);
    ob[12] = cp == kStand ? 1.f : 0.f;
    ob[13] = cp == kCrouch ? 1.f : 0.f;
    ob[14] = cp == kProne ? 1.f : 0.f;
    ob[15] = tp == kStand ? 1.f : 0.f;
    ob[16] = tp == kCrouch ? 1.f : 0.f;
    ob[17] = tp == kProne ? 1.f : 0.f;
    ob[18] = (float)st.i(kOsTrans, j) / (float)c::kPoseTransitionSpeed;
    ob[19] = (st.i(kOsFlags, j) & kFlagInZone) ? 1.f : 0.f;
    const int wt = st.i(kOsWeapon, j);
    ob[20] = wt == 0 ? 1.f : 0.f;
    ob[21] = wt == 1 ? 1.f : 0.f;
    ob[22] = wt == 2 ? 1.f : 0.f;
    return true;
}

__device__ __forceinline__ void fillCombatS(const ObsStage &st, int j, float *ob)
{
    ob[0] = st.f(kOsHP, j) / 100.f;
    ob[1] = (float)st.i(kOsMag0, j);
    ob[2] = (float)st.i(kOsMag1, j);
    ob[3] = float(st.i(kOsHeal, j)) / float(c::kOutOfCombatSteps);
}

__device__ __forceinline__ void fillOtherS(const ObsStage &st, const SelfFrame &sf, int j, float *ob)
{
    relAnglesD(sf, st.pos(j) - sf.pos, ob[23], ob[24], ob[25]);
    float rfy = st.f(kOsYaw, j) - sf.yaw;
    float rfp = st.f(kOsPitch, j) - sf.pitch;
    if (rfy > kPi) rfy -= 2.f * kPi;
    else if (rfy < -kPi) rfy += 2.f * kPi;
    ob[26] = rfy;
    ob[27] = rfp;
}

// Half-wave row stage.  `buf` holds 32 rows (stride P <= kObsSpanPad floats)
// and `offs` 32 row offsets.  Half h = lanes [32h, 32h + 32) of the wave's
// m live lanes (a tail wave's lanes past A have returned).  Pattern:
//   stage(h, ...) by the half's lanes -> waveSync -> flush*(h, ...) by every
//   live lane -> waveSync (reads done before the next rows land).
// The cross-lane exchange stays inside one wave: the wave's DS instructions
// execute in issue order, so only the compiler needs ordering, which the
// wavefront-scope fences of waveSync give.
struct HalfStage {
    float *buf;
    int64_t *offs;
    int lane, m;

    __device__ __forceinline__ int halves() const { return m > 32 ? 2 : 1; }
    __device__ __forceinline__ int rowsOf(int h) const { return m - 32 * h < 32 ? m - 32 * h : 32; }
    __device__ __forceinline__ bool mine(int h) const { return (lane >> 5) == h; }
    template <int P> __device__ __forceinline__ void stage(int h, const float *v, int n, int at = 0) const
    {
        if (mine(h))
            for (int k = 0; k < n; k++) buf[(lane & 31) * P + at + k] = v[k];
    }
    __device__ __forceinline__ void stageOff(int h, int64_t off) const
    {
        if (mine(h)) offs[lane & 31] = off;
    }
    // Rows of half h back to back from dst (row r at dst + r * n; the
    // caller passes dst at the half's first row).  float4 when dst is 16-B
    // aligned (a world group starting off a 4-agent boundary is not).
    template <int n, int P> __device__ __forceinline__ void flushSpan(int h, float *dst) const
    {
        const int total = rowsOf(h) * n;
        auto val = [&](int f) {
            const int r = f / n;
            return buf[r * P + (f - r * n)];
        };
        if ((reinterpret_cast<uintptr_t>(dst) & 15u) == 0) {
            const int q4 = total >> 2;
            // rolled, one division per float4 (the four floats walk the
            // staged row and wrap to the next): unrolled, the compiler hoisted
            // per-element LDS offsets out of the loop and held ~40 VGPRs
#pragma unroll 1
            for (int j = lane; j < q4; j += m) {
                int r = (4 * j) / n, c = 4 * j - r * n;
                float v[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    v[q] = buf[r * P + c];
                    if (++c == n) {
                        c = 0;
                        r++;
                    }
                }
                reinterpret_cast<float4 *>(dst)[j] = make_float4(v[0], v[1], v[2], v[3]);
            }
            if (lane < (total & 3)) dst[4 * q4 + lane] = val(4 * q4 + lane);
        } else {
#pragma unroll 1
            for (int f = lane; f < total; f += m) dst[f] = val(f);
        }
    }
    // 32-float rows: row r of half h to arr[((gw0 + 32h + r) * slots + k) * 32]
    // as 8 float4 pieces (each store instruction writes 8 whole rows).
    template <int P> __device__ __forceinline__ void flushRows32(int h, float *arr, int slots, int k, int64_t gw0) const
    {
        static_assert(P % 4 == 0, "float4 rows");
        const int nc = rowsOf(h) * (kOtherObs / 4);
        float *base = arr + ((gw0 + 32 * h) * slots + k) * kOtherObs;
        // <= 32 rows x 8 pieces over m >= rows lanes: at most 8 rounds (4 in a full wave)
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int c = lane + j * m;
            if (c < nc) {
                const int r = c >> 3, col = c & 7;
                const uint32_t o = (uint32_t)(r * slots * kOtherObs + col * 4); // < 32 rows x 6 slots x 32
                *reinterpret_cast<float4 *>(base + o) = reinterpret_cast<const float4 *>(buf + r * P)[col];
            }
        }
    }
    // Rows of n floats at per-row offsets (offs, staged with stageOff) into
    // dst; wbits / zbits: wave ballots of "row exists" / "row is zeros".
    template <int n, int P> __device__ __forceinline__ void flushOff(int h, float *dst, uint64_t wbits, uint64_t zbits) const
    {
        const uint32_t wb = (uint32_t)(wbits >> (32 * h)), zb = (uint32_t)(zbits >> (32 * h));
        const int total = rowsOf(h) * n;
#pragma unroll 1
        for (int c = lane; c < total; c += m) {
            const int r = c / n, col = c - r * n;
            if ((wb >> r) & 1u) dst[offs[r] + col] = ((zb >> r) & 1u) ? 0.f : buf[r * P + col];
        }
    }
    // The same for rows of n4 float4 (16-B aligned rows, P a multiple of 4).
    template <int n4, int P> __device__ __forceinline__ void flushOff4(int h, float *dst, uint64_t wbits, uint64_t zbits) const
    {
        static_assert(P % 4 == 0, "float4 rows");
        const uint32_t wb = (uint32_t)(wbits >> (32 * h)), zb = (uint32_t)(zbits >> (32 * h));
        const int total = rowsOf(h) * n4;
        for (int c = lane; c < total; c += m) {
            const int r = c / n4, col = c - r * n4;
            if ((wb >> r) & 1u)
                reinterpret_cast<float4 *>(dst + offs[r])[col] =
                    ((zb >> r) & 1u) ? make_float4(0.f, 0.f, 0.f, 0.f) : reinterpret_cast<const float4 *>(buf + r * P)[col];
        }
    }
    // A contiguous span export (lane r's n floats at dst + r * n).
    template <int n> __device__ __forceinline__ void putSpan(float *dst, const float *vals) const
    {
        constexpr int P = n | 1; // odd stride: conflict-free staging
        static_assert(P <= kObsSpanPad, "span larger than the row stage");
        for (int h = 0; h < halves(); h++) {
            stage<P>(h, vals, n);
            waveSync();
            flushSpan<n, P>(h, dst + (int64_t)32 * h * n);
            waveSync();
        }
    }
};

// kWire: the learner's rebuild of a shadow's rows from a wire message
// (wire.hip launchWireUnpack): S is a view whose input columns point into
// the message (the same SoA columns the sender's engine holds), the packed
// pose / weapon / flags word is split here, the full-team rows (not
// trainInterface outputs) are skipped, and a world whose episode counter
// moved since the previous message has every last-known row written -- the
// reset's clear on the sender (resetAgentD / resetPersistentEntitiesD),
// then this step's updates -- exactly the rows the sender's k_obs leaves.
// (One templated kernel, k_obs<false> on the step path and k_obs<true> =
// "k_obs_wire" on the learner: the same body as a __device__ function under
// two kernels compiled ~45% more instructions and ran 6% slower.)
template <bool kWire>
__global__ void __launch_bounds__(kObsBlock) __attribute__((amdgpu_waves_per_eu(3)))
k_obs(DevState S, SceneDev sc, WireObs wo)
{
    __shared__ float ost[kObsCols][kObsStageMax];
    __shared__ __attribute__((aligned(16))) float rowBuf[kObsBlock / 64][32 * kObsSpanPad];
    __shared__ int64_t offBuf[kObsBlock / 64][32];
    // a learner shadow out of wire sync keeps its rows (wire.hip wireOk);
    // the same word for every thread of the grid
    if (S.obsGate && (*S.obsGate & MPENV_WIRE_ERR_DESYNC)) return;
    const int T = S.T, N = S.N;
    const int64_t b0 = (int64_t)xcdBlockId() * kObsBlock; // < A (grid = ceil(A / kObsBlock))
    const int64_t g = b0 + threadIdx.x;
    const bool live = g < S.A;

    // ---- loads: the block's worlds' agent columns, then this lane's own
    // rotation and world fields (no store is issued before all of them)
    const int64_t a_end = b0 + kObsBlock < S.A ? b0 + kObsBlock : S.A;
    const int64_t s0 = (b0 / N) * N;
    const int ns = (int)(((a_end - 1) / N + 1) * N - s0);
    for (int k = threadIdx.x; k < ns; k += kObsBlock) {
        const int64_t j = s0 + k;
        ost[kOsPX][k] = S.px[j];
        ost[kOsPY][k] = S.py[j];
        ost[kOsPZ][k] = S.pz[j];
        ost[kOsVX][k] = S.vx[j];
        ost[kOsVY][k] = S.vy[j];
        ost[kOsVZ][k] = S.vz[j];
        ost[kOsYaw][k] = S.ayaw[j];
        ost[kOsPitch][k] = S.apitch[j];
        ost[kOsDYV][k] = S.dyv[j];
        ost[kOsDPV][k] = S.dpv[j];
        ost[kOsHP][k] = S.hp[j];
        ost[kOsFired][k] = S.firedT[j];
        ost[kOsAlive][k] = S.alive[j];
        if constexpr (kWire) {
            const uint32_t p = wo.packed[j]; // curPose | tgtPose << 8 | weapon << 16 | flags << 24
            ost[kOsCurPose][k] = __int_as_float((int32_t)(p & 0xffu));
            ost[kOsTgtPose][k] = __int_as_float((int32_t)((p >> 8) & 0xffu));
            ost[kOsWeapon][k] = __int_as_float((int32_t)((p >> 16) & 0xffu));
            ost[kOsVis][k] = __int_as_float((int32_t)S.visMask[j]);
            ost[kOsTrans][k] = __int_as_float(S.transRem[j]);
            ost[kOsFlags][k] = __int_as_float((int32_t)(p >> 24));
        } else {
            ost[kOsCurPose][k] = __int_as_float(S.curPose[j]);
            ost[kOsTgtPose][k] = __int_as_float(S.tgtPose[j]);
            ost[kOsWeapon][k] = __int_as_float(S.weapon[j]);
            ost[kOsVis][k] = __int_as_float((int32_t)S.visMask[j]);
            ost[kOsTrans][k] = __int_as_float(S.transRem[j]);
            ost[kOsFlags][k] = __int_as_float(S.flags[j]);
        }
        ost[kOsShot][k] = __int_as_float(S.wasShot[j]);
        ost[kOsHeal][k] = __int_as_float(S.autohealSteps[j]);
        ost[kOsMag0][k] = __int_as_float(S.magazine[2 * j]);
        ost[kOsMag1][k] = __int_as_float(S.magazine[2 * j + 1]);
    }
    const int64_t gs = live ? g : S.A - 1; // tail lanes load a valid agent's fields, then leave
    const int w = (int)(gs / N);
    const int i = (int)(gs - (int64_t)w * N);
    const int team = i / T, off = i - team * T;
    const Quat rot = ldRot(S, gs);
    const int cur_step = S.curStep[w];
    const int fm = team == 0 ? S.filtMatched0[w] : S.filtMatched1[w];
    const int cz = S.curZone[w];
    const int ctrl = S.controlling[w];
    const int contested = S.contested[w], captured = S.captured[w];
    const int until_point = S.stepsUntilPoint[w], zone_steps = S.zoneSteps[w];
    const AABB za = sc.tab->zoneAABB[cz];
    // the pure outputs' destinations: the engine's exports, or during a
    // gpuStreamStep the caller's buffers (OutTab; uniform loads, issued with
    // the other loads before the barrier)
    float *oMasks = S.masks, *oFilters = S.filters, *oSelf = S.selfObs, *oSelfPos = S.selfPos;
    float *oTm = S.tmObs, *oTmPos = S.tmPos, *oOpp = S.oppObs, *oOppPos = S.oppPos;
    if (!kWire && S.outTab && S.outTab->on) {
        const OutTab *t = S.outTab;
        const int64_t b = S.outBase;
        oMasks = t->masks + b * 6;
        oFilters = t->filters + b;
        oSelf = t->selfObs + b * kSelfObs;
        oSelfPos = t->selfPos + b * 3;
        oTm = t->tmObs + b * 5 * kOtherObs;
        oTmPos = t->tmPos + b * 15;
        oOpp = t->oppObs + b * 6 * kOtherObs;
        oOppPos = t->oppPos + b * 18;
    }
    bool wreset = false; // kWire: the world's episode counter moved since the previous message
    if constexpr (kWire) wreset = !wo.keyframe && wo.epPrev[w] != S.episodeCounter[w];
    __syncthreads();
    if (!live) return; // the flushes count the live lanes

    const ObsStage st { ost };
    const int lane = threadIdx.x & 63;
    const int64_t gw0 = g - lane; // first agent of the wave
    HalfStage hs;
    hs.buf = rowBuf[threadIdx.x >> 6];
    hs.offs = offBuf[threadIdx.x >> 6];
    hs.lane = lane;
    hs.m = (int)(S.A - gw0 < 64 ? S.A - gw0 : 64);
    const int64_t g0 = (int64_t)w * N;
    const int me = (int)(g - s0), l0 = (int)(g0 - s0); // stage indices: this agent, its world's first
    const bool self_alive = st.alive(me);

    // ---- masks
    float mask[kMaxTeamSize];
    for (int k = 0; k < kMaxTeamSize; k++) {
        mask[k] = 0.f;
        if (!self_alive || k >= T) continue;
        const int jo = l0 + (team ^ 1) * T + k;
        if (!st.alive(jo)) continue;
        bool can_see = (st.i(kOsVis, me) >> k) & 1;
        for (int t = 0; t < T - 1 && !can_see; t++) {
            const int jt = l0 + team * T + (t < off ? t : t + 1);
            if ((st.i(kOsVis, jt) >> k) & 1) can_see = true;
        }
        if (can_see) mask[k] = 1.f;
        if (st.f(kOsFired, jo) >= 0) mask[k] = 1.f;
    }
    hs.putSpan<6>(oMasks + gw0 * 6, mask);
    // teamKnowsLocation (mask[k] == 1) as bits for the opponent loop.
    // Reading the float array there instead gave wrong last-known updates in
    // round 2 -- a register miscompile of the float form ("k_obs
    // mask read"); the bits form is taken right here.
    uint32_t knowsBits = 0;
    for (int k = 0; k < kMaxTeamSize; k++) knowsBits |= (mask[k] == 1.f ? 1u : 0u) << k;

    oFilters[g] = (cur_step - fm < 5) ? 1.f : 0.f;

    // ---- fullTeamObservationsSystem, per (world, team): the global
    // observation and the zeroed slots past team_size (slot-0 agents)
    const int64_t mine = (int64_t)w * 2 + team, theirs = (int64_t)w * 2 + (team ^ 1);
    if (!kWire && off == 0) {
        for (int s = T; s < kMaxTeamSize; s++) {
            for (int k = 0; k < MPENV_FT_PLAYER_DIM; k++) S.ftPlayers[(mine * 6 + s) * MPENV_FT_PLAYER_DIM + k] = 0.f;
            for (int k = 0; k < MPENV_FT_ENEMY_DIM; k++) S.ftEnemies[(mine * 6 + s) * MPENV_FT_ENEMY_DIM + k] = 0.f;
            for (int k = 0; k < MPENV_FT_COMMON_DIM; k++) S.ftLastKnown[(mine * 6 + s) * MPENV_FT_COMMON_DIM + k] = 0.f;
        }
        float gob[MPENV_FT_GLOBAL_DIM];
        gob[0] = team == 0 ? 0.f : 1.f;
        gob[1] = team == 0 ? 1.f : 0.f;
        gob[2] = float(c::kEpisodeLen - cur_step) / c::kEpisodeLen;
        const Vec3 nc = normalizedPosUnclampedD(sc, (za.pMax + za.pMin) / 2.f);
        gob[3] = nc.x; gob[4] = nc.y; gob[5] = nc.z;
        gob[6] = ctrl == team ? 1.f : 0.f;
        gob[7] = (ctrl != -1 && ctrl != team) ? 1.f : 0.f;
        gob[8] = contested ? 1.f : 0.f;
        gob[9] = captured ? 1.f : 0.f;
        gob[10] = float(until_point) / float(c::kZonePointInterval);
        gob[11] = float(zone_steps) / float(c::kNumStepsPerZone);
        for (int k = 0; k < 4; k++) gob[12 + k] = cz == k ? 1.f : 0.f;
        static_assert(MPENV_FT_GLOBAL_DIM == 16, "ft global row: 4 float4");
        float4 *gdst = reinterpret_cast<float4 *>(&S.ftGlobal[mine * MPENV_FT_GLOBAL_DIM]);
        for (int q = 0; q < 4; q++) gdst[q] = make_float4(gob[4 * q], gob[4 * q + 1], gob[4 * q + 2], gob[4 * q + 3]);
    }

    // ---- self observation
    SelfFrame sf;
    sf.pos = st.pos(me);
    sf.invRot = qinv(rot);
    sf.yaw = st.f(kOsYaw, me);
    sf.pitch = st.f(kOsPitch, me);
    {
        float ob[kSelfObs];
        float pos3[3];
        for (int k = 0; k < kSelfObs; k++) ob[k] = 0.f;
        pos3[0] = pos3[1] = pos3[2] = -1000.f;
        if (fillCommonS(st, sc, sf, me, ob, pos3)) {
            fillCombatS(st, me, &ob[23]);
            float *zo = &ob[27];
            Vec3 center = (za.pMax + za.pMin) / 2.f;
            Vec3 nc = normalizedPosD(sc, center);
            zo[0] = nc.x; zo[1] = nc.y; zo[2] = nc.z;
            relAnglesD(sf, center - sf.pos, zo[3], zo[4], zo[5]);
            zo[6] = (ctrl == team) ? 1.f : 0.f;
            zo[7] = (ctrl != -1 && ctrl != team) ? 1.f : 0.f;
            zo[8] = contested ? 1.f : 0.f;
            zo[9] = captured ? 1.f : 0.f;
            zo[10] = float(until_point) / float(c::kZonePointInterval);
            zo[11] = float(zone_steps) / float(c::kNumStepsPerZone);
            zo[12] = cz == 0 ? 1.f : 0.f;
            zo[13] = cz == 1 ? 1.f : 0.f;
            zo[14] = cz == 2 ? 1.f : 0.f;
            zo[15] = cz == 3 ? 1.f : 0.f;
        }
        static_assert(kSelfObs == 43 && (kSelfObs | 1) <= kObsSpanPad, "self obs span");
        hs.putSpan<kSelfObs>(oSelf + gw0 * kSelfObs, ob);
        hs.putSpan<3>(oSelfPos + gw0 * 3, pos3);
    }
    const bool alive_ok = self_alive; // fillCommonOb's alive test of the agent itself

    // Slot positions (teammate, opponent, last-known rows) are recomputed
    // after each slot loop in fully unrolled form: written from inside the
    // rolled loops, the arrays were indexed dynamically and went to scratch,
    // whose loads would wait behind the row stores.
    auto slotPos = [&](bool exists, int j, float *p3) {
        if (exists && st.alive(j)) {
            const Vec3 np = normalizedPosD(sc, st.pos(j));
            p3[0] = np.x; p3[1] = np.y; p3[2] = np.z;
        } else {
            p3[0] = p3[1] = p3[2] = -1000.f;
        }
    };
    auto mateIdx = [&](int k) { return l0 + team * T + (k < off ? k : k + 1); };
    auto oppIdx = [&](int k) { return l0 + (team ^ 1) * T + k; };

    // ---- teammates
    {
        for (int k = 0; k < kMaxTeamSize - 1; k++) {
            float row[kOtherObs];
            float unused[3];
            for (int q = 0; q < kOtherObs; q++) row[q] = 0.f;
            if (alive_ok && k < T - 1) {
                const int jt = mateIdx(k);
                if (fillCommonS(st, sc, sf, jt, row, unused)) {
                    fillOtherS(st, sf, jt, row);
                    fillCombatS(st, jt, &row[28]);
                }
            }
            for (int h = 0; h < hs.halves(); h++) {
                hs.stage<kObsRowPad>(h, row, kOtherObs);
                waveSync();
                hs.flushRows32<kObsRowPad>(h, oTm, 5, k, gw0);
                waveSync();
            }
        }
        float tpos[15];
#pragma unroll
        for (int k = 0; k < kMaxTeamSize - 1; k++) slotPos(alive_ok && k < T - 1, mateIdx(k), &tpos[3 * k]);
        hs.putSpan<15>(oTmPos + gw0 * 15, tpos);
    }

    // ---- opponents (+ last known)
    {
        uint32_t lkWrite = 0, lkKeep = 0; // per slot: last-known row written / kept (else cleared)
        for (int k = 0; k < kMaxTeamSize; k++) {
            float row[kOtherObs];
            float unused[3];
            for (int q = 0; q < kOtherObs; q++) row[q] = 0.f;
            // last-known slot: cleared (opponent dead / just killed), then
            // overwritten with the observation when the team knows the location
            bool lk_write = false, lk_keep = false;
            if (alive_ok && k < T) {
                const int jo = oppIdx(k);
                if (!fillCommonS(st, sc, sf, jo, row, unused)) {
                    lk_write = true;
                } else {
                    fillOtherS(st, sf, jo, row);
                    if (st.i(kOsFlags, jo) & kFlagWasKilled) lk_write = true;
                    row[28] = (float)st.i(kOsShot, jo);
                    row[29] = st.f(kOsFired, jo) >= 0.f ? 1.f : 0.f;
                    row[30] = ((st.i(kOsVis, me) >> k) & 1) ? 1.f : 0.f;
                    // teamKnowsLocation (sim.cpp:2995-3003)
                    const bool knows = (knowsBits >> k) & 1u;
                    row[31] = knows ? 1.f : 0.f;
                    lk_keep = knows;
                    lk_write = lk_write || knows;
                }
            }
            lk_write = lk_write || wreset;
            lkWrite |= (lk_write ? 1u : 0u) << k;
            lkKeep |= (lk_keep ? 1u : 0u) << k;
            if (S.stats) statAdd(S.stats + kStatLkRows, lk_write ? 1u : 0u);
            const uint64_t wb = __ballot(lk_write), zb = __ballot(!lk_keep);
            for (int h = 0; h < hs.halves(); h++) {
                hs.stage<kObsRowPad>(h, row, kOtherObs);
                hs.stageOff(h, (g * 6 + k) * kOtherObs);
                waveSync();
                hs.flushRows32<kObsRowPad>(h, oOpp, 6, k, gw0);
                // the staged row is also the last-known copy
                hs.flushOff4<kOtherObs / 4, kObsRowPad>(h, S.lkObs, wb, zb);
                waveSync();
            }
        }
        float opos[18];
#pragma unroll
        for (int k = 0; k < kMaxTeamSize; k++) slotPos(alive_ok && k < T, oppIdx(k), &opos[3 * k]);
        hs.putSpan<18>(oOppPos + gw0 * 18, opos);
        // last-known positions: the written slots of each row (kept: the
        // observed position, cleared: -1000)
        {
            float lpos[18];
#pragma unroll
            for (int q = 0; q < 18; q++) lpos[q] = ((lkKeep >> (q / 3)) & 1u) ? opos[q] : -1000.f;
            constexpr int P = 19;
            for (int h = 0; h < hs.halves(); h++) {
                hs.stage<P>(h, lpos, 18);
                hs.stageOff(h, (int64_t)lkWrite); // the row's slot mask (rows at g * 18)
                waveSync();
                const int total = hs.rowsOf(h) * 18;
                float *dst = S.lkPos + (gw0 + 32 * h) * 18;
#pragma unroll 1
                for (int c = lane; c < total; c += hs.m) {
                    const int r = c / 18, col = c - r * 18;
                    if ((hs.offs[r] >> (col / 3)) & 1) dst[c] = hs.buf[r * P + col];
                }
                waveSync();
            }
        }
    }

    // ---- fullTeamObservationsSystem, the part owned by agent g (team, slot
    // off): its player slot in its own team's interface, its enemy and
    // last-known slots in the other team's interface (the common block is the
    // same in all three, the one-hot id is the slot).  Positions are
    // normalised without the clamp pvpObservations applies.  The lidar copy is
    // fused into k_lidar.
    if constexpr (!kWire) {
        const bool alive = self_alive;
        // enemy-only fields first: they decide whether the last-known slot
        // receives the common block
        const float fired = alive && st.f(kOsFired, me) >= 0.f ? 1.f : 0.f;
        bool knows = fired != 0.f;
        uint32_t los = 0;
        if (alive) {
            const int jm0 = l0 + (team ^ 1) * T;
            for (int mm = 0; mm < T; mm++) los |= ((st.i(kOsVis, jm0 + mm) >> off) & 1u) << mm;
            knows = knows || los != 0;
        }
        float cm[MPENV_FT_ENEMY_DIM]; // the common block, then the enemy tail
        cm[0] = 1.f;
        for (int k = 0; k < kMaxTeamSize; k++) cm[1 + k] = k == off ? 1.f : 0.f;
        for (int k = 7; k < MPENV_FT_COMMON_DIM; k++) cm[k] = 0.f;
        float ext[4] = { 0.f, 0.f, 0.f, 0.f };
        if (alive) {
            cm[7] = 1.f;
            const Vec3 np = normalizedPosUnclampedD(sc, st.pos(me));
            cm[8] = np.x; cm[9] = np.y; cm[10] = np.z;
            cm[11] = 0.5f * ((st.f(kOsYaw, me) / kPi) + 1.f);
            cm[12] = 0.5f * (st.f(kOsPitch, me) / (0.25f * kPi) + 1.f);
            cm[13] = st.f(kOsVX, me); cm[14] = st.f(kOsVY, me); cm[15] = st.f(kOsVZ, me);
            const int cp = st.i(kOsCurPose, me), tp = st.i(kOsTgtPose, me);
            cm[16] = cp == kStand ? 1.f : 0.f;
            cm[17] = cp == kCrouch ? 1.f : 0.f;
            cm[18] = cp == kProne ? 1.f : 0.f;
            cm[19] = tp == kStand ? 1.f : 0.f;
            cm[20] = tp == kCrouch ? 1.f : 0.f;
            cm[21] = tp == kProne ? 1.f : 0.f;
            cm[22] = (float)st.i(kOsTrans, me) / (float)c::kPoseTransitionSpeed;
            cm[23] = (st.i(kOsFlags, me) & kFlagInZone) ? 1.f : 0.f;
            ext[0] = st.f(kOsHP, me) / 100.f;
            ext[1] = (float)st.i(kOsMag0, me) / 30;
            ext[2] = (float)st.i(kOsMag1, me);
            ext[3] = float(st.i(kOsHeal, me)) / float(c::kOutOfCombatSteps);
        }
        cm[MPENV_FT_COMMON_DIM + 0] = alive ? (float)st.i(kOsShot, me) : 0.f;
        cm[MPENV_FT_COMMON_DIM + 1] = fired;
        for (int mm = 0; mm < kMaxTeamSize; mm++) cm[MPENV_FT_COMMON_DIM + 2 + mm] = (los >> mm) & 1u ? 1.f : 0.f;
        cm[MPENV_FT_COMMON_DIM + 8] = knows ? 1.f : 0.f;
        static_assert(MPENV_FT_ENEMY_DIM == MPENV_FT_COMMON_DIM + 9, "ft enemy tail");
        // one staged row serves all three slots: the common block + enemy
        // tail; the player tail is staged over the enemy tail after the
        // enemy row has left
        constexpr int P = kObsRowPad;
        static_assert(MPENV_FT_ENEMY_DIM <= P && MPENV_FT_PLAYER_DIM <= P, "ft rows");
        static_assert(MPENV_FT_COMMON_DIM % 4 == 0 && MPENV_FT_PLAYER_DIM % 4 == 0, "16-B ft rows");
        const uint64_t all = __ballot(true), zlk = __ballot(!knows);
        for (int h = 0; h < hs.halves(); h++) {
            hs.stage<P>(h, cm, MPENV_FT_ENEMY_DIM);
            hs.stageOff(h, (theirs * 6 + off) * MPENV_FT_ENEMY_DIM);
            waveSync();
            hs.flushOff<MPENV_FT_ENEMY_DIM, P>(h, S.ftEnemies, all, 0ull);
            waveSync();
            hs.stage<P>(h, ext, 4, MPENV_FT_COMMON_DIM);
            hs.stageOff(h, (theirs * 6 + off) * MPENV_FT_COMMON_DIM);
            waveSync();
            hs.flushOff4<MPENV_FT_COMMON_DIM / 4, P>(h, S.ftLastKnown, all, zlk);
            waveSync();
            hs.stageOff(h, (mine * 6 + off) * MPENV_FT_PLAYER_DIM);
            waveSync();
            hs.flushOff4<MPENV_FT_PLAYER_DIM / 4, P>(h, S.ftPlayers, all, 0ull);
            waveSync();
        }
    }
}

// pvpLidarSystem (sim.cpp:3324-3506).  Lane = ray.  Rays are dealt to
// waves in units of 4 agents = 5 wave tasks: tasks 0-3 carry one agent's 64
// forward rays each (32 angles x 2 heights, one origin and a narrow fan, so
// the wave's lanes walk similar BVH paths), task 4 the 4 agents' 16 rear rays.
// Against 64 consecutive rays of the flat [agent][80] order (which straddle
// two agents in 4 of 5 waves) this cuts the wave-lockstep node iterations by
// ~12% and triangle tests by ~19% (tools/trav_stats.cpp on recorded rays);
// every lane's arithmetic is unchanged.  A block's 4 waves take `iters`
// consecutive task quads: up to kLidarIters (amortises the BVH staging) on
// big batches, fewer on small ones so the grid still spreads over the CUs
// (at 64 worlds 1v1 a fixed 8 put the whole lidar on 5 CUs).
constexpr int kLidarIters = 6; // round 5, one world group: 4: 0.665, 5: 0.642, 6: 0.643 ms steady, step 1.185 / 1.168 / 1.163 ms (profiles/r05m_lab_lidar_iters.jsonl; round 2: 1: 0.98, 2: 0.91, 4: 0.89, 8: 0.92 ms)
// 1024-thread blocks: the 8 octant node images + the three rotated vertex
// copies (31 + 36 KB on simple_map) are staged once per 16 waves, so 2
// blocks per CU (8 waves per SIMD) fit the 160 KB of LDS.
constexpr int kLidarBlock = 1024;
constexpr int kLidarWaves = kLidarBlock / 64;
constexpr int kLidarStageMax = 112, kLidarStageCols = 12; // k_lidar's per-block agent stage
static_assert(4 * ((kLidarIters * kLidarWaves) / 5 + 2) + 2 * (2 * kMaxTeamSize - 1) <= kLidarStageMax,
              "k_lidar agent stage");

__device__ __host__ __forceinline__ int64_t lidarTasks(int64_t A) { return ((A + 3) / 4) * 5; }

// 8 waves per SIMD (64 VGPRs, a few bytes of spill outside the traversal
// loop): latency-bound LDS traversal gains more from occupancy (-7%).
#define MP_LIDAR_ATTR __attribute__((amdgpu_waves_per_eu(8)))

// Maximum over the lane's DPP row (16 lanes) of non-negative float bit
// patterns compared as signed ints (the float order; -0 sorts lowest): the
// exact float maximum of the row's hit distances, without LDS round trips.
__device__ __forceinline__ int rowMaxBits16(int v)
{
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false));  // quad_perm [1, 0, 3, 2]
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false));  // quad_perm [2, 3, 0, 1]
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x124, 0xF, 0xF, false)); // row_ror:4
    return max(v, __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false)); // row_ror:8
}

__global__ void __launch_bounds__(kLidarBlock) MP_LIDAR_ATTR k_lidar(DevState S, SceneDev sc, int iters)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // Ray-fan directions (sim.cpp:3324-3506): theta depends only on the ray
    // slot, so the 32 forward + 8 rear (-cos, sin) pairs are computed once
    // per workgroup with the same sinf_/cosf_ and read from LDS.
    __shared__ float2 fan[32 + 8];
    if (threadIdx.x < 40) {
        const bool fwd = threadIdx.x < 32;
        const int x = fwd ? threadIdx.x : threadIdx.x - 32;
        const int width = fwd ? 32 : 8;
        const float range = fwd ? 0.75f * kPi : -kPi;
        const float offset = fwd ? 0.5f * (1.f - 0.75f) * kPi : 0.f;
        const float theta = range * (float(x) / float(width - 1)) + offset;
        fan[threadIdx.x] = make_float2(-cosf_(theta), sinf_(theta));
    }
    const uint32_t N = (uint32_t)S.N, T = (uint32_t)S.T;
    const uint32_t A = (uint32_t)S.A;
    const uint32_t ntasks = (uint32_t)lidarTasks(S.A);
    // The agents this block's tasks read -- the rays' origins and frames and
    // every capsule of their worlds -- staged in LDS with the BVH: whole
    // worlds around the block's task range (<= 14 units of 4 agents plus a
    // partial world at each end: <= 78 agents, N <= 12), so no task waits
    // on HBM for them.
    __shared__ float agentStage[kLidarStageCols][kLidarStageMax];
    const uint32_t t0 = xcdBlockId() * (uint32_t)iters * kLidarWaves;
    const uint32_t t1 = min(ntasks, t0 + (uint32_t)iters * kLidarWaves);
    uint32_t s0 = 0, ns = 0;
    if (t0 < t1) {
        const uint32_t a_lo = (t0 / 5u) * 4u, a_hi = min(A, ((t1 - 1u) / 5u) * 4u + 4u);
        s0 = (a_lo / N) * N;
        ns = ((a_hi - 1u) / N + 1u) * N - s0;
        for (uint32_t k = threadIdx.x; k < ns; k += blockDim.x) {
            const uint32_t g = s0 + k;
            agentStage[0][k] = S.px[g];
            agentStage[1][k] = S.py[g];
            agentStage[2][k] = S.pz[g];
            agentStage[3][k] = S.aw[g];
            agentStage[4][k] = S.ax[g];
            agentStage[5][k] = S.ay[g];
            agentStage[6][k] = S.az[g];
            agentStage[7][k] = S.rw[g];
            agentStage[8][k] = S.rx[g];
            agentStage[9][k] = S.ry[g];
            agentStage[10][k] = S.rz[g];
            agentStage[11][k] = viewHeightD(S.curPose[g]);
        }
    }
    // gpuStreamStep's caller buffers (engine.h OutTab), read once with the staging
    const OutTab *ot = (S.outTab && S.outTab->on) ? S.outTab : nullptr;
    const LBVH bvh = stageBVHOct(smem, sc); // ends with __syncthreads
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int it = 0; it < iters; it++) {
        const uint32_t task = (xcdBlockId() * iters + it) * kLidarWaves + wave; // wave-uniform
        if (task >= ntasks) break;
        const uint32_t unit = task / 5u, sub = task - unit * 5u;
        const bool fwd = sub < 4u;
        // The ray of lane `ln`: a tail unit's lanes past A trace a copy of
        // the last agent's rays and store nothing.
        auto rayIndex = [&](uint32_t ln, uint32_t &g, bool &valid, uint32_t &kk) {
            const uint32_t g_raw = unit * 4u + (fwd ? sub : (ln >> 4));
            valid = g_raw < A;
            g = valid ? g_raw : A - 1u;
            kk = fwd ? ln : (ln & 15u); // ray slot within the forward / rear fan
        };
        auto makeRay = [&](uint32_t ln, uint32_t &g, bool &valid, uint32_t &kk, Vec3 &ray_o, Vec3 &dir) {
            rayIndex(ln, g, valid, kk);
            const uint32_t h = fwd ? (kk >> 5) : (kk >> 3), x = fwd ? (kk & 31u) : (kk & 7u);
            const uint32_t k = g - s0, qc = fwd ? 3u : 7u;
            const Quat q = quat(agentStage[qc][k], agentStage[qc + 1u][k], agentStage[qc + 2u][k],
                                agentStage[qc + 3u][k]);
            const Vec3 dir_fwd = rotateVec(q, kFwd);
            const Vec3 dir_right = rotateVec(q, kRight);
            const float top = agentStage[11][k] + c::kAgentRadius;
            ray_o = v3(agentStage[0][k], agentStage[1][k], agentStage[2][k]);
            ray_o.z += c::kAgentRadius + (top - 2.f * c::kAgentRadius) * (float(h) / float(2 - 1));
            const float2 cs = fan[fwd ? x : 32 + x];
            dir = normalize(cs.x * dir_right + cs.y * dir_fwd);
        };
        // Lane id read inside the loop (volatile: not hoisted), so the
        // lane-derived offsets are formed per task instead of living as
        // loop invariants across the traversal, which at 64 VGPRs the
        // compiler would spill to scratch.
        uint32_t lane;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
        uint32_t g, kk;
        bool valid;
        Vec3 ray_o, dir;
        // The BVH first (one traversal for both fan kinds), then the world's
        // capsules.  World / agent indices are formed after the traversal,
        // from an opaque copy of g (nothing but the ray lives across it).
        float tb;
        bool bhit;
        {
            makeRay(lane, g, valid, kk, ray_o, dir);
            // the ray's octant image: same nodes and leaves, near-first slot
            // order (scene.h octantNodeImages)
            LBVH ob = bvh;
            ob.nodes = reinterpret_cast<const MP_LDS BVHNode *>(reinterpret_cast<const MP_LDS uint4 *>(bvh.nodes) +
                                                                 rayOctant(dir) * sc.numLidarNodes * kOctNodeQ);
            bhit = bvhTraceRayT<false, kOctNodeQ, true, true>(ob, ray_o, dir, tb, kFltMax, 0.f);
        }
        // The lane id again (volatile) and the ray's indices from it: integer
        // work only, so they need not live across the traversal (at 64 VGPRs
        // they were spilled to scratch).  Shuffles below address lanes from
        // this id too (ds_bpermute), not from a lane id kept for the kernel.
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
        rayIndex(lane, g, valid, kk);
        auto shflLane = [](float v, uint32_t src) {
            return __int_as_float(__builtin_amdgcn_ds_bpermute((int)(src << 2), __float_as_int(v)));
        };
        const uint32_t w = __umulhi(g, S.nMagic); // g / N (engine.h)
        const uint32_t i = g - w * N;
        const int64_t g0 = (int64_t)w * N;
        WorldHit hw;
        if (fwd) {
            // Forward fan (one agent, one xy origin per wave): the BVH first,
            // then only the capsules some ray of the wave could hit before
            // its BVH hit.  Any point of capsule j lies within r of its
            // vertical axis, so a ray entering it at t has t >= d_xy - r
            // (d_xy = xy distance from the origin to the axis); a capsule
            // with d_xy - 1.01 r - 1 > max over the wave's rays of the BVH
            // hit t can enter no ray's `t < min_hit_t` (utils.cpp:57-69) and
            // is dropped for the whole wave (the margin dwarfs the rounding
            // of t ~ 1e-3 at these distances).  Lane j < N loads capsule j
            // once; the per-ray loop reads the survivors' bases from those
            // lanes (readlane) in ascending j, so ties resolve as before.
            float min_t = bhit ? tb : kFltMax;
            const int rm = rowMaxBits16(__float_as_int(min_t));
            const float mx = __int_as_float(max(max(__builtin_amdgcn_readlane(rm, 0), __builtin_amdgcn_readlane(rm, 16)),
                                                max(__builtin_amdgcn_readlane(rm, 32), __builtin_amdgcn_readlane(rm, 48))));
            float cx = 0.f, cy = 0.f, cz = 0.f;
            bool keep = false;
            if (lane < N) {
                const uint32_t k = (uint32_t)(g0 - s0) + lane;
                cx = agentStage[0][k]; cy = agentStage[1][k]; cz = agentStage[2][k];
                const float dx = cx - ray_o.x, dy = cy - ray_o.y;
                keep = lane != i && !(sqrtf(dx * dx + dy * dy) - c::kAgentRadius * 1.01f - 1.f > mx);
            }
            uint64_t cm = __ballot(keep);
            bool hit = bhit;
            int ent = -1;
            const float dxy2 = dir.x * dir.x + dir.y * dir.y;
            const float cull_r2 = (kCapsuleRadius * 1.01f) * (kCapsuleRadius * 1.01f);
            while (cm) {
                const int j = __builtin_ctzll(cm);
                cm &= cm - 1;
                Vec3 co = v3(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(cx), j)),
                             __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cy), j)),
                             __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cz), j)));
                co.z += kCapsuleRadius;
                const Vec3 tr = ray_o - co;
                // the per-ray conservative culls of capsulesD
                const float cr = tr.x * dir.y - tr.y * dir.x;
                if (cr * cr > cull_r2 * dxy2) continue;
                const float along = -(tr.x * dir.x + tr.y * dir.y + tr.z * dir.z);
                const float ahead = along + fmaxD(0.f, kCapsuleSegment * dir.z) + kCapsuleRadius * 1.01f;
                if (ahead < 0.f) continue;
                if (along + fminD(0.f, kCapsuleSegment * dir.z) - kCapsuleRadius * 1.01f > min_t) continue;
                const float t = intersectRayZOriginCapsule(tr, dir, kCapsuleRadius, kCapsuleSegment);
                if (t != 0 && t < min_t) {
                    min_t = t;
                    hit = true;
                    ent = j;
                }
            }
            hw.hit = hit;
            hw.t = min_t;
            hw.entity = ent;
        } else {
            // Rear fans: the same cull per 16-lane group (one agent, one xy
            // origin per group; N <= 12 capsules).  Lane q*16 + j < q*16 + N
            // loads capsule j of group q's world; the wave walks the union
            // of the groups' surviving j in ascending order and each lane
            // takes its group's copy (ds_bpermute) and tests only the j its
            // group kept -- per ray the same capsules in the same order as
            // capsulesD minus those no ray of the group can reach.
            float min_t = bhit ? tb : kFltMax;
            const float mx = __int_as_float(rowMaxBits16(__float_as_int(min_t)));
            const uint32_t gb = lane & 48u, jl = lane & 15u;
            float cx = 0.f, cy = 0.f, cz = 0.f;
            bool keep = false;
            if (jl < N) {
                const uint32_t k = (uint32_t)(g0 - s0) + jl;
                cx = agentStage[0][k]; cy = agentStage[1][k]; cz = agentStage[2][k];
                const float dx = cx - ray_o.x, dy = cy - ray_o.y;
                keep = jl != i && !(sqrtf(dx * dx + dy * dy) - c::kAgentRadius * 1.01f - 1.f > mx);
            }
            const uint64_t cm = __ballot(keep);
            uint32_t um = (uint32_t)((cm | (cm >> 16) | (cm >> 32) | (cm >> 48)) & 0xffffu);
            const uint32_t mine = (uint32_t)(cm >> gb) & 0xffffu;
            // the four agents in one world (always for 6v6: 4 divides N):
            // every group holds the same capsules, read from group 0's lanes
            const bool oneWorld = __ballot(w != (uint32_t)__builtin_amdgcn_readfirstlane((int)w)) == 0ull;
            bool hit = bhit;
            int ent = -1;
            const float dxy2 = dir.x * dir.x + dir.y * dir.y;
            const float cull_r2 = (kCapsuleRadius * 1.01f) * (kCapsuleRadius * 1.01f);
            while (um) {
                const int j = __builtin_ctz(um);
                um &= um - 1u;
                Vec3 co;
                if (oneWorld) {
                    co = v3(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(cx), j)),
                            __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cy), j)),
                            __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cz), j)));
                } else {
                    const uint32_t src = gb + (uint32_t)j;
                    co = v3(shflLane(cx, src), shflLane(cy, src), shflLane(cz, src));
                }
                if (!((mine >> j) & 1u)) continue;
                co.z += kCapsuleRadius;
                const Vec3 tr = ray_o - co;
                const float cr = tr.x * dir.y - tr.y * dir.x;
                if (cr * cr > cull_r2 * dxy2) continue;
                const float along = -(tr.x * dir.x + tr.y * dir.y + tr.z * dir.z);
                const float ahead = along + fmaxD(0.f, kCapsuleSegment * dir.z) + kCapsuleRadius * 1.01f;
                if (ahead < 0.f) continue;
                if (along + fminD(0.f, kCapsuleSegment * dir.z) - kCapsuleRadius * 1.01f > min_t) continue;
                const float t = intersectRayZOriginCapsule(tr, dir, kCapsuleRadius, kCapsuleSegment);
                if (t != 0 && t < min_t) {
                    min_t = t;
                    hit = true;
                    ent = j;
                }
            }
            hw.hit = hit;
            hw.t = min_t;
            hw.entity = ent;
        }
        if (!valid) continue;
        const bool second = i >= T; // team of the casting agent
        float4 out;
        if (hw.hit) {
            const bool wall = hw.entity == -1;
            const bool tm = !wall && ((uint32_t)hw.entity >= T) == second;
            out = make_float4(fminD(hw.t, sc.maxDist), wall ? 1.f : 0.f, tm ? 1.f : 0.f, (!wall && !tm) ? 1.f : 0.f);
        } else {
            out = make_float4(-1.f, 0.f, 0.f, 0.f);
        }
        // Addresses formed after the traversal (nothing but the ray lives
        // across it, so 64 VGPRs hold the loop without scratch spills).
        float4 *dst = fwd ? reinterpret_cast<float4 *>(S.fwdLidar) + (int64_t)g * kFwdRays + kk
                          : reinterpret_cast<float4 *>(S.rearLidar) + (int64_t)g * kRearRays + kk;
        const int64_t slot = ((int64_t)w * 2 + (second ? 1 : 0)) * kMaxTeamSize + (second ? i - T : i);
        float4 *tdst = fwd ? reinterpret_cast<float4 *>(S.ftFwdLidar) + slot * kFwdRays + kk
                           : reinterpret_cast<float4 *>(S.ftRearLidar) + slot * kRearRays + kk;
        // fullTeamObservationsSystem copies the lidar before this system
        // overwrites it (sim.cpp:5283-5310): the previous value moves into
        // the team interface's slot.
        *tdst = *dst;
        *dst = out;
        // gpuStreamStep: the caller's lidar buffer too (the engine's copy is
        // state: the bots and the next full-team copy read it), and the
        // agent's two agent maps zero-filled by its forward wave (4 KB each:
        // 4 store instructions of 64 x 16 B per map, no loads; the stores
        // drain while the wave's next traversal runs)
        if (ot) {
            const int64_t gb = S.outBase + (int64_t)g;
            float4 *cdst = fwd ? reinterpret_cast<float4 *>(ot->fwdLidar) + gb * kFwdRays + kk
                               : reinterpret_cast<float4 *>(ot->rearLidar) + gb * kRearRays + kk;
            *cdst = out;
            if (fwd) {
                const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
                float4 *m0 = reinterpret_cast<float4 *>(ot->agentMap0) + gb * 256 + kk;
                float4 *m1 = reinterpret_cast<float4 *>(ot->agentMap1) + gb * 256 + kk;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    m0[64 * q] = z;
                    m1[64 * q] = z;
                }
            }
        }
    }
}

static int check(hipError_t e) { return e == hipSuccess ? 0 : -1; }

// Debug/test hook: closest-hit BVH queries for caller rays (mode 0 = the
// traversal inlined into the step kernels, 1 = its out-of-line copy).
__global__ void __launch_bounds__(kBlock) k_trace_rays(SceneDev sc, const float *o, const float *d, int n, int mode,
                                                       float *t_out, int32_t *hit_out)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const LBVH bvh = stageBVH(smem, sc);
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const Vec3 org = v3(o[3 * r], o[3 * r + 1], o[3 * r + 2]);
    const Vec3 dir = v3(d[3 * r], d[3 * r + 1], d[3 * r + 2]);
    float t = 0.f;
    bool hit;
    if (mode == 0) {
        hit = bvhTraceRayD(bvh, org, dir, t); // inlined, as in the step kernels
    } else {
        RayHitD h = bvhTraceRayExactD(bvh, org, dir);
        hit = h.hit != 0;
        t = h.t;
    }
    t_out[r] = hit ? t : 0.f;
    hit_out[r] = hit ? 1 : 0;
}

int launchTraceRays(const SceneDev &sc, const float *o, const float *d, int n, int mode, float *t, int32_t *hit,
                    void *stream)
{
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_trace_rays, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), bvhLdsBytes(sc),
                       (hipStream_t)stream, sc, o, d, n, mode, t, hit);
    return check(hipGetLastError());
}

// Debug gather of internal state into the MPENV_EXPORT_DEBUG_* layouts.
__global__ void __launch_bounds__(256) k_debug(DevState S, float *af, int32_t *ai, int32_t *wi, float *wf,
                                               uint32_t *explore, float *crumbs)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < S.A) {
        const int64_t g = t;
        float *f = &af[g * MPENV_DBG_AF_COUNT];
        f[0] = S.px[g]; f[1] = S.py[g]; f[2] = S.pz[g];
        f[3] = S.vx[g]; f[4] = S.vy[g]; f[5] = S.vz[g];
        f[6] = S.rw[g]; f[7] = S.rx[g]; f[8] = S.ry[g]; f[9] = S.rz[g];
        f[10] = S.ayaw[g]; f[11] = S.apitch[g];
        f[12] = S.aw[g]; f[13] = S.ax[g]; f[14] = S.ay[g]; f[15] = S.az[g];
        f[16] = S.maxVel[g]; f[17] = S.minDistZone[g]; f[18] = S.firedT[g]; f[19] = S.bcPenalty[g];
        f[20] = S.sx[g]; f[21] = S.sy[g]; f[22] = S.sz[g];
        f[23] = S.minDistSub[g];
        int32_t *n = &ai[g * MPENV_DBG_AI_COUNT];
        n[0] = S.curPose[g]; n[1] = S.tgtPose[g]; n[2] = S.transRem[g];
        n[3] = S.rngA[g]; n[4] = S.rngB[g]; n[5] = S.rngCtr[g];
        n[6] = S.landedOn[g]; n[7] = S.respawnSteps[g]; n[8] = S.autohealSteps[g];
        n[9] = S.flags[g] & 63;
        n[10] = S.wasShot[g]; n[11] = S.weapon[g]; n[12] = S.bcLast[g]; n[13] = S.bcSteps[g];
        n[14] = S.visMask[g];
        n[15] = S.newCells[g];
        if (explore) {
            // 1 = visited in the agent's current episode (the reference's
            // tag == curEpisodeIdx), 0 otherwise
            const bool cur = S.exploreEp[g] == S.episode[g / S.N];
            const int ct = S.exploreTile[g];
            const uint64_t cw = (uint64_t)(uint32_t)S.exploreLo[g] | ((uint64_t)(uint32_t)S.exploreHi[g] << 32);
            for (int k = 0; k < kGridCells; k++) {
                const int cy = k / kGridW, cx = k - cy * kGridW;
                const int t = exploreTileD(cx, cy);
                const uint64_t word = t == ct ? cw : S.exploreBits[g * kExploreTiles + t];
                explore[g * kGridCells + k] = cur ? (uint32_t)((word >> exploreBitD(cx, cy)) & 1ull) : 0u;
            }
        }
    }
    if (t < S.W) {
        const int w = (int)t;
        int32_t *n = &wi[(int64_t)w * MPENV_DBG_WI_COUNT];
        n[0] = S.teamA[w]; n[1] = S.curStep[w]; n[2] = S.finished[w]; n[3] = S.curZone[w];
        n[4] = S.controlling[w]; n[5] = S.contested[w]; n[6] = S.captured[w]; n[7] = S.earned[w];
        n[8] = S.zoneSteps[w]; n[9] = S.stepsUntilPoint[w]; n[10] = S.episode[w]; n[11] = S.episodeCounter[w];
        n[12] = S.wRngA[w]; n[13] = S.wRngB[w]; n[14] = S.wRngCtr[w]; n[15] = S.numCrumbs[w];
        n[16] = S.filtAct0[w]; n[17] = S.filtAct1[w]; n[18] = S.filtMatched0[w]; n[19] = S.filtMatched1[w];
        n[20] = S.crumbOverflow[w];
        n[21] = S.subState[w];
        float *f = &wf[(int64_t)w * MPENV_DBG_WF_COUNT];
        f[0] = S.teamRew0[w]; f[1] = S.teamRew1[w]; f[2] = S.goalMin0[w]; f[3] = S.goalMin1[w];
        f[4] = S.goalTeam0[w]; f[5] = S.goalTeam1[w];
        float *cdst = &crumbs[(int64_t)w * kMaxCrumbs * 8];
        const float4 *cr = crumbPtr(S, w);
        const int nc = S.numCrumbs[w];
        for (int k = 0; k < kMaxCrumbs; k++) {
            float *e = &cdst[k * 8];
            if (k < nc) {
                float4 p = cr[2 * k], meta = cr[2 * k + 1];
                e[0] = p.x; e[1] = p.y; e[2] = p.z; e[3] = p.w;
                e[4] = meta.x; e[5] = meta.y; e[6] = (float)__float_as_int(meta.z); e[7] = 1.f;
            } else {
                for (int q = 0; q < 8; q++) e[q] = 0.f;
            }
        }
    }
}

// Copy one step of the action tape ([A][6] i32: 4 discrete + 2 aim) into the
// engine's action columns (the cudaCopyStepInputs of gpuStreamStep,
// mgr.cpp:625).
__global__ void __launch_bounds__(256) k_fill_actions(DevState S, const int32_t *src)
{
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= S.A) return;
    const int32_t *s = src + 6 * g;
    int4 d = make_int4(s[0], s[1], s[2], s[3]);
    reinterpret_cast<int4 *>(S.discreteAction)[g] = d;
    reinterpret_cast<int2 *>(S.discreteAim)[g] = make_int2(s[4], s[5]);
}

// Synthetic combat action source (bench / tests; no reference counterpart):
// the tape row of each agent, overridden by a greedy aim-bot that reads the
// agent's current observations -- the same function as the tests'
// mpenv_testlib.combat_actions (mode 0) / seek_combat_actions (mode 1), so
// engine and oracle see identical actions while parity holds.
//   an opponent visible (first k with OPPONENT_MASKS[k] > 0): discrete aim
//   toward its relative yaw / pitch (opponent obs 24 / 25) through the
//   pvpDiscreteAimSystem turn tables (sim.cpp:2284-2370), fire iff
//   |yaw| < 0.05;  mode 1 and none visible: turn toward the zone (self obs
//   31, toCenterYaw) and run forward once within 0.5 rad of it, else stand;
//   mode 1 also reloads an empty magazine (self obs 24 == 0, not reloading).
// The bucket compares run in double against the double turn tables, as
// numpy does with its float64 tables.
__device__ __forceinline__ int32_t aimBucketD(float delta, bool yaw_table, int32_t centre)
{
    const double mag = (double)fabsf(delta);
    const double pi = 3.141592653589793;
    int32_t idx = 0;
    if (yaw_table) {
        idx += (1.0 / 256.0) * pi <= mag; idx += (1.0 / 128.0) * pi <= mag; idx += (1.0 / 64.0) * pi <= mag;
        idx += (1.0 / 32.0) * pi <= mag; idx += (1.0 / 16.0) * pi <= mag; idx += (1.0 / 8.0) * pi <= mag;
    } else {
        idx += (1.0 / 128.0) * pi <= mag; idx += (1.0 / 64.0) * pi <= mag; idx += (1.0 / 32.0) * pi <= mag;
    }
    return delta > 0.f ? centre + idx : (delta < 0.f ? centre - idx : centre);
}

__global__ void __launch_bounds__(256) k_combat_actions(DevState S, const int32_t *tape, int32_t *out, int32_t mode)
{
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= S.A) return;
    const int32_t *t = tape + 6 * g;
    int32_t a[6] = { t[0], t[1], t[2], t[3], t[4], t[5] };
    const float *mk = S.masks + 6 * g;
    int k = -1;
    for (int j = 5; j >= 0; j--)
        if (mk[j] > 0.f) k = j;
    if (k >= 0) {
        const float *ob = S.oppObs + (g * 6 + k) * kOtherObs;
        const float yaw = ob[24], pitch = ob[25];
        a[4] = aimBucketD(yaw, true, 6);
        a[5] = aimBucketD(pitch, false, 3);
        a[2] = fabsf(yaw) < 0.05f ? 1 : 0;
    } else if (mode == 1) {
        const float zy = S.selfObs[g * kSelfObs + 31];
        a[4] = aimBucketD(zy, true, 6);
        if (fabsf(zy) < 0.5f) { a[0] = 2; a[1] = 0; } else { a[0] = 0; }
    }
    // mode 1: an empty magazine that is not already reloading is reloaded
    // (self obs 24 / 25: bullets, reload steps left)
    if (mode == 1 && S.selfObs[g * kSelfObs + 24] == 0.f && S.selfObs[g * kSelfObs + 25] == 0.f) a[2] = 2;
    if (out) {
        int32_t *o = out + 6 * g;
        for (int j = 0; j < 6; j++) o[j] = a[j];
    } else {
        reinterpret_cast<int4 *>(S.discreteAction)[g] = make_int4(a[0], a[1], a[2], a[3]);
        reinterpret_cast<int2 *>(S.discreteAim)[g] = make_int2(a[4], a[5]);
    }
}

// ============================================================ host side
const char *kernelName(int k)
{
    static const char *names[kNumTimedKernels] = { "k_move", "k_sim", "k_vis", "k_obs", "k_lidar" };
    return (k >= 0 && k < kNumTimedKernels) ? names[k] : "?";
}

size_t bvhLdsBytes(const SceneDev &sc) { return (size_t)sc.numNodes * 64 + (size_t)sc.numVerts * 16; }

size_t simLdsBytes(const SceneDev &sc)
{
    return simSpawnOffset(sc) + (size_t)(sc.numA + sc.numB + sc.numCommon) * sizeof(Spawn);
}
static_assert(c::kAgentRadius == kSphereR, "k_move sphere casts use the agent radius (stageBVHSphere)");

size_t bvhLdsBytesSphere(const SceneDev &sc)
{
    return bvhLdsBytes(sc) + (size_t)(sc.numVerts / 3) * 32 + (size_t)sc.numNodes * kSNodeFloats * 4;
}


size_t bvhLdsBytesOct(const SceneDev &sc)
{
    return (size_t)sc.numLidarNodes * 16 * kOctNodeQ * 8 + (size_t)sc.numLidarVerts * 16 * 3;
}

int launchConstruct(const DevState &s, const SceneDev &sc, const int32_t tc[3], void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    const int64_t total = s.A * kExploreTiles;
    int blocks = (int)std::min<int64_t>((total + 255) / 256, 65536);
    hipLaunchKernelGGL(k_init_explore, dim3(blocks), dim3(256), 0, st, s, total);
    if (check(hipGetLastError())) return -1;
    hipLaunchKernelGGL(k_construct, dim3((s.W + 63) / 64), dim3(64), 0, st, s, sc, tc[0], tc[1], tc[2]);
    return check(hipGetLastError());
}

int launchResetOnly(const DevState &s, const SceneDev &sc, void *stream)
{
    hipLaunchKernelGGL(k_reset_only, dim3((s.W + 63) / 64), dim3(64), 0, (hipStream_t)stream, s, sc);
    return check(hipGetLastError());
}

int launchMove(const DevState &s, const SceneDev &sc, void *stream)
{
    // Small batches (< 64 full blocks): one-wave blocks, so the few waves spread over CUs
    // instead of sharing a CU's SIMDs (k_move is latency-bound: 5-7
    // dependent sphere casts per lane).  Big batches keep 256-thread blocks
    // (the 24 KB LDS image per block would otherwise cap occupancy).
    // Agents per wave: 64 once the batch fills ~1.5 waves per SIMD (1,536
    // waves on 256 CUs), else the power of two (>= 8) that gets closest.
    int apw = 64;
    while (apw > 8 && (s.A + apw - 1) / apw < 1536) apw >>= 1;
    const int64_t waves = (s.A + apw - 1) / apw;
    const int bs = waves < 64 * 4 ? 64 : kBlock;
    const int64_t threads = waves * 64;
    hipLaunchKernelGGL(k_move, dim3((unsigned)((threads + bs - 1) / bs)), dim3(bs), bvhLdsBytesSphere(sc),
                       (hipStream_t)stream, s, sc, apw);
    return check(hipGetLastError());
}

int launchSimStep(const DevState &s, const SceneDev &sc, void *stream)
{
    const int wpb = kSimBlock / s.N;
    const int blocks = (s.W + wpb - 1) / wpb;
    hipLaunchKernelGGL(k_sim, dim3(blocks), dim3(kSimBlock), simLdsBytes(sc), (hipStream_t)stream, s, sc);
    return check(hipGetLastError());
}

int launchVisibility(const DevState &s, const SceneDev &sc, void *stream)
{
    const int64_t waves = (s.A + (64 / s.T) - 1) / (64 / s.T);
    const int blocks = (int)((waves * 64 + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_vis, dim3(blocks), dim3(kBlock),
                       (size_t)sc.numLidarNodes * 64 + (size_t)sc.numLidarVerts * 16 +
                           (size_t)kVisStageCols * 4 * visStageAgents(s.T, s.N), (hipStream_t)stream, s, sc);
    return check(hipGetLastError());
}

int launchObservations(const DevState &s, const SceneDev &sc, void *stream)
{
    const int blocks = (int)((s.A + kObsBlock - 1) / kObsBlock);
    hipLaunchKernelGGL(k_obs<false>, dim3(blocks), dim3(kObsBlock), 0, (hipStream_t)stream, s, sc, WireObs {});
    return check(hipGetLastError());
}

int launchObservationsWire(const DevState &view, const SceneDev &sc, const WireObs &wo, void *stream)
{
    const int blocks = (int)((view.A + kObsBlock - 1) / kObsBlock);
    hipLaunchKernelGGL(k_obs<true>, dim3(blocks), dim3(kObsBlock), 0, (hipStream_t)stream, view, sc, wo);
    return check(hipGetLastError());
}

int computeSceneFrames(SceneTables *d_tab, void *stream)
{
    hipLaunchKernelGGL(k_scene_frames, dim3(1), dim3(64), 0, (hipStream_t)stream, d_tab);
    int rc = check(hipGetLastError());
    if (!rc) rc = check(hipStreamSynchronize((hipStream_t)stream));
    return rc;
}

int computeZoneGoalTris(const SceneDev &sc, int32_t *dev_scratch, int32_t *host_out, void *stream)
{
    hipLaunchKernelGGL(k_zone_goals, dim3(1), dim3(64), 0, (hipStream_t)stream, sc, dev_scratch);
    int rc = check(hipGetLastError());
    if (!rc) rc = check(hipMemcpyAsync(host_out, dev_scratch, sizeof(int32_t) * sc.numZones, hipMemcpyDeviceToHost,
                                       (hipStream_t)stream));
    if (!rc) rc = check(hipStreamSynchronize((hipStream_t)stream));
    return rc;
}

int launchLidar(const DevState &s, const SceneDev &sc, void *stream)
{
    // ~1024 blocks before the iterations grow past 1
    const int64_t tasks = lidarTasks(s.A);
    const int iters = (int)std::max<int64_t>(1, std::min<int64_t>(kLidarIters, tasks / (kLidarWaves * 1024)));
    const int64_t per_block = (int64_t)kLidarWaves * iters;
    const int blocks = (int)((tasks + per_block - 1) / per_block);
    hipLaunchKernelGGL(k_lidar, dim3(blocks), dim3(kLidarBlock), bvhLdsBytesOct(sc), (hipStream_t)stream, s, sc,
                       iters);
    return check(hipGetLastError());
}

int launchDebugGather(const DevState &s, float *af, int32_t *ai, int32_t *wi, float *wf, uint32_t *explore,
                      float *crumbs, void *stream)
{
    const int64_t n = s.A > s.W ? s.A : s.W;
    hipLaunchKernelGGL(k_debug, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, s, af, ai, wi,
                       wf, explore, crumbs);
    return check(hipGetLastError());
}

int launchFillActions(const DevState &s, const int32_t *src6, void *stream)
{
    hipLaunchKernelGGL(k_fill_actions, dim3((unsigned)((s.A + 255) / 256)), dim3(256), 0, (hipStream_t)stream, s,
                       src6);
    return check(hipGetLastError());
}

int launchCombatActions(const DevState &s, const int32_t *tape6, int32_t *out6, int32_t mode, void *stream)
{
    hipLaunchKernelGGL(k_combat_actions, dim3((unsigned)((s.A + 255) / 256)), dim3(256), 0, (hipStream_t)stream, s,
                       tape6, out6, mode);
    return check(hipGetLastError());
}

} // namespace mpenv
