// oracle.cpp — TEST INFRASTRUCTURE ONLY (parity checker, CPU baseline).
//
// A single-threaded, plain-C++ restatement of the reference's world-batched
// Zone step: the TaskGraphID::Step graph of Sim::setupTasks
// (src/sim.cpp:5342-5842) and the Init graph (sim.cpp:5322-5340), plus the
// per-world constructor (sim.cpp:5850-5980), world generation
// (src/level_gen.cpp:19-582), the ray/sphere/visibility/spawn helpers
// (src/utils.cpp:10-948) and the compressed-BVH traversal
// (src/mesh_bvh.inl:110-1127).  Every function cites the reference lines it
// follows.  Systems run in the reference's insertion order, world by world
// (worlds never interact), so a world-partitioned thread
// pool gives the same results as the reference's per-node barriers.
//
// Only the Madrona layer (vector/quaternion math, transcendentals, RNG,
// geo:: helpers — not vendored in the reference) comes from the shared
// definition header mpenv_core.h; everything restating madrona-mp-env code
// lives here and is independent of the GPU kernels it checks.
//
// Reference quirks reproduced on purpose: the
// sphere-cast vertex test's double origin shift (mesh_bvh.inl:1073-1104),
// the escape-move sign (sim.cpp:1004), respawn scoring's integer "elapsed"
// (utils.cpp:418-428), spawn z offset after the zone-frame test
// (utils.cpp:899-903), dead agents still casting lidar and dropping
// breadcrumbs.  Deliberate, documented definitions: breadcrumb penalties
// accumulate in creation order (the reference uses an order-dependent float
// atomic, sim.cpp:4915); sphereCastLeaf reads two consecutive triangles
// per leaf as the reference does (mesh_bvh.inl:867-880) and skips only the
// read past the last triangle (undefined there); ExploreTracker cells outside
// the initialised quadrant start at 0; uninitialised locals (the first
// slope-cast normal, sim.cpp:927) start at zero.
//
// Parity unpinned against the reference's own output bitstream: the
// reference cannot be built here (Madrona, Embree, meshoptimizer absent) and
// holds no tests or golden vectors for this path.  The restatement is pinned
// instead to the reference's scene data fixtures (data/simple_map/*.bin),
// closed-form ray / sphere-cast hits on that geometry, BVH-vs-brute-force
// equality and the Threefry-2x32-20 known-answer vectors.
#include "oracle.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "mpenv.h"
#include "mpenv_core.h"

using namespace mp;

namespace {

// ----------------------------------------------------- consts.hpp:7-72
constexpr int kMaxTeamSize = 6;
constexpr int kMaxZones = 5;
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
constexpr int kFwdW = 32, kFwdH = 2, kRearW = 8, kRearH = 2;
constexpr int kGridW = 81, kGridMax = 40;

// Weapon stats (mgr.cpp:1383-1395): one weapon type.
constexpr int kMagSize = 30;
constexpr int kReloadTime = 30;
constexpr float kDmgPerBullet = 10.f;
constexpr float kAccuracyScale = 0.005f;
constexpr int kNumWeaponTypes = 1;

// Observation struct sizes (types.hpp:275-423).
constexpr int kSelfObs = 43, kOtherObs = 32, kLidarData = 4;

enum Pose { kStand = 0, kCrouch = 1, kProne = 2 };

// ----------------------------------------------- mesh_bvh.hpp:61-86 Node
struct Node {
    float minX, minY, minZ;
    int8_t expX, expY, expZ;
    uint8_t internalNodes;
    uint8_t triSize[4];
    uint8_t qMinX[4], qMinY[4], qMinZ[4];
    uint8_t qMaxX[4], qMaxY[4], qMaxZ[4];
    int32_t children[4];
    int32_t parentID;
};
static_assert(sizeof(Node) == 64, "node layout");

struct Spawn {
    AABB region;
    float yawMin, yawMax;
};

struct ZOBB {
    Vec3 pMin, pMax;
    float rotation;
};

struct GoalRegion {
    ZOBB subRegions[3];
    int numSubRegions;
    bool attackerTeam;
    float rewardStrength;
};

float viewHeight(int pose) // utils.hpp:37-56
{
    float top = pose == kStand ? kStandHeight : (pose == kCrouch ? kCrouchHeight : kProneHeight);
    return top - kAgentRadius;
}

int32_t f2iSat(float f) // float->int conversion with defined NaN/overflow
{
    if (!(f == f)) return 0;
    if (f >= 2147483520.f) return INT32_MAX;
    if (f <= -2147483648.f) return INT32_MIN;
    return (int32_t)f;
}

// ------------------------------------------------------------ state
struct Agent {
    Vec3 pos;
    Quat rot;
    Vec3 vel;
    Vec3 newPos, newVel;
    float maxVelocity;
    int curPose, tgtPose, transitionRemaining;
    float dmg[kMaxTeamSize];
    float aimYaw, aimPitch;
    Quat aimRot;
    int team, offset;
    RNG rng;
    int landedShotOn;  // agent index within world, -1 = Entity::none()
    int remainingRespawnSteps, remainingStepsBeforeAutoheal;
    bool successfulKill;
    int wasShotCount;
    bool wasKilled;
    float firedShotT;
    bool inZone;
    float minDistToZone;
    bool hasDiedDuringEpisode;
    bool reloadedFullMag;
    int weaponType;
    float totalPenalty;
    int64_t lastBreadcrumb;
    int stepsSinceLastNewBreadcrumb;
    Vec3 startPos;
    std::vector<uint32_t> visited;
    uint32_t numNewCellsVisited;
    float daimYawVel, daimPitchVel;
    bool canSee[kMaxTeamSize];
    // CombatState sub-zone fields (types.hpp:521-522), SubZones only
    bool inSubZone = false;
    float minDistToSubZone = 0.f;
};

struct Crumb {
    Vec3 pos;
    float penalty;
    int team, offset;
    uint32_t id;
};

struct World {
    // MatchInfo (types.hpp:127-134)
    int teamA, curStep;
    bool isFinished;
    bool enableSpawnCurriculum;
    uint32_t curCurriculumTier, curCurriculumSpawnIdx;
    // ZoneState (types.hpp:563-572)
    int curZone, curControllingTeam;
    bool isContested, isCaptured, earnedPoint;
    int zoneStepsRemaining, stepsUntilPoint;
    // Sim data (sim.hpp:81-191)
    uint32_t curEpisodeIdx, worldEpisodeCounter;
    RNG baseRNG;
    int zoneStats[kMaxZones][5];
    uint64_t filtersActive[2];
    int filtersLastMatches[2][64];
    int filtersLastMatchedStep[2];
    int episodeCurriculum;
    uint64_t matchID;
    uint32_t eventLoggedInStep, eventMask; // sim.hpp:162-163
    // SpawnUsageCounter (types.hpp:95-100) lives in Oracle::spawnTrack.
    // GoalRegionsState (types.hpp:808-814)
    bool regionsActive[10];
    float minDistToRegions[10];
    float teamStepRewards[2];
    // TeamRewardState
    float teamRewards[2];
    std::vector<Crumb> crumbs;
    uint32_t nextCrumbId;
    int crumbOverflow;
    // SubZone entities (types.hpp:791-796), SubZones only
    int subCtrl[8];
    bool subContested[8], subCaptured[8];
};

struct Oracle {
    oracle_config cfg;
    std::string scenePath;
    int W, N, teamSize;
    uint32_t worldOffset;
    bool autoReset;
    uint32_t simFlags;
    int task = MPENV_TASK_ZONE; // Zone or ZoneCaptureDefend
    bool flank = false;         // RewardMode::Flank
    RandKey initRandKey;

    AABB worldBounds;
    float maxDist;
    float frustum[4];
    std::vector<Node> nodes;
    std::vector<Vec3> navTris;   // 3 per triangle
    std::vector<float> navCdf;   // running triangle areas (navSamplePoint)
    std::vector<mpenv_curriculum_snapshot> curriculum; // TrajectoryCurriculum
    struct ZOBB { Vec3 pMin, pMax; float rotation; } subZones[8]; // level_gen.cpp:282-326
    std::vector<int32_t> astar;  // [T][T] (buildAStarLookup, built by the oracle)
    std::vector<int32_t> navAdj; // [T][3]
    // Lidar closest-hit rule (cfg.lidar_octant_order: kLidarSlot / kLidarOctant /
    // kLidarLex, bvhTraceRay); octOrder: per ray octant and node, the slot
    // visited k-th (octantOrder()).
    int lidarOrder = 0;
    std::vector<int8_t> octOrder; // [8][numNodes][4]
    // pvpLidar's tree (cfg.lidar_bvh_*): the octant and lex rules walk it
    std::vector<Node> lidarNodes;
    std::vector<Vec3> lidarVerts;
    std::vector<int8_t> lidarOctOrder;
    int numNavTris = 0;
    std::vector<Vec3> verts;
    std::vector<Spawn> aSpawns, bSpawns, commonRespawns;
    uint32_t numDefaultASpawns, numDefaultBSpawns;
    std::vector<AABB> zoneAABBs;
    std::vector<float> zoneRot;
    std::vector<GoalRegion> goalRegions;
    int32_t trainControl[3];

    std::vector<Agent> agents;
    std::vector<World> worlds;
    // SpawnUsageCounter per world: [W][3][spawnTrackLen] (initA, initB,
    // respawn).  The reference fixes 128 slots (types.hpp:96) and asserts the
    // list fits; here the length is max(128, longest spawn list) so a long
    // SpawnInMiddle list indexes its own slots (documented definition).
    int spawnTrackLen = 128;
    std::vector<uint32_t> spawnTrack;
    uint32_t *track(int w, int k) { return &spawnTrack[((size_t)w * 3 + k) * spawnTrackLen]; }

    // Exported buffers, laid out as the reference's exported columns.
    std::vector<int32_t> resetBuf, worldCurriculum, matchResult, exploreAction, discreteAction,
        discreteAim, policy, done, magazine, botAction;
    std::vector<float> aimAction, reward, selfObs, filtersObs, teammateObs, opponentObs, lastKnownObs,
        selfPos, teammatePos, opponentPos, lastKnownPos, masks, fwdLidar, rearLidar, agentMap, hp,
        alive, rewardCoefs;
    // FullTeamInterface columns, [W * 2] team interfaces (types.hpp:1040-1152)
    std::vector<int32_t> ftActions, ftDone, ftPolicy;
    std::vector<float> ftGlobal, ftPlayers, ftEnemies, ftLastKnown, ftFwdLidar, ftRearLidar, ftReward;
    std::vector<float> dbgAF, dbgWF, dbgCrumbs;
    // logs (record / replay / events), enabled by oracle_set_log_modes
    bool recordOn = false, replayOn = false, eventsOn = false;
    std::vector<mpenv_step_log> recordLog, replayLog;
    std::vector<mpenv_game_event> events;        // [W][2N+1]
    std::vector<mpenv_packed_step_snapshot> snapshots;
    std::vector<int32_t> snapWritten;
    std::vector<int32_t> dbgAI, dbgWI;
    std::vector<uint32_t> dbgExplore;

    Agent &agent(int w, int i) { return agents[(size_t)w * N + i]; }
    size_t gi(int w, int i) const { return (size_t)w * N + i; }
};

// ============================================================== geometry
// mesh_bvh.inl:584-741 computeRayIsectTxfm — only kx/ky/kz and the shear
// constants feed the traversal; the near/far error terms are unused by
// traceRay and are omitted.
struct RayTxfm {
    int kx, ky, kz;
    float Sx, Sy, Sz;
};

RayTxfm computeRayIsectTxfm(Vec3 d, Vec3 inv_d)
{
    float abs_x = fabs_(d.x), abs_y = fabs_(d.y), abs_z = fabs_(d.z);
    int kz;
    if (abs_x > abs_y && abs_x > abs_z) kz = 0;
    else if (abs_y > abs_z) kz = 1;
    else kz = 2;
    int kx = kz + 1; if (kx == 3) kx = 0;
    int ky = kx + 1; if (ky == 3) ky = 0;
    if (comp(d, kz) < 0.f) std::swap(kx, ky);
    RayTxfm t;
    t.kx = kx; t.ky = ky; t.kz = kz;
    t.Sx = comp(d, kx) * comp(inv_d, kz);
    t.Sy = comp(d, ky) * comp(inv_d, kz);
    t.Sz = comp(inv_d, kz);
    return t;
}

// mesh_bvh.inl:433-554 (backface culling on, line 3)
bool rayTriangleIntersection(Vec3 ta, Vec3 tb, Vec3 tc, const RayTxfm &tx, Vec3 org, float t_max,
                             float *out_t)
{
    const Vec3 A = ta - org, B = tb - org, C = tc - org;
    const float Ax = fma_(-tx.Sx, comp(A, tx.kz), comp(A, tx.kx));
    const float Ay = fma_(-tx.Sy, comp(A, tx.kz), comp(A, tx.ky));
    const float Bx = fma_(-tx.Sx, comp(B, tx.kz), comp(B, tx.kx));
    const float By = fma_(-tx.Sy, comp(B, tx.kz), comp(B, tx.ky));
    const float Cx = fma_(-tx.Sx, comp(C, tx.kz), comp(C, tx.kx));
    const float Cy = fma_(-tx.Sy, comp(C, tx.kz), comp(C, tx.ky));
    float U = fma_(Cx, By, -(Cy * Bx));
    float V = fma_(Ax, Cy, -(Ay * Cx));
    float Wb = fma_(Bx, Ay, -(By * Ax));
    if (U < 0.0f || V < 0.0f || Wb < 0.0f) return false;
    if (U == 0.0f || V == 0.0f || Wb == 0.0f) {
        double CxBy = (double)Cx * (double)By;
        double CyBx = (double)Cy * (double)Bx;
        U = (float)(CxBy - CyBx);
        double AxCy = (double)Ax * (double)Cy;
        double AyCx = (double)Ay * (double)Cx;
        V = (float)(AxCy - AyCx);
        double BxAy = (double)Bx * (double)Ay;
        double ByAx = (double)By * (double)Ax;
        Wb = (float)(BxAy - ByAx);
        if (U < 0.0f || V < 0.0f || Wb < 0.0f) return false;
    }
    float det = U + V + Wb;
    if (det == 0.f) return false;
    const float Az = tx.Sz * comp(A, tx.kz);
    const float Bz = tx.Sz * comp(B, tx.kz);
    const float Cz = tx.Sz * comp(C, tx.kz);
    const float T = fma_(U, Az, fma_(V, Bz, Wb * Cz));
    if (T < 0.0f || T > t_max * det) return false;
    const float rcpDet = 1.0f / det;
    *out_t = T * rcpDet;
    return true;
}

float expScale(int8_t e) { return u2f((uint32_t)((int32_t)e + 127) << 23); }

// Slab rounding (analysis hook oracle_set_slab_fma): 1 = q * dirQuant +
// originQuant fused (the definition the engine and the oracle share,
// DESIGN.md §2 definition 13), 0 = multiply then add, each rounded.
int g_slabFma = 1;
inline float slabT(float q, float dq, float oq) { return g_slabFma ? fma_(q, dq, oq) : q * dq + oq; }

// mesh_bvh.inl:110-208 (MeshBVH::traceRay) + 360-431 (traceRayLeaf)
// Lidar closest-hit rules (cfg.lidar_octant_order; DESIGN.md §2 definition 12):
//   kLidarSlot   -- mesh_bvh.inl:160-204 as written: slots in order, each
//                   accepted hit tightens t_max (the reference);
//   kLidarOctant -- the round-2/3 octant child order (same acceptance);
//   kLidarLex    -- order-independent: the smallest t = fl(T * fl(1 / det))
//                   of the watertight test over every triangle the ray hits
//                   (which triangle attains it is not observable), -0 below
//                   +0 (an origin on a vertex or edge hits at t = -0 or +0:
//                   lexLess compares the bit patterns as signed integers,
//                   the total order of {-0} and [+0, inf]).  Boxes and triangles are tested
//                   against t_best * (1 + 2^-20), so no triangle whose t ties
//                   or beats the current best is ever pruned, whatever the
//                   visit order (the product's fan lists rely on that).
enum { kLidarSlot = 0, kLidarOctant = 1, kLidarLex = 2 };
constexpr float kLexRelax = 1.00000095367431640625f; // 1 + 2^-20
// kLidarLex box test: t_near <= fma(|t_far|, 2^-16, t_far + 2^-8) (as the engine).  A child box
// quantised at its node's boundary has no margin (qMin clamps at 0), so a
// ray aimed exactly at such a vertex can miss the box by slab rounding
// although it hits the triangle; the slack keeps those boxes, so the
// traversal visits every triangle a brute-force loop would find nearer than
// the bound (tests/test_lidar_order.py checks equality with brute force).
constexpr float kBoxSlackRel = 1.52587890625e-5f, kBoxSlackAbs = 0.00390625f;
inline bool lexLess(float a, float b) { return (int32_t)f2u(a) < (int32_t)f2u(b); }

bool bvhTraceRay(const Oracle &o, Vec3 ray_o, Vec3 ray_d, float *t_hit, float t_max = kFltMax, bool octant = false,
                 bool lex = false, bool lidar_tree = false)
{
    // lidar_tree: pvpLidar's own tree (Oracle::lidarNodes), else the
    // collision tree every other query walks
    const std::vector<Node> &nodes = lidar_tree ? o.lidarNodes : o.nodes;
    const std::vector<Vec3> &verts = lidar_tree ? o.lidarVerts : o.verts;
    const std::vector<int8_t> &octOrder = lidar_tree ? o.lidarOctOrder : o.octOrder;
    // octant: visit each node's child slots in the order octantOrder()
    // defines for the ray's direction signs (the lidar's documented child
    // order); otherwise slot order, as mesh_bvh.inl:160-204.
    const int oct = (std::signbit(ray_d.x) ? 1 : 0) | (std::signbit(ray_d.y) ? 2 : 0) | (std::signbit(ray_d.z) ? 4 : 0);
    const float diveps = 0.0000001f;
    Vec3 inv_d = v3(1.f / ray_d.x, 1.f / ray_d.y, 1.f / ray_d.z);
    RayTxfm tx = computeRayIsectTxfm(ray_d, inv_d);

    int32_t stack[64];
    int sp = 0;
    stack[sp++] = 0;
    bool ray_hit = false;
    float t_best = t_max; // kLidarLex: the smallest t so far
    if (lex) t_max = t_best * kLexRelax;
    while (sp > 0) {
        int32_t node_idx = stack[--sp];
        const Node &node = nodes[node_idx];
        float rayXInv = copysign_(ray_d.x == 0 ? 1 / diveps : 1 / ray_d.x, ray_d.x);
        float rayYInv = copysign_(ray_d.y == 0 ? 1 / diveps : 1 / ray_d.y, ray_d.y);
        float rayZInv = copysign_(ray_d.z == 0 ? 1 / diveps : 1 / ray_d.z, ray_d.z);
        float dirQuantX = expScale(node.expX) * rayXInv;
        float dirQuantY = expScale(node.expY) * rayYInv;
        float dirQuantZ = expScale(node.expZ) * rayZInv;
        float originQuantX = (node.minX - ray_o.x) * rayXInv;
        float originQuantY = (node.minY - ray_o.y) * rayYInv;
        float originQuantZ = (node.minZ - ray_o.z) * rayZInv;
        for (int slot = 0; slot < 4; slot++) {
            const int i = octant ? octOrder[((size_t)oct * nodes.size() + node_idx) * 4 + slot] : slot;
            if (node.children[i] == -1) continue;
            // q * dirQuant + originQuant, fused: the reference's GPU build is
            // compiled with NVRTC's default --fmad=true, which contracts it
            float t_near_x = slabT((float)node.qMinX[i], dirQuantX, originQuantX);
            float t_near_y = slabT((float)node.qMinY[i], dirQuantY, originQuantY);
            float t_near_z = slabT((float)node.qMinZ[i], dirQuantZ, originQuantZ);
            float t_far_x = slabT((float)node.qMaxX[i], dirQuantX, originQuantX);
            float t_far_y = slabT((float)node.qMaxY[i], dirQuantY, originQuantY);
            float t_far_z = slabT((float)node.qMaxZ[i], dirQuantZ, originQuantZ);
            float t_near = fmax_(fmin_(t_near_x, t_far_x),
                                 fmax_(fmin_(t_near_y, t_far_y), fmax_(fmin_(t_near_z, t_far_z), 0.f)));
            float t_far = fmin_(fmax_(t_far_x, t_near_x),
                                fmin_(fmax_(t_far_y, t_near_y), fmin_(fmax_(t_far_z, t_near_z), t_max)));
            if (t_near <= (lex ? fma_(fabs_(t_far), kBoxSlackRel, t_far + kBoxSlackAbs) : t_far)) {
                if (node.children[i] & 0x80000000) {
                    int32_t leaf_idx = node.children[i] & ~0x80000000;
                    if (lex) {
                        for (int k = 0; k < node.triSize[i]; k++) {
                            const int tri = leaf_idx + k;
                            float t = 0.f;
                            if (rayTriangleIntersection(verts[tri * 3 + 0], verts[tri * 3 + 1],
                                                        verts[tri * 3 + 2], tx, ray_o, t_max, &t) &&
                                lexLess(t, t_best)) {
                                t_best = t;
                                ray_hit = true;
                                t_max = t_best * kLexRelax;
                            }
                        }
                        continue;
                    }
                    // traceRayLeaf
                    bool hit_tri = false;
                    float hit_t = 0.f;
                    float leaf_tmax = t_max;
                    for (int k = 0; k < node.triSize[i]; k++) {
                        Vec3 a = verts[(leaf_idx + k) * 3 + 0];
                        Vec3 b = verts[(leaf_idx + k) * 3 + 1];
                        Vec3 c = verts[(leaf_idx + k) * 3 + 2];
                        if (rayTriangleIntersection(a, b, c, tx, ray_o, leaf_tmax, &hit_t)) {
                            hit_tri = true;
                            leaf_tmax = hit_t;
                        }
                    }
                    if (hit_tri) {
                        ray_hit = true;
                        t_max = hit_t;
                    }
                } else {
                    stack[sp++] = node.children[i];
                }
            }
        }
    }
    *t_hit = lex ? t_best : t_max;
    return ray_hit;
}

// mesh_bvh.inl:817-855
bool sphereCastNodeCheck(Vec3 o, Vec3 inv_d, float t_max, float r, AABB aabb)
{
    AABB e = aabb;
    e.pMin.x -= r; e.pMin.y -= r; e.pMin.z -= r;
    e.pMax.x += r; e.pMax.y += r; e.pMax.z += r;
    float t_min = 0.f;
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

// mesh_bvh.inl:885-1127 (Jolt-derived swept sphere vs triangle)
float sphereCastTriangle(Vec3 ta, Vec3 tb, Vec3 tc, Vec3 ray_o, Vec3 ray_d, float t_max, float r,
                         Vec3 *out_n)
{
    const Vec3 e01 = tb - ta, e02 = tc - ta, e12 = tc - tb;
    const Vec3 v0 = ta - ray_o, v1 = tb - ray_o, v2 = tc - ray_o;
    Vec3 nu = computeTriangleGeoNormal(e01, e02, e12);
    float n_len = length(nu);
    Vec3 n = nu / n_len;
    const float n_dot_d = dot(n, ray_d);
    const float r2 = r * r;

    if (fabs_(dot(v0, n)) <= r) {
        Vec3 q = triangleClosestPointToOrigin(v0, v1, v2, e01, e02);
        float q_len2 = length2(q);
        if (q_len2 <= r2) {
            float q_len = sqrt_(q_len2);
            *out_n = q_len > 0.0f ? q / q_len : kUp;
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
                    *out_n = -sgn * n;
                    return plane_t;
                }
            }
        }
    }

    const float edge_eps = 1e-6f;
    const float d_len2 = length2(ray_d);
    auto testEdge = [&](Vec3 axis, Vec3 base, float hit_t) {
        Vec3 start = -base;
        const float s_dot_a = dot(start, axis);
        const float d_dot_a = dot(ray_d, axis);
        const float e_dot_a = s_dot_a + d_dot_a;
        if (s_dot_a < 0.0f && e_dot_a < 0.0f) return hit_t;
        const float a_len2 = length2(axis);
        if (s_dot_a > a_len2 && e_dot_a > a_len2) return hit_t;
        float a = a_len2 * d_len2 - d_dot_a * d_dot_a;
        if (fabs_(a) < edge_eps) return hit_t;
        float b = a_len2 * dot(start, ray_d) - d_dot_a * s_dot_a;
        float c = a_len2 * (length2(start) - r2) - s_dot_a * s_dot_a;
        float det = b * b - a * c;
        if (det < 0.0f) return hit_t;
        float t = -(b + sqrt_(det)) / a;
        if (t < 0.0f || t >= hit_t) return hit_t;
        if (s_dot_a + t * d_dot_a < 0.0f || s_dot_a + t * d_dot_a > a_len2) return hit_t;
        return t;
    };
    // Faithful to mesh_bvh.inl:1073-1104: v is already relative to ray_o but
    // is subtracted from ray_o again.
    auto testVert = [&](Vec3 v, float hit_t) {
        Vec3 m = ray_o - v;
        float b = dot(m, ray_d);
        float c = dot(m, m) - r2;
        if (c > 0.0f && b > 0.0f) return hit_t;
        float discr = b * b - c;
        if (discr < 0.0f) return hit_t;
        float t = -b - sqrt_(discr);
        if (t < 0.f) return 0.f;
        if (t >= hit_t) return hit_t;
        return t;
    };

    float hit_t = t_max;
    hit_t = testEdge(e01, v0, hit_t);
    hit_t = testEdge(e02, v0, hit_t);
    hit_t = testEdge(e12, v1, hit_t);
    hit_t = testVert(v0, hit_t);
    hit_t = testVert(v1, hit_t);
    hit_t = testVert(v2, hit_t);
    if (hit_t >= t_max) return t_max;
    Vec3 hp = ray_d * hit_t;
    Vec3 ct = triangleClosestPointToOrigin(v0 - hp, v1 - hp, v2 - hp, e01, e02);
    *out_n = normalize(ct);
    return hit_t;
}

// mesh_bvh.inl:743-815 (MeshBVH::sphereCast) + 857-883 (sphereCastLeaf:
// two consecutive triangles per leaf, see file header).
// Analysis counters (oracle_cast_stats): casts, casts ending at t = 0, and
// the leaf read rule (2 = the reference's two consecutive triangles,
// 1 = only triSize triangles, the round-1 definition kept for comparison).
std::atomic<uint64_t> g_casts { 0 }, g_zeroCasts { 0 };
int g_leafReadTwo = 1;

float bvhSphereCast(const Oracle &o, Vec3 ray_o, Vec3 ray_d, float r, Vec3 *out_n,
                    float t_max = kFltMax)
{
    Vec3 inv_d = v3(1.f / ray_d.x, 1.f / ray_d.y, 1.f / ray_d.z);
    int32_t stack[64];
    int sp = 0;
    stack[sp++] = 0;
    Vec3 closest = v3(0.f, 0.f, 0.f);
    float hit_t = t_max;
    while (sp > 0) {
        int32_t node_idx = stack[--sp];
        const Node &node = o.nodes[node_idx];
        for (int i = 0; i < 4; i++) {
            if (node.children[i] == -1) continue;
            float sx = u2f((uint32_t)((int32_t)node.expX + 127) << 23);
            float sy = u2f((uint32_t)((int32_t)node.expY + 127) << 23);
            float sz = u2f((uint32_t)((int32_t)node.expZ + 127) << 23);
            AABB child;
            child.pMin = v3(node.minX + sx * node.qMinX[i], node.minY + sy * node.qMinY[i],
                            node.minZ + sz * node.qMinZ[i]);
            child.pMax = v3(node.minX + sx * node.qMaxX[i], node.minY + sy * node.qMaxY[i],
                            node.minZ + sz * node.qMaxZ[i]);
            if (sphereCastNodeCheck(ray_o, inv_d, hit_t, r, child)) {
                if (node.children[i] & 0x80000000) {
                    int32_t leaf_idx = node.children[i] & ~0x80000000;
                    Vec3 leaf_n = v3(0.f, 0.f, 0.f);
                    float leaf_t = hit_t;
                    // numTrisPerLeaf (= 2) triangles in leaf order regardless
                    // of triSize (mesh_bvh.inl:867-880, fetchLeafTriangle
                    // 556-576 always succeeds); the last triangle's overrun
                    // past the vertex array is defined as "not tested".
                    const int num_tris = (int)(o.verts.size() / 3);
                    const int nread = g_leafReadTwo ? 2 : node.triSize[i];
                    for (int k = 0; k < nread && leaf_idx + k < num_tris; k++) {
                        Vec3 a = o.verts[(leaf_idx + k) * 3 + 0];
                        Vec3 b = o.verts[(leaf_idx + k) * 3 + 1];
                        Vec3 c = o.verts[(leaf_idx + k) * 3 + 2];
                        leaf_t = sphereCastTriangle(a, b, c, ray_o, ray_d, leaf_t, r, &leaf_n);
                    }
                    if (leaf_t < hit_t) {
                        hit_t = leaf_t;
                        closest = leaf_n;
                    }
                } else {
                    stack[sp++] = node.children[i];
                }
            }
        }
    }
    if (hit_t < t_max) *out_n = closest;
    g_casts.fetch_add(1, std::memory_order_relaxed);
    if (hit_t == 0.f) g_zeroCasts.fetch_add(1, std::memory_order_relaxed);
    return hit_t;
}

// ============================================================ utils.cpp
struct HitResult {
    bool hit;
    float t;
    int entity; // agent index in world, -1 none
};

// utils.cpp:10-72 traceRayAgainstWorld
HitResult traceRayAgainstWorld(const Oracle &o, int w, Vec3 org, Vec3 d, int order = kLidarSlot)
{
    float min_hit_t = kFltMax;
    float t_bvh;
    // the octant and lex rules are pvpLidar's: they walk its tree (the
    // product's k_lidar does); the slot rule, the reference's order, walks
    // the collision tree (the reference has one tree)
    bool hit = bvhTraceRay(o, org, d, &t_bvh, kFltMax, order == kLidarOctant, order == kLidarLex, order != kLidarSlot);
    if (hit) min_hit_t = t_bvh;
    int hit_entity = -1;
    for (int j = 0; j < o.N; j++) {
        const Agent &a = o.agents[o.gi(w, j)];
        Vec3 capsule_origin = a.pos;
        capsule_origin.z += kAgentRadius;
        Vec3 translated = org - capsule_origin;
        float t = intersectRayZOriginCapsule(translated, d, kAgentRadius, kStandHeight - 2.f * kAgentRadius);
        if (t != 0 && t < min_hit_t) {
            min_hit_t = t;
            hit = true;
            hit_entity = j;
        }
    }
    return { hit, min_hit_t, hit_entity };
}

// utils.cpp:75-138 sphereCastWorld (agent capsules disabled, #if 0)
float sphereCastWorld(const Oracle &o, Vec3 org, Vec3 d, float r, Vec3 &normal)
{
    return bvhSphereCast(o, org, d, r, &normal);
}

float sphereCastWorld(const Oracle &o, Vec3 org, Vec3 d, float r)
{
    Vec3 n = v3(0.f, 0.f, 0.f);
    return bvhSphereCast(o, org, d, r, &n);
}

struct AimS {
    float yaw, pitch;
    Quat rot;
};

// utils.cpp:140-167 computeAim
AimS computeAim(float yaw, float pitch)
{
    if (yaw < -kPi) yaw += 2.f * kPi;
    else if (yaw > kPi) yaw -= 2.f * kPi;
    if (pitch < -0.25f * kPi) pitch = -0.25f * kPi;
    if (pitch > 0.25f * kPi) pitch = 0.25f * kPi;
    Quat r = angleAxis(yaw, kUp) * angleAxis(pitch, kRight);
    r = qnormalize(r);
    return { yaw, pitch, r };
}

// utils.cpp:169-184
bool inFrustum(const Oracle &o, Vec3 vp)
{
    bool in = true;
    in = in && vp.y * o.frustum[1] - fabs_(vp.x) * o.frustum[0] > -kAgentRadius;
    in = in && vp.y * o.frustum[3] - fabs_(vp.z) * o.frustum[2] > -kAgentRadius;
    return in;
}

// utils.cpp:186-271 isAgentVisible (only the boolean result is consumed in
// the Zone task; the running mean of visible points is not needed)
bool isAgentVisible(const Oracle &o, int w, Vec3 org, Quat aim_rot, int target)
{
    const Agent &t = o.agents[o.gi(w, target)];
    Vec3 base = t.pos;
    auto testVisible = [&](Vec3 p) {
        Vec3 to_test = p - org;
        Vec3 view = rotateVec(qinv(aim_rot), to_test);
        if (view.y <= 0.f) return false;
        if (!inFrustum(o, view)) return false;
        float len = length(to_test);
        if (len < kAgentRadius) return false;
        to_test = to_test / len;
        HitResult h = traceRayAgainstWorld(o, w, org, to_test);
        if (!h.hit) return false;
        return h.entity == target;
    };
    float vh = viewHeight(t.curPose);
    Vec3 aim_right = rotateVec(aim_rot, kRight);
    Vec3 delta_right = aim_right * 0.9f * kAgentRadius;
    Vec3 bottom = base; bottom.z += kAgentRadius;
    Vec3 top = base; top.z += vh;
    Vec3 right = base; right.z += vh; right = right + delta_right;
    Vec3 left = base; left.z += vh; left = left - delta_right;
    int num_visible = 0;
    if (testVisible(bottom)) num_visible++;
    if (testVisible(top)) num_visible++;
    if (testVisible(left)) num_visible++;
    if (testVisible(right)) num_visible++;
    return num_visible > 0;
}

// utils.cpp:273-479 standardSpawnPoint (Zone task: no TDM episode branch)
void standardSpawnPoint(Oracle &o, int w, int ai, bool is_respawn, bool use_middle_spawn, Vec3 *out_pt,
                        float *out_yaw)
{
    World &wd = o.worlds[w];
    Agent &ag = o.agent(w, ai);
    RNG &rng = ag.rng;

    const Spawn *options;
    int num_spawns;
    auto spawnAgent = [&](int idx) {
        Spawn s = options[idx];
        float x_rnd = rngUniform(rng);
        float y_rnd = rngUniform(rng);
        float z_rnd = rngUniform(rng);
        float yaw_rnd = rngUniform(rng);
        float x_min = s.region.pMin.x, x_diff = s.region.pMax.x - x_min;
        float y_min = s.region.pMin.y, y_diff = s.region.pMax.y - y_min;
        float z_min = s.region.pMin.z, z_diff = s.region.pMax.z - z_min;
        *out_pt = v3(x_min + x_rnd * x_diff, y_min + y_rnd * y_diff, z_min + z_rnd * z_diff);
        *out_yaw = s.yawMin + yaw_rnd * (s.yawMax - s.yawMin);
    };

    if (!is_respawn || o.commonRespawns.empty()) {
        uint32_t *tracker;
        int num_default, num_extra;
        if (ag.team == wd.teamA) {
            options = o.aSpawns.data();
            num_default = (int)o.numDefaultASpawns;
            num_extra = (int)o.aSpawns.size() - num_default;
            tracker = o.track(w, 0);
        } else {
            options = o.bSpawns.data();
            num_default = (int)o.numDefaultBSpawns;
            num_extra = (int)o.bSpawns.size() - num_default;
            tracker = o.track(w, 1);
        }
        if (use_middle_spawn) {
            options += num_default;
            num_spawns = num_extra;
        } else {
            num_spawns = num_default;
        }
        int init_idx = -1;
        for (int i = 0; i < 5; i++) {
            int idx = rngI32(rng, 0, num_spawns);
            if (tracker[idx] == (uint32_t)wd.curStep) continue;
            init_idx = idx;
            break;
        }
        if (init_idx == -1) init_idx = rngI32(rng, 0, num_spawns);
        spawnAgent(init_idx);
        tracker[init_idx] = (uint32_t)wd.curStep;
        return;
    }

    options = o.commonRespawns.data();
    num_spawns = (int)o.commonRespawns.size();
    AABB zone_aabb = o.zoneAABBs[wd.curZone];
    Vec3 zone_center = 0.5f * (zone_aabb.pMin + zone_aabb.pMax);

    float best_score = kFltMax;
    int best_idx = -1;
    for (int s = 0; s < num_spawns; s++) {
        uint32_t last_used = o.track(w, 2)[s];
        if (last_used == (uint32_t)wd.curStep) continue;
        float score = 0.f;
        uint32_t elapsed = (uint32_t)(kDeltaT * float((uint32_t)wd.curStep - last_used));
        const float elapsed_weight = 0.1f, dist_weight = 0.01f;
        if (elapsed < 3.f) score += elapsed_weight * (3.f - elapsed);
        Spawn sp = options[s];
        Vec3 spawn_pt = 0.5f * (sp.region.pMin + sp.region.pMax);
        for (int j = 0; j < o.N; j++) {
            if (j == ai) continue;
            const Agent &other = o.agent(w, j);
            if (o.alive[o.gi(w, j)] == 0.f) continue;
            float dist = distance(spawn_pt, other.pos);
            if (dist < 4.f * kAgentRadius) {
                score += 100000.f;
            } else {
                if (other.team == ag.team) continue;
                score += dist_weight * (1.f / dist);
            }
        }
        float dz = distance(spawn_pt, zone_center);
        if (dz < 100.f) score += 1000000.f;
        if (score < best_score) {
            best_idx = s;
            best_score = score;
        }
    }
    if (best_idx < 0) best_idx = 0; // assert(best_spawn_idx != -1) in the reference
    spawnAgent(best_idx);
    o.track(w, 2)[best_idx] = (uint32_t)wd.curStep;
}

// AgentPolicy idx clamped to the 8 sub-zones (sim.cpp:1996-1997, 3802-3803)
int subZoneIndex(const Oracle &o, size_t g)
{
    return std::clamp(o.policy[g], 0, 7);
}

// utils.cpp:734-948 spawnAgents (Zone task)
void spawnAgents(Oracle &o, int w, bool is_respawn)
{
    World &wd = o.worlds[w];
    int dead[2 * kMaxTeamSize];
    int num_dead = 0;
    for (int i = 0; i < o.N; i++) {
        if (o.alive[o.gi(w, i)] == 0.f) dead[num_dead++] = i;
    }
    if (num_dead == 0) return;

    RNG &base = wd.baseRNG;
    (void)rngI32(base, 0, 0); // episodes[sampleI32(0, numEpisodes = 0)] (utils.cpp:788-789)

    bool use_middle = false;
    if (o.simFlags & MPENV_SIMFLAG_SPAWN_IN_MIDDLE) use_middle = rngUniform(base) < 0.5f;
    const bool randomize_hp = (o.simFlags & MPENV_SIMFLAG_RANDOMIZE_HP_MAGAZINE) != 0;
    const bool hardcoded = (o.simFlags & MPENV_SIMFLAG_HARDCODED_SPAWNS) != 0;
    const bool navmesh_spawn = (o.simFlags & MPENV_SIMFLAG_NAVMESH_SPAWN) != 0;
    const bool curriculum = (o.simFlags & MPENV_SIMFLAG_ENABLE_CURRICULUM) != 0;

    for (int d = 0; d < num_dead; d++) {
        int ai = dead[d];
        Agent &ag = o.agent(w, ai);
        size_t g = o.gi(w, ai);
        Vec3 spawn_pt;
        float spawn_yaw;
        float spawn_pitch = 0.f;
        if (hardcoded && !is_respawn) {
            // utils.cpp:480-650 hardcodedSpawnPoint (curriculum branch disabled)
            hardcodedSpawn((ag.team == wd.teamA ? 0 : 3) + ag.offset, spawn_pt, spawn_yaw);
        } else if (navmesh_spawn) {
            // utils.cpp:807-809
            spawn_pt = navSamplePoint(&o.navTris[0].x, o.navCdf.data(), o.numNavTris, rngAdvance(base));
            spawn_yaw = rngUniform(base) * 2.f * kPi;
        } else if (curriculum && wd.episodeCurriculum == 0) {
            // utils.cpp:819-837 LearnShooting: standard point, then a random
            // point on the spawn's side of y = 0
            standardSpawnPoint(o, w, ai, is_respawn, use_middle, &spawn_pt, &spawn_yaw);
            const bool north = spawn_pt.y > 0.f;
            const float x = -700.f + rngUniform(base) * 1400.f;
            const float y = rngUniform(base) * 350.f;
            spawn_pt = v3(x, north ? y : -y, 0.f);
        } else {
            standardSpawnPoint(o, w, ai, is_respawn, use_middle, &spawn_pt, &spawn_yaw);
        }

        ag.pos = spawn_pt;
        ag.rot = qnormalize(angleAxis(spawn_yaw, kUp));
        AimS aim = computeAim(spawn_yaw, spawn_pitch);
        ag.aimYaw = aim.yaw; ag.aimPitch = aim.pitch; ag.aimRot = aim.rot;
        ag.vel = v3(0.f, 0.f, 0.f);

        ag.weaponType = rngI32(base, 0, kNumWeaponTypes);
        if (randomize_hp) {
            int tenth = rngI32(base, 1, 11);
            o.hp[g] = float(tenth * 10);
            o.magazine[2 * g] = rngI32(base, 0, kMagSize);
            o.magazine[2 * g + 1] = 0;
        } else {
            o.hp[g] = 100.f;
            o.magazine[2 * g] = kMagSize;
            o.magazine[2 * g + 1] = 0;
        }
        ag.remainingRespawnSteps = is_respawn ? 0 : kRespawnInvincibleSteps;
        ag.remainingStepsBeforeAutoheal = 0;

        {
            AABB zone_aabb = o.zoneAABBs[wd.curZone];
            Vec3 zone_center = (zone_aabb.pMax + zone_aabb.pMin) / 2.f;
            float rot_angle = o.zoneRot[wd.curZone];
            Quat to_zone = qinv(angleAxis(rot_angle, kUp));
            zone_aabb.pMin = rotateVec(to_zone, zone_aabb.pMin);
            zone_aabb.pMax = rotateVec(to_zone, zone_aabb.pMax);
            Vec3 pos_in_zone = rotateVec(to_zone, spawn_pt);
            spawn_pt.z += kStandHeight / 2.f;
            ag.inZone = aabbContains(zone_aabb, pos_in_zone);
            ag.minDistToZone = distance(spawn_pt, zone_center);
        }
        if (o.simFlags & MPENV_SIMFLAG_SUB_ZONES) {
            // utils.cpp:906-926 (spawn_pt already carries the +standHeight/2
            // of the zone block above and receives it a second time)
            const Oracle::ZOBB &sz = o.subZones[subZoneIndex(o, g)];
            AABB zone_aabb = { sz.pMin, sz.pMax };
            Vec3 zone_center = (zone_aabb.pMax + zone_aabb.pMin) / 2.f;
            Quat to_zone = qinv(angleAxis(sz.rotation, kUp));
            zone_aabb.pMin = rotateVec(to_zone, zone_aabb.pMin);
            zone_aabb.pMax = rotateVec(to_zone, zone_aabb.pMax);
            Vec3 pos_in_zone = rotateVec(to_zone, spawn_pt);
            spawn_pt.z += kStandHeight / 2.f;
            ag.inSubZone = aabbContains(zone_aabb, pos_in_zone);
            ag.minDistToSubZone = distance(spawn_pt, zone_center);
        }

        ag.curPose = kStand; ag.tgtPose = kStand; ag.transitionRemaining = 0;
        ag.newPos = ag.pos;
        ag.newVel = v3(0.f, 0.f, 0.f);
        ag.maxVelocity = kMaxWalkVelocity;
        ag.daimYawVel = 0.f; ag.daimPitchVel = 0.f;
        o.alive[g] = 1.f;
    }
}

// ====================================================== level_gen.cpp
// level_gen.cpp:19-328 createPersistentEntities (agents only: static
// geometry, zone/camera/sub-zone entities are visualisation-only)
void createPersistentEntities(Oracle &o, int w)
{
    for (int i = 0; i < o.N; i++) {
        Agent &ag = o.agent(w, i);
        size_t g = o.gi(w, i);
        ag.visited.assign((size_t)kGridW * kGridW, 0u);
        for (int y = 0; y < kGridMax; y++)
            for (int x = 0; x < kGridMax; x++)
                ag.visited[(size_t)y * kGridW + x] = 0xFFFFFFFFu;
        o.policy[g] = 0;
        o.aimAction[2 * g] = 0.f; o.aimAction[2 * g + 1] = 0.f;
        o.discreteAim[2 * g] = kDiscreteAimYawBuckets / 2;
        o.discreteAim[2 * g + 1] = kDiscreteAimPitchBuckets / 2;
        ag.daimYawVel = 0.f; ag.daimPitchVel = 0.f;
        ag.team = i / o.teamSize;
        ag.offset = i - ag.team * o.teamSize;
        for (int j = 0; j < kMaxTeamSize; j++) ag.dmg[j] = 0.f;
    }
}

// level_gen.cpp:330-582 resetPersistentEntities
void resetPersistentEntities(Oracle &o, int w, RandKey episode_key)
{
    World &wd = o.worlds[w];
    RNG &base = wd.baseRNG;
    for (int i = 0; i < o.N; i++) {
        Agent &ag = o.agent(w, i);
        size_t g = o.gi(w, i);
        ag.pos = v3(kFltMax, kFltMax, kFltMax);
        ag.rng = makeRNG(splitI(episode_key, (uint32_t)(i + 1)));
        ag.landedShotOn = -1;
        ag.remainingRespawnSteps = 0;
        ag.remainingStepsBeforeAutoheal = 0;
        ag.successfulKill = false;
        ag.wasShotCount = 0;
        ag.wasKilled = false;
        ag.firedShotT = -kFltMax;
        ag.hasDiedDuringEpisode = false;
        ag.reloadedFullMag = false;
        o.alive[g] = 0.f;
        for (int j = 0; j < kMaxTeamSize; j++) {
            float *lk = &o.lastKnownObs[(g * kMaxTeamSize + j) * kOtherObs];
            std::fill(lk, lk + kOtherObs, 0.f);
            float *lkp = &o.lastKnownPos[(g * kMaxTeamSize + j) * 3];
            lkp[0] = lkp[1] = lkp[2] = -1000.f;
        }
        ag.totalPenalty = 0.f;
        ag.lastBreadcrumb = -1;
        ag.stepsSinceLastNewBreadcrumb = 0;
    }
    std::fill(o.track(w, 0), o.track(w, 0) + 3 * o.spawnTrackLen, 0xFFFFFFFFu);
    spawnAgents(o, w, false);

    for (int i = 0; i < o.N; i++) {
        Agent &ag = o.agent(w, i);
        size_t g = o.gi(w, i);
        ag.startPos = ag.pos;
        for (int k = 0; k < 4; k++) o.discreteAction[4 * g + k] = 0;
        o.aimAction[2 * g] = 0.f; o.aimAction[2 * g + 1] = 0.f;
        ag.numNewCellsVisited = 0;
        auto sampleCoef = [&base](float a, float b) { return a + (b - a) * rngUniform(base); };
        // level_gen.cpp:434-444: nine draws, then overwritten with defaults (446)
        (void)sampleCoef(0.f, 1.f);
        (void)sampleCoef(0.01f, 0.2f);
        (void)sampleCoef(0.0001f, 0.005f);
        (void)sampleCoef(0.0f, 0.05f);
        (void)sampleCoef(0.0f, 0.01f);
        (void)sampleCoef(0.0f, 0.1f);
        (void)sampleCoef(0.0f, 0.01f);
        (void)sampleCoef(0.1f, 2.0f);
        (void)sampleCoef(0.01f, 0.5f);
        float *rc = &o.rewardCoefs[9 * g];
        rc[0] = 0.f; rc[1] = 0.5f; rc[2] = 0.005f; rc[3] = 0.05f; rc[4] = 0.01f;
        rc[5] = 0.1f; rc[6] = 0.0005f; rc[7] = 1.f; rc[8] = 0.1f;
    }

    for (int i = 0; i < (int)o.goalRegions.size(); i++) {
        wd.regionsActive[i] = true;
        wd.minDistToRegions[i] = kFltMax;
    }
    wd.teamStepRewards[0] = 0.f;
    wd.teamStepRewards[1] = 0.f;

    // level_gen.cpp:498-580: start from a recorded match state half the time
    // (not in eval mode); the uniform is drawn whenever snapshots exist
    if (!o.curriculum.empty() && rngUniform(base) < 0.5f && !o.trainControl[0]) {
        const int idx = rngI32(base, 0, (int)o.curriculum.size());
        const mpenv_curriculum_snapshot &sn = o.curriculum[idx];
        wd.curZone = sn.cur_zone;
        if (sn.cur_zone_controller == -1) {
            wd.curControllingTeam = -1;
            wd.isCaptured = false;
        } else {
            wd.isCaptured = true;
            wd.curControllingTeam = sn.cur_zone_controller;
            wd.stepsUntilPoint = sn.steps_until_point;
            wd.zoneStepsRemaining = sn.zone_steps_remaining;
        }
        wd.curStep = sn.step;
        const int half = o.N / 2;
        for (int i = 0; i < o.N; i++) {
            const int j = wd.teamA == 0 ? i : (i < half ? half + i : i - half);
            Agent &ag = o.agent(w, j);
            const size_t g = o.gi(w, j);
            const mpenv_packed_player &p = sn.players[i];
            ag.pos = v3((float)p.pos[0], (float)p.pos[1], (float)p.pos[2]);
            AimS aim = computeAim((float)p.yaw * kPi / 32768.f, (float)p.pitch * kPi / 32768.f);
            ag.aimYaw = aim.yaw; ag.aimPitch = aim.pitch; ag.aimRot = aim.rot;
            ag.rot = qnormalize(angleAxis(aim.yaw, kUp));
            o.hp[g] = (float)p.hp;
            o.magazine[2 * g] = p.mag_num_bullets;
            o.magazine[2 * g + 1] = p.is_reloading;
            if (p.flags & 4) { ag.curPose = kCrouch; ag.tgtPose = kCrouch; ag.transitionRemaining = 0; }
            if (p.flags & 8) { ag.curPose = kProne; ag.tgtPose = kProne; ag.transitionRemaining = 0; }
        }
    }
}

// sim.cpp:732-833 initWorld
void initWorld(Oracle &o, int w, bool triggered_reset)
{
    World &wd = o.worlds[w];
    const uint32_t world_id = o.worldOffset + (uint32_t)w;
    wd.episodeCurriculum = o.worldCurriculum[w];
    wd.matchID = ((uint64_t)world_id << 32) | (uint64_t)wd.curEpisodeIdx;

    RandKey episode_key = splitI(o.initRandKey, wd.curEpisodeIdx, world_id);
    wd.baseRNG = makeRNG(splitI(episode_key, 0));
    RNG &base = wd.baseRNG;

    bool flip = false;
    if (o.trainControl[2]) flip = rngUniform(base) < 0.5f;
    wd.teamA = flip ? 1 : 0;
    if (triggered_reset && o.trainControl[1]) {
        wd.curStep = rngI32(base, 0, kEpisodeLen - 1);
    } else {
        wd.curStep = 0;
    }
    wd.isFinished = false;

    // CurriculumState (sim.cpp:5915-5924)
    const float use_prob = 1.0f;
    const float tier_probs[5] = { 0.f, 0.f, 0.3f, 0.3f, 0.4f };
    wd.enableSpawnCurriculum = rngUniform(base) < use_prob;
    float cdf[5];
    float running = 0.f;
    for (int i = 0; i < 5; i++) { running += tier_probs[i]; cdf[i] = running; }
    float sel = running * rngUniform(base);
    for (int i = 0; i < 5; i++) {
        if (sel < cdf[i]) { wd.curCurriculumTier = (uint32_t)i; break; }
    }
    // SpawnCurriculum tiers are only consumed by the disabled
    // curriculumSpawnPoint (utils.cpp:652-732); only the draw matters.
    wd.curCurriculumSpawnIdx = (uint32_t)rngI32(base, 0, 0);

    if (o.simFlags & MPENV_SIMFLAG_HARDCODED_SPAWNS) (void)rngI32(base, 0, 4);

    wd.curZone = rngI32(base, 0, (int)o.zoneAABBs.size());
    wd.curControllingTeam = -1;
    wd.isContested = false;
    wd.isCaptured = false;
    wd.earnedPoint = false;
    wd.zoneStepsRemaining = kNumStepsPerZone;
    wd.stepsUntilPoint = kZonePointInterval;
    for (int k = 0; k < 8; k++) { // sim.cpp:815-820
        wd.subCtrl[k] = -1;
        wd.subContested[k] = false;
        wd.subCaptured[k] = false;
    }
    if (o.task == MPENV_TASK_ZONE_CAPTURE_DEFEND) wd.curZone = 3; // sim.cpp:822-825

    resetPersistentEntities(o, w, episode_key);

    for (int t = 0; t < 2; t++) {
        wd.filtersActive[t] = 0;
        wd.filtersLastMatchedStep[t] = 0;
    }
}

// sim.cpp:835-872 resetSystem
void resetSystem(Oracle &o, int w)
{
    World &wd = o.worlds[w];
    int32_t force_reset = o.resetBuf[w];
    int32_t should_reset = force_reset;
    if (o.autoReset && wd.isFinished) should_reset = 1;
    if (should_reset != 0) {
        o.resetBuf[w] = 0;
        wd.curEpisodeIdx = wd.worldEpisodeCounter++;
        if (o.simFlags & MPENV_SIMFLAG_ENABLE_CURRICULUM) {
            if (wd.curEpisodeIdx < 50) {
                if (rngUniform(wd.baseRNG) < (wd.curEpisodeIdx + 1) / (float)50) o.worldCurriculum[w] = 1;
                else o.worldCurriculum[w] = 0;
            } else {
                o.worldCurriculum[w] = 1;
            }
        }
        initWorld(o, w, force_reset == 1);
    }
}

// ====================================================== step systems
Vec3 rotate2D(Vec3 dir, float radians) // sim.cpp:874-879
{
    float c = cosf_(radians);
    float s = sinf_(radians);
    return v3(c * dir.x - s * dir.y, s * dir.x + c * dir.y, 0);
}

// sim.cpp:2093-2199 pvpMovementSystem
void pvpMovementSystem(Oracle &o, int w, int i)
{
    Agent &ag = o.agent(w, i);
    size_t g = o.gi(w, i);
    if (o.alive[g] == 0.f) return;
    const int32_t *action = &o.discreteAction[4 * g];
    {
        Vec3 v = ag.vel;
        float v_len = length(v);
        if (v_len > 0.f) {
            Vec3 norm_v = v / v_len;
            v_len -= kDeaccelerateRate * kDeltaT;
            v_len = fmaxD(0.f, v_len);
            ag.vel = norm_v * v_len;
        }
    }
    if (ag.transitionRemaining > 0) {
        ag.transitionRemaining -= 1;
        if (ag.transitionRemaining == 0) ag.curPose = ag.tgtPose;
    }
    int action_pose = action[3];
    if (action_pose != ag.tgtPose) {
        ag.tgtPose = action_pose;
        int dst = std::abs(ag.tgtPose - ag.curPose);
        ag.transitionRemaining = dst * (kPoseTransitionSpeed / 2);
    }
    int32_t move_amount_d = action[0];
    int32_t move_angle_d = action[1];
    float accel_max = 3000;
    if (ag.curPose == kCrouch) accel_max = 100;
    else if (ag.curPose == kProne) accel_max = 50;
    float move_amount = (float)move_amount_d * (accel_max / (float)(kNumMoveAmountBuckets - 1));
    const float per_bucket = 2.f * kPi / float(kNumMoveAngleBuckets);
    float move_angle = float(move_angle_d) * per_bucket;
    float f_x = move_amount * sinf_(move_angle);
    float f_y = move_amount * cosf_(move_angle);
    ag.vel = ag.vel + rotateVec(ag.rot, v3(f_x, f_y, 0)) * kDeltaT;
    if (move_amount != 0) ag.remainingRespawnSteps = 0;
    float v_len = length(ag.vel);
    if (v_len == 0.f) return;
    {
        const float max_change = 510.f;
        float tgt;
        if (ag.curPose == kStand) tgt = move_amount_d == 2 ? kMaxRunVelocity : kMaxWalkVelocity;
        else if (ag.curPose == kCrouch) tgt = kMaxCrouchVelocity;
        else tgt = kMaxProneVelocity;
        float diff = tgt - ag.maxVelocity;
        float adj = fmaxD(fminD(diff, max_change), -max_change);
        ag.maxVelocity += adj;
    }
    Vec3 v_norm = ag.vel / v_len;
    v_len = fminD(v_len, ag.maxVelocity);
    ag.vel = v_norm * v_len;
}

// sim.cpp:2266-2282 pvpContinuousAimSystem
void pvpContinuousAimSystem(Oracle &o, int w, int i)
{
    Agent &ag = o.agent(w, i);
    size_t g = o.gi(w, i);
    if (o.alive[g] == 0.f) return;
    ag.aimYaw += o.aimAction[2 * g] * kDeltaT;
    ag.aimPitch += o.aimAction[2 * g + 1] * kDeltaT;
    AimS a = computeAim(ag.aimYaw, ag.aimPitch);
    ag.aimYaw = a.yaw; ag.aimPitch = a.pitch; ag.aimRot = a.rot;
    ag.rot = qnormalize(angleAxis(ag.aimYaw, kUp));
}

// sim.cpp:2284-2370 pvpDiscreteAimSystem
void pvpDiscreteAimSystem(Oracle &o, int w, int i)
{
    Agent &ag = o.agent(w, i);
    size_t g = o.gi(w, i);
    if (o.alive[g] == 0.f) return;
    static const float yaw_turn[7] = { 0, 0.00390625f * kPi, 0.0078125f * kPi, 0.015625f * kPi,
                                       0.03125f * kPi, 0.0625f * kPi, 0.125f * kPi };
    static const float pitch_turn[4] = { 0, 0.0078125f * kPi, 0.015625f * kPi, 0.03125f * kPi };
    int yb = o.discreteAim[2 * g] - kDiscreteAimYawBuckets / 2;
    if (yb < 0) ag.aimYaw -= yaw_turn[std::abs(yb)];
    else ag.aimYaw += yaw_turn[std::abs(yb)];
    int pb = o.discreteAim[2 * g + 1] - kDiscreteAimPitchBuckets / 2;
    if (pb < 0) ag.aimPitch -= pitch_turn[std::abs(pb)];
    else ag.aimPitch += pitch_turn[std::abs(pb)];
    AimS a = computeAim(ag.aimYaw, ag.aimPitch);
    ag.aimYaw = a.yaw; ag.aimPitch = a.pitch; ag.aimRot = a.rot;
    ag.rot = qnormalize(angleAxis(ag.aimYaw, kUp));
}

// ---- NavUtils (sim.cpp:4958-5037)
Vec3 navTriCenter(const Oracle &o, int tri)
{
    Vec3 c = v3(0.f, 0.f, 0.f);
    for (int k = 0; k < 3; k++) c = c + o.navTris[3 * tri + k] / 3.0f;
    return c;
}

// NearestNavTri (sim.cpp:4975-5010)
int nearestNavTri(const Oracle &o, Vec3 pos)
{
    float closest = kFltMax;
    int closest_idx = -1;
    for (int tri = 0; tri < o.numNavTris; tri++) {
        bool contained = true;
        bool gtz = false;
        for (int i = 0; i < 3; i++) {
            Vec3 v1 = o.navTris[3 * tri + i];
            Vec3 v2 = o.navTris[3 * tri + (i + 1) % 3];
            Vec3 v3_ = v2 - v1;
            Vec3 vp = pos - v1;
            Vec3 c = cross(v3_, vp);
            if ((c.z > 0.0f) != gtz && i > 0) contained = false;
            gtz = c.z > 0.0f;
            float distsq = length2(v1 - pos);
            if (distsq < closest) {
                float dir = dot(v3_, vp);
                Vec3 perp = vp * (-dir / dot(v3_, v3_)) + v3_;
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

// PathfindToPoint (sim.cpp:5012-5035)
Vec3 pathfindToPoint(const Oracle &o, Vec3 start, Vec3 pos)
{
    int start_tri = nearestNavTri(o, start);
    int goal_tri = nearestNavTri(o, pos);
    if (start_tri < 0 || goal_tri < 0) return v3(0.f, 0.f, 0.f); // assert in the reference
    int next_tri = o.astar[(size_t)start_tri * o.numNavTris + goal_tri];
    if (next_tri == -1) return v3(0.f, 0.f, 0.f);
    if (next_tri == goal_tri) return pos;
    return navTriCenter(o, next_tri);
}

// sim.cpp:5041-5172 planAStarAISystem
void planAStarAISystem(Oracle &o, int w, int i)
{
    size_t g = o.gi(w, i);
    if (o.policy[g] != -1) return; // consts::aStarPolicyID
    Agent &ag = o.agent(w, i);
    const World &wd = o.worlds[w];
    RNG &rng = ag.rng;
    int move_amount = rngI32(rng, 0, 2);
    int move_angle = rngI32(rng, 0, 2);
    int r_yaw = rngI32(rng, 0, 5);
    int r_pitch = rngI32(rng, 0, 2);
    int r = o.magazine[2 * g] == 0 ? 1 : 0;
    int stand = rngI32(rng, 0, 2);
    int f = 0;
    for (int k = 0; k < o.N / 2; k++)
        if (ag.canSee[k]) f = 1;
    AABB zb = o.zoneAABBs[wd.curZone];
    Vec3 center = (zb.pMin + zb.pMax) / 2.f; // AABB::centroid
    Vec3 pos = v3(ag.pos.x, ag.pos.y, 0.0f);
    center = pathfindToPoint(o, pos, center);
    center.z = 0.0f;
    Vec3 fwd = v3(-sinf_(ag.aimYaw), cosf_(ag.aimYaw), 0.f);
    Vec3 tgt_dir = normalize(center - pos);
    move_amount = dot(fwd, tgt_dir) > 0.6f ? 1 : 0;
    r_yaw = cross(fwd, tgt_dir).z < 0.0f ? 0 + move_amount : 4 - move_amount;
    move_amount *= 2;
    move_angle = 0;
    stand = 0;
    float collision_ang = 0.0f, collision_norm = 0.0f;
    for (int y = 0; y < 2; y++) {
        for (int x = 0; x < 32; x++) {
            if (o.fwdLidar[((g * 2 + y) * 32 + x) * 4] < 16.0f) {
                collision_norm++;
                collision_ang += x;
            }
        }
    }
    if (collision_norm > 0.0f) {
        collision_ang /= collision_norm;
        move_amount = 1;
        switch ((int)(collision_ang / (float)32 * 8.0f)) {
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
    if (r) f = 0;
    if (f) r_yaw = 2;
    int32_t *out = &o.botAction[7 * g];
    out[0] = move_amount; out[1] = move_angle; out[2] = r_yaw; out[3] = r_pitch;
    out[4] = f; out[5] = r; out[6] = stand;
}

// sim.cpp:2057-2091 applyBotActionsSystem
void applyBotActionsSystem(Oracle &o, int w, int i)
{
    size_t g = o.gi(w, i);
    if (o.policy[g] != -1) return;
    const int32_t *hb = &o.botAction[7 * g];
    o.discreteAction[4 * g + 0] = hb[0];
    o.discreteAction[4 * g + 1] = hb[1];
    o.discreteAction[4 * g + 2] = hb[4];
    o.discreteAction[4 * g + 3] = hb[6];
    const float turn_delta = 10.f / (float)(5 / 2);
    o.aimAction[2 * g] = turn_delta * (float)(hb[2] - 5 / 2);
    o.aimAction[2 * g + 1] = turn_delta * (float)(hb[3] - 5 / 2);
}

// sim.cpp:889-1028 applyVelocitySystem (+ updateMoveStateSystem 1030-1039)
void applyVelocitySystem(Oracle &o, int w, int i)
{
    Agent &ag = o.agent(w, i);
    Vec3 x = ag.pos;
    Vec3 v = ag.vel;
    v.z = 0;
    ag.newPos = x;
    ag.newVel = v3(0.f, 0.f, 0.f);
    float v_len = length(v);
    if (v_len == 0.f) return;
    Vec3 v_norm = v / v_len;
    float move_dist = v_len * kDeltaT;

    const float buffer = 0.05f * kAgentRadius;
    const float r = kAgentRadius;
    float top = kStandHeight - r;
    float low_check = kProneHeight;
    if (ag.curPose == kCrouch) {
        top = kCrouchHeight - r;
    } else if (ag.curPose == kProne) {
        top = low_check;
        low_check = kProneHeight - r + buffer;
    }

    Vec3 ray_o = x;
    ray_o.z += top;
    Vec3 normal = v3(0.f, 0.f, 0.f);
    sphereCastWorld(o, ray_o, -kUp, r, normal);
    if (normal.z > 0.0f && normal.z < 0.7 && dot(normal, v_norm) < 0.0f) return;

    ray_o = x + v_norm * buffer * 0.5f;
    ray_o.z += low_check;
    float low_dist = sphereCastWorld(o, ray_o, v_norm, r, normal);
    float high_dist = low_dist;
    bool high_hit = false;
    if (ag.curPose != kProne) {
        ray_o.z = x.z + top;
        Vec3 high_normal = v3(0.f, 0.f, 0.f);
        high_dist = sphereCastWorld(o, ray_o, v_norm, r, high_normal);
        if (high_dist < low_dist) {
            low_dist = high_dist;
            normal = high_normal;
            high_hit = true;
        }
    }
    bool stuck = low_dist == 0.0f || high_dist == 0.0f;
    low_dist = fmaxD(0.0f, low_dist - buffer);
    high_dist = fmaxD(0.0f, high_dist - buffer);
    Vec3 hit_pos = x + v_norm * fminD(low_dist, move_dist);

    if (move_dist > low_dist) {
        Vec3 slide_dir = normalize(cross(kUp, normal));
        if (dot(slide_dir, v_norm) < 0) slide_dir = -slide_dir;
        ray_o = x + v_norm * low_dist;
        ray_o.z += high_hit ? top : low_check;
        float slide = sphereCastWorld(o, ray_o, slide_dir, r);
        slide = fmaxD(0.0f, slide - buffer);
        float max_move = move_dist - low_dist;
        slide = fminD(slide, max_move);
        if (slide > 0.0f) hit_pos = hit_pos + slide_dir * slide;
    }

    Vec3 ground_check = hit_pos;
    ground_check.z += top;
    float ground_dist = sphereCastWorld(o, ground_check, -kUp, r);
    if (ground_dist == kFltMax) return;

    if (ground_dist <= 0.0f || stuck) {
        float furthest = 0.0f;
        int best_dir = -1;
        for (int dir = 0; dir < 4; dir++) {
            Vec3 dv = rotate2D(v_norm, (float)dir * 3.14159f * 0.5f);
            ray_o = x - dv * r * 2.0f;
            ray_o.z += low_check;
            float hd = sphereCastWorld(o, ray_o, dv, r);
            if (hd > furthest) {
                furthest = hd;
                best_dir = dir;
            }
        }
        if (best_dir != -1) {
            Vec3 dv = rotate2D(v_norm, (float)best_dir * 3.14159f * 0.5f);
            hit_pos = x + dv * (fminD(furthest - r * 2.0f, -buffer));
            ground_check = hit_pos;
            ground_check.z += top;
            ground_dist = sphereCastWorld(o, ground_check, -kUp, r);
            if (ground_dist == kFltMax) return;
        }
    }

    float fall_dist = fminD(ground_dist, top) + r;
    Vec3 new_pos = ground_check;
    new_pos.z -= fall_dist;
    Vec3 to_new = new_pos - x;
    float to_new_dist = length(to_new);
    if (to_new_dist == 0.f) return;
    ag.newPos = new_pos;
    ag.newVel = to_new / kDeltaT;
}

// sim.cpp:1041-1095 fallSystem (+ updateMoveStatePostFallSystem 1097-1104)
void fallSystem(Oracle &o, int w, int i)
{
    Agent &ag = o.agent(w, i);
    size_t g = o.gi(w, i);
    if (o.alive[g] == 0.f) {
        ag.newPos = ag.pos;
        return;
    }
    const float fall_rate = 386.08858267717f;
    const float cast_offset = kAgentRadius;
    Vec3 ray_o = ag.pos;
    ray_o.z += kAgentRadius + cast_offset;
    float ground = sphereCastWorld(o, ray_o, -kUp, kAgentRadius);
    if (ground == kFltMax || ground < cast_offset) {
        ag.newPos = ag.pos;
        return;
    }
    float fall = fminD(ground - cast_offset, fall_rate * kDeltaT);
    Vec3 np = ag.pos;
    np.z -= fall;
    ag.newPos = np;
}

// sim.cpp:1443-1615 fireSystem
// sim.cpp:23-39 logEvent into the step's per-world event slots (slot 2i,
// 2i+1: agent i; slot 2N: capture)
void logEvent(Oracle &o, int w, int slot, uint32_t type, int a, int b, int c16)
{
    if (!o.eventsOn) return;
    World &wd = o.worlds[w];
    mpenv_game_event &e = o.events[(size_t)w * (2 * o.N + 1) + slot];
    e.type = type;
    e.pad_ = 0;
    e.match_id = wd.matchID;
    e.step = (uint32_t)wd.curStep;
    e.a = (uint8_t)a;
    e.b = (uint8_t)b;
    e.c16 = (uint16_t)c16;
}

int playerId(const Agent &a) { return a.team * kMaxTeamSize + a.offset; }

void fireSystem(Oracle &o, int w, int i)
{
    Agent &ag = o.agent(w, i);
    size_t g = o.gi(w, i);
    ag.landedShotOn = -1;
    ag.successfulKill = false;
    ag.firedShotT = -kFltMax;
    ag.reloadedFullMag = false;
    if (o.alive[g] == 0.f) return;
    int32_t *mag = &o.magazine[2 * g];
    int fire = o.discreteAction[4 * g + 2];
    if (fire == 2) {
        logEvent(o, w, 2 * i, MPENV_EVENT_RELOAD, playerId(ag), mag[0], 0);
        if (mag[0] == kMagSize) ag.reloadedFullMag = true;
        mag[0] = kMagSize;
        mag[1] = kReloadTime;
    }
    bool reload_in_progress = mag[1] > 0;
    if (reload_in_progress) mag[1] -= 1;
    bool should_fire = false;
    if (!reload_in_progress && mag[0] > 0) should_fire = fire == 1;
    if (!should_fire) return;
    mag[0] -= 1;

    Vec3 fire_from = ag.pos;
    fire_from.z += viewHeight(ag.curPose);
    float u1 = rngUniform(ag.rng);
    float u2 = rngUniform(ag.rng);
    float z1 = sqrt_(-2.f * logf_(u1)) * cosf_(2.f * kPi * u2);
    float z2 = sqrt_(-2.f * logf_(u1)) * sinf_(2.f * kPi * u2);
    float acc = kAccuracyScale;
    float bias = 1.5f;
    float up_delta = fminD(fmaxD((z1 + bias) * acc, 0.f), 4.f * acc);
    float right_delta = fminD(fmaxD(z2 * acc, -4.f * acc), 4.f * acc);
    ag.aimYaw += right_delta;
    ag.aimPitch += up_delta;
    AimS a = computeAim(ag.aimYaw, ag.aimPitch);
    ag.aimYaw = a.yaw; ag.aimPitch = a.pitch; ag.aimRot = a.rot;
    Vec3 fire_dir = rotateVec(ag.aimRot, kFwd);

    HitResult h = traceRayAgainstWorld(o, w, fire_from, fire_dir);
    ag.firedShotT = h.hit ? h.t : kFltMax;
    bool success = h.hit;
    if (h.entity == -1) {
        success = false;
    } else {
        const Agent &tgt = o.agent(w, h.entity);
        if (success && tgt.team == ag.team) success = false;
        if (success && tgt.remainingRespawnSteps > 0) success = false;
    }
    if (!success) return;
    logEvent(o, w, 2 * i, MPENV_EVENT_PLAYER_SHOT, playerId(ag), playerId(o.agent(w, h.entity)), 0);
    ag.landedShotOn = h.entity;
    if (o.hp[o.gi(w, h.entity)] <= kDmgPerBullet) {
        ag.successfulKill = true;
        logEvent(o, w, 2 * i + 1, MPENV_EVENT_KILL, playerId(ag), playerId(o.agent(w, h.entity)), 0);
    }
    o.agent(w, h.entity).dmg[ag.offset] = kDmgPerBullet;
}

// sim.cpp:1794-1836 applyDmgSystem
void applyDmgSystem(Oracle &o, int w, int i)
{
    Agent &ag = o.agent(w, i);
    size_t g = o.gi(w, i);
    ag.wasShotCount = 0;
    ag.wasKilled = false;
    if (ag.remainingRespawnSteps > 0) ag.remainingRespawnSteps -= 1;
    for (int k = 0; k < o.teamSize; k++) {
        if (ag.dmg[k] > 0.f) {
            ag.wasShotCount += 1;
            ag.remainingStepsBeforeAutoheal = kOutOfCombatSteps;
        }
        o.hp[g] -= ag.dmg[k];
        ag.dmg[k] = 0.f;
    }
    if (o.alive[g] == 1.f && o.hp[g] <= 0.f) {
        ag.wasKilled = true;
        ag.hasDiedDuringEpisode = true;
    }
    if (o.hp[g] <= 0.f) {
        o.hp[g] = 0.f;
        o.alive[g] = 0.f;
        ag.pos = v3(0, 0, 10000.f);
        ag.vel = v3(0, 0, 0);
    } else {
        o.alive[g] = 1.f;
    }
}

// sim.cpp:1875-1890 autoHealSystem
void autoHealSystem(Oracle &o, int w, int i)
{
    Agent &ag = o.agent(w, i);
    size_t g = o.gi(w, i);
    if (o.alive[g] == 0.f) return;
    if (ag.remainingStepsBeforeAutoheal == 0 && o.hp[g] < 100.f) {
        o.hp[g] = fminD(100.f, o.hp[g] + kAutohealPerStep);
    } else if (ag.remainingStepsBeforeAutoheal > 0) {
        ag.remainingStepsBeforeAutoheal -= 1;
    }
}

// sim.cpp:1892-1976 zoneSystem
void zoneSystem(Oracle &o, int w)
{
    World &wd = o.worlds[w];
    if (wd.curControllingTeam != -1) wd.zoneStepsRemaining -= 1;
    if (wd.zoneStepsRemaining == 0) {
        wd.curZone += 1;
        if (wd.curZone == (int)o.zoneAABBs.size()) wd.curZone = 0;
        wd.isCaptured = false;
        wd.zoneStepsRemaining = kNumStepsPerZone;
        wd.stepsUntilPoint = kZonePointInterval;
        AABB za = o.zoneAABBs[wd.curZone];
        Vec3 center = (za.pMax + za.pMin) / 2.f;
        for (int i = 0; i < o.N; i++) {
            Agent &ag = o.agent(w, i);
            ag.minDistToZone = distance(ag.pos, center);
        }
    }
    AABB za = o.zoneAABBs[wd.curZone];
    float rot_angle = o.zoneRot[wd.curZone];
    Quat to_zone = qinv(angleAxis(rot_angle, kUp));
    za.pMin = rotateVec(to_zone, za.pMin);
    za.pMax = rotateVec(to_zone, za.pMax);
    int na = 0, nb = 0;
    for (int i = 0; i < o.N; i++) {
        Agent &ag = o.agent(w, i);
        Vec3 p = ag.pos;
        p.z += kStandHeight / 2.f;
        Vec3 pz = rotateVec(to_zone, p);
        if (!aabbContains(za, pz)) {
            ag.inZone = false;
            continue;
        }
        ag.inZone = true;
        if (ag.team == 0) na += 1;
        if (ag.team == 1) nb += 1;
    }
    wd.stepsUntilPoint -= 1;
    wd.isContested = na > 0 && nb > 0;
    if (wd.isContested || (na == 0 && nb == 0)) {
        wd.curControllingTeam = -1;
        wd.isCaptured = false;
        wd.stepsUntilPoint = kZonePointInterval;
    } else if (na > 0 && nb == 0) {
        if (wd.curControllingTeam != 0) {
            wd.curControllingTeam = 0;
            wd.isCaptured = false;
            wd.stepsUntilPoint = kZonePointInterval;
        }
    } else if (na == 0 && nb > 0) {
        if (wd.curControllingTeam != 1) {
            wd.curControllingTeam = 1;
            wd.isCaptured = false;
            wd.stepsUntilPoint = kZonePointInterval;
        }
    }
}

// sim.cpp:1978-2041 subzoneSystem, for sub-zones 0..7 in entity order
void subzoneSystem(Oracle &o, int w)
{
    World &wd = o.worlds[w];
    for (int k = 0; k < 8; k++) {
        const Oracle::ZOBB &sz = o.subZones[k];
        AABB za = { sz.pMin, sz.pMax };
        Quat to_zone = qinv(angleAxis(sz.rotation, kUp));
        za.pMin = rotateVec(to_zone, za.pMin);
        za.pMax = rotateVec(to_zone, za.pMax);
        int na = 0, nb = 0;
        for (int i = 0; i < o.N; i++) {
            if (subZoneIndex(o, o.gi(w, i)) != k) continue;
            Agent &ag = o.agent(w, i);
            Vec3 p = ag.pos;
            p.z += kStandHeight / 2.f;
            Vec3 pz = rotateVec(to_zone, p);
            if (!aabbContains(za, pz)) {
                ag.inSubZone = false;
                continue;
            }
            ag.inSubZone = true;
            ag.minDistToSubZone = 0.f;
            if (ag.team == 0) na += 1;
            if (ag.team == 1) nb += 1;
        }
        wd.subContested[k] = na > 0 && nb > 0;
        if (wd.subContested[k] || (na == 0 && nb == 0)) {
            wd.subCtrl[k] = -1;
            wd.subCaptured[k] = false;
        } else if (na > 0 && nb == 0) {
            if (wd.subCtrl[k] != 0) {
                wd.subCtrl[k] = 0;
                wd.subCaptured[k] = false;
            }
        } else if (na == 0 && nb > 0) {
            if (wd.subCtrl[k] != 1) {
                wd.subCtrl[k] = 1;
                wd.subCaptured[k] = false;
            }
        }
    }
}

// sim.cpp:4845-4889 leaveBreadcrumbsSystem
void leaveBreadcrumbsSystem(Oracle &o, int w, int i)
{
    World &wd = o.worlds[w];
    Agent &ag = o.agent(w, i);
    ag.totalPenalty = 0.f;
    const float penalty = 1.f;
    const int frequency = 10;
    bool updated = false;
    if (ag.lastBreadcrumb != -1) {
        for (Crumb &c : wd.crumbs) {
            if ((int64_t)c.id != ag.lastBreadcrumb) continue;
            if (distance(ag.pos, c.pos) < kAgentRadius * 4) {
                c.penalty = penalty;
                updated = true;
                ag.stepsSinceLastNewBreadcrumb = 0;
            }
            break;
        }
    }
    if (!updated) {
        ag.stepsSinceLastNewBreadcrumb += 1;
        if (ag.stepsSinceLastNewBreadcrumb > frequency) {
            if ((int)wd.crumbs.size() < MPENV_MAX_CRUMBS) {
                Crumb c;
                c.pos = ag.pos;
                c.penalty = penalty;
                c.team = ag.team;
                c.offset = ag.offset;
                c.id = wd.nextCrumbId++;
                wd.crumbs.push_back(c);
                ag.lastBreadcrumb = c.id;
            } else {
                wd.crumbOverflow += 1;
                ag.lastBreadcrumb = -1;
            }
            ag.stepsSinceLastNewBreadcrumb = 0;
        }
    }
}

// sim.cpp:4892-4926 accumulateBreadcrumbPenaltiesSystem (crumbs visited in
// creation order; sim.cpp:5572/5581 CompactArchetypeNode keeps that order)
void accumulateBreadcrumbPenalties(Oracle &o, int w)
{
    World &wd = o.worlds[w];
    std::vector<Crumb> kept;
    kept.reserve(wd.crumbs.size());
    for (Crumb &c : wd.crumbs) {
        for (int team = 0; team < 2; team++) {
            for (int off = 0; off < o.teamSize; off++) {
                if (c.team != team) continue;
                if (c.offset == off) continue;
                Agent &ag = o.agent(w, team * o.teamSize + off);
                if (distance(ag.pos, c.pos) <= kAgentRadius * 4.f) {
                    ag.totalPenalty += c.penalty;
                }
            }
        }
        c.penalty -= 0.025f;
        if (!(c.penalty <= 0.f)) kept.push_back(c);
    }
    wd.crumbs.swap(kept);
}

// sim.cpp:128-291 updateFiltersState
void updateFiltersState(Oracle &o, int w, int cur_step)
{
    World &wd = o.worlds[w];
    struct Filt { int type; int16_t minx, miny, maxx, maxy; int minNum; };
    // type 0 = PlayerInRegion, 1 = PlayerShotEvent (full-range regions)
    const Filt filters[3] = {
        { 0, -1272, -866, -825, 696, 5 },
        { 0, 852, -851, 1280, 593, 1 },
        { 1, -32768, -32768, 32767, 32767, 0 },
    };
    const int window = 0;
    for (int fi = 0; fi < 3; fi++) {
        const Filt &f = filters[fi];
        for (int t = 0; t < 2; t++) {
            if ((wd.filtersActive[t] & (1ull << fi)) != 0) {
                if (cur_step - wd.filtersLastMatches[t][fi] > window) {
                    wd.filtersActive[t] &= ~(1ull << fi);
                }
            }
        }
        if (f.type == 1) {
            for (int p = 0; p < o.N; p++) {
                const Agent &ag = o.agent(w, p);
                int team = p / o.teamSize;
                if (ag.landedShotOn == -1) continue;
                Vec3 ap = ag.pos;
                Vec3 tp = o.agent(w, ag.landedShotOn).pos;
                if (ap.x < f.minx || ap.y < f.miny || ap.x > f.maxx || ap.y > f.maxy ||
                    tp.x < f.minx || tp.y < f.miny || tp.x > f.maxx || tp.y > f.maxy) continue;
                wd.filtersActive[team] |= (1ull << fi);
                wd.filtersLastMatches[team][fi] = cur_step;
            }
        } else {
            int cnt[2] = { 0, 0 };
            for (int p = 0; p < o.N; p++) {
                const Agent &ag = o.agent(w, p);
                int team = p / o.teamSize;
                Vec3 pos = ag.pos;
                if (pos.x < f.minx || pos.y < f.miny || pos.x > f.maxx || pos.y > f.maxy) continue;
                cnt[team] += 1;
            }
            for (int t = 0; t < 2; t++) {
                if (cnt[t] >= f.minNum) {
                    wd.filtersActive[t] |= (1ull << fi);
                    wd.filtersLastMatches[t][fi] = cur_step;
                }
            }
        }
    }
    for (int t = 0; t < 2; t++) {
        if (__builtin_popcountll(wd.filtersActive[t]) == 3) wd.filtersLastMatchedStep[t] = cur_step;
    }
}

// sim.cpp:4470-4673 zoneMatchInfoSystem
// sim.cpp:4592-4634 (capture event) + 41-106 writePackedStepSnapshot.
// eventLoggedInStep / eventMask accumulate every logEvent of the step.
void captureAndSnapshot(Oracle &o, int w, bool new_captured)
{
    World &wd = o.worlds[w];
    const size_t base = (size_t)w * (2 * o.N + 1);
    o.snapWritten[w] = 0;
    if (wd.matchID != ~0ull && new_captured) {
        AABB za = o.zoneAABBs[wd.curZone];
        Quat to_zone = qinv(angleAxis(o.zoneRot[wd.curZone], kUp));
        za.pMin = rotateVec(to_zone, za.pMin);
        za.pMax = rotateVec(to_zone, za.pMax);
        uint32_t mask = 0;
        for (int i = 0; i < o.N; i++) {
            const Agent &ag = o.agent(w, i);
            if (ag.team != wd.curControllingTeam) continue;
            Vec3 p = ag.pos;
            p.z += kStandHeight / 2.f;
            if (aabbContains(za, rotateVec(to_zone, p))) mask |= 1u << i;
        }
        logEvent(o, w, 2 * o.N, MPENV_EVENT_CAPTURE, wd.curZone, wd.curControllingTeam, (int)mask);
    }
    for (int k = 0; k < 2 * o.N + 1; k++) {
        if (o.events[base + k].type != 0) {
            wd.eventLoggedInStep = 1;
            wd.eventMask |= o.events[base + k].type;
        }
    }
    if (wd.matchID == ~0ull) return;
    mpenv_packed_step_snapshot &sn = o.snapshots[w];
    std::memset(&sn, 0, sizeof(sn));
    sn.num_events = wd.eventLoggedInStep;
    sn.event_mask = wd.eventMask;
    wd.eventLoggedInStep = 0;
    wd.eventMask = 0;
    sn.match_id = wd.matchID;
    sn.step = (uint16_t)wd.curStep;
    sn.cur_zone = (uint8_t)wd.curZone;
    sn.cur_zone_controller = (int8_t)(wd.isCaptured ? wd.curControllingTeam : -1);
    sn.zone_steps_remaining = (uint16_t)wd.zoneStepsRemaining;
    sn.steps_until_point = (uint16_t)wd.stepsUntilPoint;
    for (int i = 0; i < o.N; i++) {
        const Agent &ag = o.agent(w, i);
        const size_t g = o.gi(w, i);
        mpenv_packed_player &pl = sn.players[i];
        pl.pos[0] = (int16_t)(int32_t)ag.pos.x;
        pl.pos[1] = (int16_t)(int32_t)ag.pos.y;
        pl.pos[2] = (int16_t)(int32_t)ag.pos.z;
        pl.yaw = (int16_t)(int32_t)(ag.aimYaw * 32768 / kPi);
        pl.pitch = (int16_t)(int32_t)(ag.aimPitch * 32768 / kPi);
        pl.mag_num_bullets = (uint8_t)(uint16_t)o.magazine[2 * g];
        pl.is_reloading = (uint8_t)o.magazine[2 * g + 1];
        pl.hp = (uint8_t)o.hp[g];
        uint8_t fl = 0;
        if (ag.landedShotOn != -1) fl |= 2;
        if (ag.curPose == 1) fl |= 4;
        else if (ag.curPose == 2) fl |= 8;
        pl.flags = fl;
    }
    o.snapWritten[w] = 1;
}

// sim.cpp:4750-4792 pvpRecordSystem
void pvpRecordSystem(Oracle &o, int w)
{
    mpenv_step_log &log = o.recordLog[w];
    log.cur_step = o.worlds[w].curStep;
    for (int i = 0; i < o.N; i++) {
        const Agent &ag = o.agent(w, i);
        const size_t g = o.gi(w, i);
        mpenv_agent_log &a = log.agents[i];
        a.position[0] = ag.pos.x; a.position[1] = ag.pos.y; a.position[2] = ag.pos.z;
        a.aim_yaw = ag.aimYaw;
        a.aim_pitch = ag.aimPitch;
        a.aim_rot[0] = ag.aimRot.w; a.aim_rot[1] = ag.aimRot.x; a.aim_rot[2] = ag.aimRot.y; a.aim_rot[3] = ag.aimRot.z;
        a.hp = o.hp[g];
        a.mag_num_bullets = o.magazine[2 * g];
        a.mag_is_reloading = o.magazine[2 * g + 1];
        a.cur_pose = ag.curPose;
        a.tgt_pose = ag.tgtPose;
        a.transition_remaining = ag.transitionRemaining;
        a.shot_agent_idx = ag.landedShotOn;
        a.fired_shot_t = ag.firedShotT;
        a.was_killed = ag.wasKilled ? 1 : 0;
        a.successful_kill = ag.successfulKill ? 1 : 0;
        a.pad_[0] = a.pad_[1] = 0;
    }
}

// sim.cpp:4794-4843 pvpReplaySystem (viewer shot entities skipped)
void pvpReplaySystem(Oracle &o, int w)
{
    const mpenv_step_log &log = o.replayLog[w];
    o.worlds[w].curStep = log.cur_step;
    for (int i = 0; i < o.N; i++) {
        Agent &ag = o.agent(w, i);
        const size_t g = o.gi(w, i);
        const mpenv_agent_log &a = log.agents[i];
        ag.pos = v3(a.position[0], a.position[1], a.position[2]);
        ag.aimYaw = a.aim_yaw;
        ag.aimPitch = a.aim_pitch;
        ag.aimRot = quat(a.aim_rot[0], a.aim_rot[1], a.aim_rot[2], a.aim_rot[3]);
        ag.rot = qnormalize(angleAxis(a.aim_yaw, kUp));
        o.hp[g] = a.hp;
        o.magazine[2 * g] = a.mag_num_bullets;
        o.magazine[2 * g + 1] = a.mag_is_reloading;
        ag.curPose = a.cur_pose;
        ag.tgtPose = a.tgt_pose;
        ag.transitionRemaining = a.transition_remaining;
        ag.landedShotOn = a.shot_agent_idx;
        ag.firedShotT = a.fired_shot_t;
        ag.wasKilled = a.was_killed != 0;
        ag.successfulKill = a.successful_kill != 0;
        if (ag.wasKilled) ag.hasDiedDuringEpisode = true;
    }
}

void zoneMatchInfoSystem(Oracle &o, int w)
{
    World &wd = o.worlds[w];
    int32_t *mr = &o.matchResult[(size_t)w * 30];
    int cur_step = wd.curStep + 1;
    bool finished = false;
    if (cur_step >= kEpisodeLen || o.resetBuf[w] == 1) finished = true;
    if (cur_step == 1) {
        mr[0] = -1; mr[1] = 0; mr[2] = 0; mr[3] = 0; mr[4] = 0;
    }
    for (int i = 0; i < o.N; i++) {
        const Agent &ag = o.agent(w, i);
        if (ag.wasKilled) mr[1 + (ag.team ^ 1)] += 1;
    }
    wd.earnedPoint = false;
    bool new_captured = false;
    if (wd.stepsUntilPoint == 0) {
        wd.stepsUntilPoint = kZonePointInterval;
        if (!wd.isCaptured) {
            wd.isCaptured = true;
            new_captured = true;
        }
        if (wd.curControllingTeam >= 0) mr[3 + wd.curControllingTeam] += 1;
        wd.earnedPoint = true;
    }
    if (mr[3] >= kZoneWinPoints || mr[4] >= kZoneWinPoints) finished = true;
    // sim.cpp:4534-4575: ZoneCaptureDefend ends on the attacker's first
    // point, the defender's 8th, or when every attacker has died once
    const int attacker = wd.teamA == 1 ? 1 : 0, defender = attacker ^ 1;
    bool all_died[2] = { true, true };
    const bool zcd = o.task == MPENV_TASK_ZONE_CAPTURE_DEFEND;
    if (zcd) {
        if (mr[3 + attacker] == 1) finished = true;
        if (mr[3 + defender] == 8) finished = true;
        for (int i = 0; i < o.N; i++) {
            const Agent &ag = o.agent(w, i);
            if (!ag.hasDiedDuringEpisode) all_died[ag.team] = false;
        }
        if (all_died[attacker]) finished = true;
    }
    {
        int *zs = wd.zoneStats[wd.curZone];
        zs[4] += 1; // numTotalActiveSteps
        if (wd.isCaptured && wd.curControllingTeam >= 0) zs[1 + wd.curControllingTeam] += 1;
        if (wd.isContested) zs[3] += 1;
        if (new_captured) zs[0] += 1;
        updateFiltersState(o, w, cur_step);
        if (o.eventsOn) captureAndSnapshot(o, w, new_captured);
    }
    if (finished) {
        if (zcd) {
            if (mr[3 + attacker] == 1) mr[0] = attacker;
            else if (mr[3 + defender] == 8 || all_died[attacker]) mr[0] = defender;
            else mr[0] = 2;
        } else if (mr[3] > mr[4]) mr[0] = 0;
        else if (mr[4] > mr[3]) mr[0] = 1;
        else mr[0] = 2;
        for (int z = 0; z < kMaxZones; z++)
            for (int k = 0; k < 5; k++) mr[5 + 5 * z + k] = wd.zoneStats[z][k];
        for (int z = 0; z < kMaxZones; z++)
            for (int k = 0; k < 5; k++) wd.zoneStats[z][k] = 0;
    }
    wd.curStep = cur_step;
    wd.isFinished = finished;
}

// sim.cpp:3998-4021 distToZOBB
float distToZOBB(ZOBB z, Vec3 pos)
{
    Quat to_frame = qinv(angleAxis(z.rotation, kUp));
    Vec3 pmin = rotateVec(to_frame, z.pMin);
    Vec3 pmax = rotateVec(to_frame, z.pMax);
    Vec3 p = rotateVec(to_frame, pos);
    float sq = 0.f;
    for (int i = 0; i < 3; i++) {
        float v = comp(p, i);
        if (v < comp(pmin, i)) { float d = comp(pmin, i) - v; sq += d * d; }
        if (v > comp(pmax, i)) { float d = v - comp(pmax, i); sq += d * d; }
    }
    return sqrt_(sq);
}

// sim.cpp:4023-4087 evaluateGoalRegionsSystem
void evaluateGoalRegionsSystem(Oracle &o, int w)
{
    World &wd = o.worlds[w];
    wd.teamStepRewards[0] = 0.f;
    wd.teamStepRewards[1] = 0.f;
    int attacker = wd.teamA;
    for (int r = 0; r < (int)o.goalRegions.size(); r++) {
        const GoalRegion &gr = o.goalRegions[r];
        int region_team = gr.attackerTeam ? attacker : (attacker ^ 1);
        float max_min = -kFltMax;
        for (int s = 0; s < gr.numSubRegions; s++) {
            float min_d = kFltMax;
            for (int i = 0; i < o.N; i++) {
                const Agent &ag = o.agent(w, i);
                if (ag.team != region_team) continue;
                float d = distToZOBB(gr.subRegions[s], ag.pos);
                if (d < min_d) min_d = d;
            }
            if (min_d > max_min) max_min = min_d;
        }
        float prev = wd.minDistToRegions[r];
        if (prev == kFltMax) {
            wd.minDistToRegions[r] = max_min;
        } else {
            float diff = prev - max_min;
            if (diff > 0.f) {
                wd.minDistToRegions[r] = max_min;
                wd.teamStepRewards[region_team] += diff * gr.rewardStrength;
            }
        }
    }
}

// sim.cpp:3508-3536 exploreVisitedSystem
void exploreVisitedSystem(Oracle &o, int w, int i)
{
    World &wd = o.worlds[w];
    Agent &ag = o.agent(w, i);
    Vec3 delta = ag.pos - ag.startPos;
    int32_t x = f2iSat((delta.x + 0.5f) / (kAgentRadius * 2.f));
    int32_t y = f2iSat((delta.y + 0.5f) / (kAgentRadius * 2.f));
    int64_t cx = (int64_t)x + kGridMax, cy = (int64_t)y + kGridMax;
    if (cx < 0 || cx >= kGridW || cy < 0 || cy >= kGridW) return;
    uint32_t &cell = ag.visited[(size_t)cy * kGridW + (size_t)cx];
    uint32_t cur = wd.curEpisodeIdx;
    if (cell != cur) {
        cell = cur;
        if (length2(delta) > 2.f) ag.numNewCellsVisited += 1;
    }
}

// sim.cpp:3707-3732 learnShootingRewardSystem
void learnShootingReward(Agent &ag, float &r)
{
    if (ag.landedShotOn != -1) r += 0.5f;
    else if (ag.firedShotT >= 0.f) r -= 0.05f;
    if (ag.reloadedFullMag) r -= 0.5f;
}

// sim.cpp:3734-3847 subzoneRewardSystem (replaces zoneRewardSystem when
// SubZones is set): kills pay 3, the agent's own sub-zone drives the
// in-zone / approach / control terms, no earned-point or area terms.
void subzoneRewardSystem(Oracle &o, int w, int i)
{
    World &wd = o.worlds[w];
    Agent &ag = o.agent(w, i);
    size_t g = o.gi(w, i);
    float r = 0.f;
    if (o.worldCurriculum[w] == 0) { // LearnShooting
        learnShootingReward(ag, r);
        o.reward[g] = r;
        return;
    }
    const float *rc = &o.rewardCoefs[9 * g];
    const float shot = rc[1], explore = rc[2], in_zone = rc[3], ctrl = rc[5], zdist = rc[6], crumb = rc[8];
    r -= crumb * ag.totalPenalty;
    if (ag.reloadedFullMag) r -= 0.5f;
    if (ag.successfulKill) r += 3.f;
    if (ag.landedShotOn != -1) r += shot * 1.f;
    if (ag.wasKilled) r -= 1.5f;
    if (ag.wasShotCount > 0) r -= shot * 1.f;
    uint32_t nn = ag.numNewCellsVisited;
    ag.numNewCellsVisited = 0;
    if (nn > 0) r += float(nn) * explore;
    const int k = subZoneIndex(o, g);
    if (ag.inSubZone) {
        r += in_zone;
    } else {
        const Oracle::ZOBB &sz = o.subZones[k];
        Vec3 center = (sz.pMax + sz.pMin) / 2.f;
        float dist = distance(center, ag.pos);
        if (dist < ag.minDistToSubZone) {
            float scale = zdist;
            if (!ag.hasDiedDuringEpisode) scale *= 10.f;
            r += scale * (ag.minDistToSubZone - dist);
            ag.minDistToSubZone = dist;
        }
    }
    if (wd.subCtrl[k] != -1) {
        if (wd.subCtrl[k] == ag.team) r += ctrl;
        else r -= ctrl;
    }
    if (o.alive[g] == 0.f) {
        ag.successfulKill = false;
        ag.landedShotOn = -1;
        ag.wasKilled = false;
        ag.wasShotCount = 0;
        ag.firedShotT = -kFltMax;
    }
    o.reward[g] = r;
}

// sim.cpp:4089-4200 zoneCaptureDefendRewardSystem: goal-region progress,
// kills and control of the zone by the agent's own team, +-20 / -5 at the
// end of the match; no curriculum, breadcrumb or area terms.
void zoneCaptureDefendRewardSystem(Oracle &o, int w, int i)
{
    World &wd = o.worlds[w];
    Agent &ag = o.agent(w, i);
    size_t g = o.gi(w, i);
    const float *rc = &o.rewardCoefs[9 * g];
    const float shot = rc[1], explore = rc[2], ctrl = rc[5], earned = rc[7];
    float r = 0.f;
    r += 0.02f * wd.teamStepRewards[ag.team];
    if (ag.reloadedFullMag) r -= 0.01f;
    if (ag.successfulKill) r += 1.f;
    if (ag.landedShotOn != -1) r += shot * 1.f;
    if (ag.wasKilled) r -= 1.f;
    if (ag.wasShotCount > 0) r -= shot * 1.f;
    uint32_t nn = ag.numNewCellsVisited;
    ag.numNewCellsVisited = 0;
    if (nn > 0) r += float(nn) * explore;
    if (!ag.inZone) {
        AABB za = o.zoneAABBs[wd.curZone];
        Vec3 center = (za.pMax + za.pMin) / 2.f;
        float dist = distance(center, ag.pos);
        if (dist < ag.minDistToZone) ag.minDistToZone = dist;
    }
    if (wd.curControllingTeam != -1 && wd.curControllingTeam == ag.team) {
        r += ctrl;
        if (wd.earnedPoint) r += earned;
    }
    if (wd.isFinished) {
        const int win = o.matchResult[(size_t)w * 30];
        if (win == 2) r -= 5.f;
        else if (win == ag.team) r += 20.f;
        else r -= 20.f;
    }
    if (o.alive[g] == 0.f) {
        ag.successfulKill = false;
        ag.landedShotOn = -1;
        ag.wasKilled = false;
        ag.wasShotCount = 0;
        ag.firedShotT = -kFltMax;
    }
    o.reward[g] = r;
}

// sim.cpp:4202-4278 flankRewardSystem (Task.Zone with train_flank): small
// bonuses for teammates out of sight or >= 100 units away and for each
// opponent that cannot see the agent (judged with the agent's own aim),
// hits / kills from behind the target (|yaw difference| > pi), exploration.
// CombatState is taken by value there, so nothing is cleared.
void flankRewardSystem(Oracle &o, int w, int i)
{
    Agent &ag = o.agent(w, i);
    size_t g = o.gi(w, i);
    const float explore = o.rewardCoefs[9 * g + 2];
    float r = 0.f;
    Vec3 vis = ag.pos;
    vis.z += viewHeight(ag.curPose);
    const float flank_dist = 100.f;
    float mates = 0.f;
    for (int k = 0; k < o.teamSize - 1; k++) {
        const int j = ag.team * o.teamSize + (k < ag.offset ? k : k + 1);
        Vec3 dir = o.agent(w, j).pos - ag.pos;
        const bool seen = isAgentVisible(o, w, vis, ag.aimRot, j);
        if (length2(dir) >= flank_dist * flank_dist || !seen) mates += 0.001f;
    }
    r += mates;
    float opps = 0.f;
    for (int k = 0; k < o.teamSize; k++) {
        const Agent &op = o.agent(w, (ag.team ^ 1) * o.teamSize + k);
        Vec3 op_pos = op.pos;
        op_pos.z += viewHeight(op.curPose);
        if (!isAgentVisible(o, w, op_pos, ag.aimRot, i)) opps += 0.001f;
    }
    r += opps;
    if (ag.landedShotOn != -1) {
        const float yaw_diff = fabs_(o.agent(w, ag.landedShotOn).aimYaw - ag.aimYaw);
        if (yaw_diff > kPi) r += ag.successfulKill ? 1.f : 0.2f;
    }
    uint32_t nn = ag.numNewCellsVisited;
    ag.numNewCellsVisited = 0;
    if (nn > 0) r += float(nn) * explore;
    o.reward[g] = r;
}

// sim.cpp:3849-3996 zoneRewardSystem
void zoneRewardSystem(Oracle &o, int w, int i)
{
    World &wd = o.worlds[w];
    Agent &ag = o.agent(w, i);
    size_t g = o.gi(w, i);
    float r = 0.f;
    if (o.worldCurriculum[w] == 0) { // LearnShooting
        learnShootingReward(ag, r);
        o.reward[g] = r;
        return;
    }
    const float *rc = &o.rewardCoefs[9 * g];
    const float shot = rc[1], explore = rc[2], in_zone = rc[3], ctrl = rc[5], zdist = rc[6],
                earned = rc[7], crumb = rc[8];
    r -= crumb * ag.totalPenalty;
    if (ag.reloadedFullMag) r -= 0.5f;
    if (ag.successfulKill) r += 1.f;
    if (ag.landedShotOn != -1) r += shot * 1.f;
    if (ag.wasKilled) r -= 1.5f;
    if (ag.wasShotCount > 0) r -= shot * 1.f;
    uint32_t nn = ag.numNewCellsVisited;
    ag.numNewCellsVisited = 0;
    if (nn > 0) r += float(nn) * explore;
    if (ag.inZone) {
        r += in_zone;
    } else {
        AABB za = o.zoneAABBs[wd.curZone];
        Vec3 center = (za.pMax + za.pMin) / 2.f;
        float dist = distance(center, ag.pos);
        if (dist < ag.minDistToZone) {
            float scale = zdist;
            if (!ag.hasDiedDuringEpisode) scale *= 10.f;
            r += scale * (ag.minDistToZone - dist);
            ag.minDistToZone = dist;
        }
    }
    if (wd.curControllingTeam != -1) {
        if (wd.curControllingTeam == ag.team) {
            r += ctrl;
            if (wd.earnedPoint) r += earned;
        } else {
            r -= ctrl;
            if (wd.earnedPoint) r -= earned;
        }
    }
    if (o.alive[g] == 0.f) {
        ag.successfulKill = false;
        ag.landedShotOn = -1;
        ag.wasKilled = false;
        ag.wasShotCount = 0;
        ag.firedShotT = -kFltMax;
        o.reward[g] = r;
        return;
    }
    {
        float poly = 0.f;
        const int num_teammates = o.teamSize - 1;
        for (int k = 0; k < num_teammates - 1; k++) {
            int t1 = ag.team * o.teamSize + (k < ag.offset ? k : k + 1);
            int t2 = ag.team * o.teamSize + (k + 1 < ag.offset ? k + 1 : k + 2);
            Vec3 p1 = o.agent(w, t1).pos, p2 = o.agent(w, t2).pos;
            float e1x = p1.x - ag.pos.x, e1y = p1.y - ag.pos.y;
            float e2x = p2.x - ag.pos.x, e2y = p2.y - ag.pos.y;
            float tri = e1x * e2y - e1y * e2x;
            poly += fabs_(tri);
        }
        float dx = o.worldBounds.pMax.x - o.worldBounds.pMin.x;
        float dy = o.worldBounds.pMax.y - o.worldBounds.pMin.y;
        float area = dx * dy;
        float frac = poly / (2.f * area);
        r += frac * 1e-2f;
    }
    o.reward[g] = r;
}

// sim.cpp:4292-4313 pvpTeamRewardSystem + 4315-4339 pvpFinalRewardSystem
void teamAndFinalReward(Oracle &o, int w)
{
    World &wd = o.worlds[w];
    float tr[2] = { 0, 0 };
    int ts[2] = { 0, 0 };
    for (int i = 0; i < o.N; i++) {
        int t = o.agent(w, i).team;
        tr[t] += o.reward[o.gi(w, i)];
        ts[t] += 1;
    }
    tr[0] /= float(ts[0]);
    tr[1] /= float(ts[1]);
    wd.teamRewards[0] = tr[0];
    wd.teamRewards[1] = tr[1];
    for (int i = 0; i < o.N; i++) {
        size_t g = o.gi(w, i);
        float my = o.reward[g];
        float team_r = wd.teamRewards[o.agent(w, i).team];
        float spirit = o.rewardCoefs[9 * g + 0];
        o.reward[g] = my * (1.f - spirit) + team_r * spirit;
    }
}

// sim.cpp:2526-2560 opponentsWriteVisibilitySystem
void opponentsWriteVisibility(Oracle &o, int w, int i)
{
    Agent &ag = o.agent(w, i);
    size_t g = o.gi(w, i);
    Vec3 ray_o = ag.pos;
    ray_o.z += viewHeight(ag.curPose);
    int opp_team = ag.team ^ 1;
    for (int k = 0; k < kMaxTeamSize; k++) {
        ag.canSee[k] = false;
        if (o.alive[g] == 0.f) continue;
        if (k >= o.teamSize) continue;
        int opp = opp_team * o.teamSize + k;
        if (o.alive[o.gi(w, opp)] == 0.f) continue;
        if (isAgentVisible(o, w, ray_o, ag.aimRot, opp)) ag.canSee[k] = true;
    }
}

// sim.cpp:2562-2614 pvpOpponentMasksSystem
void opponentMasks(Oracle &o, int w, int i)
{
    Agent &ag = o.agent(w, i);
    size_t g = o.gi(w, i);
    int opp_team = ag.team ^ 1;
    for (int k = 0; k < kMaxTeamSize; k++) {
        float &m = o.masks[g * kMaxTeamSize + k];
        m = 0.f;
        if (o.alive[g] == 0.f) continue;
        if (k >= o.teamSize) continue;
        int opp = opp_team * o.teamSize + k;
        if (o.alive[o.gi(w, opp)] == 0.f) continue;
        bool can_see = ag.canSee[k];
        for (int t = 0; t < kMaxTeamSize - 1; t++) {
            if (t >= o.teamSize - 1) continue;
            int tm = ag.team * o.teamSize + (t < ag.offset ? t : t + 1);
            if (o.agent(w, tm).canSee[k]) {
                can_see = true;
                break;
            }
        }
        if (can_see) m = 1.f;
        if (o.agent(w, opp).firedShotT >= 0) m = 1.f;
    }
}

Vec3 normalizedPos(const Oracle &o, Vec3 p) // sim.cpp:2693-2718
{
    float min_x = o.worldBounds.pMin.x, min_y = o.worldBounds.pMin.y, min_z = o.worldBounds.pMin.z;
    float max_x = o.worldBounds.pMax.x, max_y = o.worldBounds.pMax.y, max_z = o.worldBounds.pMax.z;
    float xr = max_x - min_x, yr = max_y - min_y, zr = max_z - min_z;
    float x = (p.x - min_x) / xr, y = (p.y - min_y) / yr, z = (p.z - min_z) / zr;
    return v3(clampf(x, 0.f, 1.f), clampf(y, 0.f, 1.f), clampf(z, 0.f, 1.f));
}

// sim.cpp:2645-3052 pvpObservationsSystem
void pvpObservations(Oracle &o, int w, int i)
{
    World &wd = o.worlds[w];
    Agent &self = o.agent(w, i);
    size_t g = o.gi(w, i);

    o.filtersObs[g] = (wd.curStep - wd.filtersLastMatchedStep[self.team] < 5) ? 1.f : 0.f;

    float *self_ob = &o.selfObs[g * kSelfObs];
    float *self_pos = &o.selfPos[g * 3];
    std::fill(self_ob, self_ob + kSelfObs, 0.f);
    self_pos[0] = self_pos[1] = self_pos[2] = -1000.f;
    for (int k = 0; k < kMaxTeamSize - 1; k++) {
        float *p = &o.teammatePos[(g * 5 + k) * 3];
        p[0] = p[1] = p[2] = -1000.f;
        float *ob = &o.teammateObs[(g * 5 + k) * kOtherObs];
        std::fill(ob, ob + kOtherObs, 0.f);
    }
    for (int k = 0; k < kMaxTeamSize; k++) {
        float *p = &o.opponentPos[(g * 6 + k) * 3];
        p[0] = p[1] = p[2] = -1000.f;
        float *ob = &o.opponentObs[(g * 6 + k) * kOtherObs];
        std::fill(ob, ob + kOtherObs, 0.f);
    }

    const Vec3 self_pos_v = self.pos;
    const Quat self_rot = self.rot;
    const float self_yaw = self.aimYaw, self_pitch = self.aimPitch;

    auto fillCommon = [&](float *ob, float *pos_ob, int j) {
        ob[0] = 1.f; // isValid
        size_t gj = o.gi(w, j);
        if (!o.alive[gj]) return false;
        const Agent &a = o.agent(w, j);
        ob[1] = 1.f;
        Vec3 np = normalizedPos(o, a.pos);
        ob[2] = np.x; ob[3] = np.y; ob[4] = np.z;
        pos_ob[0] = np.x; pos_ob[1] = np.y; pos_ob[2] = np.z;
        ob[5] = 0.5f * ((a.aimYaw / kPi) + 1.f);
        ob[6] = 0.5f * (a.aimPitch / (0.25f * kPi) + 1.f);
        Vec3 rv = rotateVec(qinv(self_rot), a.vel);
        ob[7] = rv.x; ob[8] = rv.y; ob[9] = rv.z;
        ob[10] = a.daimYawVel; ob[11] = a.daimPitchVel;
        ob[12] = a.curPose == kStand ? 1.f : 0.f;
        ob[13] = a.curPose == kCrouch ? 1.f : 0.f;
        ob[14] = a.curPose == kProne ? 1.f : 0.f;
        ob[15] = a.tgtPose == kStand ? 1.f : 0.f;
        ob[16] = a.tgtPose == kCrouch ? 1.f : 0.f;
        ob[17] = a.tgtPose == kProne ? 1.f : 0.f;
        ob[18] = (float)a.transitionRemaining / (float)kPoseTransitionSpeed;
        ob[19] = a.inZone ? 1.f : 0.f;
        ob[20 + a.weaponType] = 1.f;
        return true;
    };
    auto fillCombat = [&](float *ob, int j) {
        size_t gj = o.gi(w, j);
        const Agent &a = o.agent(w, j);
        ob[0] = (float)o.hp[gj] / 100.f;
        ob[1] = (float)o.magazine[2 * gj];
        ob[2] = (float)o.magazine[2 * gj + 1];
        ob[3] = float(a.remainingStepsBeforeAutoheal) / float(kOutOfCombatSteps);
    };
    auto relAngles = [&](Vec3 to, float *dist_out, float *yaw_out, float *pitch_out, float eps) {
        float d = length(to);
        if (d < eps) {
            *dist_out = 0.f; *yaw_out = 0.f; *pitch_out = 0.f;
            return;
        }
        to = to / d;
        float new_yaw = -atan2f_(to.x, to.y);
        float new_pitch = asinf_(clampf(to.z, -1.f, 1.f));
        float yaw_delta = new_yaw - self_yaw;
        float pitch_delta = new_pitch - self_pitch;
        if (yaw_delta > kPi) yaw_delta -= 2.f * kPi;
        else if (yaw_delta < -kPi) yaw_delta += 2.f * kPi;
        *dist_out = d; *yaw_out = yaw_delta; *pitch_out = pitch_delta;
    };
    auto fillOther = [&](float *ob, int j) {
        const Agent &a = o.agent(w, j);
        relAngles(a.pos - self_pos_v, &ob[23], &ob[24], &ob[25], 1e-2f);
        float rfy = a.aimYaw - self_yaw;
        float rfp = a.aimPitch - self_pitch;
        if (rfy > kPi) rfy -= 2.f * kPi;
        else if (rfy < -kPi) rfy += 2.f * kPi;
        ob[26] = rfy;
        ob[27] = rfp;
    };

    if (!fillCommon(self_ob, self_pos, i)) return;
    fillCombat(&self_ob[23], i);
    {
        float *zo = &self_ob[27];
        AABB za = o.zoneAABBs[wd.curZone];
        Vec3 center = (za.pMax + za.pMin) / 2.f;
        Vec3 nc = normalizedPos(o, center);
        zo[0] = nc.x; zo[1] = nc.y; zo[2] = nc.z;
        relAngles(center - self_pos_v, &zo[3], &zo[4], &zo[5], 1e-2f);
        zo[6] = (wd.curControllingTeam == self.team) ? 1.f : 0.f;
        zo[7] = (wd.curControllingTeam != -1 && wd.curControllingTeam != self.team) ? 1.f : 0.f;
        zo[8] = wd.isContested ? 1.f : 0.f;
        zo[9] = wd.isCaptured ? 1.f : 0.f;
        zo[10] = float(wd.stepsUntilPoint) / float(kZonePointInterval);
        zo[11] = float(wd.zoneStepsRemaining) / float(kNumStepsPerZone);
        if (wd.curZone >= 0 && wd.curZone < 4) zo[12 + wd.curZone] = 1.f;
    }

    for (int k = 0; k < o.teamSize - 1; k++) {
        int j = self.team * o.teamSize + (k < self.offset ? k : k + 1);
        float *ob = &o.teammateObs[(g * 5 + k) * kOtherObs];
        float *pos_ob = &o.teammatePos[(g * 5 + k) * 3];
        if (!fillCommon(ob, pos_ob, j)) continue;
        fillOther(ob, j);
        fillCombat(&ob[28], j);
    }

    for (int k = 0; k < o.teamSize; k++) {
        int j = (self.team ^ 1) * o.teamSize + k;
        float *ob = &o.opponentObs[(g * 6 + k) * kOtherObs];
        float *lk = &o.lastKnownObs[(g * 6 + k) * kOtherObs];
        float *pos_ob = &o.opponentPos[(g * 6 + k) * 3];
        float *lk_pos = &o.lastKnownPos[(g * 6 + k) * 3];
        if (!fillCommon(ob, pos_ob, j)) {
            std::fill(lk, lk + kOtherObs, 0.f);
            lk_pos[0] = lk_pos[1] = lk_pos[2] = -1000.f;
            continue;
        }
        fillOther(ob, j);
        const Agent &a = o.agent(w, j);
        if (a.wasKilled) {
            std::fill(lk, lk + kOtherObs, 0.f);
            lk_pos[0] = lk_pos[1] = lk_pos[2] = -1000.f;
        }
        ob[28] = (float)a.wasShotCount;
        ob[29] = a.firedShotT >= 0.f ? 1.f : 0.f;
        ob[30] = self.canSee[k] ? 1.f : 0.f;
        bool knows = o.masks[g * 6 + k] == 1.f;
        ob[31] = knows ? 1.f : 0.f;
        if (knows) {
            std::copy(ob, ob + kOtherObs, lk);
            lk_pos[0] = pos_ob[0]; lk_pos[1] = pos_ob[1]; lk_pos[2] = pos_ob[2];
        }
    }
}

// sim.cpp:3324-3506 pvpLidarSystem
void pvpLidar(Oracle &o, int w, int i)
{
    Agent &ag = o.agent(w, i);
    size_t g = o.gi(w, i);
    Vec3 fwd_fwd = rotateVec(ag.aimRot, kFwd);
    Vec3 fwd_right = rotateVec(ag.aimRot, kRight);
    Vec3 rear_fwd = rotateVec(ag.rot, kFwd);
    Vec3 rear_right = rotateVec(ag.rot, kRight);
    auto trace = [&](int idx, int num, Vec3 ray_o, Vec3 fwd, Vec3 right, float range, float offset,
                     float *out) {
        float theta = range * (float(idx) / float(num - 1)) + offset;
        float x = -cosf_(theta);
        float y = sinf_(theta);
        Vec3 dir = normalize(x * right + y * fwd);
        HitResult h = traceRayAgainstWorld(o, w, ray_o, dir, o.lidarOrder);
        if (h.hit) {
            bool wall = h.entity == -1;
            bool tm = !wall && o.agent(w, h.entity).team == ag.team;
            out[0] = fminD(h.t, o.maxDist);
            out[1] = wall ? 1.f : 0.f;
            out[2] = tm ? 1.f : 0.f;
            out[3] = (!wall && !tm) ? 1.f : 0.f;
        } else {
            out[0] = -1.f; out[1] = 0.f; out[2] = 0.f; out[3] = 0.f;
        }
    };
    float top = viewHeight(ag.curPose) + kAgentRadius;
    for (int h = 0; h < kFwdH; h++) {
        Vec3 ray_o = ag.pos;
        ray_o.z += kAgentRadius + (top - 2.f * kAgentRadius) * (float(h) / float(kFwdH - 1));
        for (int x = 0; x < kFwdW; x++) {
            trace(x, kFwdW, ray_o, fwd_fwd, fwd_right, 0.75f * kPi, 0.5f * (1.f - 0.75f) * kPi,
                  &o.fwdLidar[((g * kFwdH + h) * kFwdW + x) * kLidarData]);
        }
    }
    for (int h = 0; h < kRearH; h++) {
        Vec3 ray_o = ag.pos;
        ray_o.z += kAgentRadius + (top - 2.f * kAgentRadius) * (float(h) / float(kRearH - 1));
        for (int x = 0; x < kRearW; x++) {
            trace(x, kRearW, ray_o, rear_fwd, rear_right, -kPi, 0.f,
                  &o.rearLidar[((g * kRearH + h) * kRearW + x) * kLidarData]);
        }
    }
}

// sim.cpp:3054-3301 fullTeamObservationsSystem, for both team interfaces of
// world w.  Unlike pvpObservations, positions are normalised without a clamp
// and velocities are global; last-known enemies are cleared every step and
// hold the common part of the enemy observation only while the team knows
// the location.  The lidar copy is the agents' lidar as it stands before
// this step's pvpLidarSystem (that system is added to the graph after this
// one, sim.cpp:5294-5310).
void fullTeamObservations(Oracle &o, int w)
{
    World &wd = o.worlds[w];
    const int T = o.teamSize;
    auto norm = [&](Vec3 p) {
        float min_x = o.worldBounds.pMin.x, min_y = o.worldBounds.pMin.y, min_z = o.worldBounds.pMin.z;
        float max_x = o.worldBounds.pMax.x, max_y = o.worldBounds.pMax.y, max_z = o.worldBounds.pMax.z;
        float xr = max_x - min_x, yr = max_y - min_y, zr = max_z - min_z;
        return v3((p.x - min_x) / xr, (p.y - min_y) / yr, (p.z - min_z) / zr);
    };
    for (int team = 0; team < 2; team++) {
        const size_t ti = (size_t)w * 2 + team;
        float *players = &o.ftPlayers[ti * 6 * MPENV_FT_PLAYER_DIM];
        float *enemies = &o.ftEnemies[ti * 6 * MPENV_FT_ENEMY_DIM];
        float *last = &o.ftLastKnown[ti * 6 * MPENV_FT_COMMON_DIM];
        std::fill(players, players + 6 * MPENV_FT_PLAYER_DIM, 0.f);
        std::fill(enemies, enemies + 6 * MPENV_FT_ENEMY_DIM, 0.f);
        std::fill(last, last + 6 * MPENV_FT_COMMON_DIM, 0.f);

        float *gob = &o.ftGlobal[ti * MPENV_FT_GLOBAL_DIM];
        gob[0] = team == 0 ? 0.f : 1.f;
        gob[1] = team == 0 ? 1.f : 0.f;
        gob[2] = float(kEpisodeLen - wd.curStep) / kEpisodeLen;
        {
            const AABB za = o.zoneAABBs[wd.curZone];
            Vec3 nc = norm((za.pMax + za.pMin) / 2.f);
            float *z = &gob[3];
            z[0] = nc.x; z[1] = nc.y; z[2] = nc.z;
            z[3] = (wd.curControllingTeam == team) ? 1.f : 0.f;
            z[4] = (wd.curControllingTeam != -1 && wd.curControllingTeam != team) ? 1.f : 0.f;
            z[5] = wd.isContested ? 1.f : 0.f;
            z[6] = wd.isCaptured ? 1.f : 0.f;
            z[7] = float(wd.stepsUntilPoint) / float(kZonePointInterval);
            z[8] = float(wd.zoneStepsRemaining) / float(kNumStepsPerZone);
            for (int k = 0; k < 4; k++) z[9 + k] = wd.curZone == k ? 1.f : 0.f;
        }
        auto fillCommon = [&](float *ob, int j, int slot) {
            ob[0] = 1.f;
            ob[1 + slot] = 1.f;
            const size_t gj = o.gi(w, j);
            if (!o.alive[gj]) return false;
            const Agent &a = o.agent(w, j);
            ob[7] = 1.f;
            Vec3 np = norm(a.pos);
            ob[8] = np.x; ob[9] = np.y; ob[10] = np.z;
            ob[11] = 0.5f * ((a.aimYaw / kPi) + 1.f);
            ob[12] = 0.5f * (a.aimPitch / (0.25f * kPi) + 1.f);
            ob[13] = a.vel.x; ob[14] = a.vel.y; ob[15] = a.vel.z;
            ob[16] = a.curPose == kStand ? 1.f : 0.f;
            ob[17] = a.curPose == kCrouch ? 1.f : 0.f;
            ob[18] = a.curPose == kProne ? 1.f : 0.f;
            ob[19] = a.tgtPose == kStand ? 1.f : 0.f;
            ob[20] = a.tgtPose == kCrouch ? 1.f : 0.f;
            ob[21] = a.tgtPose == kProne ? 1.f : 0.f;
            ob[22] = (float)a.transitionRemaining / (float)kPoseTransitionSpeed;
            ob[23] = a.inZone ? 1.f : 0.f;
            return true;
        };
        for (int s = 0; s < T; s++) {
            const int j = team * T + s;
            float *ob = &players[s * MPENV_FT_PLAYER_DIM];
            if (!fillCommon(ob, j, s)) continue;
            const size_t gj = o.gi(w, j);
            ob[24] = (float)o.hp[gj] / 100.f;
            ob[25] = (float)o.magazine[2 * gj] / 30;
            ob[26] = (float)o.magazine[2 * gj + 1];
            ob[27] = float(o.agent(w, j).remainingStepsBeforeAutoheal) / float(kOutOfCombatSteps);
        }
        for (int s = 0; s < T; s++) {
            const int j = (team ^ 1) * T + s;
            float *ob = &enemies[s * MPENV_FT_ENEMY_DIM];
            float *lk = &last[s * MPENV_FT_COMMON_DIM];
            if (!fillCommon(ob, j, s)) {
                std::fill(lk, lk + MPENV_FT_COMMON_DIM, 0.f);
                continue;
            }
            const Agent &a = o.agent(w, j);
            if (a.wasKilled) std::fill(lk, lk + MPENV_FT_COMMON_DIM, 0.f);
            ob[24] = (float)a.wasShotCount;
            ob[25] = a.firedShotT >= 0.f ? 1.f : 0.f;
            bool knows = ob[25] != 0.f;
            for (int m = 0; m < T; m++) {
                if (o.agent(w, team * T + m).canSee[s]) {
                    ob[26 + m] = 1.f;
                    knows = true;
                }
            }
            ob[32] = knows ? 1.f : 0.f;
            if (knows) std::copy(ob, ob + MPENV_FT_COMMON_DIM, lk);
        }
        for (int s = 0; s < T; s++) {
            const size_t g = o.gi(w, team * T + s);
            const int fl = kFwdH * kFwdW * 4, rl = kRearH * kRearW * 4;
            std::copy(&o.fwdLidar[g * fl], &o.fwdLidar[(g + 1) * fl], &o.ftFwdLidar[(ti * 6 + s) * fl]);
            std::copy(&o.rearLidar[g * rl], &o.rearLidar[(g + 1) * rl], &o.ftRearLidar[(ti * 6 + s) * rl]);
        }
    }
}

// sim.cpp:4720-4747 fullTeamDoneRewardSystem
void fullTeamDoneReward(Oracle &o, int w)
{
    for (int team = 0; team < 2; team++) {
        float r = 0.f;
        bool done = true;
        for (int i = 0; i < o.N; i++) {
            if (o.agent(w, i).team != team) continue;
            const size_t g = o.gi(w, i);
            r += o.reward[g];
            if (!o.done[g]) done = false;
        }
        o.ftReward[(size_t)w * 2 + team] = r;
        o.ftDone[(size_t)w * 2 + team] = done ? 1 : 0;
    }
}

// sim.cpp:5174-5320 resetAndObsTasks (per world)
void resetAndObs(Oracle &o, int w)
{
    resetSystem(o, w);
    for (int i = 0; i < o.N; i++) opponentsWriteVisibility(o, w, i);
    for (int i = 0; i < o.N; i++) opponentMasks(o, w, i);
    for (int i = 0; i < o.N; i++) pvpObservations(o, w, i);
    fullTeamObservations(o, w);
    for (int i = 0; i < o.N; i++) pvpLidar(o, w, i);
}

// sim.cpp:5342-5842 setupStepTasks, Task::Zone, default flags
void replayTail(Oracle &o, int w);

void stepWorld(Oracle &o, int w)
{
    const int N = o.N;
    if (o.eventsOn) // ClearTmpNode<GameEventEntity> (sim.cpp:5344)
        for (int k = 0; k < 2 * N + 1; k++) o.events[(size_t)w * (2 * N + 1) + k].type = 0;
    for (int i = 0; i < N; i++) planAStarAISystem(o, w, i);
    if (o.replayOn) {
        // pvpReplayLogic (sim.cpp:5587-5605): replay + zoneSystem only
        pvpReplaySystem(o, w);
        zoneSystem(o, w);
        replayTail(o, w);
        return;
    }
    for (int i = 0; i < N; i++) applyBotActionsSystem(o, w, i);
    for (int i = 0; i < N; i++) pvpMovementSystem(o, w, i);
    for (int i = 0; i < N; i++) pvpContinuousAimSystem(o, w, i);
    for (int i = 0; i < N; i++) pvpDiscreteAimSystem(o, w, i);
    for (int i = 0; i < N; i++) applyVelocitySystem(o, w, i);
    for (int i = 0; i < N; i++) {
        Agent &ag = o.agent(w, i);
        ag.pos = ag.newPos;
        ag.vel = ag.newVel;
    }
    for (int i = 0; i < N; i++) fallSystem(o, w, i);
    for (int i = 0; i < N; i++) o.agent(w, i).pos = o.agent(w, i).newPos;
    for (int i = 0; i < N; i++) fireSystem(o, w, i);
    for (int i = 0; i < N; i++) applyDmgSystem(o, w, i);
    if (!(o.simFlags & MPENV_SIMFLAG_NO_RESPAWN)) spawnAgents(o, w, true);
    for (int i = 0; i < N; i++) autoHealSystem(o, w, i);
    zoneSystem(o, w);
    if (o.simFlags & MPENV_SIMFLAG_SUB_ZONES) subzoneSystem(o, w);
    if (o.recordOn) pvpRecordSystem(o, w);
    for (int i = 0; i < N; i++) leaveBreadcrumbsSystem(o, w, i);
    accumulateBreadcrumbPenalties(o, w);
    replayTail(o, w);
}

// Systems after the gameplay / replay logic (sim.cpp:5664-5750 onward)
void replayTail(Oracle &o, int w)
{
    const int N = o.N;
    zoneMatchInfoSystem(o, w);
    evaluateGoalRegionsSystem(o, w);
    for (int i = 0; i < N; i++) exploreVisitedSystem(o, w, i);
    for (int i = 0; i < N; i++) {
        if (o.task == MPENV_TASK_ZONE_CAPTURE_DEFEND) zoneCaptureDefendRewardSystem(o, w, i);
        else if (o.flank) flankRewardSystem(o, w, i);
        else if (o.simFlags & MPENV_SIMFLAG_SUB_ZONES) subzoneRewardSystem(o, w, i);
        else zoneRewardSystem(o, w, i);
    }
    teamAndFinalReward(o, w);
    for (int i = 0; i < N; i++) o.done[o.gi(w, i)] = o.worlds[w].isFinished ? 1 : 0;
    fullTeamDoneReward(o, w);
    resetAndObs(o, w);
}

// sim.cpp:5850-5980 Sim::Sim
void constructWorld(Oracle &o, int w)
{
    World &wd = o.worlds[w];
    wd.curEpisodeIdx = 0;
    wd.worldEpisodeCounter = 0;
    wd.curCurriculumTier = 0;
    wd.curCurriculumSpawnIdx = 0;
    wd.nextCrumbId = 0;
    wd.crumbOverflow = 0;
    wd.crumbs.clear();
    o.resetBuf[w] = 0;
    for (int t = 0; t < 2; t++)
        for (int k = 0; k < 64; k++) wd.filtersLastMatches[t][k] = 0;
    createPersistentEntities(o, w);
    o.worldCurriculum[w] = 1; // FullMatch (sim.cpp:5959)
    initWorld(o, w, true);
    for (int z = 0; z < kMaxZones; z++)
        for (int k = 0; k < 5; k++) wd.zoneStats[z][k] = 0;
    wd.matchID = ~0ull;
    wd.eventLoggedInStep = 0;
    wd.eventMask = 0;
    for (int t = 0; t < 2; t++) {
        wd.filtersActive[t] = 0;
        wd.filtersLastMatchedStep[t] = -1;
    }
}

template <typename T>
void readVec(std::ifstream &f, std::vector<T> &v, size_t n)
{
    v.resize(n);
    if (n) f.read(reinterpret_cast<char *>(v.data()), (std::streamsize)(n * sizeof(T)));
    if (!f) throw std::runtime_error("oracle: truncated scene file");
}

// SpawnInMiddle extra spawn cells, mgr.cpp:1240-1299: a 20x20 grid over
// x in [-280, 280], y in [-200, 200], each cell z in [1.0, 1.5]; a cell is
// kept when no collision triangle overlaps it (left half -> team A, right
// half -> team B, row-major order).  The reference asks MeshBVH::findOverlaps
// (mesh_bvh.inl:50-108), which tests the cell against *quantized leaf boxes*
// of its Embree-built tree — builder-dependent, and on simple_map likely to
// reject every cell (the floor leaf box is padded by >= one quantum) and then
// index past the spawn array.  The build defines the overlap test on the
// triangles' own AABBs instead ("documented definitions").
void addMiddleSpawnCells(Oracle &o)
{
    const Vec3 lo = v3(-280.f, -200.f, 0.5f), hi = v3(280.f, 200.f, 0.5f);
    const int dim = 20;
    const float cw = (hi.x - lo.x) / dim, chh = (hi.y - lo.y) / dim;
    for (int y = 0; y < dim; y++) {
        for (int x = 0; x < dim; x++) {
            Vec3 cmin = lo + v3(cw * x, chh * y, 0.5f);
            Vec3 cmax = cmin + v3(cw, chh, 0.5f);
            bool hit = false;
            for (size_t t = 0; t + 2 < o.verts.size() && !hit; t += 3) {
                const Vec3 &a = o.verts[t], &b = o.verts[t + 1], &c = o.verts[t + 2];
                Vec3 tmin = v3(std::min(a.x, std::min(b.x, c.x)), std::min(a.y, std::min(b.y, c.y)),
                               std::min(a.z, std::min(b.z, c.z)));
                Vec3 tmax = v3(std::max(a.x, std::max(b.x, c.x)), std::max(a.y, std::max(b.y, c.y)),
                               std::max(a.z, std::max(b.z, c.z)));
                hit = tmin.x <= cmax.x && tmax.x >= cmin.x && tmin.y <= cmax.y && tmax.y >= cmin.y &&
                      tmin.z <= cmax.z && tmax.z >= cmin.z;
            }
            if (hit) continue;
            Spawn sp;
            sp.region.pMin = cmin;
            sp.region.pMax = cmax;
            sp.yawMin = 0.f;
            sp.yawMax = 2.f * kPi;
            (x >= dim / 2 ? o.bSpawns : o.aSpawns).push_back(sp);
        }
    }
}

// ------------------------------------------------------- lidar child order
// The documented lidar child order ("child visit order"): for
// a ray whose direction sign bits are octant `oct` (bit 0 x, bit 1 y, bit 2
// z; -0 counts as negative, scene.h octantNodeImages), a node's leaf children first, by ascending key, then its
// internal children by descending key, then empty slots; key = the child
// box centre projected on the octant diagonal, sum over axes a of
// s_a * (min_a + 2^exp_a * (qMin_a + qMax_a) / 2), in double; ties keep slot
// order.  With the LIFO stack this tests leaves near-to-far and pops the
// nearest internal child first.  The reference visits slots in order
// (mesh_bvh.inl:160-204) on an Embree tree whose slot order is unpinned;
// closest hits agree with slot order up to exact ties between distinct
// coplanar triangles (tools/lidar_order_check.py).
std::vector<int8_t> octantOrder(const std::vector<Node> &nodes)
{
    const size_t n = nodes.size();
    std::vector<int8_t> ord(8 * n * 4);
    for (int oct = 0; oct < 8; oct++) {
        const double s[3] = { (oct & 1) ? -1.0 : 1.0, (oct & 2) ? -1.0 : 1.0, (oct & 4) ? -1.0 : 1.0 };
        for (size_t ni = 0; ni < n; ni++) {
            const Node &nd = nodes[ni];
            double key[4];
            for (int i = 0; i < 4; i++) {
                const double cx = (double)nd.minX + std::ldexp(0.5 * ((double)nd.qMinX[i] + (double)nd.qMaxX[i]), nd.expX);
                const double cy = (double)nd.minY + std::ldexp(0.5 * ((double)nd.qMinY[i] + (double)nd.qMaxY[i]), nd.expY);
                const double cz = (double)nd.minZ + std::ldexp(0.5 * ((double)nd.qMinZ[i] + (double)nd.qMaxZ[i]), nd.expZ);
                key[i] = 0.0;
                key[i] += s[0] * cx;
                key[i] += s[1] * cy;
                key[i] += s[2] * cz;
            }
            // class: 0 leaf, 1 internal, 2 empty; insertion sort (stable)
            int slots[4] = { 0, 1, 2, 3 };
            auto cls = [&](int i) { return nd.children[i] == -1 ? 2 : (nd.children[i] & 0x80000000) ? 0 : 1; };
            auto before = [&](int a, int b) {
                if (cls(a) != cls(b)) return cls(a) < cls(b);
                if (cls(a) == 0) return key[a] < key[b];
                if (cls(a) == 1) return key[a] > key[b];
                return false;
            };
            for (int k = 1; k < 4; k++)
                for (int j = k; j > 0 && before(slots[j], slots[j - 1]); j--) std::swap(slots[j], slots[j - 1]);
            for (int k = 0; k < 4; k++) ord[((size_t)oct * n + ni) * 4 + k] = (int8_t)slots[k];
        }
    }
    return ord;
}

// ------------------------------------------------------------ navmesh
// The oracle builds the bots' navmesh and A* next-hop table itself from
// navmesh.bin, independently of the product's csrc/navmesh.cpp, so a
// misreading of buildAStarLookup on either side shows up as a table
// mismatch (tests/test_navmesh.py compares the two byte for byte).
struct NavBuild {
    std::vector<Vec3> verts;     // deduplicated
    std::vector<uint32_t> tri;   // 3 per triangle
    std::vector<int32_t> adj;    // 3 per triangle
};

// map_importer.cpp:421-506 importNavmesh (the world-bounds filter is
// `#if 0`'d, so every face is kept), then mgr.cpp:1301-1318: vertices with
// bit-identical positions share the index of their first occurrence
// (meshopt_generateVertexRemap), then Navmesh::initFromPolygons (Madrona,
// not vendored; defined as in DESIGN.md §2 #8: polygon (v0..vn-1) fans into
// (v0, vk, vk+1); the neighbour across edge k of triangle t is the lowest
// numbered other triangle holding the same undirected edge, else -1).
NavBuild navFromFile(const std::string &path)
{
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("oracle: cannot open navmesh.bin");
    auto u32 = [&f]() {
        uint32_t v = 0;
        if (!f.read(reinterpret_cast<char *>(&v), 4)) throw std::runtime_error("oracle: navmesh.bin truncated");
        return v;
    };
    const uint32_t nv = u32();
    std::vector<float> raw((size_t)nv * 3);
    if (!f.read(reinterpret_cast<char *>(raw.data()), raw.size() * 4))
        throw std::runtime_error("oracle: navmesh.bin truncated");
    const uint32_t nf = u32();
    std::vector<uint32_t> counts(nf);
    for (auto &c : counts) c = u32();
    const uint32_t ni = u32();
    std::vector<uint32_t> idx(ni);
    for (auto &i : idx) i = u32();

    NavBuild nb;
    std::vector<uint32_t> remap(nv);
    for (uint32_t i = 0; i < nv; i++) {
        uint32_t found = UINT32_MAX;
        for (uint32_t j = 0; j < (uint32_t)nb.verts.size(); j++) {
            if (std::memcmp(&raw[3 * (size_t)i], &nb.verts[j], 12) == 0) {
                found = j;
                break;
            }
        }
        if (found == UINT32_MAX) {
            found = (uint32_t)nb.verts.size();
            nb.verts.push_back(v3(raw[3 * (size_t)i], raw[3 * (size_t)i + 1], raw[3 * (size_t)i + 2]));
        }
        remap[i] = found;
    }
    size_t start = 0;
    for (uint32_t fc : counts) {
        if (start + fc > idx.size()) throw std::runtime_error("oracle: navmesh.bin face out of range");
        for (uint32_t k = 2; k < fc; k++) {
            const uint32_t a = idx[start], b = idx[start + k - 1], c = idx[start + k];
            if (a >= nv || b >= nv || c >= nv) throw std::runtime_error("oracle: navmesh.bin index out of range");
            nb.tri.push_back(remap[a]);
            nb.tri.push_back(remap[b]);
            nb.tri.push_back(remap[c]);
        }
        start += fc;
    }
    const int T = (int)(nb.tri.size() / 3);
    nb.adj.assign((size_t)T * 3, -1);
    for (int t = 0; t < T; t++) {
        for (int e = 0; e < 3; e++) {
            const uint32_t p = nb.tri[3 * t + e], q = nb.tri[3 * t + (e + 1) % 3];
            for (int u = 0; u < T && nb.adj[3 * t + e] == -1; u++) {
                if (u == t) continue;
                for (int e2 = 0; e2 < 3; e2++) {
                    const uint32_t p2 = nb.tri[3 * u + e2], q2 = nb.tri[3 * u + (e2 + 1) % 3];
                    if ((p2 == p && q2 == q) || (p2 == q && q2 == p)) {
                        nb.adj[3 * t + e] = u;
                        break;
                    }
                }
            }
        }
    }
    return nb;
}

// mgr.cpp:948-1153 NavUtils, restated as text.
struct NavAStar {
    const NavBuild &nm;
    int numTris;
    // NavUtils::Node (mgr.cpp:953-967)
    struct NodeS {
        int idx, cameFrom;
        float startDist, score;
    };
    std::vector<NodeS> state;
    // EarlyOutData (mgr.cpp:1001-1053)
    int earlyOutForDir[9];
    float totalDistance = 0.f, reasonableDistance2 = 0.f;
    bool enabled = false;

    explicit NavAStar(const NavBuild &m) : nm(m), numTris((int)(m.tri.size() / 3)), state(numTris) {}

    // mgr.cpp:969-977: center += v / 3 per vertex, in order
    Vec3 centerOfTri(int t) const
    {
        Vec3 c = v3(0.f, 0.f, 0.f);
        for (int i = 0; i < 3; i++) c = c + nm.verts[nm.tri[t * 3 + i]] / 3.0f;
        return c;
    }

    // mgr.cpp:1008-1037
    void init()
    {
        const int reasonableNavTriCount = 400;
        if (numTris <= reasonableNavTriCount) {
            enabled = false;
            return;
        }
        enabled = true;
        Vec3 mins = v3(kFltMax, kFltMax, kFltMax), maxs = v3(-kFltMax, -kFltMax, -kFltMax);
        for (const Vec3 &v : nm.verts) {
            mins = v3(fminD(mins.x, v.x), fminD(mins.y, v.y), fminD(mins.z, v.z));
            maxs = v3(fmaxD(maxs.x, v.x), fmaxD(maxs.y, v.y), fmaxD(maxs.z, v.z));
        }
        const float d = length(maxs - mins);
        totalDistance = d;
        reasonableDistance2 = d * (float)reasonableNavTriCount / (float)numTris;
        reasonableDistance2 *= reasonableDistance2;
    }

    // mgr.cpp:1041-1051
    int getEarlyOutPath(Vec3 start, Vec3 target) const
    {
        if (!enabled) return -1;
        if (length2(start - target) < reasonableDistance2) return -1;
        Vec3 dir = normalize(target - start);
        int dx = (int)(dir.x * 1.9f), dy = (int)(dir.y * 1.9f);
        return earlyOutForDir[(dx + 1) + (dy + 1) * 3];
    }

    // mgr.cpp:1055-1114: the open set is a std::set ordered by each
    // triangle's *current* score (mutated while it sits in the set).
    int pathfindToTri(int startTri, int posTri)
    {
        const Vec3 start = centerOfTri(startTri), pos = centerOfTri(posTri);
        const int early = getEarlyOutPath(start, pos);
        if (early != -1) return early;
        for (int t = 0; t < numTris; t++) state[t] = NodeS { t, -1, kFltMax, kFltMax };
        state[startTri].startDist = 0.0f;
        auto sortHeap = [this](const int &l, const int &r) { return state[l].score < state[r].score; };
        std::set<int, decltype(sortHeap)> heap(sortHeap);
        heap.insert(startTri);
        while (!heap.empty()) {
            const int thisTri = *heap.begin();
            if (thisTri == posTri) {
                int goal = thisTri;
                while (goal != startTri && goal != -1) {
                    if (state[goal].cameFrom == startTri) return goal;
                    goal = state[goal].cameFrom;
                }
                return posTri;
            }
            heap.erase(heap.begin());
            const Vec3 center = thisTri == startTri ? start : centerOfTri(thisTri);
            for (int i = 0; i < 3; i++) {
                const int neighbor = nm.adj[thisTri * 3 + i];
                if (neighbor == -1) continue;
                const Vec3 neighpos = centerOfTri(neighbor);
                const float score = state[thisTri].startDist + length(center - neighpos);
                if (score < state[neighbor].startDist) {
                    state[neighbor].cameFrom = thisTri;
                    state[neighbor].startDist = score;
                    state[neighbor].score = score + length(neighpos - pos);
                    heap.insert(neighbor);
                }
            }
        }
        return -1;
    }

    // mgr.cpp:1116-1150
    void prepareForStartTri(int startTri)
    {
        if (!enabled) return;
        enabled = false;
        for (int dirX = -1; dirX <= 1; dirX++) {
            for (int dirY = -1; dirY <= 1; dirY++) {
                if (dirX == 0 && dirY == 0) continue;
                const Vec3 dir = normalize(v3((float)dirX, (float)dirY, 0.0f));
                const Vec3 start = centerOfTri(startTri);
                const Vec3 end = start + dir * totalDistance * 2.0f;
                float bestDist = kFltMax;
                int bestTri = -1;
                for (int t = 0; t < numTris; t++) {
                    const float d = length(centerOfTri(t) - end);
                    if (d < bestDist) {
                        bestDist = d;
                        bestTri = t;
                    }
                }
                earlyOutForDir[(dirX + 1) + (dirY + 1) * 3] = pathfindToTri(startTri, bestTri);
            }
        }
        enabled = true;
    }
};

// mgr.cpp:1155-1211 buildAStarLookup (the .astar disk cache is not read:
// the oracle always computes the table it checks the product against).
std::vector<int32_t> buildAStarLookup(const NavBuild &nm)
{
    NavAStar as(nm);
    as.init();
    const int T = as.numTris;
    std::vector<int32_t> tbl((size_t)T * T);
    for (int s = 0; s < T; s++) {
        as.prepareForStartTri(s);
        for (int g = 0; g < T; g++) tbl[(size_t)s * T + g] = as.pathfindToTri(s, g);
    }
    return tbl;
}

// map_importer.cpp:508-567 (spawns, zones) and 223-256 (world bounds)
void loadScene(Oracle &o)
{
    {
        std::ifstream f(o.scenePath + "/collisions.bin", std::ios::binary);
        if (!f) throw std::runtime_error("oracle: cannot open collisions.bin");
        float wb[6];
        f.read(reinterpret_cast<char *>(wb), sizeof(wb));
        o.worldBounds.pMin = v3(wb[0], wb[1], wb[2]);
        o.worldBounds.pMax = v3(wb[3], wb[4], wb[5]);
    }
    {
        std::ifstream f(o.scenePath + "/spawns.bin", std::ios::binary);
        if (!f) throw std::runtime_error("oracle: cannot open spawns.bin");
        std::vector<Spawn> *dst[3] = { &o.aSpawns, &o.bSpawns, &o.commonRespawns };
        for (int k = 0; k < 3; k++) {
            uint32_t n = 0;
            f.read(reinterpret_cast<char *>(&n), 4);
            readVec(f, *dst[k], n);
        }
        o.numDefaultASpawns = (uint32_t)o.aSpawns.size();
        o.numDefaultBSpawns = (uint32_t)o.bSpawns.size();
    }
    {
        std::ifstream f(o.scenePath + "/zones.bin", std::ios::binary);
        if (!f) throw std::runtime_error("oracle: cannot open zones.bin");
        uint32_t n = 0;
        f.read(reinterpret_cast<char *>(&n), 4);
        readVec(f, o.zoneAABBs, n);
        readVec(f, o.zoneRot, n);
    }
    // mgr.cpp:913-944 hardcodedGoalRegions
    const float top = -56.f + kStandHeight * 1.5f;
    GoalRegion g0 = {};
    g0.subRegions[0] = { v3(625, 510, -64), v3(900, 540, top), 0.f };
    g0.numSubRegions = 1; g0.attackerTeam = true; g0.rewardStrength = 1.f;
    GoalRegion g1 = {};
    g1.subRegions[0] = { v3(938, 440, -56), v3(1030, 539, top), 0.f };
    g1.subRegions[1] = { v3(545, 102, -64), v3(630, 134, top), 0.f };
    g1.numSubRegions = 2; g1.attackerTeam = true; g1.rewardStrength = 1.f;
    o.goalRegions = { g0, g1 };
}

void refreshDebug(Oracle &o)
{
    const size_t A = (size_t)o.W * o.N;
    for (size_t g = 0; g < A; g++) {
        const Agent &a = o.agents[g];
        float *f = &o.dbgAF[g * MPENV_DBG_AF_COUNT];
        f[0] = a.pos.x; f[1] = a.pos.y; f[2] = a.pos.z;
        f[3] = a.vel.x; f[4] = a.vel.y; f[5] = a.vel.z;
        f[6] = a.rot.w; f[7] = a.rot.x; f[8] = a.rot.y; f[9] = a.rot.z;
        f[10] = a.aimYaw; f[11] = a.aimPitch;
        f[12] = a.aimRot.w; f[13] = a.aimRot.x; f[14] = a.aimRot.y; f[15] = a.aimRot.z;
        f[16] = a.maxVelocity; f[17] = a.minDistToZone; f[18] = a.firedShotT; f[19] = a.totalPenalty;
        f[20] = a.startPos.x; f[21] = a.startPos.y; f[22] = a.startPos.z;
        f[23] = a.minDistToSubZone;
        int32_t *n = &o.dbgAI[g * MPENV_DBG_AI_COUNT];
        n[0] = a.curPose; n[1] = a.tgtPose; n[2] = a.transitionRemaining;
        n[3] = (int32_t)a.rng.key.a; n[4] = (int32_t)a.rng.key.b; n[5] = (int32_t)a.rng.ctr;
        n[6] = a.landedShotOn; n[7] = a.remainingRespawnSteps; n[8] = a.remainingStepsBeforeAutoheal;
        n[9] = (a.successfulKill ? 1 : 0) | (a.wasKilled ? 2 : 0) | (a.inZone ? 4 : 0) |
               (a.hasDiedDuringEpisode ? 8 : 0) | (a.reloadedFullMag ? 16 : 0) | (a.inSubZone ? 32 : 0);
        n[10] = a.wasShotCount; n[11] = a.weaponType; n[12] = (int32_t)a.lastBreadcrumb;
        n[13] = a.stepsSinceLastNewBreadcrumb;
        int cs = 0;
        for (int k = 0; k < kMaxTeamSize; k++) cs |= a.canSee[k] ? (1 << k) : 0;
        n[14] = cs; n[15] = (int32_t)a.numNewCellsVisited;
        std::copy(a.visited.begin(), a.visited.end(), &o.dbgExplore[g * kGridW * kGridW]);
    }
    for (int w = 0; w < o.W; w++) {
        const World &wd = o.worlds[w];
        int32_t *n = &o.dbgWI[(size_t)w * MPENV_DBG_WI_COUNT];
        n[0] = wd.teamA; n[1] = wd.curStep; n[2] = wd.isFinished; n[3] = wd.curZone;
        n[4] = wd.curControllingTeam; n[5] = wd.isContested; n[6] = wd.isCaptured; n[7] = wd.earnedPoint;
        n[8] = wd.zoneStepsRemaining; n[9] = wd.stepsUntilPoint; n[10] = (int32_t)wd.curEpisodeIdx;
        n[11] = (int32_t)wd.worldEpisodeCounter; n[12] = (int32_t)wd.baseRNG.key.a;
        n[13] = (int32_t)wd.baseRNG.key.b; n[14] = (int32_t)wd.baseRNG.ctr; n[15] = (int32_t)wd.crumbs.size();
        n[16] = (int32_t)wd.filtersActive[0]; n[17] = (int32_t)wd.filtersActive[1];
        n[18] = wd.filtersLastMatchedStep[0]; n[19] = wd.filtersLastMatchedStep[1];
        n[20] = wd.crumbOverflow;
        uint32_t sub = 0;
        for (int k = 0; k < 8; k++)
            sub |= (uint32_t)((wd.subCtrl[k] + 1) | (wd.subContested[k] ? 4 : 0) | (wd.subCaptured[k] ? 8 : 0)) << (4 * k);
        n[21] = (int32_t)sub;
        float *f = &o.dbgWF[(size_t)w * MPENV_DBG_WF_COUNT];
        f[0] = wd.teamRewards[0]; f[1] = wd.teamRewards[1];
        f[2] = wd.minDistToRegions[0]; f[3] = wd.minDistToRegions[1];
        f[4] = wd.teamStepRewards[0]; f[5] = wd.teamStepRewards[1];
        float *c = &o.dbgCrumbs[(size_t)w * MPENV_MAX_CRUMBS * 8];
        std::fill(c, c + MPENV_MAX_CRUMBS * 8, 0.f);
        for (size_t k = 0; k < wd.crumbs.size(); k++) {
            const Crumb &cr = wd.crumbs[k];
            float *e = &c[k * 8];
            e[0] = cr.pos.x; e[1] = cr.pos.y; e[2] = cr.pos.z; e[3] = cr.penalty;
            e[4] = (float)cr.team; e[5] = (float)cr.offset; e[6] = (float)cr.id; e[7] = 1.f;
        }
    }
}

} // namespace

extern "C" {

void *oracle_create(const oracle_config *cfg)
{
    try {
        Oracle *o = new Oracle();
        o->cfg = *cfg;
        o->scenePath = cfg->scene_path;
        o->W = (int)cfg->num_worlds;
        o->teamSize = (int)cfg->team_size;
        o->N = 2 * o->teamSize;
        o->worldOffset = cfg->world_id_offset;
        o->autoReset = cfg->auto_reset != 0;
        o->simFlags = cfg->sim_flags;
        o->task = cfg->task_type;
        o->flank = cfg->train_flank != 0;
        if (o->task != MPENV_TASK_ZONE && o->task != MPENV_TASK_ZONE_CAPTURE_DEFEND)
            throw std::runtime_error("oracle: task must be Zone or ZoneCaptureDefend");
        // mgr.cpp:1736-1738
        RandKey init_key = initKey(cfg->rand_seed);
        o->initRandKey = splitI(init_key, 0);
        // mgr.cpp:1397-1413 TrainControl from flags
        o->trainControl[0] = (cfg->sim_flags & MPENV_SIMFLAG_SIM_EVAL_MODE) ? 1 : 0;
        o->trainControl[1] = (cfg->sim_flags & MPENV_SIMFLAG_STAGGER_STARTS) ? 1 : 0;
        o->trainControl[2] = (cfg->sim_flags & MPENV_SIMFLAG_RANDOM_FLIP_TEAMS) ? 1 : 0;
        loadScene(*o);
        if (o->task == MPENV_TASK_ZONE_CAPTURE_DEFEND && o->zoneAABBs.size() < 4)
            throw std::runtime_error("ZoneCaptureDefend needs a scene with >= 4 zones");
        if (o->simFlags & MPENV_SIMFLAG_SUB_ZONES) {
            if (o->zoneAABBs.size() < 3) throw std::runtime_error("SubZones needs a scene with >= 3 zones");
            subZoneTable(o->zoneAABBs.data(), o->zoneRot.data(), o->subZones);
        }
        o->nodes.resize(cfg->num_nodes);
        std::memcpy(o->nodes.data(), cfg->bvh_nodes, sizeof(Node) * cfg->num_nodes);
        o->verts.resize(cfg->num_bvh_verts);
        for (int i = 0; i < cfg->num_bvh_verts; i++)
            o->verts[i] = v3(cfg->bvh_verts[3 * i], cfg->bvh_verts[3 * i + 1], cfg->bvh_verts[3 * i + 2]);
        if (o->simFlags & MPENV_SIMFLAG_SPAWN_IN_MIDDLE) addMiddleSpawnCells(*o);
        o->lidarOrder = cfg->lidar_octant_order;
        o->octOrder = octantOrder(o->nodes);
        if (cfg->lidar_bvh_nodes && cfg->num_lidar_nodes > 0) {
            o->lidarNodes.resize(cfg->num_lidar_nodes);
            std::memcpy(o->lidarNodes.data(), cfg->lidar_bvh_nodes, sizeof(Node) * cfg->num_lidar_nodes);
            o->lidarVerts.resize(cfg->num_lidar_bvh_verts);
            for (int i = 0; i < cfg->num_lidar_bvh_verts; i++)
                o->lidarVerts[i] = v3(cfg->lidar_bvh_verts[3 * i], cfg->lidar_bvh_verts[3 * i + 1],
                                      cfg->lidar_bvh_verts[3 * i + 2]);
            o->lidarOctOrder = octantOrder(o->lidarNodes);
        } else {
            o->lidarNodes = o->nodes;
            o->lidarVerts = o->verts;
            o->lidarOctOrder = o->octOrder;
        }
        {
            // bots' navmesh and A* table, built here from navmesh.bin
            NavBuild nb = navFromFile(o->scenePath + "/navmesh.bin");
            const int T = (int)(nb.tri.size() / 3);
            o->numNavTris = T;
            o->navTris.resize((size_t)T * 3);
            std::vector<float> flat((size_t)T * 9);
            for (int i = 0; i < T * 3; i++) {
                o->navTris[i] = nb.verts[nb.tri[i]];
                flat[3 * i] = o->navTris[i].x;
                flat[3 * i + 1] = o->navTris[i].y;
                flat[3 * i + 2] = o->navTris[i].z;
            }
            o->navAdj = nb.adj;
            o->astar = buildAStarLookup(nb);
            o->navCdf.resize(T);
            if (T > 0) navAreaCDF(flat.data(), T, o->navCdf.data());
        }
        // sim.cpp:5855 maxDist; 5869-5882 frustumData
        o->maxDist = length(o->worldBounds.pMax - o->worldBounds.pMin);
        {
            float aspect = 16.f / 9.f;
            float ang = 90.f / 2.f * (kPi / 180.f);
            float f = 1.f / (sinf_(ang) / cosf_(ang));
            float wx = f / aspect, wy = 1.f;
            float hx = f, hy = 1.f;
            float wi = 1.f / sqrt_(wx * wx + wy * wy);
            float hi = 1.f / sqrt_(hx * hx + hy * hy);
            o->frustum[0] = wx * wi; o->frustum[1] = wy * wi;
            o->frustum[2] = hx * hi; o->frustum[3] = hy * hi;
        }
        const size_t A = (size_t)o->W * o->N, W = (size_t)o->W;
        o->agents.resize(A);
        for (Agent &a : o->agents) {
            std::memset(&a.pos, 0, offsetof(Agent, visited) - offsetof(Agent, pos));
            a.rot = quat(1, 0, 0, 0);
            a.aimRot = quat(1, 0, 0, 0);
            a.landedShotOn = -1;
            a.lastBreadcrumb = -1;
            a.numNewCellsVisited = 0;
            a.daimYawVel = a.daimPitchVel = 0.f;
            for (bool &b : a.canSee) b = false;
        }
        o->worlds.resize(W);
        o->spawnTrackLen = (int)std::max<size_t>(
            128, std::max(o->aSpawns.size(), std::max(o->bSpawns.size(), o->commonRespawns.size())));
        o->spawnTrack.assign(W * 3 * (size_t)o->spawnTrackLen, 0xFFFFFFFFu);
        o->resetBuf.assign(W, 0);
        o->worldCurriculum.assign(W, 0);
        o->matchResult.assign(W * 30, 0);
        o->exploreAction.assign(A * 4, 0);
        o->discreteAction.assign(A * 4, 0);
        o->discreteAim.assign(A * 2, 0);
        o->policy.assign(A, 0);
        o->done.assign(A, 0);
        o->magazine.assign(A * 2, 0);
        o->botAction.assign(A * 7, 0);
        o->aimAction.assign(A * 2, 0.f);
        o->reward.assign(A, 0.f);
        o->selfObs.assign(A * kSelfObs, 0.f);
        o->filtersObs.assign(A, 0.f);
        o->teammateObs.assign(A * 5 * kOtherObs, 0.f);
        o->opponentObs.assign(A * 6 * kOtherObs, 0.f);
        o->lastKnownObs.assign(A * 6 * kOtherObs, 0.f);
        o->selfPos.assign(A * 3, -1000.f);
        o->teammatePos.assign(A * 5 * 3, -1000.f);
        o->opponentPos.assign(A * 6 * 3, -1000.f);
        o->lastKnownPos.assign(A * 6 * 3, -1000.f);
        o->masks.assign(A * 6, 0.f);
        o->fwdLidar.assign(A * kFwdH * kFwdW * 4, 0.f);
        o->rearLidar.assign(A * kRearH * kRearW * 4, 0.f);
        o->ftActions.assign(W * 2 * 6 * 4, 0);
        o->ftGlobal.assign(W * 2 * MPENV_FT_GLOBAL_DIM, 0.f);
        o->ftPlayers.assign(W * 2 * 6 * MPENV_FT_PLAYER_DIM, 0.f);
        o->ftEnemies.assign(W * 2 * 6 * MPENV_FT_ENEMY_DIM, 0.f);
        o->ftLastKnown.assign(W * 2 * 6 * MPENV_FT_COMMON_DIM, 0.f);
        o->ftFwdLidar.assign(W * 2 * 6 * kFwdH * kFwdW * 4, 0.f);
        o->ftRearLidar.assign(W * 2 * 6 * kRearH * kRearW * 4, 0.f);
        o->ftReward.assign(W * 2, 0.f);
        o->ftDone.assign(W * 2, 0);
        o->ftPolicy.assign(W * 2, 0);
        o->agentMap.assign(A * 16 * 16 * 4, 0.f);
        o->hp.assign(A, 0.f);
        o->alive.assign(A, 0.f);
        o->rewardCoefs.assign(A * 9, 0.f);
        o->dbgAF.assign(A * MPENV_DBG_AF_COUNT, 0.f);
        o->dbgAI.assign(A * MPENV_DBG_AI_COUNT, 0);
        o->dbgWI.assign(W * MPENV_DBG_WI_COUNT, 0);
        o->dbgWF.assign(W * MPENV_DBG_WF_COUNT, 0.f);
        o->dbgExplore.assign(A * kGridW * kGridW, 0u);
        o->dbgCrumbs.assign(W * MPENV_MAX_CRUMBS * 8, 0.f);
        for (int w = 0; w < o->W; w++) constructWorld(*o, w);
        return o;
    } catch (const std::exception &e) {
        fprintf(stderr, "oracle_create failed: %s\n", e.what());
        return nullptr;
    }
}

void oracle_destroy(void *h) { delete static_cast<Oracle *>(h); }

int oracle_export(void *h, int32_t id, void **ptr, int32_t *dtype, int32_t *ndim, int64_t *dims)
{
    Oracle &o = *static_cast<Oracle *>(h);
    const int64_t A = (int64_t)o.W * o.N, W = o.W;
    auto set = [&](void *p, int32_t dt, std::initializer_list<int64_t> d) {
        *ptr = p;
        *dtype = dt;
        *ndim = (int32_t)d.size();
        int k = 0;
        for (int64_t x : d) dims[k++] = x;
        return 0;
    };
    switch (id) {
    case MPENV_EXPORT_RESET: return set(o.resetBuf.data(), MPENV_DTYPE_INT32, { W, 1 });
    case MPENV_EXPORT_WORLD_CURRICULUM: return set(o.worldCurriculum.data(), MPENV_DTYPE_INT32, { W, 1 });
    case MPENV_EXPORT_EXPLORE_ACTION: return set(o.exploreAction.data(), MPENV_DTYPE_INT32, { A, 4 });
    case MPENV_EXPORT_PVP_DISCRETE_ACTION: return set(o.discreteAction.data(), MPENV_DTYPE_INT32, { A, 4 });
    case MPENV_EXPORT_PVP_AIM_ACTION: return set(o.aimAction.data(), MPENV_DTYPE_FLOAT32, { A, 1, 2 });
    case MPENV_EXPORT_PVP_DISCRETE_AIM_ACTION: return set(o.discreteAim.data(), MPENV_DTYPE_INT32, { A, 2 });
    case MPENV_EXPORT_REWARD: return set(o.reward.data(), MPENV_DTYPE_FLOAT32, { A, 1 });
    case MPENV_EXPORT_DONE: return set(o.done.data(), MPENV_DTYPE_INT32, { A, 1 });
    case MPENV_EXPORT_MATCH_RESULT: return set(o.matchResult.data(), MPENV_DTYPE_INT32, { W, 30 });
    case MPENV_EXPORT_AGENT_POLICY: return set(o.policy.data(), MPENV_DTYPE_INT32, { A, 1 });
    case MPENV_EXPORT_SELF_OBSERVATION: return set(o.selfObs.data(), MPENV_DTYPE_FLOAT32, { A, kSelfObs });
    case MPENV_EXPORT_TEAMMATE_OBSERVATIONS: return set(o.teammateObs.data(), MPENV_DTYPE_FLOAT32, { A, 5, kOtherObs });
    case MPENV_EXPORT_OPPONENT_OBSERVATIONS: return set(o.opponentObs.data(), MPENV_DTYPE_FLOAT32, { A, 6, kOtherObs });
    case MPENV_EXPORT_OPPONENT_LAST_KNOWN_OBSERVATIONS: return set(o.lastKnownObs.data(), MPENV_DTYPE_FLOAT32, { A, 6, kOtherObs });
    case MPENV_EXPORT_SELF_POSITION: return set(o.selfPos.data(), MPENV_DTYPE_FLOAT32, { A, 3 });
    case MPENV_EXPORT_TEAMMATE_POSITIONS: return set(o.teammatePos.data(), MPENV_DTYPE_FLOAT32, { A, 5, 3 });
    case MPENV_EXPORT_OPPONENT_POSITIONS: return set(o.opponentPos.data(), MPENV_DTYPE_FLOAT32, { A, 6, 3 });
    case MPENV_EXPORT_OPPONENT_LAST_KNOWN_POSITIONS: return set(o.lastKnownPos.data(), MPENV_DTYPE_FLOAT32, { A, 6, 3 });
    case MPENV_EXPORT_OPPONENT_MASKS: return set(o.masks.data(), MPENV_DTYPE_FLOAT32, { A, 6, 1 });
    case MPENV_EXPORT_FWD_LIDAR: return set(o.fwdLidar.data(), MPENV_DTYPE_FLOAT32, { A, kFwdH, kFwdW, 4 });
    case MPENV_EXPORT_REAR_LIDAR: return set(o.rearLidar.data(), MPENV_DTYPE_FLOAT32, { A, kRearH, kRearW, 4 });
    case MPENV_EXPORT_AGENT_MAP:
    case MPENV_EXPORT_UNMASKED_AGENT_MAP: return set(o.agentMap.data(), MPENV_DTYPE_FLOAT32, { A, 16, 16, 4 });
    case MPENV_EXPORT_HP: return set(o.hp.data(), MPENV_DTYPE_FLOAT32, { A, 1 });
    case MPENV_EXPORT_ALIVE: return set(o.alive.data(), MPENV_DTYPE_FLOAT32, { A, 1 });
    case MPENV_EXPORT_MAGAZINE: return set(o.magazine.data(), MPENV_DTYPE_INT32, { A, 2 });
    case MPENV_EXPORT_FULL_TEAM_ACTIONS: return set(o.ftActions.data(), MPENV_DTYPE_INT32, { W * 2, 6, 4 });
    case MPENV_EXPORT_FULL_TEAM_GLOBAL: return set(o.ftGlobal.data(), MPENV_DTYPE_FLOAT32, { W * 2, MPENV_FT_GLOBAL_DIM });
    case MPENV_EXPORT_FULL_TEAM_PLAYERS:
        return set(o.ftPlayers.data(), MPENV_DTYPE_FLOAT32, { W * 2, 6, MPENV_FT_PLAYER_DIM });
    case MPENV_EXPORT_FULL_TEAM_ENEMIES:
        return set(o.ftEnemies.data(), MPENV_DTYPE_FLOAT32, { W * 2, 6, MPENV_FT_ENEMY_DIM });
    case MPENV_EXPORT_FULL_TEAM_LAST_KNOWN_ENEMIES:
        return set(o.ftLastKnown.data(), MPENV_DTYPE_FLOAT32, { W * 2, 6, MPENV_FT_COMMON_DIM });
    case MPENV_EXPORT_FULL_TEAM_FWD_LIDAR:
        return set(o.ftFwdLidar.data(), MPENV_DTYPE_FLOAT32, { W * 2, 6, kFwdH, kFwdW, 4 });
    case MPENV_EXPORT_FULL_TEAM_REAR_LIDAR:
        return set(o.ftRearLidar.data(), MPENV_DTYPE_FLOAT32, { W * 2, 6, kRearH, kRearW, 4 });
    case MPENV_EXPORT_FULL_TEAM_REWARD: return set(o.ftReward.data(), MPENV_DTYPE_FLOAT32, { W * 2, 1 });
    case MPENV_EXPORT_FULL_TEAM_DONE: return set(o.ftDone.data(), MPENV_DTYPE_INT32, { W * 2, 1 });
    case MPENV_EXPORT_FULL_TEAM_POLICY_ASSIGNMENTS: return set(o.ftPolicy.data(), MPENV_DTYPE_INT32, { W * 2, 1 });
    case MPENV_EXPORT_FILTERS_STATE: return set(o.filtersObs.data(), MPENV_DTYPE_FLOAT32, { A, 1 });
    case MPENV_EXPORT_REWARD_HYPER_PARAMS: return set(o.rewardCoefs.data(), MPENV_DTYPE_FLOAT32, { A, 9 });
    case MPENV_EXPORT_EVENT_LOG:
        if (!o.eventsOn) return -1;
        return set(o.events.data(), MPENV_DTYPE_INT32, { W, 2 * (int64_t)o.N + 1, 6 });
    case MPENV_EXPORT_PACKED_STEP_SNAPSHOT:
        if (!o.eventsOn) return -1;
        return set(o.snapshots.data(), MPENV_DTYPE_INT32, { W, 48 });
    case MPENV_EXPORT_SNAPSHOT_WRITTEN:
        if (!o.eventsOn) return -1;
        return set(o.snapWritten.data(), MPENV_DTYPE_INT32, { W, 1 });
    case MPENV_EXPORT_RECORD_LOG:
        if (!o.recordOn) return -1;
        return set(o.recordLog.data(), MPENV_DTYPE_INT32, { W, 217 });
    case MPENV_EXPORT_REPLAY_LOG:
        if (!o.replayOn) return -1;
        return set(o.replayLog.data(), MPENV_DTYPE_INT32, { W, 217 });
    case MPENV_EXPORT_SIM_CONTROL: return set(o.trainControl, MPENV_DTYPE_INT32, { 3 });
    case MPENV_EXPORT_DEBUG_AGENT_F32: return set(o.dbgAF.data(), MPENV_DTYPE_FLOAT32, { A, MPENV_DBG_AF_COUNT });
    case MPENV_EXPORT_DEBUG_AGENT_I32: return set(o.dbgAI.data(), MPENV_DTYPE_INT32, { A, MPENV_DBG_AI_COUNT });
    case MPENV_EXPORT_DEBUG_WORLD_I32: return set(o.dbgWI.data(), MPENV_DTYPE_INT32, { W, MPENV_DBG_WI_COUNT });
    case MPENV_EXPORT_DEBUG_WORLD_F32: return set(o.dbgWF.data(), MPENV_DTYPE_FLOAT32, { W, MPENV_DBG_WF_COUNT });
    case MPENV_EXPORT_DEBUG_EXPLORE: return set(o.dbgExplore.data(), MPENV_DTYPE_UINT32, { A, kGridW * kGridW });
    case MPENV_EXPORT_DEBUG_CRUMBS: return set(o.dbgCrumbs.data(), MPENV_DTYPE_FLOAT32, { W, MPENV_MAX_CRUMBS, 8 });
    default: return -1;
    }
}

void oracle_init(void *h)
{
    Oracle &o = *static_cast<Oracle *>(h);
    for (int w = 0; w < o.W; w++) o.resetBuf[w] = 1; // triggerReset (mgr.cpp:1936-1938)
    for (int w = 0; w < o.W; w++) resetAndObs(o, w); // Init graph (sim.cpp:5322-5340)
}

void oracle_step(void *h)
{
    Oracle &o = *static_cast<Oracle *>(h);
    for (int w = 0; w < o.W; w++) stepWorld(o, w);
}

void oracle_step_worlds(void *h, int32_t w0, int32_t w1)
{
    Oracle &o = *static_cast<Oracle *>(h);
    for (int w = w0; w < w1; w++) stepWorld(o, w);
}

void oracle_refresh_debug(void *h) { refreshDebug(*static_cast<Oracle *>(h)); }

void oracle_set_curriculum(void *h, const void *snapshots, int32_t n)
{
    Oracle &o = *static_cast<Oracle *>(h);
    const auto *p = static_cast<const mpenv_curriculum_snapshot *>(snapshots);
    o.curriculum.assign(p, p + (n > 0 ? n : 0));
}

void oracle_set_log_modes(void *h, int32_t record, int32_t replay, int32_t events)
{
    Oracle &o = *static_cast<Oracle *>(h);
    const size_t W = (size_t)o.W;
    o.recordOn = record != 0;
    o.replayOn = replay != 0;
    o.eventsOn = events != 0;
    if (o.recordOn) o.recordLog.assign(W, mpenv_step_log {});
    if (o.replayOn) o.replayLog.assign(W, mpenv_step_log {});
    if (o.eventsOn) {
        o.events.assign(W * (2 * o.N + 1), mpenv_game_event {});
        o.snapshots.assign(W, mpenv_packed_step_snapshot {});
        o.snapWritten.assign(W, 0);
    }
}

double oracle_run_threaded(void *h, int32_t nsteps, int32_t nthreads, const int32_t *ring, int32_t ring_len)
{
    Oracle &o = *static_cast<Oracle *>(h);
    const size_t A = (size_t)o.W * o.N;
    if (nthreads < 1) nthreads = 1;
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> pool;
    for (int t = 0; t < nthreads; t++) {
        int w0 = (int)((int64_t)o.W * t / nthreads), w1 = (int)((int64_t)o.W * (t + 1) / nthreads);
        pool.emplace_back([&o, w0, w1, nsteps, ring, ring_len, A]() {
            for (int s = 0; s < nsteps; s++) {
                const int32_t *src = ring + (size_t)(s % ring_len) * A * 6;
                for (size_t g = (size_t)w0 * o.N; g < (size_t)w1 * o.N; g++) {
                    for (int k = 0; k < 4; k++) o.discreteAction[4 * g + k] = src[6 * g + k];
                    o.discreteAim[2 * g] = src[6 * g + 4];
                    o.discreteAim[2 * g + 1] = src[6 * g + 5];
                }
                for (int w = w0; w < w1; w++) stepWorld(o, w);
            }
        });
    }
    for (auto &th : pool) th.join();
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double>(t1 - t0).count();
}

void oracle_cast_stats(int32_t leaf_read_two, uint64_t *out2)
{
    if (out2) {
        out2[0] = g_casts.load();
        out2[1] = g_zeroCasts.load();
    }
    if (leaf_read_two >= 0) {
        g_leafReadTwo = leaf_read_two;
        g_casts = 0;
        g_zeroCasts = 0;
    }
}

int oracle_navmesh(void *h, float *tris_out, int32_t *adj_out, int32_t *astar_out, int32_t *num_tris)
{
    const Oracle &o = *static_cast<Oracle *>(h);
    const int T = o.numNavTris;
    if (num_tris) *num_tris = T;
    if (tris_out)
        for (int i = 0; i < T * 3; i++) {
            tris_out[3 * i] = o.navTris[i].x;
            tris_out[3 * i + 1] = o.navTris[i].y;
            tris_out[3 * i + 2] = o.navTris[i].z;
        }
    if (adj_out) std::copy(o.navAdj.begin(), o.navAdj.end(), adj_out);
    if (astar_out) std::copy(o.astar.begin(), o.astar.end(), astar_out);
    return 0;
}

int oracle_trace_ray(void *h, const float *org, const float *d, float *t_out)
{
    Oracle &o = *static_cast<Oracle *>(h);
    return bvhTraceRay(o, v3(org[0], org[1], org[2]), v3(d[0], d[1], d[2]), t_out) ? 1 : 0;
}

float oracle_sphere_cast(void *h, const float *org, const float *d, float r, float *n_out)
{
    Oracle &o = *static_cast<Oracle *>(h);
    Vec3 n = v3(0.f, 0.f, 0.f);
    float t = bvhSphereCast(o, v3(org[0], org[1], org[2]), v3(d[0], d[1], d[2]), r, &n);
    n_out[0] = n.x; n_out[1] = n.y; n_out[2] = n.z;
    return t;
}

void oracle_set_slab_fma(int32_t on) { g_slabFma = on ? 1 : 0; }

void oracle_trace_ray_batch(void *h, int32_t n, const float *org, const float *d, int32_t order, float *t_out,
                            int32_t *hit_out)
{
    Oracle &o = *static_cast<Oracle *>(h);
    const int ntri = (int)o.verts.size() / 3;
    for (int32_t k = 0; k < n; k++) {
        float t = 0.f;
        const Vec3 ro = v3(org[3 * k], org[3 * k + 1], org[3 * k + 2]), rd = v3(d[3 * k], d[3 * k + 1], d[3 * k + 2]);
        if (order == 3) {
            // brute force under the kLidarLex rule: the smallest t over
            // every triangle, each tested with t_max = FLT_MAX
            const RayTxfm tx = computeRayIsectTxfm(rd, v3(1.f / rd.x, 1.f / rd.y, 1.f / rd.z));
            float tb = kFltMax;
            int ib = -1;
            for (int tri = 0; tri < ntri; tri++) {
                float th = 0.f;
                if (rayTriangleIntersection(o.verts[tri * 3], o.verts[tri * 3 + 1], o.verts[tri * 3 + 2], tx, ro,
                                            kFltMax, &th) && lexLess(th, tb)) {
                    tb = th;
                    ib = tri;
                }
            }
            hit_out[k] = ib >= 0 ? 1 : 0;
            t_out[k] = tb;
            continue;
        }
        hit_out[k] = bvhTraceRay(o, ro, rd, &t, kFltMax, order == kLidarOctant, order == kLidarLex,
                                 order != kLidarSlot) ? 1 : 0;
        t_out[k] = t;
    }
}

void oracle_sphere_cast_batch(void *h, int32_t n, const float *org, const float *d, float r,
                              const float *t_max, float *t_out, float *n_out)
{
    Oracle &o = *static_cast<Oracle *>(h);
    for (int32_t k = 0; k < n; k++) {
        Vec3 nn = v3(0.f, 0.f, 0.f);
        const float tm = t_max ? t_max[k] : kFltMax;
        t_out[k] = bvhSphereCast(o, v3(org[3 * k], org[3 * k + 1], org[3 * k + 2]),
                                 v3(d[3 * k], d[3 * k + 1], d[3 * k + 2]), r, &nn, tm);
        n_out[3 * k] = nn.x; n_out[3 * k + 1] = nn.y; n_out[3 * k + 2] = nn.z;
    }
}

int oracle_trace_ray_brute(void *h, const float *org, const float *d, float *t_out)
{
    Oracle &o = *static_cast<Oracle *>(h);
    Vec3 ro = v3(org[0], org[1], org[2]), rd = v3(d[0], d[1], d[2]);
    Vec3 inv_d = v3(1.f / rd.x, 1.f / rd.y, 1.f / rd.z);
    RayTxfm tx = computeRayIsectTxfm(rd, inv_d);
    float t_max = kFltMax;
    bool hit = false;
    for (size_t t = 0; t + 2 < o.verts.size(); t += 3) {
        float th;
        if (rayTriangleIntersection(o.verts[t], o.verts[t + 1], o.verts[t + 2], tx, ro, t_max, &th)) {
            hit = true;
            t_max = th;
        }
    }
    *t_out = t_max;
    return hit ? 1 : 0;
}

float oracle_sphere_cast_brute(void *h, const float *org, const float *d, float r)
{
    Oracle &o = *static_cast<Oracle *>(h);
    Vec3 ro = v3(org[0], org[1], org[2]), rd = v3(d[0], d[1], d[2]);
    float t_max = kFltMax;
    for (size_t t = 0; t + 2 < o.verts.size(); t += 3) {
        Vec3 n;
        t_max = sphereCastTriangle(o.verts[t], o.verts[t + 1], o.verts[t + 2], ro, rd, t_max, r, &n);
    }
    return t_max;
}

void oracle_eval_math(int32_t fn, const float *in, const float *in2, float *out, int32_t n)
{
    for (int32_t k = 0; k < n; k++) {
        float x = in[k];
        switch (fn) {
        case 0: out[k] = sinf_(x); break;
        case 1: out[k] = cosf_(x); break;
        case 2: out[k] = atan2f_(x, in2[k]); break;
        case 3: out[k] = asinf_(x); break;
        case 4: out[k] = logf_(x); break;
        case 5: out[k] = sqrt_(x); break;
        case 6: out[k] = x / in2[k]; break;
        default: out[k] = 0.f; break;
        }
    }
}

void oracle_threefry(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1, uint32_t *out2)
{
    RandKey r = threefry2x32(initKey(k0, k1), c0, c1);
    out2[0] = r.a;
    out2[1] = r.b;
}

void oracle_tape_actions(uint32_t seed, uint32_t step, uint32_t first_agent, int32_t n, int32_t *out6)
{
    for (int32_t k = 0; k < n; k++) tapeActions(seed, step, first_agent + (uint32_t)k, &out6[6 * k], &out6[6 * k + 4]);
}

float oracle_capsule(const float *o, const float *d, float r, float h)
{
    return intersectRayZOriginCapsule(v3(o[0], o[1], o[2]), v3(d[0], d[1], d[2]), r, h);
}

} // extern "C"
