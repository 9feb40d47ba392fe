// engine.h — device state layout of the MI355X engine.
//
// The reference stores per-entity components in Madrona ECS archetype
// columns (PvPAgent, types.hpp:932-995) and per-world singletons
// (sim.hpp:81-191).  Here every per-agent internal field is its own
// structure-of-arrays column indexed by the global agent id
// g = world * N + agent (N = 2 * teamSize, team 0 offsets first,
// level_gen.cpp:148-162), so lanes that own consecutive agents issue
// coalesced loads.  Exported components keep the reference's
// array-of-struct column layout (tensor dims of mgr.cpp:1965-2381) because
// they are the drop-in boundary.
#pragma once

#include <cstdint>

#include "mpenv.h"
#include "mpenv_core.h"
#include "scene.h"

namespace mpenv {

constexpr int kMaxTeamSize = 6;
constexpr int kMaxAgents = 2 * kMaxTeamSize;
constexpr int kMaxZones = 5;
constexpr int kGridW = 81;
constexpr int kGridCells = kGridW * kGridW;
// ExploreTracker as a per-agent bitset over the 81 x 81 cells: bit = the
// cell holds the agent's current episode index (exploreEp).  Exact for
// exploreVisitedSystem (sim.cpp:3508-3536), see DESIGN.md §2.  Cells are
// grouped in 8 x 8 tiles, one u64 each (11 x 11 tiles, 968 B per agent);
// the tile the agent stands in lives in SoA columns (exploreTile,
// exploreLo / exploreHi), so consecutive steps inside one tile (240 x 240
// units) touch only coalesced columns and the row is read / written once
// per tile change.
constexpr int kExploreTilesX = 11;
constexpr int kExploreTiles = kExploreTilesX * kExploreTilesX;
constexpr int kSelfObs = 43;
constexpr int kOtherObs = 32;
constexpr int kFwdRays = 64;   // 2 x 32
constexpr int kRearRays = 16;  // 2 x 8
constexpr int kLidarRays = kFwdRays + kRearRays;
constexpr int kMaxCrumbs = 128;
constexpr int kMinSpawnTrack = 128; // SpawnUsageCounter::maxNumSpawns (types.hpp:96)
constexpr int kMaxBVHStack = 16; // register byte-stack capacity

#define MP_AGENT_F32(X) \
    X(px) X(py) X(pz) X(vx) X(vy) X(vz) X(rw) X(rx) X(ry) X(rz) \
    X(ayaw) X(apitch) X(aw) X(ax) X(ay) X(az) X(maxVel) X(minDistZone) \
    X(firedT) X(bcPenalty) X(sx) X(sy) X(sz) X(dyv) X(dpv) X(minDistSub)

#define MP_AGENT_I32(X) \
    X(curPose) X(tgtPose) X(transRem) X(rngA) X(rngB) X(rngCtr) X(landedOn) \
    X(respawnSteps) X(autohealSteps) X(flags) X(wasShot) X(weapon) X(bcLast) \
    X(bcSteps) X(newCells) X(exploreEp) X(exploreTile) X(exploreLo) X(exploreHi)

#define MP_WORLD_I32(X) \
    X(teamA) X(curStep) X(finished) X(curZone) X(controlling) X(contested) \
    X(captured) X(earned) X(zoneSteps) X(stepsUntilPoint) X(episode) \
    X(episodeCounter) X(wRngA) X(wRngB) X(wRngCtr) X(filtAct0) X(filtAct1) \
    X(filtMatched0) X(filtMatched1) X(episodeCurr) X(numCrumbs) X(nextCrumbId) \
    X(crumbOverflow) X(curTier) X(curSpawnIdx) X(spawnCurriculum) \
    X(matchValid) X(evLogged) X(evMask) X(snapWritten) X(subState)

#define MP_WORLD_F32(X) \
    X(teamRew0) X(teamRew1) X(goalMin0) X(goalMin1) X(goalTeam0) X(goalTeam1)

// Agent flag bits (CombatState booleans, types.hpp:510-528)
enum : int32_t {
    kFlagSuccessfulKill = 1,
    kFlagWasKilled = 2,
    kFlagInZone = 4,
    kFlagHasDied = 8,
    kFlagReloadedFullMag = 16,
    kFlagInSubZone = 32,
};

struct DevState {
    int32_t W, N, T;
    uint32_t nMagic;       // ceil(2^32 / N): g / N = umulhi(g, nMagic) for g < 2^32 / N^2
    int64_t A;
    int64_t dmgStride;     // row stride of dmg (all agents of the manager)

#define MP_DECL_F(n) float *n;
#define MP_DECL_I(n) int32_t *n;
    MP_AGENT_F32(MP_DECL_F)
    MP_AGENT_I32(MP_DECL_I)
    MP_WORLD_I32(MP_DECL_I)
    MP_WORLD_F32(MP_DECL_F)
#undef MP_DECL_F
#undef MP_DECL_I

    float *dmg;            // [6][A] DamageDealt
    uint8_t *visMask;      // [A] OpponentsVisibility, bit k = sees opponent k
    // [A][T][4] k_vis occluder hint per (agent, opponent slot, sample
    // point): the triangle that last ended that line-of-sight ray (0xffff:
    // none).  A performance hint only -- any value gives the same answer
    // (geom_dev.h visibleRayD) -- so it is never reset.
    uint16_t *visOcc;
    uint64_t *exploreBits; // [A][kExploreTiles] ExploreTracker tiles for episode exploreEp
                           // (the tile exploreTile is current in exploreLo / exploreHi)
    int32_t *filtLast;     // [W][2][3] FiltersMatchState::lastMatches (3 filters used)
    int32_t *zoneStats;    // [W][5][5]
    uint32_t *spawnTrack;  // [W][3][spawnTrackLen] SpawnUsageCounter
    float4 *crumbs;        // [W][kMaxCrumbs][2] {x,y,z,penalty},{team,offset,id,-}

    // Exported columns (reference layouts)
    int32_t *reset;        // [W]
    int32_t *worldCurr;    // [W]
    int32_t *matchResult;  // [W][30]
    int32_t *exploreAction;// [A][4]
    int32_t *discreteAction; // [A][4]
    float *aimAction;      // [A][2]
    int32_t *discreteAim;  // [A][2]
    int32_t *policy;       // [A]
    int32_t *botAction;    // [A][7]
    float *reward;         // [A]
    int32_t *done;         // [A]
    float *selfObs;        // [A][43]
    float *filters;        // [A]
    float *tmObs;          // [A][5][32]
    float *oppObs;         // [A][6][32]
    float *lkObs;          // [A][6][32]
    float *selfPos;        // [A][3]
    float *tmPos;          // [A][5][3]
    float *oppPos;         // [A][6][3]
    float *lkPos;          // [A][6][3]
    float *masks;          // [A][6]
    float *fwdLidar;       // [A][2][32][4]
    float *rearLidar;      // [A][2][8][4]
    float *agentMap;       // [A][16][16][4] (never written, as in the reference)
    float *hp;             // [A]
    float *alive;          // [A]
    int32_t *magazine;     // [A][2]
    float *rewardCoefs;    // [A][9]
    int32_t *trainCtrl;    // [3]
    // FullTeamInterface columns, one row per (world, team) (types.hpp:1040-1152)
    int32_t *ftActions;    // [W*2][6][4] (input, never read by the step)
    float *ftGlobal;       // [W*2][16]
    float *ftPlayers;      // [W*2][6][28]
    float *ftEnemies;      // [W*2][6][33]
    float *ftLastKnown;    // [W*2][6][24]
    float *ftFwdLidar;     // [W*2][6][64][4]
    float *ftRearLidar;    // [W*2][6][16][4]
    float *ftReward;       // [W*2]
    int32_t *ftDone;       // [W*2]
    int32_t *ftPolicy;     // [W*2] (input, never read by the step)

    // Record / replay / event logs (allocated only when enabled)
    mpenv_step_log *recordLog;             // [W] written by the step
    const mpenv_step_log *replayLog;       // [W] read by the step
    mpenv_game_event *events;              // [W][evStride] slots: 2 per agent + capture
    mpenv_packed_step_snapshot *snapshots; // [W]
    int32_t evStride;                      // 2 * N + 1

    // Per agent: combat RNG key + first draw keys of a coming reset (k_sim)
    mp::RandKey *resetKeys; // [A][11]

    // Workload counters (mpenv_enable_stats), null when off: see StatId.
    unsigned long long *stats;
    // k_obs does nothing while (*obsGate & MPENV_WIRE_ERR_DESYNC): a learner
    // shadow whose wire history broke (wire.hip wireOk); null on the step path.
    const uint32_t *obsGate;
    // gpuStreamStep's caller buffers (OutTab): while outTab->on, k_obs writes
    // its pure outputs there instead of into the engine's exports, and
    // k_lidar writes the lidar rows there too; outBase = this state's first
    // agent in those buffers (world groups).  Null on a wire view.
    const struct OutTab *outTab;
    int64_t outBase;
};

// The caller's trainInterface output buffers k_obs / k_lidar write directly
// during a gpuStreamStep (mgr.cpp:614-645 copies them from the engine's
// exports instead).  A device table, so the captured step graph's kernel
// arguments never change: gpuStreamStep sets it (on = 1, the call's
// pointers) in front of the step and clears it behind it, both from inside
// its input / output copy launches (CopyBatch::tabDst).
struct OutTab {
    int32_t on, pad;
    float *masks, *filters, *selfObs, *selfPos, *tmObs, *tmPos, *oppObs, *oppPos, *fwdLidar, *rearLidar;
    // the two agent-map outputs (constant zeros, as the reference copies
    // them): zero-filled by k_lidar's forward waves, 8 KB per agent of
    // stores that need no loads, issued beside its VALU-bound traversals
    float *agentMap0, *agentMap1;
};

// Per-step workload counters accumulated by the kernels in stats mode
// (bench.py's workload window; never on in the timed region).
enum StatId {
    kStatAliveAgents = 0, // agents alive when k_move runs
    kStatLosPairs = 1,    // (viewer, opponent) pairs with both alive
    kStatLosRays = 2,     // visibility rays traced after the view/frustum tests
    kStatLosSeen = 3,     // of those, rays that found their target
    kStatSphereCasts = 4, // MeshBVH::sphereCast calls (k_move)
    kStatShots = 5,       // fireSystem rays (k_sim)
    kStatHits = 6,        // agents that took damage (applyDmgSystem)
    kStatKills = 7,       // agents killed (alive -> hp <= 0)
    kStatLkRows = 8,      // last-known rows k_obs wrote (knows / cleared on death)
    kStatLosTraced = 9,   // LOS rays that needed a BVH traversal (not decided by the target test or hint)
    kNumStats = 10,
};

struct ZOBBDev {
    mp::Vec3 pMin, pMax;
    float rotation;
};

struct GoalRegionDev {
    ZOBBDev sub[3];
    int32_t numSub;
    int32_t attackerTeam;
    float rewardStrength;
};

// Zone / sub-zone / goal tables in global memory.  Device code indexes them
// with per-world values (the current zone, a sub-zone id): indexing the
// by-value kernel-argument arrays of SceneDev dynamically makes the compiler
// copy the whole argument struct into registers (k_sim's zoneSystem alone
// needed ~200 VGPRs that way).
// A rotated box's frame: qinv(angleAxis(rot, up)) and its corners rotated
// into it -- what zoneSystem / distToZOBB recompute per call.  Filled on the
// device by k_scene_frames with the same functions, so every bit matches.
struct FrameDev {
    mp::Quat toFrame;
    mp::Vec3 pMin, pMax;
};

struct SceneTables {
    mp::AABB zoneAABB[kMaxZones];
    float zoneRot[kMaxZones];
    ZOBBDev subZones[8];
    GoalRegionDev goals[4];
    int32_t zoneGoalTri[kMaxZones];
    FrameDev zoneFrame[kMaxZones];
    FrameDev goalFrame[4][3];
};

// Read-only scene + task constants, passed by value as a kernel argument.
struct SceneDev {
    const SceneTables *tab; // device copy of the arrays below (set after scene upload)
    const BVHNode *nodes;
    const BVHNode *octNodes; // [8][numLidarNodes] octant node images of the lidar tree (scene.h octantNodeImages)
    const BVHNode *lidarNodes; // the lidar tree in slot order (k_vis)
    const float *lidarVerts; // the lidar tree's triangles, 3 floats per vertex (scene.h Scene::lidarVerts)
    int32_t numLidarNodes, numLidarVerts;
    const float *verts;     // 3 floats per vertex, 3 vertices per triangle
    // Per triangle, ray-independent terms of sphereCastTriangle
    // (mesh_bvh.inl:885-1127): unit normal xyz, |normal|, |e01|^2, |e02|^2,
    // |e12|^2, 0 -- computed on the host with the same mpenv_core.h
    // expressions the traversal would evaluate (bit-identical).
    const float *triPre;
    int32_t numNodes;
    int32_t numVerts;
    mp::AABB worldBounds;
    float maxDist;
    float frustum[4];
    const Spawn *aSpawns;
    const Spawn *bSpawns;
    const Spawn *commonRespawns;
    int32_t numA, numB, numCommon, numDefaultA, numDefaultB;
    int32_t spawnTrackLen; // slots per SpawnUsageCounter list: max(128, longest list)
    mp::AABB zoneAABB[kMaxZones];
    float zoneRot[kMaxZones];
    int32_t numZones;
    int32_t task;           // MPENV_TASK_ZONE or MPENV_TASK_ZONE_CAPTURE_DEFEND
    int32_t flank;          // RewardMode::Flank (train_flank)
    ZOBBDev subZones[8];    // SubZones only (level_gen.cpp:282-326)
    GoalRegionDev goals[4];
    int32_t numGoals;
    uint32_t simFlags;
    int32_t autoReset;
    uint32_t worldOffset;
    mp::RandKey initRandKey;
    // navmesh for the scripted bots (sim.cpp:4958-5172)
    const float *navTris;   // 9 floats per triangle (deduplicated vertices)
    const int32_t *astar;   // [numNavTris][numNavTris] next hop
    const float *navCdf;    // [numNavTris] running triangle areas (NavmeshSpawn)
    // TrajectoryCurriculum (level_gen.cpp:498-581), curriculum_data_path
    const mpenv_curriculum_snapshot *curriculum;
    int32_t numSnapshots;
    int32_t numNavTris;
    // NearestNavTri of each zone's centroid (computed once at scene upload
    // by k_zone_goals with the same device function planAStarD would run)
    int32_t zoneGoalTri[kMaxZones];
    // logs (sim.cpp:4750-4843 record/replay, 23-106 + 4592-4634 events)
    int32_t recordOn, replayOn, eventsOn;
    // Sphere-cast vertex-quirk grid (k_move): bit per qgCell x qgCell cell
    // of the xy plane, set where some BVH vertex lies within
    // agentRadius + 2 of the cell (scene.h quirkGrid); a cast from o can only
    // meet the testVert quirk when the cell of 2o is set.
    const uint32_t *quirkGrid;
    float qgMinX, qgMinY, qgInvCell;
    int32_t qgW, qgH;
};

// Host launchers (kernels.hip)
struct LaunchCtx {
    void *stream;       // hipStream_t
    void *events[16];   // optional per-kernel timing events (start/stop pairs)
    int timing;         // record events when nonzero
};

enum KernelId { kKMove = 0, kKSim = 1, kKVis = 2, kKObs = 3, kKLidar = 4, kNumTimedKernels = 5 };

const char *kernelName(int k);
size_t bvhLdsBytes(const SceneDev &sc);
size_t bvhLdsBytesSphere(const SceneDev &sc); // + triPre (sphere-casting kernels)
size_t bvhLdsBytesOct(const SceneDev &sc);    // octant node images + vertices (k_lidar)

int launchConstruct(const DevState &s, const SceneDev &sc, const int32_t ctor_train_ctrl[3], void *stream);
int launchResetOnly(const DevState &s, const SceneDev &sc, void *stream);
int launchMove(const DevState &s, const SceneDev &sc, void *stream);
int launchSimStep(const DevState &s, const SceneDev &sc, void *stream);
int launchVisibility(const DevState &s, const SceneDev &sc, void *stream);
int launchObservations(const DevState &s, const SceneDev &sc, void *stream);
// k_obs over a wire message (wire.hip launchWireUnpack): `view` is the
// shadow's DevState with its input columns pointing into the message.
struct WireObs {
    const uint32_t *packed;  // [A] curPose | tgtPose << 8 | weapon << 16 | flags << 24
    const int32_t *epPrev;   // [W] the previous message's episode counters (the shadow's copy)
    int32_t keyframe;        // a keyframe carries the last-known rows: nothing is cleared
};
int launchObservationsWire(const DevState &view, const SceneDev &sc, const WireObs &wo, void *stream);
int launchLidar(const DevState &s, const SceneDev &sc, void *stream);
// synchronous on `stream`, at scene upload; dev_scratch holds kMaxZones ints
int computeZoneGoalTris(const SceneDev &sc, int32_t *dev_scratch, int32_t *host_out, void *stream);
int launchTraceRays(const SceneDev &sc, const float *o, const float *d, int n, int mode, float *t, int32_t *hit,
                    void *stream);
int launchDebugGather(const DevState &s, float *af, int32_t *ai, int32_t *wi, float *wf, uint32_t *explore,
                      float *crumbs, void *stream);
int launchFillActions(const DevState &s, const int32_t *src6, void *stream);
int launchCombatActions(const DevState &s, const int32_t *tape6, int32_t *out6, int32_t mode, void *stream);
int computeSceneFrames(SceneTables *d_tab, void *stream); // fills zoneFrame / goalFrame in place

// Batched device copies (wire.hip): up to kMaxCopySegs segments in one
// launch; src == nullptr zero-fills.  Pointers must be 16-B aligned.
constexpr int kMaxCopySegs = 32;
struct CopySeg {
    const void *src;
    void *dst;
    int64_t bytes;
};
struct CopyBatch {
    CopySeg seg[kMaxCopySegs];
    int n;
    int64_t first[kMaxCopySegs + 1]; // first block of each segment (filled by launchCopyBatch)
    // gpuStreamStep's out table rides the copy launches: block 0 stores
    // `tab` to *tabDst (null: nothing), so setting it before the step and
    // clearing it after costs no launch of its own
    OutTab *tabDst;
    OutTab tab;
};
int launchCopyBatch(const CopyBatch &b, void *stream);

// Learner-exchange wire format (wire.hip)
int64_t wireBytes(const DevState &s, bool keyframe);
int launchWirePack(const DevState &s, char *dst, bool keyframe, uint32_t worldOffset, void *stream);
// epPrev / epNext: the shadow's double-buffered copies of the previous and
// this message's episode counters ([W] each, swapped by the caller per unpack)
int launchWireErrClear(uint32_t *err, void *stream); // keeps only the desync bit
int launchWireUnpack(const DevState &s, const SceneDev &sc, const char *src, bool keyframe, uint32_t *err,
                     uint32_t worldOffset, const int32_t *epPrev, int32_t *epNext, void *stream);

} // namespace mpenv
