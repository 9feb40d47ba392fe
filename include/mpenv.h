/*
 * mpenv.h — C ABI of the MI355X-native madrona-mp-env engine.
 *
 * Drop-in boundary for the world-batched Zone step.  Every entry point maps
 * to a method of the reference's Manager class (src/mgr.hpp:31-161) or its
 * Python binding (src/bindings.cpp:11-160); the cited lines are what each
 * function replaces.  Plain pointers and sizes only — no torch/HIP types in
 * the signatures (the stream is passed as an opaque hipStream_t pointer).
 *
 * Errors: every int-returning function returns 0 on success and a negative
 * MPENV_ERR_* code on failure; mpenv_last_error() gives the message.  The
 * reference FATALs on I/O failure (mgr.cpp:205,214) and asserts otherwise.
 */
#ifndef MPENV_H
#define MPENV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPENV_ABI_VERSION 1

/* Error codes */
#define MPENV_OK 0
#define MPENV_ERR_INVALID -1
#define MPENV_ERR_IO -2
#define MPENV_ERR_HIP -3
#define MPENV_ERR_UNSUPPORTED -4

/* ExecMode (madrona::ExecMode, used at scripts/jax_train.py:111).  This build
 * is HIP-only: MPENV_EXEC_CPU is rejected with MPENV_ERR_UNSUPPORTED (no
 * silent CPU fallback). */
#define MPENV_EXEC_CPU 0
#define MPENV_EXEC_CUDA 1 /* = HIP on gfx950 */

/* Task (types.hpp:45-51) */
#define MPENV_TASK_EXPLORE 0
#define MPENV_TASK_TDM 1
#define MPENV_TASK_ZONE 2
#define MPENV_TASK_TURRET 3
#define MPENV_TASK_ZONE_CAPTURE_DEFEND 4

/* SimFlags (sim_flags.hpp:7-20) */
#define MPENV_SIMFLAG_DEFAULT 0u
#define MPENV_SIMFLAG_SPAWN_IN_MIDDLE (1u << 0)
#define MPENV_SIMFLAG_RANDOMIZE_HP_MAGAZINE (1u << 1)
#define MPENV_SIMFLAG_NAVMESH_SPAWN (1u << 2)
#define MPENV_SIMFLAG_NO_RESPAWN (1u << 3)
#define MPENV_SIMFLAG_STAGGER_STARTS (1u << 4)
#define MPENV_SIMFLAG_ENABLE_CURRICULUM (1u << 5)
#define MPENV_SIMFLAG_HARDCODED_SPAWNS (1u << 6)
#define MPENV_SIMFLAG_RANDOM_FLIP_TEAMS (1u << 7)
#define MPENV_SIMFLAG_STATIC_FLIP_TEAMS (1u << 8)
#define MPENV_SIMFLAG_FULL_TEAM_POLICY (1u << 9)
#define MPENV_SIMFLAG_SIM_EVAL_MODE (1u << 10)
#define MPENV_SIMFLAG_SUB_ZONES (1u << 11)

/* ExportID (sim.hpp:15-66), same numbering. */
enum mpenv_export_id {
    MPENV_EXPORT_RESET = 0,
    MPENV_EXPORT_WORLD_CURRICULUM = 1,
    MPENV_EXPORT_EXPLORE_ACTION = 2,
    MPENV_EXPORT_PVP_DISCRETE_ACTION = 3,
    MPENV_EXPORT_PVP_AIM_ACTION = 4,
    MPENV_EXPORT_PVP_DISCRETE_AIM_ACTION = 5,
    MPENV_EXPORT_REWARD = 6,
    MPENV_EXPORT_DONE = 7,
    MPENV_EXPORT_MATCH_RESULT = 8,
    MPENV_EXPORT_AGENT_POLICY = 9,
    MPENV_EXPORT_SELF_OBSERVATION = 10,
    MPENV_EXPORT_TEAMMATE_OBSERVATIONS = 11,
    MPENV_EXPORT_OPPONENT_OBSERVATIONS = 12,
    MPENV_EXPORT_OPPONENT_LAST_KNOWN_OBSERVATIONS = 13,
    MPENV_EXPORT_SELF_POSITION = 14,
    MPENV_EXPORT_TEAMMATE_POSITIONS = 15,
    MPENV_EXPORT_OPPONENT_POSITIONS = 16,
    MPENV_EXPORT_OPPONENT_LAST_KNOWN_POSITIONS = 17,
    MPENV_EXPORT_OPPONENT_MASKS = 18,
    MPENV_EXPORT_FWD_LIDAR = 19,
    MPENV_EXPORT_REAR_LIDAR = 20,
    MPENV_EXPORT_AGENT_MAP = 21,
    MPENV_EXPORT_UNMASKED_AGENT_MAP = 22,
    MPENV_EXPORT_HP = 23,
    MPENV_EXPORT_ALIVE = 24,
    MPENV_EXPORT_MAGAZINE = 25,
    MPENV_EXPORT_FULL_TEAM_ACTIONS = 26,
    MPENV_EXPORT_FULL_TEAM_GLOBAL = 27,
    MPENV_EXPORT_FULL_TEAM_PLAYERS = 28,
    MPENV_EXPORT_FULL_TEAM_ENEMIES = 29,
    MPENV_EXPORT_FULL_TEAM_LAST_KNOWN_ENEMIES = 30,
    MPENV_EXPORT_FULL_TEAM_FWD_LIDAR = 31,
    MPENV_EXPORT_FULL_TEAM_REAR_LIDAR = 32,
    MPENV_EXPORT_FULL_TEAM_REWARD = 33,
    MPENV_EXPORT_FULL_TEAM_DONE = 34,
    MPENV_EXPORT_FULL_TEAM_POLICY_ASSIGNMENTS = 35,
    MPENV_EXPORT_EVENT_LOG = 36,
    MPENV_EXPORT_PACKED_STEP_SNAPSHOT = 37,
    MPENV_EXPORT_FILTERS_STATE = 38,
    MPENV_EXPORT_REWARD_HYPER_PARAMS = 39,
    MPENV_NUM_REFERENCE_EXPORTS = 40,

    /* Extensions (not in the reference ExportID): */
    MPENV_EXPORT_SIM_CONTROL = 64,   /* TrainControl i32[3] (mgr.cpp:1975-1978) */
    MPENV_EXPORT_DEBUG_AGENT_F32 = 65, /* [A][MPENV_DBG_AF_COUNT] internal state */
    MPENV_EXPORT_DEBUG_AGENT_I32 = 66, /* [A][MPENV_DBG_AI_COUNT] */
    MPENV_EXPORT_DEBUG_WORLD_I32 = 67, /* [W][MPENV_DBG_WI_COUNT] */
    MPENV_EXPORT_DEBUG_WORLD_F32 = 68, /* [W][MPENV_DBG_WF_COUNT] */
    MPENV_EXPORT_DEBUG_EXPLORE = 69,   /* [A][81*81] u32: 1 = cell visited in the agent's
                                          current episode (ExploreTracker.visited == curEpisodeIdx) */
    MPENV_EXPORT_DEBUG_CRUMBS = 70,    /* [W][MPENV_MAX_CRUMBS][8] f32 breadcrumb pool */
    MPENV_EXPORT_RECORD_LOG = 71,      /* [W] mpenv_step_log as i32[W][217] (record mode) */
    MPENV_EXPORT_REPLAY_LOG = 72,      /* [W] mpenv_step_log as i32[W][217] (replay mode) */
    MPENV_EXPORT_SNAPSHOT_WRITTEN = 73 /* [W][1] i32: snapshot written this step (event log) */
};
/* FULL_TEAM_* (26-35): one row per (world, team) = [W * 2], six player slots
 * (slots >= team_size stay zero), floats per slot (types.hpp:1048-1100):
 *   common (24): isValid, id[6] (one-hot slot), isAlive, global xyz
 *     (normalised, unclamped), facing yaw, pitch, velocity xyz (world frame),
 *     stand[7] (cur S/C/P, tgt S/C/P, transition), inZone
 *   player = common + hp/100, bullets/30, isReloading, autoheal fraction
 *   enemy  = common + wasHit, firedShot, hasLOS[6] (per own slot), teamKnowsLocation
 *   global (16): teamID[2], fraction of match remaining, zone: center xyz,
 *     mine / enemy controlling, contested, captured, steps until point,
 *     steps remaining, id[4]
 * FULL_TEAM_FWD/REAR_LIDAR hold the agents' lidar as of the previous step
 * (the reference copies it before pvpLidarSystem runs).  FULL_TEAM_ACTIONS
 * and FULL_TEAM_POLICY_ASSIGNMENTS are inputs the step never reads
 * (readFullTeamActionsPolicies is compiled out, sim.cpp:4928-4957). */
#define MPENV_FT_COMMON_DIM 24
#define MPENV_FT_PLAYER_DIM 28
#define MPENV_FT_ENEMY_DIM 33
#define MPENV_FT_GLOBAL_DIM 16

/* EVENT_LOG (36): this step's GameEvent slots as i32[W][2N+1][6] (slot 2i, 2i+1
 * = agent i's reload / shot / kill, slot 2N = capture; type 0 = empty).
 * PACKED_STEP_SNAPSHOT (37): i32[W][48] mpenv_packed_step_snapshot.  Both
 * exist only when an event log directory is configured. */

/* Debug-state column layouts (parity tests compare these bit-exactly). */
enum mpenv_dbg_agent_f32 {
    MPENV_DBG_AF_POS = 0,     /* 3 */
    MPENV_DBG_AF_VEL = 3,     /* 3 */
    MPENV_DBG_AF_ROT = 6,     /* 4 (w,x,y,z) */
    MPENV_DBG_AF_AIM = 10,    /* yaw, pitch, rot w,x,y,z */
    MPENV_DBG_AF_MAXVEL = 16,
    MPENV_DBG_AF_MINDIST_ZONE = 17,
    MPENV_DBG_AF_FIRED_T = 18,
    MPENV_DBG_AF_BC_PENALTY = 19,
    MPENV_DBG_AF_START = 20,  /* 3 */
    MPENV_DBG_AF_MINDIST_SUBZONE = 23,
    MPENV_DBG_AF_COUNT = 24
};
enum mpenv_dbg_agent_i32 {
    MPENV_DBG_AI_CUR_POSE = 0,
    MPENV_DBG_AI_TGT_POSE = 1,
    MPENV_DBG_AI_TRANSITION = 2,
    MPENV_DBG_AI_RNG_A = 3,
    MPENV_DBG_AI_RNG_B = 4,
    MPENV_DBG_AI_RNG_CTR = 5,
    MPENV_DBG_AI_LANDED_ON = 6,     /* agent index in world, or -1 */
    MPENV_DBG_AI_RESPAWN_STEPS = 7,
    MPENV_DBG_AI_AUTOHEAL_STEPS = 8,
    MPENV_DBG_AI_FLAGS = 9,         /* bit0 successfulKill, 1 wasKilled, 2 inZone, 3 hasDied, 4 reloadedFullMag, 5 inSubZone */
    MPENV_DBG_AI_WAS_SHOT = 10,
    MPENV_DBG_AI_WEAPON = 11,
    MPENV_DBG_AI_BC_LAST = 12,
    MPENV_DBG_AI_BC_STEPS = 13,
    MPENV_DBG_AI_CANSEE = 14,       /* bitmask over opponents */
    MPENV_DBG_AI_NEW_CELLS = 15,
    MPENV_DBG_AI_COUNT = 16
};
enum mpenv_dbg_world_i32 {
    MPENV_DBG_WI_TEAM_A = 0,
    MPENV_DBG_WI_CUR_STEP = 1,
    MPENV_DBG_WI_FINISHED = 2,
    MPENV_DBG_WI_CUR_ZONE = 3,
    MPENV_DBG_WI_CONTROLLING = 4,
    MPENV_DBG_WI_CONTESTED = 5,
    MPENV_DBG_WI_CAPTURED = 6,
    MPENV_DBG_WI_EARNED = 7,
    MPENV_DBG_WI_ZONE_STEPS = 8,
    MPENV_DBG_WI_STEPS_UNTIL_POINT = 9,
    MPENV_DBG_WI_EPISODE = 10,
    MPENV_DBG_WI_EPISODE_COUNTER = 11,
    MPENV_DBG_WI_RNG_A = 12,
    MPENV_DBG_WI_RNG_B = 13,
    MPENV_DBG_WI_RNG_CTR = 14,
    MPENV_DBG_WI_NUM_CRUMBS = 15,
    MPENV_DBG_WI_FILTER_ACTIVE0 = 16,
    MPENV_DBG_WI_FILTER_ACTIVE1 = 17,
    MPENV_DBG_WI_FILTER_LAST0 = 18,
    MPENV_DBG_WI_FILTER_LAST1 = 19,
    MPENV_DBG_WI_CRUMB_OVERFLOW = 20,
    MPENV_DBG_WI_SUBZONES = 21,     /* 4 bits per sub-zone k at 4k: controlling team + 1, contested << 2, captured << 3 */
    MPENV_DBG_WI_COUNT = 22
};
enum mpenv_dbg_world_f32 {
    MPENV_DBG_WF_TEAM_REWARD0 = 0,
    MPENV_DBG_WF_TEAM_REWARD1 = 1,
    MPENV_DBG_WF_GOAL_MIN0 = 2,
    MPENV_DBG_WF_GOAL_MIN1 = 3,
    MPENV_DBG_WF_GOAL_TEAM0 = 4,
    MPENV_DBG_WF_GOAL_TEAM1 = 5,
    MPENV_DBG_WF_COUNT = 6
};

/* Fixed-capacity per-world breadcrumb pool (reference: dynamic
 * BreadcrumbEntity archetype, sim.cpp:4845-4926).  Live crumbs per world are
 * bounded by ~6 per agent; creations beyond capacity are
 * dropped and counted in MPENV_DBG_WI_CRUMB_OVERFLOW. */
#define MPENV_MAX_CRUMBS 128

/* ---- Record / replay / event-log wire formats ----
 * Byte-compatible with the reference's structs (little-endian, natural
 * alignment), so files written here and by the reference interchange. */

/* AgentLogData (types.hpp:574-584): 72 bytes */
typedef struct mpenv_agent_log {
    float position[3];
    float aim_yaw, aim_pitch;
    float aim_rot[4];          /* Quat w, x, y, z */
    float hp;
    int32_t mag_num_bullets, mag_is_reloading;
    int32_t cur_pose, tgt_pose, transition_remaining; /* StandState */
    int32_t shot_agent_idx;    /* -1 = none */
    float fired_shot_t;
    uint8_t was_killed, successful_kill;
    uint8_t pad_[2];
} mpenv_agent_log;

/* StepLog (types.hpp:586-589): 868 bytes, one per world per step in the
 * record / replay file (world-major). */
typedef struct mpenv_step_log {
    mpenv_agent_log agents[12];
    int32_t cur_step;
} mpenv_step_log;

/* EventType (types.hpp:614-620) */
#define MPENV_EVENT_CAPTURE 1u
#define MPENV_EVENT_RELOAD 2u
#define MPENV_EVENT_KILL 4u
#define MPENV_EVENT_PLAYER_SHOT 8u

/* GameEvent (types.hpp:729-760): 24 bytes.  a/b/c16 hold the union:
 *   Capture    {u8 zoneIDX, u8 captureTeam, u16 inZoneMask}
 *   Reload     {u8 player,  u8 numBulletsAtReloadTime}
 *   Kill       {u8 killer,  u8 killed}
 *   PlayerShot {u8 attacker, u8 target}
 * Player ids are team * 6 + offset within the team. */
typedef struct mpenv_game_event {
    uint32_t type;
    uint32_t pad_;
    uint64_t match_id;
    uint32_t step;
    uint8_t a, b;
    uint16_t c16;
} mpenv_game_event;

/* PackedPlayerSnapshot (types.hpp:603-612): 14 bytes */
typedef struct mpenv_packed_player {
    int16_t pos[3];
    int16_t yaw, pitch;
    uint8_t mag_num_bullets, is_reloading, hp, flags; /* flags: 2 FiredShot, 4 Crouch, 8 Prone */
} mpenv_packed_player;

/* PackedStepSnapshot (types.hpp:622-636): 192 bytes, one per world per step
 * in steps.bin. */
typedef struct mpenv_packed_step_snapshot {
    uint32_t num_events;       /* the reference stores a 0/1 "any event" flag */
    uint32_t event_mask;
    uint64_t match_id;
    uint16_t step;
    uint8_t cur_zone;
    int8_t cur_zone_controller;
    uint16_t zone_steps_remaining;
    uint16_t steps_until_point;
    mpenv_packed_player players[12];
} mpenv_packed_step_snapshot;

/* CurriculumSnapshot (types.hpp:816-819): 176 bytes.  A curriculum_data_path
 * file is a bare array of them (mgr.cpp:1424-1441; size / 176 snapshots),
 * e.g. the match state + players of steps.bin records. */
typedef struct mpenv_curriculum_snapshot {
    uint16_t step;
    uint8_t cur_zone;
    int8_t cur_zone_controller;
    uint16_t zone_steps_remaining;
    uint16_t steps_until_point;
    mpenv_packed_player players[12];
} mpenv_curriculum_snapshot;

#ifdef __cplusplus
static_assert(sizeof(mpenv_curriculum_snapshot) == 176, "CurriculumSnapshot layout");
static_assert(sizeof(mpenv_agent_log) == 72, "AgentLogData layout");
static_assert(sizeof(mpenv_step_log) == 868, "StepLog layout");
static_assert(sizeof(mpenv_game_event) == 24, "GameEvent layout");
static_assert(sizeof(mpenv_packed_player) == 14, "PackedPlayerSnapshot layout");
static_assert(sizeof(mpenv_packed_step_snapshot) == 192, "PackedStepSnapshot layout");
#endif

/* Tensor element types (madrona::py::TensorElementType subset) */
#define MPENV_DTYPE_INT32 0
#define MPENV_DTYPE_FLOAT32 1
#define MPENV_DTYPE_UINT32 2

typedef struct mpenv_config {
    int32_t exec_mode;          /* MPENV_EXEC_* */
    int32_t gpu_id;
    uint32_t num_worlds;        /* worlds owned by this manager */
    uint32_t rand_seed;
    int32_t auto_reset;
    uint32_t sim_flags;
    int32_t task_type;          /* MPENV_TASK_* (only ZONE is implemented) */
    uint32_t team_size;         /* 1..6 */
    uint32_t num_pbt_policies;
    uint32_t policy_history_size;
    const char *scene_path;     /* dir with collisions/navmesh/spawns/zones.bin */
    int32_t train_flank;
    const char *replay_log_path;     /* NULL = none */
    const char *record_log_path;     /* NULL = none */
    const char *event_log_path;      /* NULL = none */
    const char *curriculum_data_path;/* NULL = none */
    /* Extension for sharding worlds across GPUs: the global index of this
     * manager's world 0.  RNG keys use global world IDs (sim.cpp:743-746),
     * so a shard reproduces exactly the worlds of a single big run. */
    uint32_t world_id_offset;
} mpenv_config;

typedef struct mpenv_manager mpenv_manager;

/* Manager::Manager (mgr.hpp:57-58 / mgr.cpp:1914-1919) */
int mpenv_create(const mpenv_config *cfg, mpenv_manager **out);
/* Manager::~Manager (mgr.cpp:1921) */
void mpenv_destroy(mpenv_manager *mgr);
/* Manager::init (mgr.cpp:1923-1946): forced reset of every world + Init graph */
int mpenv_init(mpenv_manager *mgr);
/* Manager::step (mgr.cpp:1948-1951): one synchronous world-batched step */
int mpenv_step(mpenv_manager *mgr);
/* Asynchronous step on a caller-owned hipStream_t (no host sync). */
int mpenv_step_async(mpenv_manager *mgr, void *hip_stream);
/* Manager::gpuStreamInit / gpuStreamStep (mgr.cpp:507-645): XLA custom-call
 * ABI.  buffers = TrainInterface inputs then outputs, in the order of
 * mpenv_train_interface(). */
int mpenv_gpu_stream_init(mpenv_manager *mgr, void *hip_stream, void **buffers);
int mpenv_gpu_stream_step(mpenv_manager *mgr, void *hip_stream, void **buffers);

/* The XLA GPU custom-call targets behind SimManager.jax() (reference:
 * madrona::py::JAXInterface::buildEntry over gpuStreamInit / gpuStreamStep,
 * src/bindings.cpp:149-158, src/mgr.cpp:507-645).  XLA's GPU custom-call
 * signature, API version 1 ("original"): buffers = the call's operands then
 * its results -- the flat trainInterface array of mpenv_gpu_stream_* (inputs
 * then outputs, mpenv_train_interface order); opaque = the bytes of an
 * mpenv_xla_opaque naming the manager (mpenv_xla_opaque_make).  The opaque
 * is checked against the live managers before use (a destroyed manager is
 * an error, not a read of freed memory).  API version 1 has no error return:
 * like the reference's REQ_CUDA / FATAL (mgr.cpp:514-531, 620-638) a bad
 * opaque or a failed launch prints "mpenv: XLA custom call ... failed: <why>"
 * on stderr and aborts.  The *_status variants take XLA's
 * API_VERSION_STATUS_RETURNING signature (a trailing XlaCustomCallStatus *)
 * and report the failure through XlaCustomCallStatusSetFailure, resolved at
 * run time from the XLA runtime loaded in the process (counted in
 * mpenv_xla_errors()); when that symbol is absent they abort as above. */
typedef struct mpenv_xla_opaque {
    uint32_t magic;   /* MPENV_XLA_MAGIC */
    uint32_t version; /* MPENV_XLA_VERSION */
    uint64_t manager; /* mpenv_manager * */
    int32_t num_buffers; /* trainInterface inputs + outputs */
    int32_t reserved;
} mpenv_xla_opaque;
#define MPENV_XLA_MAGIC 0x4a4c4d58u /* "XMLJ" */
#define MPENV_XLA_VERSION 1u
int mpenv_xla_opaque_make(mpenv_manager *mgr, mpenv_xla_opaque *out);
void mpenv_xla_gpu_stream_init(void *hip_stream, void **buffers, const char *opaque, size_t opaque_len);
void mpenv_xla_gpu_stream_step(void *hip_stream, void **buffers, const char *opaque, size_t opaque_len);
void mpenv_xla_gpu_stream_init_status(void *hip_stream, void **buffers, const char *opaque, size_t opaque_len,
                                      void *xla_status);
void mpenv_xla_gpu_stream_step_status(void *hip_stream, void **buffers, const char *opaque, size_t opaque_len,
                                      void *xla_status);
int64_t mpenv_xla_errors(void);

/* Manager::*Tensor() getters (mgr.cpp:1965-2381): zero-copy view of an
 * engine-owned buffer.  dims must hold 8 entries. gpu_id = -1 for host. */
int mpenv_export_tensor(mpenv_manager *mgr, int32_t export_id, void **ptr,
                        int32_t *dtype, int32_t *ndim, int64_t *dims,
                        int32_t *gpu_id);

/* TrainInterface (mgr.cpp:2383-2431): number of named inputs / outputs and
 * their (name, export id).  Index order is the gpuStream buffers order. */
int mpenv_train_interface_size(int32_t *num_inputs, int32_t *num_outputs);
int mpenv_train_interface_entry(int32_t is_output, int32_t idx,
                                const char **name, int32_t *export_id);

/* Step-input copy (TrainInterface::cudaCopyStepInputs of gpuStreamStep,
 * mgr.cpp:625) from a device buffer laid out [A][6] i32 (4 discrete +
 * 2 discrete-aim actions per agent), asynchronous on hip_stream. */
int mpenv_copy_actions(mpenv_manager *mgr, const int32_t *src_device, void *hip_stream);

/* Extension (synthetic action source for benchmarks and tests; no reference
 * counterpart): the tape rows tape_device [A][6] i32 overridden by a greedy
 * aim-bot computed from the engine's current observations (opponent masks
 * and relative yaw / pitch; mode 1 also turns and runs toward the zone when
 * no opponent is visible).  out_device [A][6] i32, or null to write the
 * step-input columns directly (as mpenv_copy_actions would).  Asynchronous
 * on hip_stream. */
int mpenv_combat_actions(mpenv_manager *mgr, const int32_t *tape_device, int32_t *out_device, int32_t mode,
                         void *hip_stream);

/* Test hook (no reference counterpart): closest-hit BVH queries
 * (MeshBVH::traceRay, mesh_bvh.inl:110-208) for n caller rays in device
 * memory (o, d: [n][3] f32).  mode 0 = the traversal inlined in the step
 * kernels, 1 = an out-of-line copy.  Outputs t (0 on miss) and hit. */
int mpenv_debug_trace_rays(mpenv_manager *mgr, const float *o_device, const float *d_device, int32_t n,
                           int32_t mode, float *t_device, int32_t *hit_device, void *hip_stream);

/* Extension, the learner exchange's compact wire format (DESIGN.md §6;
 * replaces shipping the trainInterface outputs of mgr.cpp:2383-2431 as they
 * are exported, 3,924 B per agent, with ~477 B per agent + 160 B per world).
 * pack: one message of this step's outputs into dst (device memory of
 * mpenv_wire_bytes bytes), asynchronous on hip_stream; keyframe != 0 also
 * carries the last-known rows (the first message of an exchange).
 * unpack: on the learner, into a manager of the same configuration (the
 * sender's shadow): the lidar, rewards and other per-agent outputs, then the
 * observation system reading the message's state columns in place, so every
 * trainInterface output of the shadow equals the sender's bit for bit (the
 * shadow's internal state columns and full-team rows are not rebuilt: they
 * are not trainInterface outputs).  Message buffers must be 16-B aligned;
 * the buffer must stay unmodified until the unpack has run on hip_stream.
 * A message for another
 * configuration or shard (header world offset != the shadow's
 * world_id_offset), of the other kind, or one whose values did not fit the
 * packed fields is not unpacked; it raises MPENV_WIRE_ERR_REFUSED and
 * MPENV_WIRE_ERR_DESYNC in the error word mpenv_wire_error returns (it
 * synchronises the device).  The read clears REFUSED; DESYNC stays set --
 * later plain messages are refused too (REFUSED again) and the shadow's
 * observation rows are not rebuilt -- until a keyframe is unpacked. */
#define MPENV_WIRE_ERR_REFUSED 1u
#define MPENV_WIRE_ERR_DESYNC 2u
int mpenv_wire_bytes(mpenv_manager *mgr, int32_t keyframe, int64_t *bytes);
int mpenv_wire_pack(mpenv_manager *mgr, void *dst_device, int32_t keyframe, void *hip_stream);
int mpenv_wire_unpack(mpenv_manager *mgr, const void *src_device, int32_t keyframe, void *hip_stream);
int mpenv_wire_error(mpenv_manager *mgr, uint32_t *out);
/* The same read without a device synchronisation: ordered on hip_stream
 * (the stream the shadow's unpacks run on); with `out` in pinned host memory
 * the call returns at once and *out holds the word once the stream has
 * reached the read (record an event after it).  Clears REFUSED like
 * mpenv_wire_error. */
int mpenv_wire_error_async(mpenv_manager *mgr, uint32_t *out, void *hip_stream);

/* Measurement hook: how many times the Step graph has been captured (the
 * graph is re-captured whenever a kernel argument struct changes: world
 * groups, stats or timing buffers; every other step replays it). */
int mpenv_graph_captures(mpenv_manager *mgr, int64_t *out);
/* Whether steps replay the captured graph (1) or launch kernel by kernel
 * (0), and why not: a capture that fails (capture invalidated, unjoined
 * fork, end-capture or instantiate error) is abandoned -- the step runs its
 * kernels directly -- and the reason is kept here (reason: a buffer of
 * reason_len bytes, may be null). */
int mpenv_graph_status(mpenv_manager *mgr, int32_t *graph_on, char *reason, int32_t reason_len);

/* Extension: step the worlds as `groups` contiguous ranges on concurrent
 * HIP streams (fork/join on the step stream; results identical for any
 * split).  Default 1 (round 5: one group measured fastest); env
 * MPENV_WORLD_GROUPS overrides at creation.  Capped at 3. */
int mpenv_set_world_groups(mpenv_manager *mgr, int32_t groups);
int mpenv_world_groups(mpenv_manager *mgr, int32_t *groups);
/* Extension: with one world group, run k_lidar on a branch stream beside
 * k_vis -> k_obs (fork after k_sim, join at the end of the step; results
 * identical).  Default off; env MPENV_LIDAR_BRANCH=1 at creation. */
int mpenv_set_lidar_branch(mpenv_manager *mgr, int32_t on);

/* Manager::triggerReset (mgr.cpp:2484-2500) */
int mpenv_trigger_reset(mpenv_manager *mgr, int32_t world_idx);
/* Manager::setPvPAction (mgr.cpp:2518-2566) */
int mpenv_set_pvp_action(mpenv_manager *mgr, int32_t world_idx, int32_t agent_idx,
                         const int32_t discrete[4], const float aim[2],
                         const int32_t aim_discrete[2]);
/* Manager::setHP (mgr.cpp:2585-2601) */
int mpenv_set_hp(mpenv_manager *mgr, int32_t world_idx, int32_t agent_idx, int32_t hp);
/* Manager::setAgentPolicy / setUniformAgentPolicy (mgr.cpp:2619-2658) */
int mpenv_set_agent_policy(mpenv_manager *mgr, int32_t world_idx, int32_t agent_idx,
                           int32_t policy);
int mpenv_set_uniform_agent_policy(mpenv_manager *mgr, int32_t policy);
/* Manager::isReplayFinished (mgr.cpp:2603-2617) */
int mpenv_is_replay_finished(mpenv_manager *mgr, int32_t *finished);

/* Number of worlds / agents per world of a manager. */
int mpenv_dims(mpenv_manager *mgr, int32_t *num_worlds, int32_t *agents_per_world);

/* Measurement hook: average device time (ms) of each step kernel over the
 * steps since the last call, measured with HIP events on the step stream.
 * names[i] point to static strings.  Returns the number of kernels. */
int mpenv_kernel_timings(mpenv_manager *mgr, int32_t max_n, const char **names,
                         float *avg_ms, int32_t *launches);
int mpenv_enable_kernel_timing(mpenv_manager *mgr, int32_t enable);

/* Measurement hook (no reference counterpart): per-step workload counters
 * accumulated by the step kernels while enabled (enabling zeroes them):
 * [0] alive agents at k_move, [1] (viewer, opponent) pairs both alive,
 * [2] visibility rays after the view / frustum tests, [3] visibility rays
 * that saw their target, [4] sphere casts, [5] shot rays, [6] agents that
 * took damage, [7] agents killed, [8] last-known observation rows written by
 * the observation system, [9] visibility rays that needed a BVH traversal
 * (not decided by the target-capsule test or the occluder hint).
 * read_stats copies min(n, 10) counters and returns the number of counters
 * (10). */
int mpenv_enable_stats(mpenv_manager *mgr, int32_t enable);
int mpenv_read_stats(mpenv_manager *mgr, uint64_t *out, int32_t n);

/* Scene BVH as the engine builds it (map_importer.cpp:364-419 replacement):
 * 64-byte nodes and float3 vertices (3 per triangle).  Call with null
 * outputs to query sizes.  Used by the parity oracle and tests. */
int mpenv_scene_bvh(const char *scene_path, void *nodes_out, int32_t *num_nodes,
                    float *verts_out, int32_t *num_verts, int32_t *max_stack);
/* k_lidar's own tree of the scene's triangles (scene.h lidarBVHOpts), same
 * format: closest hits are tree-independent up to coplanar ties, so the
 * lidar walks a tree built for its near-horizontal fans. */
int mpenv_scene_lidar_bvh(const char *scene_path, void *nodes_out, int32_t *num_nodes,
                          float *verts_out, int32_t *num_verts, int32_t *max_stack);
/* The same for another build of the scene's triangles (scene.h
 * BVHBuildOpts): opts[0] max leaf size (1-2), [1] SAH bins (0 = full sweep),
 * [2] measure (0 surface area, 1 lidar-weighted), [3] traversal cost x 100,
 * [4] the lidar measure's floor weight x 100, then pairs (heap index of a
 * binary build node, root 1; rank of the SAH candidate split to take there,
 * BVHBuildOpts::splitRank); missing entries keep the defaults.  For
 * tools/trav_stats.cpp (tree models and the TRAV_TUNE search). */
int mpenv_scene_bvh_variant(const char *scene_path, const int32_t *opts, int32_t num_opts, void *nodes_out,
                            int32_t *num_nodes, float *verts_out, int32_t *num_verts, int32_t *max_stack);

/* The sphere-cast quirk guard k_move uses (scene.h quirkGrid, radius 15,
 * margin 2, 16-unit cells): header[0..2] = minX, minY, cell (float bits),
 * header[3..4] = w, h; bits [ceil(w*h/32)] row-major.  Pass *num_words = 0
 * to query the size.  For tests. */
int mpenv_scene_quirk_grid(const char *scene_path, int32_t *header_out, uint32_t *bits_out, int32_t *num_words);

/* Host-side navmesh (Navmesh::initFromPolygons, mgr.cpp:1301-1327) and A*
 * next-hop table (buildAStarLookup, mgr.cpp:1155-1211) of a scene, for
 * tests and the oracle.  Two-call pattern: pass *num_tris = 0 to query the
 * count; with *num_tris >= T fills tri_verts [T][3][3], adj [T][3] and
 * astar [T][T] (each optional). */
int mpenv_scene_navmesh(const char *scene_path, float *tri_verts_out, int32_t *num_tris, int32_t *adj_out,
                        int32_t *astar_out);

const char *mpenv_last_error(void);
int32_t mpenv_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* MPENV_H */
