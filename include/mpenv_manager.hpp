// mpenv_manager.hpp — the reference's C++ Manager class (src/mgr.hpp:14-161)
// over the C ABI of mpenv.h, header-only, for C++ callers (headless/viewer
// style programs) that were written against madronaMPEnv::Manager.
//
// Same names, Config fields and method set; differences:
//   * madrona::py::Tensor -> madronaMPEnv::Tensor (ptr, type, dims, gpu id),
//     still a zero-copy view of engine-owned device memory (mgr.cpp:295-301).
//   * Errors throw std::runtime_error (the reference FATALs / asserts).
//   * Out of scope, declared with the reference's signatures
//     so callers written against mgr.hpp compile, and throwing
//     std::runtime_error when called: ExecMode::CPU (rejected at
//     construction), a non-null VizState* (the viewer), vizStep,
//     getWorldContext (Madrona's per-world ECS context, opaque Engine here),
//     setExploreAction and setCoarsePvPAction (Task::Explore and the
//     coarse-action path, neither on the Zone step graph).  Full-team
//     tensors, record/replay and event logs are implemented (fullTeam*Tensor
//     getters, Config log paths).  cpuJAXInit/Step are no-ops as in mgr.hpp.
//   * gpuStreamInit/Step take the HIP stream as void*.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "mpenv.h"

namespace madronaMPEnv {

enum class ExecMode : int32_t { CPU = MPENV_EXEC_CPU, CUDA = MPENV_EXEC_CUDA };

// types.hpp:45-51
enum class Task : uint32_t { Explore = 0, TDM = 1, Zone = 2, Turret = 3, ZoneCaptureDefend = 4 };

// sim_flags.hpp:7-20
enum class SimFlags : uint32_t {
    Default = 0,
    SpawnInMiddle = MPENV_SIMFLAG_SPAWN_IN_MIDDLE,
    RandomizeHPMagazine = MPENV_SIMFLAG_RANDOMIZE_HP_MAGAZINE,
    NavmeshSpawn = MPENV_SIMFLAG_NAVMESH_SPAWN,
    NoRespawn = MPENV_SIMFLAG_NO_RESPAWN,
    StaggerStarts = MPENV_SIMFLAG_STAGGER_STARTS,
    EnableCurriculum = MPENV_SIMFLAG_ENABLE_CURRICULUM,
    HardcodedSpawns = MPENV_SIMFLAG_HARDCODED_SPAWNS,
    RandomFlipTeams = MPENV_SIMFLAG_RANDOM_FLIP_TEAMS,
    StaticFlipTeams = MPENV_SIMFLAG_STATIC_FLIP_TEAMS,
    FullTeamPolicy = MPENV_SIMFLAG_FULL_TEAM_POLICY,
    SimEvalMode = MPENV_SIMFLAG_SIM_EVAL_MODE,
    SubZones = MPENV_SIMFLAG_SUB_ZONES,
};
inline SimFlags operator|(SimFlags a, SimFlags b) { return SimFlags((uint32_t)a | (uint32_t)b); }
inline SimFlags &operator|=(SimFlags &a, SimFlags b) { return a = a | b; }
inline SimFlags operator&(SimFlags a, SimFlags b) { return SimFlags((uint32_t)a & (uint32_t)b); }

struct Vector3 {
    float x, y, z;
    static Vector3 zero() { return { 0.f, 0.f, 0.f }; }
};

// Action components (types.hpp:173-183) and AgentPolicy.
struct PvPDiscreteAction { int32_t moveAmount, moveAngle, fire, stand; };
struct PvPAimAction { float yaw, pitch; };
struct PvPDiscreteAimAction { int32_t yaw, pitch; };
struct AgentPolicy { int32_t idx; };
struct ExploreAction { int32_t moveAmount, moveAngle, rotate, mantle; }; // types.hpp:166-171
struct CoarsePvPAction { int32_t moveAmount, moveAngle, facing; };       // types.hpp:205-209

// Opaque: the viewer's state (viz.hpp:16) and Madrona's per-world context
// (mgr.hpp:130); neither exists in this engine.
struct VizState;
struct Engine;

// mgr.hpp:16-24
struct MapConfig {
    const char *name;
    const char *collisionDataFile;
    const char *navmeshFile;
    const char *spawnDataFile;
    const char *zoneDataFile;
    Vector3 mapOffset;
    float mapRotation;
};

// madrona::py::Tensor equivalent: a view of engine-owned memory.
struct Tensor {
    enum class ElementType : int32_t { Int32 = MPENV_DTYPE_INT32, Float32 = MPENV_DTYPE_FLOAT32, UInt32 = MPENV_DTYPE_UINT32 };
    void *ptr = nullptr;
    ElementType type = ElementType::Float32;
    std::vector<int64_t> dims;
    int32_t gpuID = -1;
    void *devicePtr() const { return ptr; }
    int64_t numElements() const
    {
        int64_t n = 1;
        for (int64_t d : dims) n *= d;
        return n;
    }
    int64_t numBytes() const { return 4 * numElements(); }
};

// madrona::py::TrainInterface equivalent (mgr.cpp:2383-2431).
struct NamedTensor {
    std::string name;
    Tensor tensor;
};
struct TrainInterface {
    std::vector<NamedTensor> inputs;
    std::vector<NamedTensor> outputs;
};

class Manager {
public:
    // mgr.hpp:33-52
    struct Config {
        ExecMode execMode;
        int gpuID;
        uint32_t numWorlds;
        uint32_t randSeed;
        bool autoReset;
        SimFlags simFlags;
        Task taskType;
        uint32_t teamSize;
        uint32_t numPBTPolicies;
        uint32_t policyHistorySize;
        MapConfig map;
        bool highlevelMove = false;
        bool trainFlank = false;
        const char *replayLogPath = nullptr;
        const char *recordLogPath = nullptr;
        const char *eventLogPath = nullptr;
        const char *curriculumDataPath = nullptr;
        const char *policyWeightsPath = nullptr;
        uint32_t worldIDOffset = 0; // extension: first global world id (sharding)
    };

    // mgr.hpp:54-56; viz must be null (there is no viewer)
    explicit Manager(const Config &cfg, VizState *viz = nullptr)
    {
        if (viz != nullptr) throw std::runtime_error("mpenv: the viewer (VizState) is not part of this engine");
        const std::string dir = sceneDir(cfg.map);
        if (cfg.map.mapOffset.x != 0.f || cfg.map.mapOffset.y != 0.f || cfg.map.mapOffset.z != 0.f ||
            cfg.map.mapRotation != 0.f)
            throw std::runtime_error("mpenv: mapOffset/mapRotation must be zero (bindings.cpp:79-80)");
        if (cfg.highlevelMove) throw std::runtime_error("mpenv: highlevelMove is not implemented");
        mpenv_config c {};
        c.exec_mode = (int32_t)cfg.execMode;
        c.gpu_id = cfg.gpuID;
        c.num_worlds = cfg.numWorlds;
        c.rand_seed = cfg.randSeed;
        c.auto_reset = cfg.autoReset ? 1 : 0;
        c.sim_flags = (uint32_t)cfg.simFlags;
        c.task_type = (int32_t)cfg.taskType;
        c.team_size = cfg.teamSize;
        c.num_pbt_policies = cfg.numPBTPolicies;
        c.policy_history_size = cfg.policyHistorySize;
        c.scene_path = dir.c_str();
        c.train_flank = cfg.trainFlank ? 1 : 0;
        c.replay_log_path = cfg.replayLogPath;
        c.record_log_path = cfg.recordLogPath;
        c.event_log_path = cfg.eventLogPath;
        c.curriculum_data_path = cfg.curriculumDataPath;
        c.world_id_offset = cfg.worldIDOffset;
        check(mpenv_create(&c, &mgr_));
        execMode_ = cfg.execMode;
    }
    ~Manager() { mpenv_destroy(mgr_); }
    Manager(const Manager &) = delete;
    Manager &operator=(const Manager &) = delete;

    void init() { check(mpenv_init(mgr_)); }
    void step() { check(mpenv_step(mgr_)); }
    void vizStep() { outOfScope("vizStep (viewer)"); }
    inline void cpuJAXInit(void **, void **) {} // mgr.hpp:64-65: no-ops there too
    inline void cpuJAXStep(void **, void **) {}
    void gpuStreamInit(void *strm, void **buffers) { check(mpenv_gpu_stream_init(mgr_, strm, buffers)); }
    void gpuStreamStep(void *strm, void **buffers) { check(mpenv_gpu_stream_step(mgr_, strm, buffers)); }
    // extension: the Step graph enqueued on a caller stream without a sync
    void stepAsync(void *strm) { check(mpenv_step_async(mgr_, strm)); }

    Tensor resetTensor() const { return get(MPENV_EXPORT_RESET); }
    Tensor simControlTensor() const { return get(MPENV_EXPORT_SIM_CONTROL); }
    Tensor matchResultTensor() const { return get(MPENV_EXPORT_MATCH_RESULT); }
    Tensor pvpDiscreteActionTensor() const { return get(MPENV_EXPORT_PVP_DISCRETE_ACTION); }
    Tensor pvpAimActionTensor() const { return get(MPENV_EXPORT_PVP_AIM_ACTION); }
    Tensor pvpDiscreteAimActionTensor() const { return get(MPENV_EXPORT_PVP_DISCRETE_AIM_ACTION); }
    Tensor exploreActionTensor() const { return get(MPENV_EXPORT_EXPLORE_ACTION); }
    Tensor rewardTensor() const { return get(MPENV_EXPORT_REWARD); }
    Tensor doneTensor() const { return get(MPENV_EXPORT_DONE); }
    Tensor policyAssignmentTensor() const { return get(MPENV_EXPORT_AGENT_POLICY); }
    Tensor worldCurriculumTensor() const { return get(MPENV_EXPORT_WORLD_CURRICULUM); }
    Tensor selfObservationTensor() const { return get(MPENV_EXPORT_SELF_OBSERVATION); }
    Tensor filtersStateObservationTensor() const { return get(MPENV_EXPORT_FILTERS_STATE); }
    Tensor teammateObservationsTensor() const { return get(MPENV_EXPORT_TEAMMATE_OBSERVATIONS); }
    Tensor opponentObservationsTensor() const { return get(MPENV_EXPORT_OPPONENT_OBSERVATIONS); }
    Tensor opponentLastKnownObservationsTensor() const { return get(MPENV_EXPORT_OPPONENT_LAST_KNOWN_OBSERVATIONS); }
    Tensor selfPositionTensor() const { return get(MPENV_EXPORT_SELF_POSITION); }
    Tensor teammatePositionObservationsTensor() const { return get(MPENV_EXPORT_TEAMMATE_POSITIONS); }
    Tensor opponentPositionObservationsTensor() const { return get(MPENV_EXPORT_OPPONENT_POSITIONS); }
    Tensor opponentLastKnownPositionObservationsTensor() const
    {
        return get(MPENV_EXPORT_OPPONENT_LAST_KNOWN_POSITIONS);
    }
    Tensor opponentMasksTensor() const { return get(MPENV_EXPORT_OPPONENT_MASKS); }
    Tensor fwdLidarTensor() const { return get(MPENV_EXPORT_FWD_LIDAR); }
    Tensor rearLidarTensor() const { return get(MPENV_EXPORT_REAR_LIDAR); }
    Tensor agentMapTensor() const { return get(MPENV_EXPORT_AGENT_MAP); }
    Tensor unmaskedAgentMapTensor() const { return get(MPENV_EXPORT_UNMASKED_AGENT_MAP); }
    Tensor hpTensor() const { return get(MPENV_EXPORT_HP); }
    Tensor magazineTensor() const { return get(MPENV_EXPORT_MAGAZINE); }
    Tensor aliveTensor() const { return get(MPENV_EXPORT_ALIVE); }
    Tensor rewardHyperParamsTensor() const { return get(MPENV_EXPORT_REWARD_HYPER_PARAMS); }
    // FullTeamInterface (mgr.hpp:110-120)
    Tensor fullTeamActionTensor() const { return get(MPENV_EXPORT_FULL_TEAM_ACTIONS); }
    Tensor fullTeamGlobalObservationsTensor() const { return get(MPENV_EXPORT_FULL_TEAM_GLOBAL); }
    Tensor fullTeamPlayerObservationsTensor() const { return get(MPENV_EXPORT_FULL_TEAM_PLAYERS); }
    Tensor fullTeamEnemyObservationsTensor() const { return get(MPENV_EXPORT_FULL_TEAM_ENEMIES); }
    Tensor fullTeamLastKnownEnemyObservationsTensor() const
    {
        return get(MPENV_EXPORT_FULL_TEAM_LAST_KNOWN_ENEMIES);
    }
    Tensor fullTeamFwdLidarTensor() const { return get(MPENV_EXPORT_FULL_TEAM_FWD_LIDAR); }
    Tensor fullTeamRearLidarTensor() const { return get(MPENV_EXPORT_FULL_TEAM_REAR_LIDAR); }
    Tensor fullTeamRewardTensor() const { return get(MPENV_EXPORT_FULL_TEAM_REWARD); }
    Tensor fullTeamDoneTensor() const { return get(MPENV_EXPORT_FULL_TEAM_DONE); }
    Tensor fullTeamPolicyAssignmentTensor() const { return get(MPENV_EXPORT_FULL_TEAM_POLICY_ASSIGNMENTS); }

    TrainInterface trainInterface() const
    {
        TrainInterface ti;
        int32_t ni = 0, no = 0;
        check(mpenv_train_interface_size(&ni, &no));
        for (int io = 0; io < 2; io++) {
            for (int32_t k = 0; k < (io ? no : ni); k++) {
                const char *name = nullptr;
                int32_t id = 0;
                check(mpenv_train_interface_entry(io, k, &name, &id));
                (io ? ti.outputs : ti.inputs).push_back({ name, get(id) });
            }
        }
        return ti;
    }

    ExecMode execMode() const { return execMode_; }

    Engine &getWorldContext(int32_t) { outOfScope("getWorldContext (Madrona ECS context)"); }

    void triggerReset(int32_t world_idx) { check(mpenv_trigger_reset(mgr_, world_idx)); }
    void setExploreAction(int32_t, ExploreAction) { outOfScope("setExploreAction (Task::Explore)"); }
    void setCoarsePvPAction(int32_t, int32_t, CoarsePvPAction) { outOfScope("setCoarsePvPAction"); }
    void setPvPAction(int32_t world_idx, int32_t agent_idx, PvPDiscreteAction discrete, PvPAimAction aim,
                      PvPDiscreteAimAction aim_discrete)
    {
        const int32_t d[4] = { discrete.moveAmount, discrete.moveAngle, discrete.fire, discrete.stand };
        const float a[2] = { aim.yaw, aim.pitch };
        const int32_t ad[2] = { aim_discrete.yaw, aim_discrete.pitch };
        check(mpenv_set_pvp_action(mgr_, world_idx, agent_idx, d, a, ad));
    }
    void setHP(int32_t world_idx, int32_t agent_idx, int32_t hp) { check(mpenv_set_hp(mgr_, world_idx, agent_idx, hp)); }
    bool isReplayFinished()
    {
        int32_t f = 0;
        check(mpenv_is_replay_finished(mgr_, &f));
        return f != 0;
    }
    void setAgentPolicy(int32_t world_idx, int32_t agent_idx, AgentPolicy policy)
    {
        check(mpenv_set_agent_policy(mgr_, world_idx, agent_idx, policy.idx));
    }
    void setUniformAgentPolicy(AgentPolicy policy) { check(mpenv_set_uniform_agent_policy(mgr_, policy.idx)); }

    mpenv_manager *handle() const { return mgr_; }

private:
    [[noreturn]] static void outOfScope(const char *what)
    {
        throw std::runtime_error(std::string("mpenv: ") + what + " is out of scope for this engine (DESIGN.md §8)");
    }

    static void check(int rc)
    {
        if (rc != MPENV_OK) throw std::runtime_error(std::string("mpenv: ") + mpenv_last_error());
    }

    // bindings.cpp:56-78 builds the four paths from one scene directory;
    // accept exactly that layout.
    static std::string sceneDir(const MapConfig &m)
    {
        if (!m.collisionDataFile) throw std::runtime_error("mpenv: MapConfig.collisionDataFile is required");
        std::string c = m.collisionDataFile;
        const std::string suffix = "/collisions.bin";
        if (c.size() < suffix.size() || c.compare(c.size() - suffix.size(), suffix.size(), suffix) != 0)
            throw std::runtime_error("mpenv: collisionDataFile must be <scene>/collisions.bin");
        std::string dir = c.substr(0, c.size() - suffix.size());
        auto same = [&](const char *p, const char *name) {
            return p == nullptr || std::string(p) == dir + "/" + name;
        };
        if (!same(m.navmeshFile, "navmesh.bin") || !same(m.spawnDataFile, "spawns.bin") ||
            !same(m.zoneDataFile, "zones.bin"))
            throw std::runtime_error("mpenv: scene files must share one directory (bindings.cpp:56-78 layout)");
        return dir;
    }

    Tensor get(int32_t id) const
    {
        Tensor t;
        int32_t dt = 0, nd = 0, gpu = -1;
        int64_t dims[8];
        check(mpenv_export_tensor(mgr_, id, &t.ptr, &dt, &nd, dims, &gpu));
        t.type = Tensor::ElementType(dt);
        t.dims.assign(dims, dims + nd);
        t.gpuID = gpu;
        return t;
    }

    mpenv_manager *mgr_ = nullptr;
    ExecMode execMode_ = ExecMode::CUDA;
};

} // namespace madronaMPEnv
