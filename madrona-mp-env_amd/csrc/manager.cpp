// manager.cpp — the Manager (src/mgr.hpp:31-161, src/mgr.cpp) for the gfx950
// engine, exposed through the C ABI of include/mpenv.h.
//
// Owns every device buffer (engine-owned tensors, zero-copy views handed to
// callers as in mgr.cpp:295-301/655-661), the scene upload, and the step
// launch sequence on a HIP stream.  There is no CPU execution path: a CPU
// ExecMode is rejected (the reference's CPU TaskGraph executor is restated
// only by the test oracle).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <unordered_set>

#include <dlfcn.h>
#include <string>
#include <vector>

#include "engine.h"
#include "mpenv.h"
#include "scene.h"

using namespace mpenv;

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string &msg)
{
    g_last_error = msg;
    return code;
}

#define HIP_CHECK(expr)                                                                   \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess) {                                                           \
            throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e_) + \
                                     " at " #expr);                                       \
        }                                                                                 \
    } while (0)

// Order of TrainInterface inputs/outputs (mgr.cpp:2383-2431).
struct TIEntry {
    const char *name;
    int32_t id;
};
const TIEntry kTIInputs[] = {
    { "discrete", MPENV_EXPORT_PVP_DISCRETE_ACTION },
    { "aim", MPENV_EXPORT_PVP_DISCRETE_AIM_ACTION },
    { "resets", MPENV_EXPORT_RESET },
    { "simCtrl", MPENV_EXPORT_SIM_CONTROL },
    { "pbt.policy_assignments", MPENV_EXPORT_AGENT_POLICY },
};
const TIEntry kTIOutputs[] = {
    { "fwd_lidar", MPENV_EXPORT_FWD_LIDAR },
    { "rear_lidar", MPENV_EXPORT_REAR_LIDAR },
    { "hp", MPENV_EXPORT_HP },
    { "magazine", MPENV_EXPORT_MAGAZINE },
    { "alive", MPENV_EXPORT_ALIVE },
    { "self", MPENV_EXPORT_SELF_OBSERVATION },
    { "filters_state", MPENV_EXPORT_FILTERS_STATE },
    { "teammates", MPENV_EXPORT_TEAMMATE_OBSERVATIONS },
    { "opponents", MPENV_EXPORT_OPPONENT_OBSERVATIONS },
    { "opponents_last_known", MPENV_EXPORT_OPPONENT_LAST_KNOWN_OBSERVATIONS },
    { "self_pos", MPENV_EXPORT_SELF_POSITION },
    { "teammate_positions", MPENV_EXPORT_TEAMMATE_POSITIONS },
    { "opponent_positions", MPENV_EXPORT_OPPONENT_POSITIONS },
    { "opponent_last_known_positions", MPENV_EXPORT_OPPONENT_LAST_KNOWN_POSITIONS },
    { "opponent_masks", MPENV_EXPORT_OPPONENT_MASKS },
    { "agent_map", MPENV_EXPORT_AGENT_MAP },
    { "unmasked_agent_map", MPENV_EXPORT_AGENT_MAP },
    { "reward_coefs", MPENV_EXPORT_REWARD_HYPER_PARAMS },
    { "rewards", MPENV_EXPORT_REWARD },
    { "dones", MPENV_EXPORT_DONE },
    { "pbt.episode_results", MPENV_EXPORT_MATCH_RESULT },
};
constexpr int kNumTIInputs = sizeof(kTIInputs) / sizeof(kTIInputs[0]);
constexpr int kNumTIOutputs = sizeof(kTIOutputs) / sizeof(kTIOutputs[0]);

struct TensorDesc {
    void *ptr = nullptr;
    int32_t dtype = MPENV_DTYPE_FLOAT32;
    std::vector<int64_t> dims;
    size_t bytes() const
    {
        size_t n = 4;
        for (int64_t d : dims) n *= (size_t)d;
        return n;
    }
};

} // namespace

struct mpenv_manager {
    mpenv_config cfg;
    std::string scenePath;
    int gpu = 0;
    Scene scene;
    SceneDev sc;
    DevState S;
    hipStream_t stream = nullptr;
    std::vector<void *> allocations;

    // Debug gather buffers (allocated lazily)
    float *dbgAF = nullptr, *dbgWF = nullptr, *dbgCrumbs = nullptr;
    int32_t *dbgAI = nullptr, *dbgWI = nullptr;
    uint32_t *dbgExplore = nullptr;

    // World groups: contiguous world ranges stepped on their own streams
    // (fork/join with events) so independent kernels overlap on the GPU.
    int groups = 1;
    std::vector<hipStream_t> gstreams;
    std::vector<DevState> gS;
    std::vector<SceneDev> gsc;
    hipEvent_t forkEv = nullptr;
    std::vector<hipEvent_t> joinEv;
    // One group only: k_lidar on a branch stream beside k_vis -> k_obs (no
    // data dependence between them after k_sim).  MPENV_LIDAR_BRANCH=1.
    bool lidarBranch = false;
    hipStream_t bStream = nullptr;
    hipEvent_t bForkEv = nullptr, bJoinEv = nullptr;
    // gpuStreamStep: the agent maps' zero fills (no dependence on the step)
    // on a side stream of their own, overlapping the step's kernels; joined
    // back into the caller's stream before the call returns.
    hipStream_t zStream = nullptr;
    hipEvent_t zForkEv = nullptr, zJoinEv = nullptr;

    // Record / replay / event logs (mgr.cpp:155-300: per-step file I/O
    // around the Step graph)
    FILE *replayFile = nullptr, *recordFile = nullptr, *eventsFile = nullptr, *stepsFile = nullptr;
    bool replayEof = false;
    std::vector<mpenv_step_log> hostLog;
    std::vector<mpenv_game_event> hostEvents;
    std::vector<mpenv_packed_step_snapshot> hostSnaps;
    std::vector<int32_t> hostSnapWritten;

    // Workload counters (DevState::stats, kNumStats u64), allocated on first use
    unsigned long long *statsBuf = nullptr;

    // Kernel timing
    bool timing = false;
    std::vector<hipEvent_t> eventPool;
    size_t eventsUsed = 0;

    // The Step graph as a captured HIP graph (all world groups, fork/join
    // included), replayed with one hipGraphLaunch per step.  Kernel
    // arguments are captured by value, so the graph is keyed on the bytes of
    // every argument struct and re-captured when any of them changes (world
    // groups, stats buffer, ...).  MPENV_STEP_GRAPH=0 launches kernel by
    // kernel instead; timed steps (events between kernels) always do.
    bool useGraph = true;
    hipStream_t capStream = nullptr;
    hipGraph_t stepGraph = nullptr;
    hipGraphExec_t stepExec = nullptr;
    std::vector<char> graphKey;
    // recorded after every hipGraphLaunch on the launch's stream: a
    // re-capture waits on it before destroying the previous exec (its last
    // launch may still run on a caller stream the manager does not own)
    hipEvent_t graphDoneEv = nullptr;
    int64_t graphCaptures = 0; // mpenv_graph_captures
    std::string graphOffReason; // why the step is not replayed from a graph (mpenv_graph_status)
    uint32_t *wireErr = nullptr; // device word raised by a rejected wire message (wire.hip)
    int32_t *wireEp = nullptr;   // [2][W] a shadow's episode counters of the last two messages
    int wireParity = 0;          // which half of wireEp holds the previous message's
    OutTab *outTabDev = nullptr; // gpuStreamStep's caller output buffers (engine.h OutTab)

    ~mpenv_manager()
    {
        if (stream) (void)hipStreamSynchronize(stream);
        for (hipStream_t gs : gstreams) (void)hipStreamSynchronize(gs);
        if (graphDoneEv) {
            (void)hipEventSynchronize(graphDoneEv);
            (void)hipEventDestroy(graphDoneEv);
        }
        if (stepExec) (void)hipGraphExecDestroy(stepExec);
        if (stepGraph) (void)hipGraphDestroy(stepGraph);
        if (capStream) (void)hipStreamDestroy(capStream);
        for (hipEvent_t e : eventPool) (void)hipEventDestroy(e);
        for (hipEvent_t e : joinEv) (void)hipEventDestroy(e);
        if (forkEv) (void)hipEventDestroy(forkEv);
        for (hipStream_t gs : gstreams) (void)hipStreamDestroy(gs);
        if (bStream) {
            (void)hipStreamSynchronize(bStream);
            (void)hipStreamDestroy(bStream);
        }
        if (bForkEv) (void)hipEventDestroy(bForkEv);
        if (bJoinEv) (void)hipEventDestroy(bJoinEv);
        if (zStream) {
            (void)hipStreamSynchronize(zStream);
            (void)hipStreamDestroy(zStream);
        }
        if (zForkEv) (void)hipEventDestroy(zForkEv);
        if (zJoinEv) (void)hipEventDestroy(zJoinEv);
        for (FILE *f : { replayFile, recordFile, eventsFile, stepsFile })
            if (f) std::fclose(f);
        for (void *p : allocations) (void)hipFree(p);
        if (stream) (void)hipStreamDestroy(stream);
    }

    template <typename T>
    T *alloc(size_t count)
    {
        size_t bytes = std::max<size_t>(count * sizeof(T), 16);
        void *p = nullptr;
        HIP_CHECK(hipMalloc(&p, bytes));
        HIP_CHECK(hipMemsetAsync(p, 0, bytes, stream));
        allocations.push_back(p);
        return static_cast<T *>(p);
    }

    // Host->device copy ordered on the manager stream (after the zeroing
    // memsets issued by alloc() and any in-flight step), then waited for.
    void upload(void *dst, const void *src, size_t bytes)
    {
        HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream));
        HIP_CHECK(hipStreamSynchronize(stream));
    }

    hipEvent_t nextEvent()
    {
        if (eventsUsed == eventPool.size()) {
            hipEvent_t e;
            HIP_CHECK(hipEventCreate(&e));
            eventPool.push_back(e);
        }
        return eventPool[eventsUsed++];
    }

    void record(hipStream_t st)
    {
        if (timing) HIP_CHECK(hipEventRecord(nextEvent(), st));
    }

    // The Step graph over one world range on one stream.  With timing on,
    // kNumTimedKernels + 1 events bracket the kernels (one segment per
    // range per step, contiguous in the pool).
    void stepRange(const DevState &R, const SceneDev &rsc, hipStream_t st)
    {
        record(st);
        if (launchMove(R, rsc, st)) throw std::runtime_error("k_move launch failed");
        record(st);
        if (launchSimStep(R, rsc, st)) throw std::runtime_error("k_sim launch failed");
        record(st);
        if (lidarBranch && groups == 1 && !timing) {
            HIP_CHECK(hipEventRecord(bForkEv, st));
            HIP_CHECK(hipStreamWaitEvent(bStream, bForkEv, 0));
            if (launchLidar(R, rsc, bStream)) throw std::runtime_error("k_lidar launch failed");
            HIP_CHECK(hipEventRecord(bJoinEv, bStream));
            if (launchVisibility(R, rsc, st)) throw std::runtime_error("k_vis launch failed");
            if (launchObservations(R, rsc, st)) throw std::runtime_error("k_obs launch failed");
            HIP_CHECK(hipStreamWaitEvent(st, bJoinEv, 0));
            return;
        }
        if (launchVisibility(R, rsc, st)) throw std::runtime_error("k_vis launch failed");
        record(st);
        if (launchObservations(R, rsc, st)) throw std::runtime_error("k_obs launch failed");
        record(st);
        if (launchLidar(R, rsc, st)) throw std::runtime_error("k_lidar launch failed");
        record(st);
    }

    // Replay: next W StepLogs from the file (a short read at EOF keeps the
    // rest of the previous step's records, as the reference's fstream read).
    void preStep(hipStream_t st)
    {
        if (!replayFile) return;
        const size_t n = std::fread(hostLog.data(), sizeof(mpenv_step_log), hostLog.size(), replayFile);
        if (n < hostLog.size()) replayEof = true;
        HIP_CHECK(hipMemcpyAsync((void *)S.replayLog, hostLog.data(), sizeof(mpenv_step_log) * hostLog.size(),
                                 hipMemcpyHostToDevice, st));
    }

    // Record: W StepLogs per step.  Events: the step's events world-major
    // (per world: agent slots in order, then the capture) to events.bin and
    // the written snapshots to steps.bin (writeGameEvents, mgr.cpp:104-116).
    void postStep(hipStream_t st)
    {
        if (!recordFile && !eventsFile) return;
        HIP_CHECK(hipStreamSynchronize(st));
        if (recordFile) {
            HIP_CHECK(hipMemcpy(hostLog.data(), S.recordLog, sizeof(mpenv_step_log) * hostLog.size(),
                                hipMemcpyDeviceToHost));
            std::fwrite(hostLog.data(), sizeof(mpenv_step_log), hostLog.size(), recordFile);
        }
        if (eventsFile) {
            HIP_CHECK(hipMemcpy(hostEvents.data(), S.events, sizeof(mpenv_game_event) * hostEvents.size(),
                                hipMemcpyDeviceToHost));
            HIP_CHECK(hipMemcpy(hostSnaps.data(), S.snapshots, sizeof(mpenv_packed_step_snapshot) * hostSnaps.size(),
                                hipMemcpyDeviceToHost));
            HIP_CHECK(hipMemcpy(hostSnapWritten.data(), S.snapWritten, sizeof(int32_t) * hostSnapWritten.size(),
                                hipMemcpyDeviceToHost));
            for (const mpenv_game_event &e : hostEvents)
                if (e.type != 0) std::fwrite(&e, sizeof(e), 1, eventsFile);
            for (size_t w = 0; w < hostSnaps.size(); w++)
                if (hostSnapWritten[w]) std::fwrite(&hostSnaps[w], sizeof(hostSnaps[w]), 1, stepsFile);
        }
    }

    void runStep(hipStream_t st)
    {
        preStep(st);
        launchStep(st);
        postStep(st);
    }

    std::vector<char> argKey() const
    {
        std::vector<char> k;
        auto put = [&](const void *p, size_t n) {
            const char *c = static_cast<const char *>(p);
            k.insert(k.end(), c, c + n);
        };
        put(&groups, sizeof(groups));
        put(&lidarBranch, sizeof(lidarBranch));
        put(&S, sizeof(S));
        put(&sc, sizeof(sc));
        for (const DevState &G : gS) put(&G, sizeof(G));
        for (const SceneDev &g : gsc) put(&g, sizeof(g));
        return k;
    }

    void launchStep(hipStream_t st)
    {
        if (!useGraph || timing) {
            launchStepDirect(st);
            return;
        }
        std::vector<char> key = argKey();
        if (!stepExec || key != graphKey) {
            if (graphDoneEv) HIP_CHECK(hipEventSynchronize(graphDoneEv));
            if (stepExec) HIP_CHECK(hipGraphExecDestroy(stepExec));
            if (stepGraph) HIP_CHECK(hipGraphDestroy(stepGraph));
            stepExec = nullptr;
            stepGraph = nullptr;
            if (!capStream) HIP_CHECK(hipStreamCreateWithFlags(&capStream, hipStreamNonBlocking));
            // capture on a private stream (the caller's may be the legacy
            // default stream, which cannot be captured); the group streams
            // join the capture through the fork event
            if (!captureStep()) {
                // abandoned capture: this and later steps launch directly
                launchStepDirect(st);
                return;
            }
            graphKey = std::move(key);
            graphCaptures++;
        }
        HIP_CHECK(hipGraphLaunch(stepExec, st));
        if (!graphDoneEv) HIP_CHECK(hipEventCreateWithFlags(&graphDoneEv, hipEventDisableTiming));
        HIP_CHECK(hipEventRecord(graphDoneEv, st));
    }

    // Captures the Step graph into stepGraph / stepExec.  Every capture call
    // is checked, and so is the capture's state before it ends (an enqueue
    // that invalidated it, a fork not joined back): on any failure the
    // capture is ended and discarded, the graph is switched off with the
    // reason kept (mpenv_graph_status), and false is returned -- a bad
    // capture is never instantiated or launched.
    bool captureStep()
    {
        auto abandon = [&](const std::string &why) {
            hipGraph_t g = nullptr;
            hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
            if (hipStreamIsCapturing(capStream, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
                (void)hipStreamEndCapture(capStream, &g);
            if (g) (void)hipGraphDestroy(g);
            if (stepExec) (void)hipGraphExecDestroy(stepExec);
            if (stepGraph) (void)hipGraphDestroy(stepGraph);
            stepExec = nullptr;
            stepGraph = nullptr;
            (void)hipGetLastError(); // clear the sticky launch error of a failed capture call
            useGraph = false;
            graphOffReason = why;
            std::fprintf(stderr, "mpenv: step graph off (%s); launching kernels directly\n", why.c_str());
            return false;
        };
        hipError_t e = hipStreamBeginCapture(capStream, hipStreamCaptureModeThreadLocal);
        if (e != hipSuccess) return abandon(std::string("hipStreamBeginCapture: ") + hipGetErrorString(e));
        try {
            launchStepDirect(capStream);
        } catch (const std::exception &ex) {
            return abandon(std::string("enqueue during capture: ") + ex.what());
        }
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        unsigned long long id = 0;
        e = hipStreamGetCaptureInfo(capStream, &cs, &id);
        if (e != hipSuccess) return abandon(std::string("hipStreamGetCaptureInfo: ") + hipGetErrorString(e));
        if (cs != hipStreamCaptureStatusActive) return abandon("capture invalidated before its end");
        e = hipStreamEndCapture(capStream, &stepGraph);
        if (e != hipSuccess || !stepGraph) return abandon(std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
        e = hipGraphInstantiate(&stepExec, stepGraph, nullptr, nullptr, 0);
        if (e != hipSuccess || !stepExec) return abandon(std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
        return true;
    }

    void launchStepDirect(hipStream_t st)
    {
        if (groups <= 1) {
            stepRange(S, sc, st);
            return;
        }
        // group 0 runs on the caller's stream itself, so G groups occupy G
        // hardware queues (GPU_MAX_HW_QUEUES is 4 per process by default)
        HIP_CHECK(hipEventRecord(forkEv, st));
        for (int i = 1; i < groups; i++) HIP_CHECK(hipStreamWaitEvent(gstreams[i], forkEv, 0));
        for (int i = 1; i < groups; i++) {
            stepRange(gS[i], gsc[i], gstreams[i]);
            HIP_CHECK(hipEventRecord(joinEv[i], gstreams[i]));
        }
        stepRange(gS[0], gsc[0], st);
        for (int i = 1; i < groups; i++) HIP_CHECK(hipStreamWaitEvent(st, joinEv[i], 0));
    }

    void setupGroups(int want);

    void runInitGraph(hipStream_t st)
    {
        // triggerReset on every world (mgr.cpp:1936-1938) then the Init graph
        // (sim.cpp:5322-5340): resetSystem + observations + lidar.
        HIP_CHECK(hipMemsetD32Async((hipDeviceptr_t)S.reset, 1, (size_t)S.W, st));
        if (launchResetOnly(S, sc, st)) throw std::runtime_error("k_reset launch failed");
        if (launchVisibility(S, sc, st)) throw std::runtime_error("k_vis launch failed");
        if (launchObservations(S, sc, st)) throw std::runtime_error("k_obs launch failed");
        if (launchLidar(S, sc, st)) throw std::runtime_error("k_lidar launch failed");
    }

    bool exportDesc(int32_t id, TensorDesc &d);
    void gatherDebug(bool explore = false);
};

bool mpenv_manager::exportDesc(int32_t id, TensorDesc &d)
{
    const int64_t A = S.A, W = S.W;
    auto set = [&](void *p, int32_t dt, std::initializer_list<int64_t> dims) {
        d.ptr = p;
        d.dtype = dt;
        d.dims.assign(dims.begin(), dims.end());
        return true;
    };
    switch (id) {
    case MPENV_EXPORT_RESET: return set(S.reset, MPENV_DTYPE_INT32, { W, 1 });
    case MPENV_EXPORT_WORLD_CURRICULUM: return set(S.worldCurr, MPENV_DTYPE_INT32, { W, 1 });
    case MPENV_EXPORT_EXPLORE_ACTION: return set(S.exploreAction, MPENV_DTYPE_INT32, { A, 4 });
    case MPENV_EXPORT_PVP_DISCRETE_ACTION: return set(S.discreteAction, MPENV_DTYPE_INT32, { A, 4 });
    case MPENV_EXPORT_PVP_AIM_ACTION: return set(S.aimAction, MPENV_DTYPE_FLOAT32, { A, 1, 2 });
    case MPENV_EXPORT_PVP_DISCRETE_AIM_ACTION: return set(S.discreteAim, MPENV_DTYPE_INT32, { A, 2 });
    case MPENV_EXPORT_REWARD: return set(S.reward, MPENV_DTYPE_FLOAT32, { A, 1 });
    case MPENV_EXPORT_DONE: return set(S.done, MPENV_DTYPE_INT32, { A, 1 });
    case MPENV_EXPORT_MATCH_RESULT: return set(S.matchResult, MPENV_DTYPE_INT32, { W, 30 });
    case MPENV_EXPORT_AGENT_POLICY: return set(S.policy, MPENV_DTYPE_INT32, { A, 1 });
    case MPENV_EXPORT_SELF_OBSERVATION: return set(S.selfObs, MPENV_DTYPE_FLOAT32, { A, kSelfObs });
    case MPENV_EXPORT_TEAMMATE_OBSERVATIONS: return set(S.tmObs, MPENV_DTYPE_FLOAT32, { A, 5, kOtherObs });
    case MPENV_EXPORT_OPPONENT_OBSERVATIONS: return set(S.oppObs, MPENV_DTYPE_FLOAT32, { A, 6, kOtherObs });
    case MPENV_EXPORT_OPPONENT_LAST_KNOWN_OBSERVATIONS: return set(S.lkObs, MPENV_DTYPE_FLOAT32, { A, 6, kOtherObs });
    case MPENV_EXPORT_SELF_POSITION: return set(S.selfPos, MPENV_DTYPE_FLOAT32, { A, 3 });
    case MPENV_EXPORT_TEAMMATE_POSITIONS: return set(S.tmPos, MPENV_DTYPE_FLOAT32, { A, 5, 3 });
    case MPENV_EXPORT_OPPONENT_POSITIONS: return set(S.oppPos, MPENV_DTYPE_FLOAT32, { A, 6, 3 });
    case MPENV_EXPORT_OPPONENT_LAST_KNOWN_POSITIONS: return set(S.lkPos, MPENV_DTYPE_FLOAT32, { A, 6, 3 });
    case MPENV_EXPORT_OPPONENT_MASKS: return set(S.masks, MPENV_DTYPE_FLOAT32, { A, 6, 1 });
    case MPENV_EXPORT_FWD_LIDAR: return set(S.fwdLidar, MPENV_DTYPE_FLOAT32, { A, 2, 32, 4 });
    case MPENV_EXPORT_REAR_LIDAR: return set(S.rearLidar, MPENV_DTYPE_FLOAT32, { A, 2, 8, 4 });
    case MPENV_EXPORT_AGENT_MAP:
    case MPENV_EXPORT_UNMASKED_AGENT_MAP: return set(S.agentMap, MPENV_DTYPE_FLOAT32, { A, 16, 16, 4 });
    case MPENV_EXPORT_HP: return set(S.hp, MPENV_DTYPE_FLOAT32, { A, 1 });
    case MPENV_EXPORT_ALIVE: return set(S.alive, MPENV_DTYPE_FLOAT32, { A, 1 });
    case MPENV_EXPORT_MAGAZINE: return set(S.magazine, MPENV_DTYPE_INT32, { A, 2 });
    case MPENV_EXPORT_FULL_TEAM_ACTIONS: return set(S.ftActions, MPENV_DTYPE_INT32, { W * 2, 6, 4 });
    case MPENV_EXPORT_FULL_TEAM_GLOBAL: return set(S.ftGlobal, MPENV_DTYPE_FLOAT32, { W * 2, MPENV_FT_GLOBAL_DIM });
    case MPENV_EXPORT_FULL_TEAM_PLAYERS:
        return set(S.ftPlayers, MPENV_DTYPE_FLOAT32, { W * 2, 6, MPENV_FT_PLAYER_DIM });
    case MPENV_EXPORT_FULL_TEAM_ENEMIES:
        return set(S.ftEnemies, MPENV_DTYPE_FLOAT32, { W * 2, 6, MPENV_FT_ENEMY_DIM });
    case MPENV_EXPORT_FULL_TEAM_LAST_KNOWN_ENEMIES:
        return set(S.ftLastKnown, MPENV_DTYPE_FLOAT32, { W * 2, 6, MPENV_FT_COMMON_DIM });
    case MPENV_EXPORT_FULL_TEAM_FWD_LIDAR: return set(S.ftFwdLidar, MPENV_DTYPE_FLOAT32, { W * 2, 6, 2, 32, 4 });
    case MPENV_EXPORT_FULL_TEAM_REAR_LIDAR: return set(S.ftRearLidar, MPENV_DTYPE_FLOAT32, { W * 2, 6, 2, 8, 4 });
    case MPENV_EXPORT_FULL_TEAM_REWARD: return set(S.ftReward, MPENV_DTYPE_FLOAT32, { W * 2, 1 });
    case MPENV_EXPORT_FULL_TEAM_DONE: return set(S.ftDone, MPENV_DTYPE_INT32, { W * 2, 1 });
    case MPENV_EXPORT_FULL_TEAM_POLICY_ASSIGNMENTS: return set(S.ftPolicy, MPENV_DTYPE_INT32, { W * 2, 1 });
    case MPENV_EXPORT_FILTERS_STATE: return set(S.filters, MPENV_DTYPE_FLOAT32, { A, 1 });
    case MPENV_EXPORT_REWARD_HYPER_PARAMS: return set(S.rewardCoefs, MPENV_DTYPE_FLOAT32, { A, 9 });
    case MPENV_EXPORT_EVENT_LOG:
        if (!S.events) return false;
        return set(S.events, MPENV_DTYPE_INT32, { W, S.evStride, 6 });
    case MPENV_EXPORT_PACKED_STEP_SNAPSHOT:
        if (!S.snapshots) return false;
        return set(S.snapshots, MPENV_DTYPE_INT32, { W, 48 });
    case MPENV_EXPORT_RECORD_LOG:
        if (!S.recordLog) return false;
        return set(S.recordLog, MPENV_DTYPE_INT32, { W, 217 });
    case MPENV_EXPORT_REPLAY_LOG:
        if (!S.replayLog) return false;
        return set((void *)S.replayLog, MPENV_DTYPE_INT32, { W, 217 });
    case MPENV_EXPORT_SNAPSHOT_WRITTEN:
        if (!S.snapshots) return false;
        return set(S.snapWritten, MPENV_DTYPE_INT32, { W, 1 });
    case MPENV_EXPORT_SIM_CONTROL: return set(S.trainCtrl, MPENV_DTYPE_INT32, { 3 });
    case MPENV_EXPORT_DEBUG_AGENT_F32: gatherDebug(); return set(dbgAF, MPENV_DTYPE_FLOAT32, { A, MPENV_DBG_AF_COUNT });
    case MPENV_EXPORT_DEBUG_AGENT_I32: gatherDebug(); return set(dbgAI, MPENV_DTYPE_INT32, { A, MPENV_DBG_AI_COUNT });
    case MPENV_EXPORT_DEBUG_WORLD_I32: gatherDebug(); return set(dbgWI, MPENV_DTYPE_INT32, { W, MPENV_DBG_WI_COUNT });
    case MPENV_EXPORT_DEBUG_WORLD_F32: gatherDebug(); return set(dbgWF, MPENV_DTYPE_FLOAT32, { W, MPENV_DBG_WF_COUNT });
    case MPENV_EXPORT_DEBUG_EXPLORE: gatherDebug(true); return set(dbgExplore, MPENV_DTYPE_UINT32, { A, kGridCells });
    case MPENV_EXPORT_DEBUG_CRUMBS: gatherDebug(); return set(dbgCrumbs, MPENV_DTYPE_FLOAT32, { W, kMaxCrumbs, 8 });
    default: return false;
    }
}

void mpenv_manager::gatherDebug(bool explore)
{
    if (!dbgAF) {
        dbgAF = alloc<float>((size_t)S.A * MPENV_DBG_AF_COUNT);
        dbgAI = alloc<int32_t>((size_t)S.A * MPENV_DBG_AI_COUNT);
        dbgWI = alloc<int32_t>((size_t)S.W * MPENV_DBG_WI_COUNT);
        dbgWF = alloc<float>((size_t)S.W * MPENV_DBG_WF_COUNT);
        dbgCrumbs = alloc<float>((size_t)S.W * kMaxCrumbs * 8);
    }
    // the expanded explore grid (4 B per cell, 26 KB per agent) only on request
    if (explore && !dbgExplore) dbgExplore = alloc<uint32_t>((size_t)S.A * kGridCells);
    if (launchDebugGather(S, dbgAF, dbgAI, dbgWI, dbgWF, explore ? dbgExplore : nullptr, dbgCrumbs, stream))
        throw std::runtime_error("debug gather launch failed");
    HIP_CHECK(hipStreamSynchronize(stream));
}

static void buildSceneDev(mpenv_manager &m)
{
    Scene &s = m.scene;
    SceneDev &sc = m.sc;
    std::memset(&sc, 0, sizeof(sc));
    if (s.nodes.size() > 256) throw std::runtime_error("BVH has more than 256 nodes (byte-stack limit)");
    if (s.maxStack > kMaxBVHStack || s.maxStackAnyOrder > kMaxBVHStack)
        throw std::runtime_error("BVH too deep for the 16-entry register stack");
    if (s.lidarNodes.size() > 256) throw std::runtime_error("lidar BVH has more than 256 nodes (byte-stack limit)");
    if (s.lidarMaxStack > kMaxBVHStack) throw std::runtime_error("lidar BVH too deep for the 16-entry register stack");
    if (s.zoneAABBs.empty() || s.zoneAABBs.size() > (size_t)kMaxZones) throw std::runtime_error("bad zone count");
    if (s.numDefaultASpawns == 0 || s.numDefaultBSpawns == 0) throw std::runtime_error("scene needs A and B spawns");
    if ((m.cfg.sim_flags & MPENV_SIMFLAG_SPAWN_IN_MIDDLE) &&
        (s.aSpawns.size() == s.numDefaultASpawns || s.bSpawns.size() == s.numDefaultBSpawns))
        // the reference would index past its spawn array here (utils.cpp:358-366)
        throw std::runtime_error("SpawnInMiddle: no free middle cells in this scene");

    BVHNode *d_nodes = m.alloc<BVHNode>(s.nodes.size());
    m.upload(d_nodes, s.nodes.data(), sizeof(BVHNode) * s.nodes.size());
    {
        // k_lidar: octant images of the lidar tree and its triangles
        const std::vector<BVHNode> oct = octantNodeImages(s.lidarNodes);
        BVHNode *d_oct = m.alloc<BVHNode>(oct.size());
        m.upload(d_oct, oct.data(), sizeof(BVHNode) * oct.size());
        sc.octNodes = d_oct;
        BVHNode *d_ln = m.alloc<BVHNode>(s.lidarNodes.size());
        m.upload(d_ln, s.lidarNodes.data(), sizeof(BVHNode) * s.lidarNodes.size());
        sc.lidarNodes = d_ln;
        float *d_lv = m.alloc<float>(s.lidarVerts.size() * 3);
        m.upload(d_lv, s.lidarVerts.data(), sizeof(float) * 3 * s.lidarVerts.size());
        sc.lidarVerts = d_lv;
        sc.numLidarNodes = (int32_t)s.lidarNodes.size();
        sc.numLidarVerts = (int32_t)s.lidarVerts.size();
    }
    float *d_verts = m.alloc<float>(s.bvhVerts.size() * 3);
    m.upload(d_verts, s.bvhVerts.data(), sizeof(float) * 3 * s.bvhVerts.size());
    auto upSpawns = [&](const std::vector<Spawn> &v) {
        Spawn *p = m.alloc<Spawn>(std::max<size_t>(v.size(), 1));
        if (!v.empty()) m.upload(p, v.data(), sizeof(Spawn) * v.size());
        return p;
    };
    {
        const NavMesh &nm = s.nav;
        const size_t T = nm.numTris();
        std::vector<float> tv(std::max<size_t>(T * 9, 1), 0.f);
        for (size_t t = 0; t < T; t++)
            for (int k = 0; k < 3; k++) {
                const mp::Vec3 v = nm.verts[nm.tris[3 * t + k]];
                tv[9 * t + 3 * k + 0] = v.x;
                tv[9 * t + 3 * k + 1] = v.y;
                tv[9 * t + 3 * k + 2] = v.z;
            }
        float *d_nav = m.alloc<float>(tv.size());
        m.upload(d_nav, tv.data(), sizeof(float) * tv.size());
        int32_t *d_astar = m.alloc<int32_t>(std::max<size_t>(nm.astar.size(), 1));
        if (!nm.astar.empty()) m.upload(d_astar, nm.astar.data(), sizeof(int32_t) * nm.astar.size());
        std::vector<float> cdf(std::max<size_t>(T, 1), 0.f);
        mp::navAreaCDF(tv.data(), (int)T, cdf.data());
        float *d_cdf = m.alloc<float>(cdf.size());
        m.upload(d_cdf, cdf.data(), sizeof(float) * cdf.size());
        sc.navCdf = d_cdf;
        sc.navTris = d_nav;
        sc.astar = d_astar;
        sc.numNavTris = (int32_t)T;
    }
    {
        // sphere-cast triangle constants (geom_dev.h sphereTriD)
        const size_t nt = s.bvhVerts.size() / 3;
        std::vector<float> pre(std::max<size_t>(nt, 1) * 8, 0.f);
        for (size_t t = 0; t < nt; t++) {
            const mp::Vec3 a = s.bvhVerts[3 * t], b = s.bvhVerts[3 * t + 1], c = s.bvhVerts[3 * t + 2];
            const mp::Vec3 e01 = b - a, e02 = c - a, e12 = c - b;
            const mp::Vec3 nu = mp::computeTriangleGeoNormal(e01, e02, e12);
            const float n_len = mp::length(nu);
            const mp::Vec3 n = nu / n_len;
            float *o = &pre[8 * t];
            o[0] = n.x; o[1] = n.y; o[2] = n.z; o[3] = n_len;
            o[4] = mp::length2(e01); o[5] = mp::length2(e02); o[6] = mp::length2(e12); o[7] = 0.f;
        }
        float *d_pre = m.alloc<float>(pre.size());
        m.upload(d_pre, pre.data(), sizeof(float) * pre.size());
        sc.triPre = d_pre;
    }
    {
        // the sphere-cast radius is always consts::agentRadius (k_move)
        const QuirkGrid q = quirkGrid(s.bvhVerts, 15.f, 2.f, 16.f);
        uint32_t *d_q = m.alloc<uint32_t>(std::max<size_t>(q.bits.size(), 1));
        if (!q.bits.empty()) m.upload(d_q, q.bits.data(), sizeof(uint32_t) * q.bits.size());
        sc.quirkGrid = d_q;
        sc.qgMinX = q.minX;
        sc.qgMinY = q.minY;
        sc.qgInvCell = 1.f / q.cell;
        sc.qgW = q.w;
        sc.qgH = q.h;
    }
    sc.nodes = d_nodes;
    sc.verts = d_verts;
    sc.numNodes = (int32_t)s.nodes.size();
    sc.numVerts = (int32_t)s.bvhVerts.size();
    sc.worldBounds = s.worldBounds;
    // sim.cpp:5855 maxDist; 5869-5882 frustumData
    sc.maxDist = mp::length(s.worldBounds.pMax - s.worldBounds.pMin);
    {
        float aspect = 16.f / 9.f;
        float ang = 90.f / 2.f * (mp::kPi / 180.f);
        float f = 1.f / (mp::sinf_(ang) / mp::cosf_(ang));
        float wx = f / aspect, wy = 1.f, hx = f, hy = 1.f;
        float wi = 1.f / mp::sqrt_(wx * wx + wy * wy);
        float hi = 1.f / mp::sqrt_(hx * hx + hy * hy);
        sc.frustum[0] = wx * wi; sc.frustum[1] = wy * wi;
        sc.frustum[2] = hx * hi; sc.frustum[3] = hy * hi;
    }
    sc.aSpawns = upSpawns(s.aSpawns);
    sc.bSpawns = upSpawns(s.bSpawns);
    sc.commonRespawns = upSpawns(s.commonRespawns);
    sc.numA = (int32_t)s.aSpawns.size();
    sc.numB = (int32_t)s.bSpawns.size();
    sc.numCommon = (int32_t)s.commonRespawns.size();
    sc.numDefaultA = (int32_t)s.numDefaultASpawns;
    sc.numDefaultB = (int32_t)s.numDefaultBSpawns;
    sc.spawnTrackLen = (int32_t)std::max<size_t>(
        kMinSpawnTrack, std::max(s.aSpawns.size(), std::max(s.bSpawns.size(), s.commonRespawns.size())));
    sc.numZones = (int32_t)s.zoneAABBs.size();
    sc.task = m.cfg.task_type;
    sc.flank = m.cfg.train_flank ? 1 : 0; // RewardMode::Flank applies to Task.Zone (sim.cpp:5733-5748)
    if (m.cfg.curriculum_data_path) {
        // mgr.cpp:1424-1441: the file is an array of CurriculumSnapshot
        // (size / 176 of them).  Snapshots naming a zone or controller the
        // scene does not have are rejected (the reference would index past
        // its zone arrays).
        FILE *f = std::fopen(m.cfg.curriculum_data_path, "rb");
        if (!f) throw std::runtime_error(std::string("cannot open curriculum data ") + m.cfg.curriculum_data_path);
        std::fseek(f, 0, SEEK_END);
        const long size = std::ftell(f);
        std::fseek(f, 0, SEEK_SET);
        std::vector<mpenv_curriculum_snapshot> snaps((size_t)std::max<long>(size, 0) / sizeof(mpenv_curriculum_snapshot));
        const size_t got = snaps.empty() ? 0 : std::fread(snaps.data(), sizeof(mpenv_curriculum_snapshot), snaps.size(), f);
        std::fclose(f);
        if (got != snaps.size()) throw std::runtime_error("short read of curriculum data");
        for (const mpenv_curriculum_snapshot &sn : snaps) {
            if (sn.cur_zone >= s.zoneAABBs.size() || sn.cur_zone_controller < -1 || sn.cur_zone_controller > 1)
                throw std::runtime_error("curriculum snapshot names a zone or controller outside the scene");
        }
        if (!snaps.empty()) {
            auto *d = m.alloc<mpenv_curriculum_snapshot>(snaps.size());
            m.upload(d, snaps.data(), sizeof(mpenv_curriculum_snapshot) * snaps.size());
            sc.curriculum = d;
        }
        sc.numSnapshots = (int32_t)snaps.size();
    }
    // initWorld starts every ZoneCaptureDefend episode at zone 3 (sim.cpp:822-825)
    if (sc.task == MPENV_TASK_ZONE_CAPTURE_DEFEND && s.zoneAABBs.size() < 4)
        throw std::runtime_error("ZoneCaptureDefend needs a scene with >= 4 zones");
    if (m.cfg.sim_flags & MPENV_SIMFLAG_SUB_ZONES) {
        // sub-zones 0 and 1 are zones 1 and 2 (level_gen.cpp:283-293)
        if (s.zoneAABBs.size() < 3) throw std::runtime_error("SubZones needs a scene with >= 3 zones");
        mp::subZoneTable(s.zoneAABBs.data(), s.zoneRotations.data(), sc.subZones);
    }
    for (int z = 0; z < sc.numZones; z++) {
        sc.zoneAABB[z] = s.zoneAABBs[z];
        sc.zoneRot[z] = s.zoneRotations[z];
    }
    for (int z = 0; z < kMaxZones; z++) sc.zoneGoalTri[z] = -1;
    if (sc.numNavTris > 0 && computeZoneGoalTris(sc, m.alloc<int32_t>(kMaxZones), sc.zoneGoalTri, m.stream))
        throw std::runtime_error("zone goal triangle kernel failed");
    sc.numGoals = (int32_t)s.goalRegions.size();
    for (int gi = 0; gi < sc.numGoals && gi < 4; gi++) {
        const GoalRegion &g = s.goalRegions[gi];
        GoalRegionDev &d = sc.goals[gi];
        for (int k = 0; k < 3; k++) {
            d.sub[k].pMin = g.subRegions[k].pMin;
            d.sub[k].pMax = g.subRegions[k].pMax;
            d.sub[k].rotation = g.subRegions[k].rotation;
        }
        d.numSub = g.numSubRegions;
        d.attackerTeam = g.attackerTeam;
        d.rewardStrength = g.rewardStrength;
    }
    {
        SceneTables t;
        std::memcpy(t.zoneAABB, sc.zoneAABB, sizeof(t.zoneAABB));
        std::memcpy(t.zoneRot, sc.zoneRot, sizeof(t.zoneRot));
        std::memcpy(t.subZones, sc.subZones, sizeof(t.subZones));
        std::memcpy(t.goals, sc.goals, sizeof(t.goals));
        std::memcpy(t.zoneGoalTri, sc.zoneGoalTri, sizeof(t.zoneGoalTri));
        SceneTables *d_tab = m.alloc<SceneTables>(1);
        m.upload(d_tab, &t, sizeof(t));
        if (computeSceneFrames(d_tab, m.stream)) throw std::runtime_error("k_scene_frames launch failed");
        sc.tab = d_tab;
    }
    sc.simFlags = m.cfg.sim_flags;
    sc.autoReset = m.cfg.auto_reset;
    sc.worldOffset = m.cfg.world_id_offset;
    // mgr.cpp:1736-1737
    sc.initRandKey = mp::splitI(mp::initKey(m.cfg.rand_seed), 0);
}

static void allocState(mpenv_manager &m)
{
    DevState &S = m.S;
    const size_t A = (size_t)S.A, W = (size_t)S.W;
#define MP_ALLOC_AF(n) S.n = m.alloc<float>(A);
#define MP_ALLOC_AI(n) S.n = m.alloc<int32_t>(A);
#define MP_ALLOC_WI(n) S.n = m.alloc<int32_t>(W);
#define MP_ALLOC_WF(n) S.n = m.alloc<float>(W);
    MP_AGENT_F32(MP_ALLOC_AF)
    MP_AGENT_I32(MP_ALLOC_AI)
    MP_WORLD_I32(MP_ALLOC_WI)
    MP_WORLD_F32(MP_ALLOC_WF)
#undef MP_ALLOC_AF
#undef MP_ALLOC_AI
#undef MP_ALLOC_WI
#undef MP_ALLOC_WF
    S.dmg = m.alloc<float>(A * kMaxTeamSize);
    S.dmgStride = (int64_t)A;
    S.visMask = m.alloc<uint8_t>(A);
    m.wireErr = m.alloc<uint32_t>(1);
    HIP_CHECK(hipMemsetAsync(m.wireErr, 0, sizeof(uint32_t), m.stream));
    m.outTabDev = m.alloc<OutTab>(1); // zeros: off
    S.outTab = m.outTabDev;
    m.wireEp = m.alloc<int32_t>(2 * W);
    HIP_CHECK(hipMemsetAsync(m.wireEp, 0, sizeof(int32_t) * 2 * W, m.stream));
    S.visOcc = m.alloc<uint16_t>((size_t)A * S.T * 4);
    HIP_CHECK(hipMemsetAsync(S.visOcc, 0xff, sizeof(uint16_t) * (size_t)A * S.T * 4, m.stream));
    S.exploreBits = m.alloc<uint64_t>(A * kExploreTiles);
    S.filtLast = m.alloc<int32_t>(W * 6);
    S.zoneStats = m.alloc<int32_t>(W * 25);
    S.resetKeys = m.alloc<mp::RandKey>(A * 11);
    S.spawnTrack = m.alloc<uint32_t>(W * 3 * (size_t)m.sc.spawnTrackLen);
    S.crumbs = m.alloc<float4>(W * kMaxCrumbs * 2);
    S.reset = m.alloc<int32_t>(W);
    S.worldCurr = m.alloc<int32_t>(W);
    S.matchResult = m.alloc<int32_t>(W * 30);
    S.exploreAction = m.alloc<int32_t>(A * 4);
    S.discreteAction = m.alloc<int32_t>(A * 4);
    S.aimAction = m.alloc<float>(A * 2);
    S.discreteAim = m.alloc<int32_t>(A * 2);
    S.policy = m.alloc<int32_t>(A);
    S.botAction = m.alloc<int32_t>(A * 7);
    S.reward = m.alloc<float>(A);
    S.done = m.alloc<int32_t>(A);
    S.selfObs = m.alloc<float>(A * kSelfObs);
    S.filters = m.alloc<float>(A);
    S.tmObs = m.alloc<float>(A * 5 * kOtherObs);
    S.oppObs = m.alloc<float>(A * 6 * kOtherObs);
    S.lkObs = m.alloc<float>(A * 6 * kOtherObs);
    S.selfPos = m.alloc<float>(A * 3);
    S.tmPos = m.alloc<float>(A * 15);
    S.oppPos = m.alloc<float>(A * 18);
    S.lkPos = m.alloc<float>(A * 18);
    S.masks = m.alloc<float>(A * 6);
    S.fwdLidar = m.alloc<float>(A * kFwdRays * 4);
    S.rearLidar = m.alloc<float>(A * kRearRays * 4);
    S.agentMap = m.alloc<float>(A * 16 * 16 * 4);
    S.hp = m.alloc<float>(A);
    S.alive = m.alloc<float>(A);
    S.magazine = m.alloc<int32_t>(A * 2);
    S.rewardCoefs = m.alloc<float>(A * 9);
    S.trainCtrl = m.alloc<int32_t>(3);
    S.ftActions = m.alloc<int32_t>(W * 2 * 6 * 4);
    S.ftGlobal = m.alloc<float>(W * 2 * MPENV_FT_GLOBAL_DIM);
    S.ftPlayers = m.alloc<float>(W * 2 * 6 * MPENV_FT_PLAYER_DIM);
    S.ftEnemies = m.alloc<float>(W * 2 * 6 * MPENV_FT_ENEMY_DIM);
    S.ftLastKnown = m.alloc<float>(W * 2 * 6 * MPENV_FT_COMMON_DIM);
    S.ftFwdLidar = m.alloc<float>(W * 2 * 6 * kFwdRays * 4);
    S.ftRearLidar = m.alloc<float>(W * 2 * 6 * kRearRays * 4);
    S.ftReward = m.alloc<float>(W * 2);
    S.ftDone = m.alloc<int32_t>(W * 2);
    S.ftPolicy = m.alloc<int32_t>(W * 2);
}

static void openLogs(mpenv_manager &m, const mpenv_config *cfg)
{
    DevState &S = m.S;
    const size_t W = (size_t)S.W;
    S.evStride = 2 * S.N + 1;
    if (cfg->replay_log_path) {
        m.replayFile = std::fopen(cfg->replay_log_path, "rb");
        if (!m.replayFile) throw std::runtime_error(std::string("cannot open replay log ") + cfg->replay_log_path);
        S.replayLog = m.alloc<mpenv_step_log>(W);
        m.sc.replayOn = 1;
    }
    if (cfg->record_log_path) {
        m.recordFile = std::fopen(cfg->record_log_path, "wb");
        if (!m.recordFile) throw std::runtime_error(std::string("cannot open record log ") + cfg->record_log_path);
        S.recordLog = m.alloc<mpenv_step_log>(W);
        m.sc.recordOn = 1;
    }
    if (m.replayFile || m.recordFile) m.hostLog.assign(W, mpenv_step_log {});
    if (cfg->event_log_path) {
        const std::string dir = cfg->event_log_path;
        m.eventsFile = std::fopen((dir + "/events.bin").c_str(), "wb");
        m.stepsFile = std::fopen((dir + "/steps.bin").c_str(), "wb");
        if (!m.eventsFile || !m.stepsFile) throw std::runtime_error("cannot open event logs in " + dir);
        S.events = m.alloc<mpenv_game_event>(W * S.evStride);
        S.snapshots = m.alloc<mpenv_packed_step_snapshot>(W);
        m.hostEvents.assign(W * S.evStride, mpenv_game_event {});
        m.hostSnaps.assign(W, mpenv_packed_step_snapshot {});
        m.hostSnapWritten.assign(W, 0);
        m.sc.eventsOn = 1;
    }
}

// A contiguous world range [w0, w0 + nw) of the manager viewed as a complete
// engine: every per-agent / per-world column offset to the range, W/A set
// to its size, and the scene's world-id offset advanced so RNG keys stay
// global.  Worlds never read each other, so step kernels launched on
// different ranges are independent and can run on concurrent streams.
static void sliceState(const DevState &S, const SceneDev &sc, int64_t w0, int64_t nw, int32_t track_len,
                       DevState &G, SceneDev &gsc)
{
    G = S;
    gsc = sc;
    const int64_t g0 = w0 * S.N;
    G.W = (int32_t)nw;
    G.A = nw * S.N;
    gsc.worldOffset = sc.worldOffset + (uint32_t)w0;
#define MP_SL_A(n) G.n = S.n + g0;
#define MP_SL_W(n) G.n = S.n + w0;
    MP_AGENT_F32(MP_SL_A)
    MP_AGENT_I32(MP_SL_A)
    MP_WORLD_I32(MP_SL_W)
    MP_WORLD_F32(MP_SL_W)
#undef MP_SL_A
#undef MP_SL_W
    G.outBase = S.outBase + g0;
    G.dmg = S.dmg + g0; // stride stays S.dmgStride
    G.visMask = S.visMask + g0;
    G.visOcc = S.visOcc + g0 * S.T * 4;
    G.exploreBits = S.exploreBits + g0 * kExploreTiles;
    G.filtLast = S.filtLast + w0 * 6;
    G.resetKeys = S.resetKeys + g0 * 11;
    G.zoneStats = S.zoneStats + w0 * 25;
    G.spawnTrack = S.spawnTrack + w0 * 3 * track_len;
    G.crumbs = S.crumbs + w0 * kMaxCrumbs * 2;
    G.reset = S.reset + w0;
    G.worldCurr = S.worldCurr + w0;
    G.matchResult = S.matchResult + w0 * 30;
    G.exploreAction = S.exploreAction + g0 * 4;
    G.discreteAction = S.discreteAction + g0 * 4;
    G.aimAction = S.aimAction + g0 * 2;
    G.discreteAim = S.discreteAim + g0 * 2;
    G.policy = S.policy + g0;
    G.botAction = S.botAction + g0 * 7;
    G.reward = S.reward + g0;
    G.done = S.done + g0;
    G.selfObs = S.selfObs + g0 * kSelfObs;
    G.filters = S.filters + g0;
    G.tmObs = S.tmObs + g0 * 5 * kOtherObs;
    G.oppObs = S.oppObs + g0 * 6 * kOtherObs;
    G.lkObs = S.lkObs + g0 * 6 * kOtherObs;
    G.selfPos = S.selfPos + g0 * 3;
    G.tmPos = S.tmPos + g0 * 15;
    G.oppPos = S.oppPos + g0 * 18;
    G.lkPos = S.lkPos + g0 * 18;
    G.masks = S.masks + g0 * 6;
    G.fwdLidar = S.fwdLidar + g0 * kFwdRays * 4;
    G.rearLidar = S.rearLidar + g0 * kRearRays * 4;
    G.agentMap = S.agentMap + g0 * 16 * 16 * 4;
    G.hp = S.hp + g0;
    G.alive = S.alive + g0;
    G.magazine = S.magazine + g0 * 2;
    G.rewardCoefs = S.rewardCoefs + g0 * 9;
    G.ftActions = S.ftActions + w0 * 2 * 6 * 4;
    G.ftGlobal = S.ftGlobal + w0 * 2 * MPENV_FT_GLOBAL_DIM;
    G.ftPlayers = S.ftPlayers + w0 * 2 * 6 * MPENV_FT_PLAYER_DIM;
    G.ftEnemies = S.ftEnemies + w0 * 2 * 6 * MPENV_FT_ENEMY_DIM;
    G.ftLastKnown = S.ftLastKnown + w0 * 2 * 6 * MPENV_FT_COMMON_DIM;
    G.ftFwdLidar = S.ftFwdLidar + w0 * 2 * 6 * kFwdRays * 4;
    G.ftRearLidar = S.ftRearLidar + w0 * 2 * 6 * kRearRays * 4;
    G.ftReward = S.ftReward + w0 * 2;
    G.ftDone = S.ftDone + w0 * 2;
    G.ftPolicy = S.ftPolicy + w0 * 2;
    if (S.recordLog) G.recordLog = S.recordLog + w0;
    if (S.replayLog) G.replayLog = S.replayLog + w0;
    if (S.events) G.events = S.events + w0 * S.evStride;
    if (S.snapshots) G.snapshots = S.snapshots + w0;
}

void mpenv_manager::setupGroups(int want)
{
    // release a previous split
    for (hipStream_t gs : gstreams) {
        HIP_CHECK(hipStreamSynchronize(gs));
        HIP_CHECK(hipStreamDestroy(gs));
    }
    for (hipEvent_t e : joinEv) HIP_CHECK(hipEventDestroy(e));
    if (forkEv) HIP_CHECK(hipEventDestroy(forkEv));
    gstreams.clear();
    joinEv.clear();

    gS.clear();
    gsc.clear();
    forkEv = nullptr;
    // at most 3 (4 measured slower: 66 vs 86 M agent-steps/s at C3)
    groups = std::max(1, std::min(std::min(want, 3), S.W));
    if (groups == 1) return;
    HIP_CHECK(hipEventCreateWithFlags(&forkEv, hipEventDisableTiming));
    for (int i = 0; i < groups; i++) {
        const int64_t w0 = (int64_t)S.W * i / groups, w1 = (int64_t)S.W * (i + 1) / groups;
        DevState G;
        SceneDev gs;
        sliceState(S, sc, w0, w1 - w0, sc.spawnTrackLen, G, gs);
        gS.push_back(G);
        gsc.push_back(gs);
        hipStream_t st;
        HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        gstreams.push_back(st);
        hipEvent_t ev;
        HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        joinEv.push_back(ev);
    }
}

// Live managers: the XLA targets receive a manager pointer inside opaque
// bytes XLA keeps, so they check it against this set before using it (a
// dropped SimManager, or foreign bytes, is then an error, not a read of freed
// memory).
static std::mutex g_liveMu;
static std::unordered_set<const mpenv_manager *> g_live;

static void liveAdd(const mpenv_manager *m)
{
    std::lock_guard<std::mutex> lk(g_liveMu);
    g_live.insert(m);
}

static void liveRemove(const mpenv_manager *m)
{
    std::lock_guard<std::mutex> lk(g_liveMu);
    g_live.erase(m);
}

static bool liveHas(const mpenv_manager *m)
{
    std::lock_guard<std::mutex> lk(g_liveMu);
    return g_live.count(m) != 0;
}

extern "C" {

int32_t mpenv_abi_version(void) { return MPENV_ABI_VERSION; }

const char *mpenv_last_error(void) { return g_last_error.c_str(); }

int mpenv_create(const mpenv_config *cfg, mpenv_manager **out)
{
    if (!cfg || !out) return fail(MPENV_ERR_INVALID, "null argument");
    *out = nullptr;
    if (cfg->exec_mode != MPENV_EXEC_CUDA)
        return fail(MPENV_ERR_UNSUPPORTED, "ExecMode.CPU is not supported: this engine runs only on the GPU (HIP)");
    if (cfg->task_type != MPENV_TASK_ZONE && cfg->task_type != MPENV_TASK_ZONE_CAPTURE_DEFEND)
        return fail(MPENV_ERR_UNSUPPORTED, "only Task.Zone and Task.ZoneCaptureDefend are implemented");
    if (cfg->team_size < 1 || cfg->team_size > kMaxTeamSize)
        return fail(MPENV_ERR_INVALID, "team_size must be in [1, 6]");
    if (cfg->num_worlds == 0) return fail(MPENV_ERR_INVALID, "num_worlds must be > 0");
    if (!cfg->scene_path) return fail(MPENV_ERR_INVALID, "scene_path is required");
    if (cfg->sim_flags >> 12) return fail(MPENV_ERR_INVALID, "sim_flags has bits beyond SubZones (1 << 11)");
    if (cfg->replay_log_path && cfg->record_log_path)
        return fail(MPENV_ERR_UNSUPPORTED, "record and replay logs together are not supported");

    mpenv_manager *m = nullptr;
    try {
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
            return fail(MPENV_ERR_HIP, "no HIP device available");
        if (cfg->gpu_id < 0 || cfg->gpu_id >= ndev) return fail(MPENV_ERR_INVALID, "gpu_id out of range");
        HIP_CHECK(hipSetDevice(cfg->gpu_id));
        m = new mpenv_manager();
        m->S.stats = nullptr;
        m->S.obsGate = nullptr;
        m->S.outTab = nullptr;
        m->S.outBase = 0;
        m->cfg = *cfg;
        m->scenePath = cfg->scene_path;
        m->cfg.scene_path = m->scenePath.c_str();
        m->gpu = cfg->gpu_id;
        // A blocking stream: ordered after work the caller queued on the
        // legacy default stream (e.g. torch writes into the action tensors),
        // matching the synchronous Manager::step contract (mgr.cpp:1949-1960).
        HIP_CHECK(hipStreamCreateWithFlags(&m->stream, hipStreamDefault));
        m->scene = loadScene(m->scenePath, (cfg->sim_flags & MPENV_SIMFLAG_SPAWN_IN_MIDDLE) != 0);
        buildSceneDev(*m);
        m->S.W = (int32_t)cfg->num_worlds;
        m->S.T = (int32_t)cfg->team_size;
        m->S.N = 2 * m->S.T;
        m->S.A = (int64_t)m->S.W * m->S.N;
        m->S.nMagic = (uint32_t)((0x100000000ull + (uint64_t)m->S.N - 1) / (uint64_t)m->S.N);
        if ((uint64_t)m->S.A * (uint64_t)m->S.N * (uint64_t)m->S.N >= 0x100000000ull)
            throw std::runtime_error("mpenv: num_worlds too large for one device (agent index division)");
        allocState(*m);
        openLogs(*m, cfg);
        // the caller's path strings are not kept past create
        m->cfg.replay_log_path = m->cfg.record_log_path = m->cfg.event_log_path = nullptr;
        m->cfg.curriculum_data_path = nullptr;
        {
            // World groups (concurrent streams).  MPENV_WORLD_GROUPS overrides.
            // Two measured best at C3 in rounds 2-4 (round 2: 1.447 ms/step
            // against 1.468 with one); since round 5's load-first k_obs one
            // group is faster (driver window 1.23 vs 1.30 ms, steady 1.178 vs
            // 1.215; profiles/r05e_ab_world_groups.jsonl).
            int want = 1;
            if (const char *e = std::getenv("MPENV_WORLD_GROUPS")) want = std::atoi(e);
            m->setupGroups(want);
        }
        if (const char *e = std::getenv("MPENV_STEP_GRAPH")) m->useGraph = std::atoi(e) != 0;
        if (const char *e = std::getenv("MPENV_LIDAR_BRANCH"))
            if (std::atoi(e) != 0 && mpenv_set_lidar_branch(m, 1) != MPENV_OK) throw std::runtime_error(g_last_error);
        // TrainControl from sim flags (mgr.cpp:1397-1413)
        int32_t tc[3] = { (cfg->sim_flags & MPENV_SIMFLAG_SIM_EVAL_MODE) ? 1 : 0,
                          (cfg->sim_flags & MPENV_SIMFLAG_STAGGER_STARTS) ? 1 : 0,
                          (cfg->sim_flags & MPENV_SIMFLAG_RANDOM_FLIP_TEAMS) ? 1 : 0 };
        HIP_CHECK(hipMemcpyAsync(m->S.trainCtrl, tc, sizeof(tc), hipMemcpyHostToDevice, m->stream));
        if (launchConstruct(m->S, m->sc, tc, m->stream)) throw std::runtime_error("construct launch failed");
        HIP_CHECK(hipStreamSynchronize(m->stream));
        liveAdd(m);
        *out = m;
        return MPENV_OK;
    } catch (const std::exception &e) {
        delete m;
        std::string msg = e.what();
        bool io = msg.find("open") != std::string::npos || msg.find("truncated") != std::string::npos;
        return fail(io ? MPENV_ERR_IO : MPENV_ERR_HIP, msg);
    }
}

void mpenv_destroy(mpenv_manager *m)
{
    if (m) liveRemove(m);
    delete m;
}

int mpenv_init(mpenv_manager *m)
{
    if (!m) return fail(MPENV_ERR_INVALID, "null manager");
    try {
        m->runInitGraph(m->stream);
        HIP_CHECK(hipStreamSynchronize(m->stream));
    } catch (const std::exception &e) {
        return fail(MPENV_ERR_HIP, e.what());
    }
    return MPENV_OK;
}

int mpenv_step_async(mpenv_manager *m, void *stream)
{
    if (!m) return fail(MPENV_ERR_INVALID, "null manager");
    try {
        m->runStep(stream ? (hipStream_t)stream : m->stream);
    } catch (const std::exception &e) {
        return fail(MPENV_ERR_HIP, e.what());
    }
    return MPENV_OK;
}

int mpenv_step(mpenv_manager *m)
{
    if (!m) return fail(MPENV_ERR_INVALID, "null manager");
    try {
        m->runStep(m->stream);
        HIP_CHECK(hipStreamSynchronize(m->stream));
    } catch (const std::exception &e) {
        return fail(MPENV_ERR_HIP, e.what());
    }
    return MPENV_OK;
}

int mpenv_export_tensor(mpenv_manager *m, int32_t id, void **ptr, int32_t *dtype, int32_t *ndim, int64_t *dims,
                        int32_t *gpu_id)
{
    if (!m || !ptr || !dtype || !ndim || !dims) return fail(MPENV_ERR_INVALID, "null argument");
    TensorDesc d;
    try {
        if (!m->exportDesc(id, d)) return fail(MPENV_ERR_INVALID, "unknown export id " + std::to_string(id));
    } catch (const std::exception &e) {
        return fail(MPENV_ERR_HIP, e.what());
    }
    *ptr = d.ptr;
    *dtype = d.dtype;
    *ndim = (int32_t)d.dims.size();
    for (size_t k = 0; k < d.dims.size(); k++) dims[k] = d.dims[k];
    if (gpu_id) *gpu_id = m->gpu;
    return MPENV_OK;
}

int mpenv_train_interface_size(int32_t *num_inputs, int32_t *num_outputs)
{
    if (num_inputs) *num_inputs = kNumTIInputs;
    if (num_outputs) *num_outputs = kNumTIOutputs;
    return MPENV_OK;
}

int mpenv_train_interface_entry(int32_t is_output, int32_t idx, const char **name, int32_t *export_id)
{
    const TIEntry *tab = is_output ? kTIOutputs : kTIInputs;
    int n = is_output ? kNumTIOutputs : kNumTIInputs;
    if (idx < 0 || idx >= n) return fail(MPENV_ERR_INVALID, "train interface index out of range");
    if (name) *name = tab[idx].name;
    if (export_id) *export_id = tab[idx].id;
    return MPENV_OK;
}

// cudaCopyStepInputs / cudaCopyStepOutputs (mgr.cpp:614-645): every
// trainInterface input from the caller's buffers, or every output into
// them, as one batched copy launch (the agent maps are never written by the
// step and stay all zeros, so their copies are zero fills); a segment whose
// pointers are not 16-B aligned falls back to hipMemcpyAsync.
// zeros: 1 = only the agent maps' zero fills, 0 or -2 = the other outputs
// only, -1 = every output.
// The outputs gpuStreamStep has k_obs / k_lidar write straight into the
// caller's buffers (engine.h OutTab) instead of copying them afterwards.
static bool directOutput(int32_t id)
{
    switch (id) {
    case MPENV_EXPORT_OPPONENT_MASKS: case MPENV_EXPORT_FILTERS_STATE: case MPENV_EXPORT_SELF_OBSERVATION:
    case MPENV_EXPORT_SELF_POSITION: case MPENV_EXPORT_TEAMMATE_OBSERVATIONS:
    case MPENV_EXPORT_TEAMMATE_POSITIONS: case MPENV_EXPORT_OPPONENT_OBSERVATIONS:
    case MPENV_EXPORT_OPPONENT_POSITIONS: case MPENV_EXPORT_FWD_LIDAR: case MPENV_EXPORT_REAR_LIDAR:
        return true;
    default:
        return false;
    }
}

// The call's OutTab, or false when some direct output's buffer is missing
// or not 16-B aligned (the kernels store float4 rows): then every output is
// copied as before.
static bool directTable(void **buffers, OutTab &t)
{
    t = OutTab {};
    t.on = 1;
    int maps = 0;
    for (int i = 0; i < kNumTIOutputs; i++) {
        const int32_t id = kTIOutputs[i].id;
        if (!directOutput(id) && id != MPENV_EXPORT_AGENT_MAP) continue;
        float *p = static_cast<float *>(buffers[kNumTIInputs + i]);
        if (!p || ((uintptr_t)p & 15u)) return false;
        if (id == MPENV_EXPORT_AGENT_MAP) {
            (maps++ == 0 ? t.agentMap0 : t.agentMap1) = p;
            continue;
        }
        switch (id) {
        case MPENV_EXPORT_OPPONENT_MASKS: t.masks = p; break;
        case MPENV_EXPORT_FILTERS_STATE: t.filters = p; break;
        case MPENV_EXPORT_SELF_OBSERVATION: t.selfObs = p; break;
        case MPENV_EXPORT_SELF_POSITION: t.selfPos = p; break;
        case MPENV_EXPORT_TEAMMATE_OBSERVATIONS: t.tmObs = p; break;
        case MPENV_EXPORT_TEAMMATE_POSITIONS: t.tmPos = p; break;
        case MPENV_EXPORT_OPPONENT_OBSERVATIONS: t.oppObs = p; break;
        case MPENV_EXPORT_OPPONENT_POSITIONS: t.oppPos = p; break;
        case MPENV_EXPORT_FWD_LIDAR: t.fwdLidar = p; break;
        case MPENV_EXPORT_REAR_LIDAR: t.rearLidar = p; break;
        default: break;
        }
    }
    return maps == 2;
}

static int copyTI(mpenv_manager *m, hipStream_t st, void **buffers, bool inputs, bool outputs, int zeros = -1,
                  bool skip_direct = false, const OutTab *tab = nullptr)
{
    CopyBatch b {};
    if (tab) { // the out table rides the first copy launch (engine.h CopyBatch)
        b.tabDst = m->outTabDev;
        b.tab = *tab;
    }
    auto add = [&](const void *src, void *dst, size_t bytes) {
        if (((uintptr_t)src | (uintptr_t)dst) & 15u) {
            if (src) HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st));
            else HIP_CHECK(hipMemsetAsync(dst, 0, bytes, st));
            return;
        }
        if (b.n == kMaxCopySegs) {
            if (launchCopyBatch(b, st)) throw std::runtime_error("copy launch failed");
            b.n = 0;
            b.tabDst = nullptr;
        }
        b.seg[b.n++] = CopySeg { src, dst, (int64_t)bytes };
    };
    int k = 0;
    for (int i = 0; i < kNumTIInputs; i++, k++) {
        if (!inputs || !buffers[k]) continue;
        TensorDesc d;
        m->exportDesc(kTIInputs[i].id, d);
        add(buffers[k], d.ptr, d.bytes());
    }
    for (int i = 0; i < kNumTIOutputs; i++, k++) {
        if (!outputs || !buffers[k]) continue;
        const bool zero = kTIOutputs[i].id == MPENV_EXPORT_AGENT_MAP;
        if ((zeros == 1 && !zero) || ((zeros == 0 || zeros == -2) && zero)) continue;
        if (skip_direct && directOutput(kTIOutputs[i].id)) continue;
        TensorDesc d;
        m->exportDesc(kTIOutputs[i].id, d);
        add(zero ? nullptr : d.ptr, buffers[k], d.bytes());
    }
    if ((b.n > 0 || b.tabDst) && launchCopyBatch(b, st)) throw std::runtime_error("copy launch failed");
    return 0;
}

// gpuStreamStep's side stream for the zero fills and its fork / join events,
// made by gpuStreamInit (outside any graph capture of the steps that follow)
static void ensureZStream(mpenv_manager *m)
{
    if (m->zStream) return;
    HIP_CHECK(hipStreamCreateWithFlags(&m->zStream, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreateWithFlags(&m->zForkEv, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&m->zJoinEv, hipEventDisableTiming));
}

// mgr.cpp:507-612
int mpenv_gpu_stream_init(mpenv_manager *m, void *stream, void **buffers)
{
    if (!m || !buffers) return fail(MPENV_ERR_INVALID, "null argument");
    try {
        ensureZStream(m);
        hipStream_t st = stream ? (hipStream_t)stream : m->stream;
        m->runInitGraph(st);
        copyTI(m, st, buffers, false, true);
    } catch (const std::exception &e) {
        return fail(MPENV_ERR_HIP, e.what());
    }
    return MPENV_OK;
}

// mgr.cpp:614-645
int mpenv_gpu_stream_step(mpenv_manager *m, void *stream, void **buffers)
{
    if (!m || !buffers) return fail(MPENV_ERR_INVALID, "null argument");
    try {
        hipStream_t st = stream ? (hipStream_t)stream : m->stream;
        ensureZStream(m);
        // The observation rows, the lidar and the agent maps' zeros go
        // straight into the caller's buffers (OutTab, set in front of the
        // step and cleared behind it, so the captured step graph is the same
        // for every call); the rest -- the state-backed outputs (hp,
        // magazine, alive, last-known rows, rewards, dones, episode results)
        // -- is copied after the step.
        OutTab tab;
        const bool direct = directTable(buffers, tab);
        if (!direct) {
            // every output copied: the zero fills (1.6 GB of stores at C3)
            // beside the step, ordered after whatever the caller queued
            HIP_CHECK(hipEventRecord(m->zForkEv, st));
            HIP_CHECK(hipStreamWaitEvent(m->zStream, m->zForkEv, 0));
            copyTI(m, m->zStream, buffers, false, true, 1);
            HIP_CHECK(hipEventRecord(m->zJoinEv, m->zStream));
        }
        const OutTab off {};
        copyTI(m, st, buffers, true, false, -1, false, direct ? &tab : nullptr); // sets the table
        m->runStep(st);
        copyTI(m, st, buffers, false, true, 0, direct, direct ? &off : nullptr); // clears it
        if (!direct) HIP_CHECK(hipStreamWaitEvent(st, m->zJoinEv, 0));
    } catch (const std::exception &e) {
        return fail(MPENV_ERR_HIP, e.what());
    }
    return MPENV_OK;
}

int mpenv_debug_trace_rays(mpenv_manager *m, const float *o, const float *d, int32_t n, int32_t mode, float *t_out,
                           int32_t *hit_out, void *stream)
{
    if (!m || !o || !d || !t_out || !hit_out || n < 0) return fail(MPENV_ERR_INVALID, "bad argument");
    hipStream_t st = stream ? (hipStream_t)stream : m->stream;
    if (launchTraceRays(m->sc, o, d, n, mode, t_out, hit_out, st) || hipStreamSynchronize(st) != hipSuccess)
        return fail(MPENV_ERR_HIP, "trace-ray launch failed");
    return MPENV_OK;
}

// XLA GPU custom-call targets (SimManager.jax(); include/mpenv.h)
static std::atomic<int64_t> g_xlaErrors { 0 };

int mpenv_xla_opaque_make(mpenv_manager *m, mpenv_xla_opaque *out)
{
    if (!m || !out) return fail(MPENV_ERR_INVALID, "null argument");
    *out = mpenv_xla_opaque {};
    out->magic = MPENV_XLA_MAGIC;
    out->version = MPENV_XLA_VERSION;
    out->manager = (uint64_t)(uintptr_t)m;
    out->num_buffers = kNumTIInputs + kNumTIOutputs;
    return MPENV_OK;
}

// The manager an opaque names, or null (with mpenv_last_error set) when the
// bytes are not an opaque of this build or name no live manager.
static mpenv_manager *xlaManager(const char *opaque, size_t len)
{
    mpenv_xla_opaque o;
    if (!opaque || len != sizeof(o)) {
        fail(MPENV_ERR_INVALID, "bad XLA opaque: " + std::to_string(len) + " bytes, expected " +
                                    std::to_string(sizeof(o)));
        return nullptr;
    }
    std::memcpy(&o, opaque, sizeof(o));
    if (o.magic != MPENV_XLA_MAGIC || o.version != MPENV_XLA_VERSION || o.num_buffers != kNumTIInputs + kNumTIOutputs) {
        fail(MPENV_ERR_INVALID, "bad XLA opaque: not made by mpenv_xla_opaque_make of this build");
        return nullptr;
    }
    mpenv_manager *m = reinterpret_cast<mpenv_manager *>((uintptr_t)o.manager);
    if (!liveHas(m)) {
        fail(MPENV_ERR_INVALID, "bad XLA opaque: its manager was destroyed (keep the SimManager alive while the "
                                "registered custom call is in use)");
        return nullptr;
    }
    return m;
}

static int xlaRun(bool step, void *stream, void **buffers, const char *opaque, size_t opaque_len)
{
    mpenv_manager *m = xlaManager(opaque, opaque_len);
    if (!m) return MPENV_ERR_INVALID;
    return step ? mpenv_gpu_stream_step(m, stream, buffers) : mpenv_gpu_stream_init(m, stream, buffers);
}

// API version 1 has no error channel: like the reference's REQ_CUDA / FATAL
// (mgr.cpp:514-531, 620-638) a failure is reported on stderr and aborts the
// process rather than leaving XLA with result buffers that were never written.
[[noreturn]] static void xlaFatal(const char *what)
{
    std::fprintf(stderr, "mpenv: XLA custom call %s failed: %s\n", what, g_last_error.c_str());
    std::fflush(stderr);
    std::abort();
}

void mpenv_xla_gpu_stream_init(void *stream, void **buffers, const char *opaque, size_t opaque_len)
{
    if (xlaRun(false, stream, buffers, opaque, opaque_len) != MPENV_OK) xlaFatal("gpuStreamInit");
}

void mpenv_xla_gpu_stream_step(void *stream, void **buffers, const char *opaque, size_t opaque_len)
{
    if (xlaRun(true, stream, buffers, opaque, opaque_len) != MPENV_OK) xlaFatal("gpuStreamStep");
}

// API_VERSION_STATUS_RETURNING: the failure goes to XLA through
// XlaCustomCallStatusSetFailure, exported by the XLA runtime that calls the
// target (jaxlib); it is looked up at run time so this library links without
// XLA.  Without it there is no one to hand the status to: abort as above.
typedef void (*XlaStatusSetFailureFn)(void *status, const char *message, size_t message_len);

static void xlaStatusFail(const char *what, void *status)
{
    static XlaStatusSetFailureFn fn =
        reinterpret_cast<XlaStatusSetFailureFn>(dlsym(RTLD_DEFAULT, "XlaCustomCallStatusSetFailure"));
    if (!fn || !status) xlaFatal(what);
    g_xlaErrors.fetch_add(1);
    const std::string msg = std::string("mpenv: ") + what + ": " + g_last_error;
    fn(status, msg.data(), msg.size());
}

void mpenv_xla_gpu_stream_init_status(void *stream, void **buffers, const char *opaque, size_t opaque_len,
                                      void *status)
{
    if (xlaRun(false, stream, buffers, opaque, opaque_len) != MPENV_OK) xlaStatusFail("gpuStreamInit", status);
}

void mpenv_xla_gpu_stream_step_status(void *stream, void **buffers, const char *opaque, size_t opaque_len,
                                      void *status)
{
    if (xlaRun(true, stream, buffers, opaque, opaque_len) != MPENV_OK) xlaStatusFail("gpuStreamStep", status);
}

int64_t mpenv_xla_errors(void) { return g_xlaErrors.load(); }

// Learner exchange wire format (wire.hip)
int mpenv_wire_bytes(mpenv_manager *m, int32_t keyframe, int64_t *bytes)
{
    if (!m || !bytes) return fail(MPENV_ERR_INVALID, "null argument");
    *bytes = wireBytes(m->S, keyframe != 0);
    return MPENV_OK;
}

int mpenv_wire_pack(mpenv_manager *m, void *dst, int32_t keyframe, void *stream)
{
    if (!m || !dst) return fail(MPENV_ERR_INVALID, "null argument");
    if ((uintptr_t)dst & 15u) return fail(MPENV_ERR_INVALID, "wire message buffer must be 16-B aligned");
    if (launchWirePack(m->S, static_cast<char *>(dst), keyframe != 0, m->sc.worldOffset,
                       stream ? stream : (void *)m->stream))
        return fail(MPENV_ERR_HIP, "wire pack launch failed");
    return MPENV_OK;
}

int mpenv_wire_unpack(mpenv_manager *m, const void *src, int32_t keyframe, void *stream)
{
    if (!m || !src) return fail(MPENV_ERR_INVALID, "null argument");
    if ((uintptr_t)src & 15u) return fail(MPENV_ERR_INVALID, "wire message buffer must be 16-B aligned");
    void *st = stream ? stream : (void *)m->stream;
    const int W = m->S.W;
    int32_t *prev = m->wireEp + (size_t)m->wireParity * W, *next = m->wireEp + (size_t)(m->wireParity ^ 1) * W;
    if (launchWireUnpack(m->S, m->sc, static_cast<const char *>(src), keyframe != 0, m->wireErr, m->sc.worldOffset,
                         prev, next, st))
        return fail(MPENV_ERR_HIP, "wire unpack launch failed");
    m->wireParity ^= 1;
    return MPENV_OK;
}

// The error word's bits now; the refused bit is cleared by this read, the
// desync bit stays until a keyframe is unpacked (wire.hip wireOk).  `stream`
// null: the whole device is synchronised first (every unpack queued so far
// has run); otherwise the read is ordered on that stream only, and with a
// pinned `out` (hipHostMalloc / torch pin_memory) the call does not block:
// the value lands when the stream reaches it (record an event after the
// call and wait on it before reading *out).
int mpenv_wire_error_async(mpenv_manager *m, uint32_t *out, void *stream)
{
    if (!m || !out) return fail(MPENV_ERR_INVALID, "null argument");
    try {
        hipStream_t st = (hipStream_t)stream;
        HIP_CHECK(hipMemcpyAsync(out, m->wireErr, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        // clear REFUSED, keep DESYNC: one atomic AND on the device word
        if (launchWireErrClear(m->wireErr, st)) throw std::runtime_error("wire error clear launch failed");
    } catch (const std::exception &e) {
        return fail(MPENV_ERR_HIP, e.what());
    }
    return MPENV_OK;
}

int mpenv_wire_error(mpenv_manager *m, uint32_t *out)
{
    if (!m || !out) return fail(MPENV_ERR_INVALID, "null argument");
    try {
        HIP_CHECK(hipDeviceSynchronize());
        uint32_t v = 0;
        HIP_CHECK(hipMemcpy(&v, m->wireErr, sizeof(uint32_t), hipMemcpyDeviceToHost));
        *out = v;
        // the refused bit is cleared by this read; the desync bit stays until a
        // keyframe is unpacked (wire.hip wireOk)
        const uint32_t keep = v & MPENV_WIRE_ERR_DESYNC;
        HIP_CHECK(hipMemcpy(m->wireErr, &keep, sizeof(uint32_t), hipMemcpyHostToDevice));
    } catch (const std::exception &e) {
        return fail(MPENV_ERR_HIP, e.what());
    }
    return MPENV_OK;
}

int mpenv_graph_captures(mpenv_manager *m, int64_t *out)
{
    if (!m || !out) return fail(MPENV_ERR_INVALID, "null argument");
    *out = m->graphCaptures;
    return MPENV_OK;
}

int mpenv_graph_status(mpenv_manager *m, int32_t *graph_on, char *reason, int32_t reason_len)
{
    if (!m || !graph_on) return fail(MPENV_ERR_INVALID, "null argument");
    *graph_on = m->useGraph ? 1 : 0;
    if (reason && reason_len > 0) {
        std::snprintf(reason, (size_t)reason_len, "%s", m->graphOffReason.c_str());
    }
    return MPENV_OK;
}

int mpenv_set_lidar_branch(mpenv_manager *m, int32_t on)
{
    if (!m) return fail(MPENV_ERR_INVALID, "null argument");
    try {
        HIP_CHECK(hipStreamSynchronize(m->stream));
        if (on && !m->bStream) {
            HIP_CHECK(hipStreamCreateWithFlags(&m->bStream, hipStreamNonBlocking));
            HIP_CHECK(hipEventCreateWithFlags(&m->bForkEv, hipEventDisableTiming));
            HIP_CHECK(hipEventCreateWithFlags(&m->bJoinEv, hipEventDisableTiming));
        }
        m->lidarBranch = on != 0;
    } catch (const std::exception &e) {
        return fail(MPENV_ERR_HIP, e.what());
    }
    return MPENV_OK;
}

int mpenv_set_world_groups(mpenv_manager *m, int32_t groups)
{
    if (!m || groups < 1) return fail(MPENV_ERR_INVALID, "bad argument");
    try {
        HIP_CHECK(hipStreamSynchronize(m->stream));
        m->setupGroups(groups);
    } catch (const std::exception &e) {
        return fail(MPENV_ERR_HIP, e.what());
    }
    return MPENV_OK;
}

int mpenv_world_groups(mpenv_manager *m, int32_t *groups)
{
    if (!m || !groups) return fail(MPENV_ERR_INVALID, "bad argument");
    *groups = m->groups;
    return MPENV_OK;
}

int mpenv_copy_actions(mpenv_manager *m, const int32_t *src, void *stream)
{
    if (!m || !src) return fail(MPENV_ERR_INVALID, "null argument");
    if (launchFillActions(m->S, src, stream ? stream : (void *)m->stream))
        return fail(MPENV_ERR_HIP, "action copy launch failed");
    return MPENV_OK;
}

int mpenv_combat_actions(mpenv_manager *m, const int32_t *tape, int32_t *out, int32_t mode, void *stream)
{
    if (!m || !tape) return fail(MPENV_ERR_INVALID, "null argument");
    if (mode != 0 && mode != 1) return fail(MPENV_ERR_INVALID, "combat action mode must be 0 or 1");
    if (launchCombatActions(m->S, tape, out, mode, stream ? stream : (void *)m->stream))
        return fail(MPENV_ERR_HIP, "combat action launch failed");
    return MPENV_OK;
}

static int checkAgent(mpenv_manager *m, int32_t w, int32_t a)
{
    if (!m) return fail(MPENV_ERR_INVALID, "null manager");
    if (w < 0 || w >= m->S.W) return fail(MPENV_ERR_INVALID, "world index out of range");
    if (a < 0 || a >= m->S.N) return fail(MPENV_ERR_INVALID, "agent index out of range");
    return MPENV_OK;
}

// Setter upload: ordered after in-flight work on the manager stream.
static bool put(mpenv_manager *m, void *dst, const void *src, size_t bytes)
{
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, m->stream) == hipSuccess &&
           hipStreamSynchronize(m->stream) == hipSuccess;
}

int mpenv_trigger_reset(mpenv_manager *m, int32_t w)
{
    if (int rc = checkAgent(m, w, 0)) return rc;
    int32_t one = 1;
    if (!put(m, m->S.reset + w, &one, 4))
        return fail(MPENV_ERR_HIP, "hipMemcpy failed");
    return MPENV_OK;
}

int mpenv_set_pvp_action(mpenv_manager *m, int32_t w, int32_t a, const int32_t discrete[4], const float aim[2],
                         const int32_t aim_discrete[2])
{
    if (int rc = checkAgent(m, w, a)) return rc;
    const int64_t g = (int64_t)w * m->S.N + a;
    bool ok = true;
    if (discrete) ok &= put(m, m->S.discreteAction + 4 * g, discrete, 16);
    if (aim) ok &= put(m, m->S.aimAction + 2 * g, aim, 8);
    if (aim_discrete) ok &= put(m, m->S.discreteAim + 2 * g, aim_discrete, 8);
    return ok ? MPENV_OK : fail(MPENV_ERR_HIP, "hipMemcpy failed");
}

int mpenv_set_hp(mpenv_manager *m, int32_t w, int32_t a, int32_t hp)
{
    if (int rc = checkAgent(m, w, a)) return rc;
    float v = (float)hp;
    if (!put(m, m->S.hp + (int64_t)w * m->S.N + a, &v, 4))
        return fail(MPENV_ERR_HIP, "hipMemcpy failed");
    return MPENV_OK;
}

int mpenv_set_agent_policy(mpenv_manager *m, int32_t w, int32_t a, int32_t policy)
{
    if (int rc = checkAgent(m, w, a)) return rc;
    if (!put(m, m->S.policy + (int64_t)w * m->S.N + a, &policy, 4))
        return fail(MPENV_ERR_HIP, "hipMemcpy failed");
    return MPENV_OK;
}

int mpenv_set_uniform_agent_policy(mpenv_manager *m, int32_t policy)
{
    if (!m) return fail(MPENV_ERR_INVALID, "null manager");
    if (hipMemsetD32Async((hipDeviceptr_t)m->S.policy, policy, (size_t)m->S.A, m->stream) != hipSuccess ||
        hipStreamSynchronize(m->stream) != hipSuccess)
        return fail(MPENV_ERR_HIP, "hipMemsetD32 failed");
    return MPENV_OK;
}

// Manager::isReplayFinished (mgr.cpp:2603-2617): the replay file hit EOF
int mpenv_is_replay_finished(mpenv_manager *m, int32_t *finished)
{
    if (!m || !finished) return fail(MPENV_ERR_INVALID, "null argument");
    if (!m->replayFile) return fail(MPENV_ERR_INVALID, "no replay log configured");
    if (!m->replayEof) {
        const int c = std::fgetc(m->replayFile);
        if (c == EOF) m->replayEof = true;
        else std::ungetc(c, m->replayFile);
    }
    *finished = m->replayEof ? 1 : 0;
    return MPENV_OK;
}

int mpenv_dims(mpenv_manager *m, int32_t *num_worlds, int32_t *agents_per_world)
{
    if (!m) return fail(MPENV_ERR_INVALID, "null manager");
    if (num_worlds) *num_worlds = m->S.W;
    if (agents_per_world) *agents_per_world = m->S.N;
    return MPENV_OK;
}

int mpenv_enable_kernel_timing(mpenv_manager *m, int32_t enable)
{
    if (!m) return fail(MPENV_ERR_INVALID, "null manager");
    m->timing = enable != 0;
    m->eventsUsed = 0;
    return MPENV_OK;
}

int mpenv_enable_stats(mpenv_manager *m, int32_t enable)
{
    if (!m) return fail(MPENV_ERR_INVALID, "null manager");
    try {
        HIP_CHECK(hipStreamSynchronize(m->stream));
        for (hipStream_t gs : m->gstreams) HIP_CHECK(hipStreamSynchronize(gs));
        if (enable && !m->statsBuf) m->statsBuf = m->alloc<unsigned long long>(kNumStats);
        if (enable) HIP_CHECK(hipMemsetAsync(m->statsBuf, 0, sizeof(unsigned long long) * kNumStats, m->stream));
        HIP_CHECK(hipStreamSynchronize(m->stream));
    } catch (const std::exception &e) {
        return fail(MPENV_ERR_HIP, e.what());
    }
    unsigned long long *p = enable ? m->statsBuf : nullptr;
    m->S.stats = p;
    for (DevState &G : m->gS) G.stats = p;
    return MPENV_OK;
}

int mpenv_read_stats(mpenv_manager *m, uint64_t *out, int32_t n)
{
    if (!m || !out) return fail(MPENV_ERR_INVALID, "null argument");
    std::vector<unsigned long long> h(kNumStats, 0ull);
    try {
        HIP_CHECK(hipDeviceSynchronize());
        if (m->statsBuf)
            HIP_CHECK(hipMemcpy(h.data(), m->statsBuf, sizeof(unsigned long long) * kNumStats,
                                hipMemcpyDeviceToHost));
    } catch (const std::exception &e) {
        return fail(MPENV_ERR_HIP, e.what());
    }
    for (int k = 0; k < n && k < kNumStats; k++) out[k] = h[k];
    return kNumStats;
}

int mpenv_kernel_timings(mpenv_manager *m, int32_t max_n, const char **names, float *avg_ms, int32_t *launches)
{
    if (!m) return fail(MPENV_ERR_INVALID, "null manager");
    const int nk = kNumTimedKernels;
    std::vector<double> sum(nk, 0.0);
    int steps = 0;
    try {
        HIP_CHECK(hipDeviceSynchronize());
        // events per step: nk + 1 boundaries
        const size_t per = (size_t)nk + 1;
        for (size_t base = 0; base + per <= m->eventsUsed; base += per) {
            for (int k = 0; k < nk; k++) {
                float ms = 0.f;
                HIP_CHECK(hipEventElapsedTime(&ms, m->eventPool[base + k], m->eventPool[base + k + 1]));
                sum[k] += ms;
            }
            steps++;
        }
    } catch (const std::exception &e) {
        return fail(MPENV_ERR_HIP, e.what());
    }
    m->eventsUsed = 0;
    for (int k = 0; k < nk && k < max_n; k++) {
        if (names) names[k] = kernelName(k);
        if (avg_ms) avg_ms[k] = steps ? (float)(sum[k] / steps) : 0.f;
        if (launches) launches[k] = steps;
    }
    return nk;
}

// Host-side access to the navmesh and A* table (tests / oracle input).
int mpenv_scene_navmesh(const char *scene_path, float *tri_verts_out, int32_t *num_tris, int32_t *adj_out,
                        int32_t *astar_out)
{
    try {
        Scene s = loadScene(scene_path);
        const NavMesh &nm = s.nav;
        const int32_t T = (int32_t)nm.numTris();
        if (num_tris) {
            if (*num_tris >= T) {
                for (int32_t t = 0; t < T; t++)
                    for (int k = 0; k < 3; k++) {
                        const mp::Vec3 v = nm.verts[nm.tris[3 * t + k]];
                        if (tri_verts_out) {
                            tri_verts_out[9 * t + 3 * k + 0] = v.x;
                            tri_verts_out[9 * t + 3 * k + 1] = v.y;
                            tri_verts_out[9 * t + 3 * k + 2] = v.z;
                        }
                        if (adj_out) adj_out[3 * t + k] = nm.adj[3 * t + k];
                    }
                if (astar_out) std::memcpy(astar_out, nm.astar.data(), sizeof(int32_t) * nm.astar.size());
            }
            *num_tris = T;
        }
    } catch (const std::exception &e) {
        return fail(MPENV_ERR_IO, e.what());
    }
    return MPENV_OK;
}

// The quirk guard k_move uploads (for tests).
int mpenv_scene_quirk_grid(const char *scene_path, int32_t *header_out, uint32_t *bits_out, int32_t *num_words)
{
    if (!num_words) return fail(MPENV_ERR_INVALID, "num_words is null");
    try {
        Scene s = loadScene(scene_path);
        const QuirkGrid q = quirkGrid(s.bvhVerts, 15.f, 2.f, 16.f);
        if (header_out) {
            std::memcpy(&header_out[0], &q.minX, 4);
            std::memcpy(&header_out[1], &q.minY, 4);
            std::memcpy(&header_out[2], &q.cell, 4);
            header_out[3] = q.w;
            header_out[4] = q.h;
        }
        if (bits_out && *num_words >= (int32_t)q.bits.size())
            std::memcpy(bits_out, q.bits.data(), q.bits.size() * 4);
        *num_words = (int32_t)q.bits.size();
    } catch (const std::exception &e) {
        return fail(MPENV_ERR_IO, e.what());
    }
    return MPENV_OK;
}

// Host-side access to the scene BVH (for the parity oracle and tests).
int mpenv_scene_bvh_variant(const char *scene_path, const int32_t *opts, int32_t num_opts, void *nodes_out,
                            int32_t *num_nodes, float *verts_out, int32_t *num_verts, int32_t *max_stack)
{
    try {
        Scene s = loadScene(scene_path);
        BVHBuildOpts o;
        if (opts && num_opts > 0) o.maxLeaf = opts[0];
        if (opts && num_opts > 1) o.bins = opts[1];
        if (opts && num_opts > 2) o.measure = opts[2];
        if (opts && num_opts > 3) o.travCost = (float)opts[3] / 100.f;
        if (opts && num_opts > 4) o.floorWeight = (float)opts[4] / 100.f;
        for (int32_t k = 5; opts && k + 1 < num_opts; k += 2) {
            if (opts[k] >= 0) o.splitRank[(uint64_t)opts[k]] = opts[k + 1];
            else o.collapseChoice[(uint64_t)(-(int64_t)opts[k])] = opts[k + 1];
        }
        Scene t;
        buildBVH(s.triVerts, t, o);
        if (num_nodes) {
            if (nodes_out && *num_nodes >= (int32_t)t.nodes.size())
                std::memcpy(nodes_out, t.nodes.data(), t.nodes.size() * sizeof(BVHNode));
            *num_nodes = (int32_t)t.nodes.size();
        }
        if (num_verts) {
            if (verts_out && *num_verts >= (int32_t)t.bvhVerts.size())
                std::memcpy(verts_out, t.bvhVerts.data(), t.bvhVerts.size() * 12);
            *num_verts = (int32_t)t.bvhVerts.size();
        }
        if (max_stack) *max_stack = std::max(t.maxStack, t.maxStackAnyOrder);
    } catch (const std::exception &e) {
        return fail(MPENV_ERR_IO, e.what());
    }
    return MPENV_OK;
}

int mpenv_scene_lidar_bvh(const char *scene_path, void *nodes_out, int32_t *num_nodes, float *verts_out,
                          int32_t *num_verts, int32_t *max_stack)
{
    try {
        Scene s = loadScene(scene_path);
        if (num_nodes) {
            if (nodes_out && *num_nodes >= (int32_t)s.lidarNodes.size())
                std::memcpy(nodes_out, s.lidarNodes.data(), s.lidarNodes.size() * sizeof(BVHNode));
            *num_nodes = (int32_t)s.lidarNodes.size();
        }
        if (num_verts) {
            if (verts_out && *num_verts >= (int32_t)s.lidarVerts.size())
                std::memcpy(verts_out, s.lidarVerts.data(), s.lidarVerts.size() * 12);
            *num_verts = (int32_t)s.lidarVerts.size();
        }
        if (max_stack) *max_stack = s.lidarMaxStack;
    } catch (const std::exception &e) {
        return fail(MPENV_ERR_IO, e.what());
    }
    return MPENV_OK;
}

int mpenv_scene_bvh(const char *scene_path, void *nodes_out, int32_t *num_nodes, float *verts_out,
                    int32_t *num_verts, int32_t *max_stack)
{
    try {
        Scene s = loadScene(scene_path);
        if (num_nodes) {
            if (nodes_out && *num_nodes >= (int32_t)s.nodes.size())
                std::memcpy(nodes_out, s.nodes.data(), s.nodes.size() * sizeof(BVHNode));
            *num_nodes = (int32_t)s.nodes.size();
        }
        if (num_verts) {
            if (verts_out && *num_verts >= (int32_t)s.bvhVerts.size())
                std::memcpy(verts_out, s.bvhVerts.data(), s.bvhVerts.size() * 12);
            *num_verts = (int32_t)s.bvhVerts.size();
        }
        if (max_stack) *max_stack = std::max(s.maxStack, s.maxStackAnyOrder);
    } catch (const std::exception &e) {
        return fail(MPENV_ERR_IO, e.what());
    }
    return MPENV_OK;
}

} // extern "C"
