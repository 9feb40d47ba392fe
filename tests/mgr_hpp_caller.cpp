// A caller written against the reference's Manager (src/mgr.hpp:31-161):
// it names every public method with the reference's signature (member
// pointers, so a missing or mistyped declaration fails to compile), then
// checks at run time, without a GPU, that the out-of-scope parts throw
// instead of misbehaving.  Built and run by tests/test_abi.py.
#include <cstdio>
#include <cstring>
#include <stdexcept>

#include "mpenv_manager.hpp"

using namespace madronaMPEnv;

template <typename T> static void use(T) {}

int main(int argc, char **argv)
{
    // mgr.hpp signatures, one member pointer each
    use<void (Manager::*)()>(&Manager::init);
    use<void (Manager::*)()>(&Manager::step);
    use<void (Manager::*)()>(&Manager::vizStep);
    use<void (Manager::*)(void **, void **)>(&Manager::cpuJAXInit);
    use<void (Manager::*)(void **, void **)>(&Manager::cpuJAXStep);
    use<void (Manager::*)(void *, void **)>(&Manager::gpuStreamInit);
    use<void (Manager::*)(void *, void **)>(&Manager::gpuStreamStep);
    using Getter = Tensor (Manager::*)() const;
    const Getter getters[] = {
        &Manager::resetTensor, &Manager::simControlTensor, &Manager::matchResultTensor,
        &Manager::pvpDiscreteActionTensor, &Manager::pvpAimActionTensor, &Manager::pvpDiscreteAimActionTensor,
        &Manager::exploreActionTensor, &Manager::rewardTensor, &Manager::doneTensor,
        &Manager::policyAssignmentTensor, &Manager::worldCurriculumTensor, &Manager::selfObservationTensor,
        &Manager::filtersStateObservationTensor, &Manager::teammateObservationsTensor,
        &Manager::opponentObservationsTensor, &Manager::opponentLastKnownObservationsTensor,
        &Manager::selfPositionTensor, &Manager::teammatePositionObservationsTensor,
        &Manager::opponentPositionObservationsTensor, &Manager::opponentLastKnownPositionObservationsTensor,
        &Manager::opponentMasksTensor, &Manager::fwdLidarTensor, &Manager::rearLidarTensor,
        &Manager::agentMapTensor, &Manager::unmaskedAgentMapTensor, &Manager::hpTensor,
        &Manager::magazineTensor, &Manager::aliveTensor, &Manager::rewardHyperParamsTensor,
        &Manager::fullTeamActionTensor, &Manager::fullTeamGlobalObservationsTensor,
        &Manager::fullTeamPlayerObservationsTensor, &Manager::fullTeamEnemyObservationsTensor,
        &Manager::fullTeamLastKnownEnemyObservationsTensor, &Manager::fullTeamFwdLidarTensor,
        &Manager::fullTeamRearLidarTensor, &Manager::fullTeamRewardTensor, &Manager::fullTeamDoneTensor,
        &Manager::fullTeamPolicyAssignmentTensor,
    };
    use<TrainInterface (Manager::*)() const>(&Manager::trainInterface);
    use<ExecMode (Manager::*)() const>(&Manager::execMode);
    use<Engine &(Manager::*)(int32_t)>(&Manager::getWorldContext);
    use<void (Manager::*)(int32_t)>(&Manager::triggerReset);
    use<void (Manager::*)(int32_t, ExploreAction)>(&Manager::setExploreAction);
    use<void (Manager::*)(int32_t, int32_t, PvPDiscreteAction, PvPAimAction, PvPDiscreteAimAction)>(
        &Manager::setPvPAction);
    use<void (Manager::*)(int32_t, int32_t, CoarsePvPAction)>(&Manager::setCoarsePvPAction);
    use<void (Manager::*)(int32_t, int32_t, int32_t)>(&Manager::setHP);
    use<bool (Manager::*)()>(&Manager::isReplayFinished);
    use<void (Manager::*)(int32_t, int32_t, AgentPolicy)>(&Manager::setAgentPolicy);
    use<void (Manager::*)(AgentPolicy)>(&Manager::setUniformAgentPolicy);
    (void)getters;

    const char *scene = argc > 1 ? argv[1] : "scenes/simple_map";
    std::string col = std::string(scene) + "/collisions.bin";
    Manager::Config cfg {};
    cfg.execMode = ExecMode::CUDA;
    cfg.gpuID = 0;
    cfg.numWorlds = 2;
    cfg.randSeed = 5;
    cfg.autoReset = true;
    cfg.simFlags = SimFlags::Default;
    cfg.taskType = Task::Zone;
    cfg.teamSize = 1;
    cfg.map = MapConfig { "simple_map", col.c_str(), nullptr, nullptr, nullptr, Vector3::zero(), 0.f };

    // Manager(cfg, viz): a viewer state is refused before any device work
    int fails = 0;
    try {
        Manager mgr(cfg, reinterpret_cast<VizState *>(&cfg));
        std::fprintf(stderr, "FAIL: a non-null VizState was accepted\n");
        fails++;
    } catch (const std::runtime_error &e) {
        if (!std::strstr(e.what(), "VizState")) {
            std::fprintf(stderr, "FAIL: unexpected message: %s\n", e.what());
            fails++;
        }
    }
    // ExecMode::CPU is rejected (there is no CPU executor)
    cfg.execMode = ExecMode::CPU;
    try {
        Manager mgr(cfg);
        std::fprintf(stderr, "FAIL: ExecMode::CPU was accepted\n");
        fails++;
    } catch (const std::runtime_error &e) {
        if (!std::strstr(e.what(), "CPU")) {
            std::fprintf(stderr, "FAIL: unexpected message: %s\n", e.what());
            fails++;
        }
    }
    if (fails == 0) std::printf("mgr.hpp caller ok\n");
    return fails;
}
