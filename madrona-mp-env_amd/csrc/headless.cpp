// headless — command-line driver over the C++ Manager (the role of the
// reference's src/headless.cpp:24-139): create a Manager, init, run steps,
// print world-steps/s ("FPS") and agent-steps/s.
//
//   headless CUDA NUM_WORLDS NUM_STEPS SCENE_DIR [--rand-actions] [--team-size N]
//
// --rand-actions draws actions from the hash tape (mpenv_core.h tapeActions)
// into a device buffer and copies them in before every step, as the
// TrainInterface input copy of gpuStreamStep does.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "mpenv_core.h"
#include "mpenv_manager.hpp"

using namespace madronaMPEnv;

int main(int argc, char *argv[])
{
    if (argc < 5) {
        fprintf(stderr, "%s TYPE NUM_WORLDS NUM_STEPS SCENE_DIR [--rand-actions] [--team-size N]\n", argv[0]);
        return 1;
    }
    const std::string type = argv[1];
    if (type != "CUDA" && type != "HIP") {
        fprintf(stderr, "only the GPU exec mode (CUDA/HIP) is implemented\n");
        return 1;
    }
    const uint32_t num_worlds = (uint32_t)std::stoul(argv[2]);
    const uint32_t num_steps = (uint32_t)std::stoul(argv[3]);
    const std::string scene = argv[4];
    bool rand_actions = false;
    uint32_t team_size = 6;
    for (int i = 5; i < argc; i++) {
        if (!strcmp(argv[i], "--rand-actions")) rand_actions = true;
        else if (!strcmp(argv[i], "--team-size") && i + 1 < argc) team_size = (uint32_t)std::stoul(argv[++i]);
    }
    const std::string col = scene + "/collisions.bin", nav = scene + "/navmesh.bin",
                      spw = scene + "/spawns.bin", zon = scene + "/zones.bin";
    try {
        Manager::Config cfg {};
        cfg.execMode = ExecMode::CUDA;
        cfg.gpuID = 0;
        cfg.numWorlds = num_worlds;
        cfg.randSeed = 10;
        cfg.autoReset = true;
        cfg.simFlags = SimFlags::Default;
        cfg.taskType = Task::Zone;
        cfg.teamSize = team_size;
        cfg.numPBTPolicies = 0;
        cfg.policyHistorySize = 1;
        cfg.map = { scene.c_str(), col.c_str(), nav.c_str(), spw.c_str(), zon.c_str(), Vector3::zero(), 0.f };
        Manager mgr(cfg);
        mgr.init();

        const int64_t A = (int64_t)num_worlds * 2 * team_size;
        const int ring = 16;
        int32_t *d_ring = nullptr;
        if (rand_actions) {
            std::vector<int32_t> h((size_t)ring * A * 6);
            for (int s = 0; s < ring; s++)
                for (int64_t g = 0; g < A; g++)
                    mp::tapeActions(1234u, (uint32_t)s, (uint32_t)g, &h[((size_t)s * A + g) * 6],
                                    &h[((size_t)s * A + g) * 6 + 4]);
            if (hipMalloc(&d_ring, h.size() * 4) != hipSuccess ||
                hipMemcpy(d_ring, h.data(), h.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
                fprintf(stderr, "device action ring allocation failed\n");
                return 1;
            }
        }
        auto start = std::chrono::steady_clock::now();
        for (uint32_t i = 0; i < num_steps; i++) {
            if (d_ring) mpenv_copy_actions(mgr.handle(), d_ring + (size_t)(i % ring) * A * 6, nullptr);
            mgr.step();
        }
        auto end = std::chrono::steady_clock::now();
        const double secs = std::chrono::duration<double>(end - start).count();
        printf("FPS %f\n", (double)num_steps * num_worlds / secs);
        printf("agent-steps/s %f\n", (double)num_steps * A / secs);
        if (d_ring) (void)hipFree(d_ring);
    } catch (const std::exception &e) {
        fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
