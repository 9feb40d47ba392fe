// pybind_module.cpp — the `madrona_mp_env` Python module (reference:
// src/bindings.cpp:11-160, nanobind; nanobind is absent, pybind11 is used).
//
// Same names, enum values and SimManager.__init__ keyword arguments as the
// reference, layered over the C ABI of include/mpenv.h.  Tensor getters
// return zero-copy views of engine-owned device memory; .to_torch() hands
// them to PyTorch through DLPack (kDLROCM), like madrona::py::Tensor
// (mgr.cpp:295-301, 655-661).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <memory>
#include <string>
#include <vector>

#include "mpenv.h"

namespace py = pybind11;

namespace {

// ---- minimal DLPack ABI (dlpack.h v0.8)
struct DLDevice { int32_t device_type; int32_t device_id; };
struct DLDataType { uint8_t code; uint8_t bits; uint16_t lanes; };
struct DLTensor {
    void *data;
    DLDevice device;
    int32_t ndim;
    DLDataType dtype;
    int64_t *shape;
    int64_t *strides;
    uint64_t byte_offset;
};
struct DLManagedTensor {
    DLTensor dl_tensor;
    void *manager_ctx;
    void (*deleter)(DLManagedTensor *self);
};
constexpr int32_t kDLCPU = 1;
constexpr int32_t kDLROCM = 10;

struct ManagerHandle {
    mpenv_manager *mgr = nullptr;
    ~ManagerHandle()
    {
        if (mgr) mpenv_destroy(mgr);
    }
};

void check(int rc)
{
    if (rc != MPENV_OK) throw std::runtime_error(std::string("madrona_mp_env: ") + mpenv_last_error());
}

struct PyTensor {
    std::shared_ptr<ManagerHandle> owner;
    void *ptr = nullptr;
    int32_t dtype = MPENV_DTYPE_FLOAT32;
    std::vector<int64_t> dims;
    int32_t gpu = -1;

    struct Ctx {
        std::shared_ptr<ManagerHandle> owner;
        std::vector<int64_t> shape;
    };

    py::capsule dlpack() const
    {
        auto *mt = new DLManagedTensor();
        auto *ctx = new Ctx { owner, dims };
        mt->dl_tensor.data = ptr;
        mt->dl_tensor.device = { gpu >= 0 ? kDLROCM : kDLCPU, gpu >= 0 ? gpu : 0 };
        mt->dl_tensor.ndim = (int32_t)dims.size();
        uint8_t code = dtype == MPENV_DTYPE_FLOAT32 ? 2 : (dtype == MPENV_DTYPE_UINT32 ? 1 : 0);
        mt->dl_tensor.dtype = { code, 32, 1 };
        mt->dl_tensor.shape = ctx->shape.data();
        mt->dl_tensor.strides = nullptr;
        mt->dl_tensor.byte_offset = 0;
        mt->manager_ctx = ctx;
        mt->deleter = [](DLManagedTensor *self) {
            delete static_cast<Ctx *>(self->manager_ctx);
            delete self;
        };
        return py::capsule(mt, "dltensor", [](PyObject *cap) {
            if (PyCapsule_IsValid(cap, "dltensor")) {
                auto *m = static_cast<DLManagedTensor *>(PyCapsule_GetPointer(cap, "dltensor"));
                if (m && m->deleter) m->deleter(m);
            }
        });
    }
};

struct PySimManager {
    std::shared_ptr<ManagerHandle> h;

    PyTensor tensor(int32_t id) const
    {
        PyTensor t;
        t.owner = h;
        int32_t ndim = 0;
        int64_t dims[8];
        check(mpenv_export_tensor(h->mgr, id, &t.ptr, &t.dtype, &ndim, dims, &t.gpu));
        t.dims.assign(dims, dims + ndim);
        return t;
    }
};

// Unscoped so that pybind11 generates |, &, ^ (sim_flags |= SimFlags.X,
// scripts/jax_train.py:80-100).
enum SimFlagsE : uint32_t {
    SimFlagsE_Default = 0,
    SimFlagsE_SpawnInMiddle = 1u << 0,
    SimFlagsE_RandomizeHPMagazine = 1u << 1,
    SimFlagsE_NavmeshSpawn = 1u << 2,
    SimFlagsE_NoRespawn = 1u << 3,
    SimFlagsE_StaggerStarts = 1u << 4,
    SimFlagsE_EnableCurriculum = 1u << 5,
    SimFlagsE_HardcodedSpawns = 1u << 6,
    SimFlagsE_RandomFlipTeams = 1u << 7,
    SimFlagsE_StaticFlipTeams = 1u << 8,
    SimFlagsE_FullTeamPolicy = 1u << 9,
    SimFlagsE_SimEvalMode = 1u << 10,
    SimFlagsE_SubZones = 1u << 11,
};

// The flat buffer array of gpuStreamInit / gpuStreamStep: exactly one
// pointer per trainInterface input and output (the C ABI reads that many).
std::vector<void *> streamBuffers(const std::vector<uintptr_t> &bufs)
{
    int32_t ni = 0, no = 0;
    mpenv_train_interface_size(&ni, &no);
    if (bufs.size() != (size_t)(ni + no))
        throw py::value_error("gpu_stream_*: buffers must hold " + std::to_string(ni + no) +
                              " pointers (trainInterface inputs then outputs), got " + std::to_string(bufs.size()));
    std::vector<void *> b(bufs.size());
    for (size_t k = 0; k < bufs.size(); k++) b[k] = reinterpret_cast<void *>(bufs[k]);
    return b;
}

} // namespace

PYBIND11_MODULE(madrona_mp_env, m)
{
    m.doc() = "MI355X-native madrona-mp-env engine (Zone task, gfx950 HIP kernels)";

    // madrona.ExecMode submodule (madrona::py::setupMadronaSubmodule)
    py::module_ madrona = m.def_submodule("madrona", "madrona runtime enums");
    enum class ExecMode : int32_t { CPU = MPENV_EXEC_CPU, CUDA = MPENV_EXEC_CUDA };
    py::enum_<ExecMode>(madrona, "ExecMode").value("CPU", ExecMode::CPU).value("CUDA", ExecMode::CUDA);

    enum class Task : uint32_t { Explore = 0, TDM = 1, Zone = 2, Turret = 3, ZoneCaptureDefend = 4 };
    py::enum_<Task>(m, "Task")
        .value("Explore", Task::Explore)
        .value("TDM", Task::TDM)
        .value("Zone", Task::Zone)
        .value("Turret", Task::Turret)
        .value("ZoneCaptureDefend", Task::ZoneCaptureDefend);

    py::enum_<SimFlagsE>(m, "SimFlags", py::arithmetic())
        .value("Default", SimFlagsE_Default)
        .value("SpawnInMiddle", SimFlagsE_SpawnInMiddle)
        .value("RandomizeHPMagazine", SimFlagsE_RandomizeHPMagazine)
        .value("NavmeshSpawn", SimFlagsE_NavmeshSpawn)
        .value("NoRespawn", SimFlagsE_NoRespawn)
        .value("StaggerStarts", SimFlagsE_StaggerStarts)
        .value("EnableCurriculum", SimFlagsE_EnableCurriculum)
        .value("HardcodedSpawns", SimFlagsE_HardcodedSpawns)
        .value("RandomFlipTeams", SimFlagsE_RandomFlipTeams)
        .value("StaticFlipTeams", SimFlagsE_StaticFlipTeams)
        .value("FullTeamPolicy", SimFlagsE_FullTeamPolicy)
        .value("SimEvalMode", SimFlagsE_SimEvalMode)
        .value("SubZones", SimFlagsE_SubZones);

    py::class_<PyTensor>(m, "Tensor")
        .def_property_readonly("shape", [](const PyTensor &t) { return py::tuple(py::cast(t.dims)); })
        .def_property_readonly("dtype", [](const PyTensor &t) {
            return t.dtype == MPENV_DTYPE_FLOAT32 ? "float32" : (t.dtype == MPENV_DTYPE_UINT32 ? "uint32" : "int32");
        })
        .def_property_readonly("gpu_id", [](const PyTensor &t) { return t.gpu; })
        .def("data_ptr", [](const PyTensor &t) { return reinterpret_cast<uintptr_t>(t.ptr); })
        .def("__dlpack__", [](const PyTensor &t, py::object) { return t.dlpack(); }, py::arg("stream") = py::none())
        .def("__dlpack_device__", [](const PyTensor &t) {
            return py::make_tuple(t.gpu >= 0 ? kDLROCM : kDLCPU, t.gpu >= 0 ? t.gpu : 0);
        })
        .def("to_torch", [](const PyTensor &t) {
            py::object from_dlpack = py::module_::import("torch.utils.dlpack").attr("from_dlpack");
            return from_dlpack(t.dlpack());
        });

    py::class_<PySimManager>(m, "SimManager")
        .def(py::init([](ExecMode exec_mode, int64_t gpu_id, int64_t num_worlds, int64_t rand_seed, bool auto_reset,
                         uint32_t sim_flags, Task task, uint32_t team_size, uint32_t num_pbt_policies,
                         uint32_t policy_history_size, const std::string &scene_path, bool train_flank,
                         py::object replay_log_path, py::object record_log_path, py::object event_log_path,
                         py::object curriculum_data_path, uint32_t world_id_offset) {
                 std::string replay, record, event, curric;
                 mpenv_config cfg = {};
                 cfg.exec_mode = (int32_t)exec_mode;
                 cfg.gpu_id = (int32_t)gpu_id;
                 cfg.num_worlds = (uint32_t)num_worlds;
                 cfg.rand_seed = (uint32_t)rand_seed;
                 cfg.auto_reset = auto_reset ? 1 : 0;
                 cfg.sim_flags = sim_flags;
                 cfg.task_type = (int32_t)task;
                 cfg.team_size = team_size;
                 cfg.num_pbt_policies = num_pbt_policies;
                 cfg.policy_history_size = policy_history_size;
                 cfg.scene_path = scene_path.c_str();
                 cfg.train_flank = train_flank ? 1 : 0;
                 if (!replay_log_path.is_none()) { replay = py::str(replay_log_path); cfg.replay_log_path = replay.c_str(); }
                 if (!record_log_path.is_none()) { record = py::str(record_log_path); cfg.record_log_path = record.c_str(); }
                 if (!event_log_path.is_none()) { event = py::str(event_log_path); cfg.event_log_path = event.c_str(); }
                 if (!curriculum_data_path.is_none()) {
                     curric = py::str(curriculum_data_path);
                     cfg.curriculum_data_path = curric.c_str();
                 }
                 cfg.world_id_offset = world_id_offset;
                 auto h = std::make_shared<ManagerHandle>();
                 {
                     py::gil_scoped_release nogil;
                     check(mpenv_create(&cfg, &h->mgr));
                 }
                 return PySimManager { h };
             }),
             py::arg("exec_mode"), py::arg("gpu_id"), py::arg("num_worlds"), py::arg("rand_seed"),
             py::arg("auto_reset"), py::arg("sim_flags"), py::arg("task_type"), py::arg("team_size"),
             py::arg("num_pbt_policies"), py::arg("policy_history_size"), py::arg("scene_path"),
             py::arg("train_flank") = false, py::arg("replay_log_path") = py::none(),
             py::arg("record_log_path") = py::none(), py::arg("event_log_path") = py::none(),
             py::arg("curriculum_data_path") = py::none(), py::arg("world_id_offset") = 0)
        .def("init", [](PySimManager &s) { py::gil_scoped_release nogil; check(mpenv_init(s.h->mgr)); })
        .def("step", [](PySimManager &s) { py::gil_scoped_release nogil; check(mpenv_step(s.h->mgr)); })
        .def("step_async", [](PySimManager &s, uintptr_t stream) {
            check(mpenv_step_async(s.h->mgr, reinterpret_cast<void *>(stream)));
        }, py::arg("stream") = 0)
        .def("copy_actions", [](PySimManager &s, uintptr_t src, uintptr_t stream) {
            check(mpenv_copy_actions(s.h->mgr, reinterpret_cast<const int32_t *>(src), reinterpret_cast<void *>(stream)));
        }, py::arg("src"), py::arg("stream") = 0)
        .def("combat_actions", [](PySimManager &s, uintptr_t tape, uintptr_t out, int32_t mode, uintptr_t stream) {
            check(mpenv_combat_actions(s.h->mgr, reinterpret_cast<const int32_t *>(tape),
                                       reinterpret_cast<int32_t *>(out), mode, reinterpret_cast<void *>(stream)));
        }, py::arg("tape"), py::arg("out") = 0, py::arg("mode") = 1, py::arg("stream") = 0)
        // Manager::gpuStreamInit / gpuStreamStep (mgr.cpp:507-645): the flat
        // buffer array of the XLA custom call -- trainInterface inputs then
        // outputs, caller-owned device pointers (0 = skip that tensor).
        .def("gpu_stream_init", [](PySimManager &s, uintptr_t stream, const std::vector<uintptr_t> &bufs) {
            std::vector<void *> b = streamBuffers(bufs);
            check(mpenv_gpu_stream_init(s.h->mgr, reinterpret_cast<void *>(stream), b.data()));
        }, py::arg("stream"), py::arg("buffers"))
        .def("gpu_stream_step", [](PySimManager &s, uintptr_t stream, const std::vector<uintptr_t> &bufs) {
            std::vector<void *> b = streamBuffers(bufs);
            check(mpenv_gpu_stream_step(s.h->mgr, reinterpret_cast<void *>(stream), b.data()));
        }, py::arg("stream"), py::arg("buffers"))
        // the learner exchange's compact wire format (include/mpenv.h
        // mpenv_wire_*): sizes, pack into / unpack from device buffers
        .def("wire_bytes", [](PySimManager &s, bool keyframe) {
            int64_t b = 0;
            check(mpenv_wire_bytes(s.h->mgr, keyframe ? 1 : 0, &b));
            return b;
        }, py::arg("keyframe") = false)
        .def("wire_pack", [](PySimManager &s, uintptr_t dst, bool keyframe, uintptr_t stream) {
            check(mpenv_wire_pack(s.h->mgr, reinterpret_cast<void *>(dst), keyframe ? 1 : 0,
                                  reinterpret_cast<void *>(stream)));
        }, py::arg("dst"), py::arg("keyframe") = false, py::arg("stream") = 0)
        .def("wire_unpack", [](PySimManager &s, uintptr_t src, bool keyframe, uintptr_t stream) {
            check(mpenv_wire_unpack(s.h->mgr, reinterpret_cast<const void *>(src), keyframe ? 1 : 0,
                                    reinterpret_cast<void *>(stream)));
        }, py::arg("src"), py::arg("keyframe") = false, py::arg("stream") = 0)
        .def("wire_error", [](PySimManager &s) {
            uint32_t e = 0;
            check(mpenv_wire_error(s.h->mgr, &e));
            return e;
        })
        .def("wire_error_async", [](PySimManager &s, uintptr_t out, uintptr_t stream) {
            check(mpenv_wire_error_async(s.h->mgr, reinterpret_cast<uint32_t *>(out), reinterpret_cast<void *>(stream)));
        }, py::arg("out"), py::arg("stream"))
        .def("set_world_groups", [](PySimManager &s, int32_t g) { check(mpenv_set_world_groups(s.h->mgr, g)); })
        .def("set_lidar_branch", [](PySimManager &s, bool on) { check(mpenv_set_lidar_branch(s.h->mgr, on ? 1 : 0)); })
        .def("graph_status", [](PySimManager &s) {
            int32_t on = 0;
            char why[512] = {};
            check(mpenv_graph_status(s.h->mgr, &on, why, sizeof(why)));
            return py::make_tuple(on != 0, std::string(why));
        })
        .def("world_groups", [](PySimManager &s) { int32_t g = 0; check(mpenv_world_groups(s.h->mgr, &g)); return g; })
        .def("enable_kernel_timing", [](PySimManager &s, bool on) { check(mpenv_enable_kernel_timing(s.h->mgr, on)); })
        .def("enable_stats", [](PySimManager &s, bool on) { check(mpenv_enable_stats(s.h->mgr, on)); })
        .def("read_stats", [](PySimManager &s) {
            uint64_t v[10] = {};
            int n = mpenv_read_stats(s.h->mgr, v, 10);
            if (n < 0) check(n);
            static const char *names[10] = { "alive_agents", "los_pairs", "los_rays", "los_seen",
                                             "sphere_casts", "shot_rays", "hit_agents", "kills", "lk_rows",
                                             "los_traced" };
            py::dict d;
            for (int k = 0; k < 10; k++) d[py::str(names[k])] = v[k];
            return d;
        })
        .def("kernel_timings", [](PySimManager &s) {
            const char *names[16];
            float ms[16];
            int32_t launches[16];
            int n = mpenv_kernel_timings(s.h->mgr, 16, names, ms, launches);
            if (n < 0) check(n);
            py::dict d;
            for (int k = 0; k < n; k++) d[py::str(names[k])] = py::make_tuple(ms[k], launches[k]);
            return d;
        })
        .def_property_readonly("num_worlds", [](PySimManager &s) { int32_t w, n; mpenv_dims(s.h->mgr, &w, &n); return w; })
        .def_property_readonly("agents_per_world", [](PySimManager &s) { int32_t w, n; mpenv_dims(s.h->mgr, &w, &n); return n; })
        .def("fwd_lidar", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_FWD_LIDAR); })
        .def("rear_lidar", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_REAR_LIDAR); })
        .def("hp", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_HP); })
        .def("magazine", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_MAGAZINE); })
        .def("alive", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_ALIVE); })
        .def("self_obs", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_SELF_OBSERVATION); })
        .def("filters_state", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_FILTERS_STATE); })
        .def("teammates", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_TEAMMATE_OBSERVATIONS); })
        .def("opponents", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_OPPONENT_OBSERVATIONS); })
        .def("opponents_last_known",
             [](PySimManager &s) { return s.tensor(MPENV_EXPORT_OPPONENT_LAST_KNOWN_OBSERVATIONS); })
        .def("self_pos", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_SELF_POSITION); })
        .def("teammate_positions", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_TEAMMATE_POSITIONS); })
        .def("opponent_positions", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_OPPONENT_POSITIONS); })
        .def("opponent_last_known_positions",
             [](PySimManager &s) { return s.tensor(MPENV_EXPORT_OPPONENT_LAST_KNOWN_POSITIONS); })
        .def("opponent_masks", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_OPPONENT_MASKS); })
        .def("agent_map", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_AGENT_MAP); })
        .def("unmasked_agent_map", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_AGENT_MAP); })
        .def("reward_coefs", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_REWARD_HYPER_PARAMS); })
        .def("explore_action_tensor", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_EXPLORE_ACTION); })
        .def("pvp_action_tensor", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_PVP_DISCRETE_ACTION); })
        .def("aim_action_tensor", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_PVP_DISCRETE_AIM_ACTION); })
        .def("reward_tensor", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_REWARD); })
        .def("done_tensor", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_DONE); })
        .def("reset_tensor", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_RESET); })
        .def("self_observation_tensor", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_SELF_OBSERVATION); })
        // Extensions beyond bindings.cpp (Manager methods of mgr.hpp):
        .def("sim_control_tensor", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_SIM_CONTROL); })
        .def("match_result_tensor", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_MATCH_RESULT); })
        .def("policy_assignment_tensor", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_AGENT_POLICY); })
        .def("world_curriculum_tensor", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_WORLD_CURRICULUM); })
        .def("pvp_aim_action_tensor", [](PySimManager &s) { return s.tensor(MPENV_EXPORT_PVP_AIM_ACTION); })
        .def("export_tensor", [](PySimManager &s, int32_t id) { return s.tensor(id); })
        .def("trigger_reset", [](PySimManager &s, int32_t w) { check(mpenv_trigger_reset(s.h->mgr, w)); })
        .def("set_hp", [](PySimManager &s, int32_t w, int32_t a, int32_t hp) { check(mpenv_set_hp(s.h->mgr, w, a, hp)); })
        .def("set_agent_policy",
             [](PySimManager &s, int32_t w, int32_t a, int32_t p) { check(mpenv_set_agent_policy(s.h->mgr, w, a, p)); })
        .def("set_uniform_agent_policy",
             [](PySimManager &s, int32_t p) { check(mpenv_set_uniform_agent_policy(s.h->mgr, p)); })
        .def("train_interface", [](PySimManager &s) {
            int32_t ni = 0, no = 0;
            mpenv_train_interface_size(&ni, &no);
            py::dict inputs, outputs;
            for (int k = 0; k < ni; k++) {
                const char *name; int32_t id;
                mpenv_train_interface_entry(0, k, &name, &id);
                inputs[py::str(name)] = py::cast(s.tensor(id));
            }
            for (int k = 0; k < no; k++) {
                const char *name; int32_t id;
                mpenv_train_interface_entry(1, k, &name, &id);
                outputs[py::str(name)] = py::cast(s.tensor(id));
            }
            py::dict ti;
            ti["inputs"] = inputs;
            ti["outputs"] = outputs;
            return ti;
        })
        // JAXInterface::buildEntry (bindings.cpp:149-158): the XLA GPU
        // custom-call targets over gpuStreamInit / gpuStreamStep as PyCapsules
        // named "xla._CUSTOM_CALL_TARGET" (what jax's
        // xla_client.register_custom_call_target takes), the opaque bytes that
        // name this manager, and the trainInterface the call's operand
        // (inputs) and result (outputs) shapes come from.  Registering them
        // needs jax, absent from this image; the targets themselves are plain
        // C functions of XLA's API-version-1 signature, plus status-returning
        // twins (include/mpenv.h).
        .def("jax", [](PySimManager &s, bool xla_gpu) -> py::object {
            if (!xla_gpu)
                throw std::runtime_error("madrona_mp_env.SimManager.jax: only the XLA GPU (ROCm) target is built; "
                                         "ExecMode.CPU is not supported by this engine");
            mpenv_xla_opaque o;
            check(mpenv_xla_opaque_make(s.h->mgr, &o));
            const char *kName = "xla._CUSTOM_CALL_TARGET";
            py::dict d;
            d["init"] = py::capsule(reinterpret_cast<void *>(&mpenv_xla_gpu_stream_init), kName);
            d["step"] = py::capsule(reinterpret_cast<void *>(&mpenv_xla_gpu_stream_step), kName);
            d["opaque"] = py::bytes(reinterpret_cast<const char *>(&o), sizeof(o));
            // the same targets in XLA's status-returning form (API version 2,
            // API_VERSION_STATUS_RETURNING): failures reach XLA instead of
            // aborting the process
            d["init_status"] = py::capsule(reinterpret_cast<void *>(&mpenv_xla_gpu_stream_init_status), kName);
            d["step_status"] = py::capsule(reinterpret_cast<void *>(&mpenv_xla_gpu_stream_step_status), kName);
            d["platform"] = "ROCM";
            d["api_version"] = 1;
            d["status_api_version"] = 2;
            int32_t ni = 0, no = 0;
            mpenv_train_interface_size(&ni, &no);
            py::list in_names, out_names;
            for (int k = 0; k < ni; k++) {
                const char *name; int32_t id;
                mpenv_train_interface_entry(0, k, &name, &id);
                in_names.append(py::str(name));
            }
            for (int k = 0; k < no; k++) {
                const char *name; int32_t id;
                mpenv_train_interface_entry(1, k, &name, &id);
                out_names.append(py::str(name));
            }
            d["input_names"] = in_names;
            d["output_names"] = out_names;
            // keeps the manager alive as long as the registration data is
            d["sim"] = py::cast(s);
            return d;
        }, py::arg("xla_gpu") = true);
}
