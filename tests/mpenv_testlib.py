"""ctypes harness over the two C ABIs used by the tests.

* libmpenv.so (the product, include/mpenv.h) — the gfx950 engine.
* liboracle.so (oracle/oracle.h) — TEST INFRASTRUCTURE: the CPU restatement
  of the reference step used as the parity checker.

Nothing here is imported by the product.
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "madrona-mp-env_amd")
SCENE = os.environ.get("MPENV_SCENE", os.path.join(ROOT, "scenes", "simple_map"))

if PKG not in sys.path:
    sys.path.insert(0, PKG)

import build_native  # noqa: E402
import mpenv_tape  # noqa: E402

# ---------------------------------------------------------------- constants
EXPORT = dict(
    RESET=0, WORLD_CURRICULUM=1, EXPLORE_ACTION=2, PVP_DISCRETE_ACTION=3, PVP_AIM_ACTION=4,
    PVP_DISCRETE_AIM_ACTION=5, REWARD=6, DONE=7, MATCH_RESULT=8, AGENT_POLICY=9,
    SELF_OBSERVATION=10, TEAMMATE_OBSERVATIONS=11, OPPONENT_OBSERVATIONS=12,
    OPPONENT_LAST_KNOWN_OBSERVATIONS=13, SELF_POSITION=14, TEAMMATE_POSITIONS=15,
    OPPONENT_POSITIONS=16, OPPONENT_LAST_KNOWN_POSITIONS=17, OPPONENT_MASKS=18, FWD_LIDAR=19,
    REAR_LIDAR=20, AGENT_MAP=21, UNMASKED_AGENT_MAP=22, HP=23, ALIVE=24, MAGAZINE=25,
    FILTERS_STATE=38, REWARD_HYPER_PARAMS=39, SIM_CONTROL=64, DEBUG_AGENT_F32=65,
    DEBUG_AGENT_I32=66, DEBUG_WORLD_I32=67, DEBUG_WORLD_F32=68, DEBUG_EXPLORE=69,
    DEBUG_CRUMBS=70, EVENT_LOG=36, PACKED_STEP_SNAPSHOT=37, RECORD_LOG=71, REPLAY_LOG=72,
    SNAPSHOT_WRITTEN=73, FULL_TEAM_ACTIONS=26, FULL_TEAM_GLOBAL=27, FULL_TEAM_PLAYERS=28,
    FULL_TEAM_ENEMIES=29, FULL_TEAM_LAST_KNOWN_ENEMIES=30, FULL_TEAM_FWD_LIDAR=31,
    FULL_TEAM_REAR_LIDAR=32, FULL_TEAM_REWARD=33, FULL_TEAM_DONE=34, FULL_TEAM_POLICY_ASSIGNMENTS=35,
)

# FullTeamInterface outputs (fullTeamObservationsSystem, fullTeamDoneRewardSystem)
FULL_TEAM_OUTPUTS = [
    "FULL_TEAM_GLOBAL", "FULL_TEAM_PLAYERS", "FULL_TEAM_ENEMIES", "FULL_TEAM_LAST_KNOWN_ENEMIES",
    "FULL_TEAM_FWD_LIDAR", "FULL_TEAM_REAR_LIDAR", "FULL_TEAM_REWARD", "FULL_TEAM_DONE",
]

# Exports compared between engine and oracle after every step.
STEP_OUTPUTS = [
    "FWD_LIDAR", "REAR_LIDAR", "HP", "MAGAZINE", "ALIVE", "SELF_OBSERVATION", "FILTERS_STATE",
    "TEAMMATE_OBSERVATIONS", "OPPONENT_OBSERVATIONS", "OPPONENT_LAST_KNOWN_OBSERVATIONS",
    "SELF_POSITION", "TEAMMATE_POSITIONS", "OPPONENT_POSITIONS", "OPPONENT_LAST_KNOWN_POSITIONS",
    "OPPONENT_MASKS", "REWARD", "DONE", "MATCH_RESULT", "REWARD_HYPER_PARAMS", "RESET",
    "WORLD_CURRICULUM", "PVP_DISCRETE_ACTION", "PVP_DISCRETE_AIM_ACTION", "PVP_AIM_ACTION",
] + FULL_TEAM_OUTPUTS
# trainInterface outputs (mgr.cpp:2383-2431, csrc/manager.cpp kTIOutputs) ->
# export names; agent_map / unmasked_agent_map (never written) are not shipped.
TRAIN_OUTPUTS = {
    "fwd_lidar": "FWD_LIDAR", "rear_lidar": "REAR_LIDAR", "hp": "HP", "magazine": "MAGAZINE",
    "alive": "ALIVE", "self": "SELF_OBSERVATION", "filters_state": "FILTERS_STATE",
    "teammates": "TEAMMATE_OBSERVATIONS", "opponents": "OPPONENT_OBSERVATIONS",
    "opponents_last_known": "OPPONENT_LAST_KNOWN_OBSERVATIONS", "self_pos": "SELF_POSITION",
    "teammate_positions": "TEAMMATE_POSITIONS", "opponent_positions": "OPPONENT_POSITIONS",
    "opponent_last_known_positions": "OPPONENT_LAST_KNOWN_POSITIONS", "opponent_masks": "OPPONENT_MASKS",
    "reward_coefs": "REWARD_HYPER_PARAMS", "rewards": "REWARD", "dones": "DONE",
    "pbt.episode_results": "MATCH_RESULT",
}
DEBUG_OUTPUTS = ["DEBUG_AGENT_F32", "DEBUG_AGENT_I32", "DEBUG_WORLD_I32", "DEBUG_WORLD_F32",
                 "DEBUG_CRUMBS"]

DTYPES = {0: np.int32, 1: np.float32, 2: np.uint32}

# Task (sim.hpp Task enum, include/mpenv.h MPENV_TASK_*)
TASK_TDM, TASK_ZONE, TASK_TURRET, TASK_ZONE_CAPTURE_DEFEND = 1, 2, 3, 4

SIMFLAG_STAGGER_STARTS = 1 << 4
SIMFLAG_RANDOM_FLIP_TEAMS = 1 << 7


class OracleConfig(C.Structure):
    _fields_ = [
        ("num_worlds", C.c_uint32), ("rand_seed", C.c_uint32), ("auto_reset", C.c_int32),
        ("sim_flags", C.c_uint32), ("team_size", C.c_uint32), ("world_id_offset", C.c_uint32),
        ("scene_path", C.c_char_p), ("bvh_nodes", C.c_void_p), ("num_nodes", C.c_int32),
        ("bvh_verts", C.c_void_p), ("num_bvh_verts", C.c_int32),
        ("task_type", C.c_int32), ("train_flank", C.c_int32), ("lidar_octant_order", C.c_int32),
        ("lidar_bvh_nodes", C.c_void_p), ("num_lidar_nodes", C.c_int32),
        ("lidar_bvh_verts", C.c_void_p), ("num_lidar_bvh_verts", C.c_int32),
    ]


class MpenvConfig(C.Structure):
    _fields_ = [
        ("exec_mode", C.c_int32), ("gpu_id", C.c_int32), ("num_worlds", C.c_uint32),
        ("rand_seed", C.c_uint32), ("auto_reset", C.c_int32), ("sim_flags", C.c_uint32),
        ("task_type", C.c_int32), ("team_size", C.c_uint32), ("num_pbt_policies", C.c_uint32),
        ("policy_history_size", C.c_uint32), ("scene_path", C.c_char_p), ("train_flank", C.c_int32),
        ("replay_log_path", C.c_char_p), ("record_log_path", C.c_char_p),
        ("event_log_path", C.c_char_p), ("curriculum_data_path", C.c_char_p),
        ("world_id_offset", C.c_uint32),
    ]


_libs = {}


def usable_cpus():
    """CPUs this process may use: affinity, capped by a cgroup v2 CPU quota
    (the GPU box shows the whole host's CPUs but grants 16)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def ensure_built():
    build_native.build_all(force=False)


def lib_mpenv():
    if "mpenv" not in _libs:
        ensure_built()
        # MPENV_LIB: a kernel_lab variant of the library (development only)
        lib = C.CDLL(os.environ.get("MPENV_LIB", build_native.LIB))
        lib.mpenv_create.argtypes = [C.POINTER(MpenvConfig), C.POINTER(C.c_void_p)]
        lib.mpenv_destroy.argtypes = [C.c_void_p]
        for fn in ("mpenv_init", "mpenv_step"):
            getattr(lib, fn).argtypes = [C.c_void_p]
        lib.mpenv_step_async.argtypes = [C.c_void_p, C.c_void_p]
        lib.mpenv_export_tensor.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_void_p),
                                            C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                            C.POINTER(C.c_int64), C.POINTER(C.c_int32)]
        lib.mpenv_last_error.restype = C.c_char_p
        lib.mpenv_scene_bvh.argtypes = [C.c_char_p, C.c_void_p, C.POINTER(C.c_int32), C.c_void_p,
                                        C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        lib.mpenv_scene_navmesh.argtypes = [C.c_char_p, C.c_void_p, C.POINTER(C.c_int32), C.c_void_p,
                                            C.c_void_p]
        lib.mpenv_trigger_reset.argtypes = [C.c_void_p, C.c_int32]
        lib.mpenv_copy_actions.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        lib.mpenv_set_hp.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32]
        lib.mpenv_enable_kernel_timing.argtypes = [C.c_void_p, C.c_int32]
        lib.mpenv_kernel_timings.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_char_p),
                                             C.POINTER(C.c_float), C.POINTER(C.c_int32)]
        _libs["mpenv"] = lib
    return _libs["mpenv"]


def lib_oracle():
    if "oracle" not in _libs:
        ensure_built()
        lib = C.CDLL(build_native.ORACLE_LIB)
        lib.oracle_create.argtypes = [C.POINTER(OracleConfig)]
        lib.oracle_create.restype = C.c_void_p
        lib.oracle_destroy.argtypes = [C.c_void_p]
        lib.oracle_export.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_void_p),
                                      C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                      C.POINTER(C.c_int64)]
        for fn in ("oracle_init", "oracle_step", "oracle_refresh_debug"):
            getattr(lib, fn).argtypes = [C.c_void_p]
        lib.oracle_step_worlds.argtypes = [C.c_void_p, C.c_int32, C.c_int32]
        lib.oracle_set_log_modes.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32]
        lib.oracle_set_curriculum.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
        lib.oracle_run_threaded.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int32]
        lib.oracle_run_threaded.restype = C.c_double
        fp = C.POINTER(C.c_float)
        lib.oracle_trace_ray.argtypes = [C.c_void_p, fp, fp, fp]
        lib.oracle_trace_ray_brute.argtypes = [C.c_void_p, fp, fp, fp]
        lib.oracle_sphere_cast.argtypes = [C.c_void_p, fp, fp, C.c_float, fp]
        lib.oracle_sphere_cast.restype = C.c_float
        lib.oracle_set_slab_fma.argtypes = [C.c_int32]
        lib.oracle_trace_ray_batch.argtypes = [C.c_void_p, C.c_int32, fp, fp, C.c_int32, fp, C.c_void_p]
        lib.oracle_sphere_cast_batch.argtypes = [C.c_void_p, C.c_int32, fp, fp, C.c_float, fp, fp, fp]
        lib.oracle_sphere_cast_brute.argtypes = [C.c_void_p, fp, fp, C.c_float]
        lib.oracle_sphere_cast_brute.restype = C.c_float
        lib.oracle_navmesh.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.POINTER(C.c_int32)]
        lib.oracle_eval_math.argtypes = [C.c_int32, fp, fp, fp, C.c_int32]
        lib.oracle_threefry.argtypes = [C.c_uint32] * 4 + [C.POINTER(C.c_uint32)]
        lib.oracle_tape_actions.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_int32,
                                            C.POINTER(C.c_int32)]
        lib.oracle_capsule.argtypes = [fp, fp, C.c_float, C.c_float]
        lib.oracle_capsule.restype = C.c_float
        _libs["oracle"] = lib
    return _libs["oracle"]


def fptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def scene_navmesh(scene=SCENE):
    """(tri_verts [T,3,3] f32, adjacency [T,3] i32, astar [T,T] i32) from the
    product's navmesh builder."""
    lib = lib_mpenv()
    nt = C.c_int32(0)
    rc = lib.mpenv_scene_navmesh(scene.encode(), None, C.byref(nt), None, None)
    assert rc == 0, lib.mpenv_last_error()
    T = nt.value
    tv = np.zeros((T, 3, 3), np.float32)
    adj = np.zeros((T, 3), np.int32)
    astar = np.zeros((T, T), np.int32)
    rc = lib.mpenv_scene_navmesh(scene.encode(), tv.ctypes.data, C.byref(nt), adj.ctypes.data,
                                 astar.ctypes.data)
    assert rc == 0, lib.mpenv_last_error()
    return tv, adj, astar


def scene_bvh(scene=SCENE, lidar=False):
    """The collision tree, or (lidar=True) k_lidar's own tree."""
    lib = lib_mpenv()
    fn = lib.mpenv_scene_lidar_bvh if lidar else lib.mpenv_scene_bvh
    fn.argtypes = [C.c_char_p, C.c_void_p, C.POINTER(C.c_int32), C.c_void_p, C.POINTER(C.c_int32),
                   C.POINTER(C.c_int32)]
    nn, nv, ms = C.c_int32(0), C.c_int32(0), C.c_int32(0)
    rc = fn(scene.encode(), None, C.byref(nn), None, C.byref(nv), C.byref(ms))
    assert rc == 0, lib.mpenv_last_error()
    nodes = np.zeros(nn.value * 64, dtype=np.uint8)
    verts = np.zeros(nv.value * 3, dtype=np.float32)
    rc = fn(scene.encode(), nodes.ctypes.data, C.byref(nn), verts.ctypes.data, C.byref(nv), C.byref(ms))
    assert rc == 0, lib.mpenv_last_error()
    return nodes, verts, ms.value


def four_zone_scene(dst):
    """simple_map with a fourth zone appended to zones.bin (the reference's
    ZoneCaptureDefend starts every episode at zone 3, sim.cpp:822-825, and
    simple_map has three): a 250 x 250 box between the hardcoded spawns.
    Written under dst; returns the scene directory."""
    import shutil
    d = os.path.join(str(dst), "four_zones")
    os.makedirs(d, exist_ok=True)
    for f in ("collisions.bin", "navmesh.bin", "spawns.bin"):
        shutil.copy(os.path.join(SCENE, f), d)
    raw = open(os.path.join(SCENE, "zones.bin"), "rb").read()
    n = int(np.frombuffer(raw[:4], np.uint32)[0])
    boxes = np.frombuffer(raw[4:4 + 24 * n], np.float32).reshape(n, 6)
    rots = np.frombuffer(raw[4 + 24 * n:], np.float32)[:n]
    extra = np.array([[700.0, 250.0, -80.0, 950.0, 500.0, 300.0]], np.float32)
    with open(os.path.join(d, "zones.bin"), "wb") as f:
        f.write(np.uint32(n + 1).tobytes())
        f.write(np.concatenate([boxes, extra]).tobytes())
        f.write(np.concatenate([rots, np.zeros(1, np.float32)]).tobytes())
    return d


CURRICULUM_SNAPSHOT = np.dtype([("step", "<u2"), ("cur_zone", "u1"), ("controller", "i1"),
                                ("zone_steps_remaining", "<u2"), ("steps_until_point", "<u2"),
                                ("players", [("pos", "<i2", 3), ("yaw", "<i2"), ("pitch", "<i2"),
                                             ("mag", "u1"), ("reloading", "u1"), ("hp", "u1"),
                                             ("flags", "u1")], 12)])


def make_curriculum_file(path, n=64, seed=7):
    """A curriculum_data_path file (n CurriculumSnapshots, 176 B each,
    types.hpp:816-819).  Player positions come from a 6v6 oracle rollout so
    they sit on the map; the rest of each snapshot is drawn at random:
    controller -1/0/1, crouch / prone flags, hp, magazine, step."""
    assert CURRICULUM_SNAPSHOT.itemsize == 176
    rng = np.random.default_rng(seed)
    o = Oracle(4, 6, sim_flags=1)
    o.put_ctrl([0, 1, 1])
    o.init()
    pos = []
    for s in range(60):
        o.set_actions(mpenv_tape.tape_actions(99, s, 0, 4 * 12))
        o.step()
        if s % 4 == 3:
            o.lib.oracle_refresh_debug(o.h)
            pos.append(o.get("DEBUG_AGENT_F32")[:, :3].reshape(4, 12, 3).copy())
    o.close()
    pos = np.concatenate(pos)  # [k, 12, 3]
    out = np.zeros(n, CURRICULUM_SNAPSHOT)
    for k in range(n):
        sn = out[k]
        sn["step"] = rng.integers(0, 2900)
        sn["cur_zone"] = rng.integers(0, 3)
        sn["controller"] = rng.integers(-1, 2)
        sn["zone_steps_remaining"] = rng.integers(1, 601)
        sn["steps_until_point"] = rng.integers(1, 21)
        pl = sn["players"]
        pl["pos"] = np.round(pos[k % len(pos)]).astype(np.int16)
        pl["yaw"] = rng.integers(-32768, 32768, 12)
        pl["pitch"] = rng.integers(-6000, 6000, 12)
        pl["mag"] = rng.integers(0, 31, 12)
        pl["reloading"] = rng.integers(0, 3, 12)
        pl["hp"] = rng.integers(1, 101, 12)
        pl["flags"] = rng.choice([0, 2, 4, 8], 12)
    out.tofile(path)
    return path


class Oracle:
    """CPU restatement of the reference step (test infrastructure)."""

    def __init__(self, num_worlds, team_size, rand_seed=5, sim_flags=0, auto_reset=True,
                 world_id_offset=0, scene=SCENE, task=TASK_ZONE, curriculum=None, flank=False,
                 lidar_order="octant"):
        self.lib = lib_oracle()
        self.nodes, self.verts, _ = scene_bvh(scene)
        self.lnodes, self.lverts, _ = scene_bvh(scene, lidar=True)  # k_lidar's own tree
        cfg = OracleConfig(num_worlds, rand_seed, int(auto_reset), sim_flags, team_size,
                           world_id_offset, scene.encode(), self.nodes.ctypes.data,
                           len(self.nodes) // 64, self.verts.ctypes.data, len(self.verts) // 3, task,
                           int(flank), {"slot": 0, "octant": 1, "lex": 2}[lidar_order],
                           self.lnodes.ctypes.data, len(self.lnodes) // 64, self.lverts.ctypes.data,
                           len(self.lverts) // 3)
        self.h = self.lib.oracle_create(C.byref(cfg))
        assert self.h, "oracle_create failed"
        if curriculum:
            data = np.fromfile(curriculum, np.uint8)
            n = len(data) // 176
            self.lib.oracle_set_curriculum(self.h, data.ctypes.data, n)
        self.W, self.N = num_worlds, 2 * team_size

    def close(self):
        if self.h:
            self.lib.oracle_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def view(self, name):
        """Zero-copy numpy view of an oracle export."""
        ptr, dt, nd = C.c_void_p(), C.c_int32(), C.c_int32()
        dims = (C.c_int64 * 8)()
        rc = self.lib.oracle_export(self.h, EXPORT[name], C.byref(ptr), C.byref(dt), C.byref(nd), dims)
        assert rc == 0, name
        shape = tuple(dims[i] for i in range(nd.value))
        n = int(np.prod(shape))
        ctype = {0: C.c_int32, 1: C.c_float, 2: C.c_uint32}[dt.value]
        buf = (ctype * n).from_address(ptr.value)
        return np.ctypeslib.as_array(buf).reshape(shape)

    def get(self, name):
        if name.startswith("DEBUG"):
            self.lib.oracle_refresh_debug(self.h)
        return self.view(name).copy()

    def navmesh(self):
        """The oracle's own (tri_verts [T,3,3], adjacency [T,3], astar [T,T])."""
        nt = C.c_int32(0)
        self.lib.oracle_navmesh(self.h, None, None, None, C.byref(nt))
        T = nt.value
        tv = np.zeros((T, 3, 3), np.float32)
        adj = np.zeros((T, 3), np.int32)
        astar = np.zeros((T, T), np.int32)
        self.lib.oracle_navmesh(self.h, tv.ctypes.data, adj.ctypes.data, astar.ctypes.data, C.byref(nt))
        return tv, adj, astar

    def put_ctrl(self, ctrl):
        self.view("SIM_CONTROL")[:] = np.asarray(ctrl, np.int32).reshape(self.view("SIM_CONTROL").shape)

    def set_actions(self, acts6):
        self.view("PVP_DISCRETE_ACTION")[:] = acts6[:, :4]
        self.view("PVP_DISCRETE_AIM_ACTION")[:] = acts6[:, 4:6]

    def init(self):
        self.lib.oracle_init(self.h)

    def step(self):
        self.lib.oracle_step(self.h)


class HipMem:
    """Device->host copies through libamdhip64 (no torch needed)."""

    def __init__(self):
        self.hip = C.CDLL("libamdhip64.so")
        self.hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        self.hip.hipDeviceSynchronize.argtypes = []
        self.hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        self.hip.hipFree.argtypes = [C.c_void_p]

    def upload(self, arr):
        """A device copy of arr (caller frees with free())."""
        arr = np.ascontiguousarray(arr)
        p = C.c_void_p()
        assert self.hip.hipMalloc(C.byref(p), arr.nbytes) == 0, "hipMalloc failed"
        self.h2d(p.value, arr)
        return p.value

    def free(self, ptr):
        self.hip.hipFree(ptr)

    def d2h(self, ptr, nbytes, out):
        rc = self.hip.hipMemcpy(out.ctypes.data, ptr, nbytes, 2)
        assert rc == 0, f"hipMemcpy D2H failed: {rc}"

    def h2d(self, ptr, arr):
        arr = np.ascontiguousarray(arr)
        rc = self.hip.hipMemcpy(ptr, arr.ctypes.data, arr.nbytes, 1)
        assert rc == 0, f"hipMemcpy H2D failed: {rc}"


class Engine:
    """The gfx950 engine through its C ABI (include/mpenv.h)."""

    def __init__(self, num_worlds, team_size, rand_seed=5, sim_flags=0, auto_reset=True,
                 world_id_offset=0, scene=SCENE, gpu_id=0, replay=None, record=None, events=None,
                 task=TASK_ZONE, curriculum=None, flank=False):
        self.lib = lib_mpenv()
        self.mem = HipMem()
        self._scene = scene.encode()
        self._paths = [p.encode() if p else None for p in (replay, record, events, curriculum)]
        cfg = MpenvConfig(1, gpu_id, num_worlds, rand_seed, int(auto_reset), sim_flags, task,
                          team_size, 0, 0, self._scene, int(flank), self._paths[0], self._paths[1], self._paths[2],
                          self._paths[3], world_id_offset)
        h = C.c_void_p()
        rc = self.lib.mpenv_create(C.byref(cfg), C.byref(h))
        assert rc == 0, self.lib.mpenv_last_error().decode()
        self.h = h
        self.W, self.N = num_worlds, 2 * team_size

    def close(self):
        if self.h:
            self.lib.mpenv_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def desc(self, name):
        ptr, dt, nd, gpu = C.c_void_p(), C.c_int32(), C.c_int32(), C.c_int32()
        dims = (C.c_int64 * 8)()
        rc = self.lib.mpenv_export_tensor(self.h, EXPORT[name], C.byref(ptr), C.byref(dt),
                                          C.byref(nd), dims, C.byref(gpu))
        assert rc == 0, self.lib.mpenv_last_error().decode()
        return ptr.value, DTYPES[dt.value], tuple(dims[i] for i in range(nd.value))

    def get(self, name):
        ptr, dt, shape = self.desc(name)
        out = np.empty(shape, dtype=dt)
        self.mem.d2h(ptr, out.nbytes, out)
        return out

    def get_rows(self, name, r0, r1):
        """Rows [r0, r1) of the leading dimension (agents or worlds)."""
        ptr, dt, shape = self.desc(name)
        row = int(np.prod(shape[1:])) * 4
        out = np.empty((r1 - r0,) + tuple(shape[1:]), dtype=dt)
        self.mem.d2h(ptr + r0 * row, out.nbytes, out)
        return out

    def put_rows(self, name, r0, arr):
        """Overwrite rows [r0, r0 + len(arr)) of the leading dimension."""
        ptr, dt, shape = self.desc(name)
        row = int(np.prod(shape[1:])) * 4
        self.mem.h2d(ptr + r0 * row, np.ascontiguousarray(arr, dtype=dt))

    def combat_actions(self, tape_dev, out_dev=None, mode=1):
        """mpenv_combat_actions: the device aim-bot over the tape rows at
        tape_dev ([A][6] i32), into out_dev or straight into the step inputs."""
        self.lib.mpenv_combat_actions.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
        assert self.lib.mpenv_combat_actions(self.h, tape_dev, out_dev, mode, None) == 0, \
            self.lib.mpenv_last_error().decode()
        if out_dev is not None:
            self.mem.hip.hipDeviceSynchronize()

    def set_world_groups(self, groups):
        self.lib.mpenv_set_world_groups.argtypes = [C.c_void_p, C.c_int32]
        assert self.lib.mpenv_set_world_groups(self.h, groups) == 0, self.lib.mpenv_last_error().decode()

    def enable_stats(self, on=True):
        self.lib.mpenv_enable_stats.argtypes = [C.c_void_p, C.c_int32]
        assert self.lib.mpenv_enable_stats(self.h, int(on)) == 0, self.lib.mpenv_last_error().decode()

    def read_stats(self):
        """Workload counters (include/mpenv.h mpenv_read_stats)."""
        self.lib.mpenv_read_stats.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
        v = np.zeros(10, np.uint64)
        assert self.lib.mpenv_read_stats(self.h, v.ctypes.data, 10) >= 0, self.lib.mpenv_last_error().decode()
        names = ("alive_agents", "los_pairs", "los_rays", "los_seen", "sphere_casts", "shot_rays",
                 "hit_agents", "kills", "lk_rows", "los_traced")
        return dict(zip(names, (int(x) for x in v)))

    def copy_actions(self, dev_ptr):
        """Step inputs from device memory [A][6] i32 (gpuStreamStep's copy)."""
        assert self.lib.mpenv_copy_actions(self.h, dev_ptr, None) == 0, self.lib.mpenv_last_error().decode()

    def trigger_reset(self, w):
        assert self.lib.mpenv_trigger_reset(self.h, w) == 0

    def set_hp(self, w, a, hp):
        assert self.lib.mpenv_set_hp(self.h, w, a, hp) == 0

    def put(self, name, arr):
        ptr, dt, shape = self.desc(name)
        arr = np.ascontiguousarray(arr, dtype=dt).reshape(shape)
        self.mem.h2d(ptr, arr)

    def put_ctrl(self, ctrl):
        self.put("SIM_CONTROL", ctrl)

    def set_actions(self, acts6):
        self.put("PVP_DISCRETE_ACTION", acts6[:, :4])
        self.put("PVP_DISCRETE_AIM_ACTION", acts6[:, 4:6])

    def init(self):
        rc = self.lib.mpenv_init(self.h)
        assert rc == 0, self.lib.mpenv_last_error().decode()

    def step(self):
        rc = self.lib.mpenv_step(self.h)
        assert rc == 0, self.lib.mpenv_last_error().decode()


def explore_visited(sim):
    """[A, 81*81] u32: 1 where the ExploreTracker cell holds the agent's
    current episode index.  The engine exports exactly this (its bitset);
    the oracle keeps the reference's u32 tags, reduced here with the world's
    current episode (DEBUG_WORLD_I32[10])."""
    if isinstance(sim, Oracle):
        tags = sim.get("DEBUG_EXPLORE")
        ep = np.repeat(sim.get("DEBUG_WORLD_I32")[:, 10].astype(np.uint32), sim.N)
        return (tags == ep[:, None]).astype(np.uint32)
    return sim.get("DEBUG_EXPLORE")


def compare(a, b, name, float_rtol=0.0):
    """Byte-exact: integers by value, floats by their bit patterns (as
    uint32), so +0 / -0 differ and a NaN only matches a NaN with the same
    payload and sign.  float_rtol > 0 (no caller uses it; the north star's
    1e-5 ceiling) relaxes non-NaN floats to that relative tolerance."""
    assert a.shape == b.shape, (name, a.shape, b.shape)
    if a.dtype.kind == "f":
        assert a.dtype == np.float32 and b.dtype == np.float32, (name, a.dtype, b.dtype)
        same = np.ascontiguousarray(a).view(np.uint32) == np.ascontiguousarray(b).view(np.uint32)
        if float_rtol > 0:
            same |= np.abs(a - b) <= float_rtol * np.maximum(np.abs(a), np.abs(b))
        if not same.all():
            idx = np.argwhere(~same)
            i0 = tuple(idx[0])
            ab = np.ascontiguousarray(a).view(np.uint32)[i0]
            bb = np.ascontiguousarray(b).view(np.uint32)[i0]
            raise AssertionError(
                f"{name}: {len(idx)} mismatches, first at {i0}: engine={a[i0]!r} (0x{ab:08x}) "
                f"oracle={b[i0]!r} (0x{bb:08x})")
    else:
        if not np.array_equal(a, b):
            idx = np.argwhere(a != b)
            i0 = tuple(idx[0])
            raise AssertionError(
                f"{name}: {len(idx)} mismatches, first at {i0}: engine={a[i0]!r} oracle={b[i0]!r}")


# Discrete-aim turn table (sim.cpp:2284-2370 pvpDiscreteAimSystem).
_YAW_TURN = np.array([0, 1 / 256, 1 / 128, 1 / 64, 1 / 32, 1 / 16, 1 / 8]) * np.pi
_PITCH_TURN = np.array([0, 1 / 128, 1 / 64, 1 / 32]) * np.pi


def combat_actions(sim, step, seed=1234, base=None):
    """Tape actions overridden by a greedy aim-bot for agents that see an
    opponent: turn toward the first visible opponent (relative yaw/pitch are
    opponent-observation fields 24/25, sim.cpp obs layout) and fire when
    roughly on target.  A deterministic function of the observations, so it
    drives engine and oracle identically while parity holds; it exists to
    exercise kills, respawns and combat rewards, which a pure random tape on
    simple_map rarely reaches."""
    A = sim.W * sim.N
    # base: the tape rows to override (default: the hash tape from agent 0)
    acts = mpenv_tape.tape_actions(seed, step, 0, A) if base is None else np.array(base, np.int32)
    opp = sim.get("OPPONENT_OBSERVATIONS")  # [A, 6, 32]
    mask = sim.get("OPPONENT_MASKS").reshape(A, -1)
    vis = mask[:, :opp.shape[1]] > 0
    has = vis.any(1)
    k = np.argmax(vis, 1)
    yaw = opp[np.arange(A), k, 24]
    pitch = opp[np.arange(A), k, 25]

    yb = _bucket(yaw, _YAW_TURN, 6)
    pb = _bucket(pitch, _PITCH_TURN, 3)
    acts[has, 4] = yb[has]
    acts[has, 5] = pb[has]
    acts[has, 2] = np.where(np.abs(yaw[has]) < 0.05, 1, 0)
    return acts


def _bucket(delta, table, centre):
    mag = np.abs(delta)[:, None]
    idx = np.sum(table[None, 1:] <= mag, axis=1)
    return (centre + np.sign(delta) * idx).astype(np.int32)


def seek_combat_actions(sim, step, seed=1234, base=None):
    """combat_actions, and agents that see no opponent turn toward the zone
    (self-observation 31, ZoneObservation.toCenterYaw) and run forward once
    within 0.5 rad of it, else stand still: both teams converge on the zone,
    so fights, kills and respawns are frequent; an empty magazine (self obs
    24 == 0, not reloading: obs 25 == 0) is reloaded.  The engine's
    mpenv_combat_actions(mode 1) computes the same function on the device."""
    A = sim.W * sim.N
    acts = combat_actions(sim, step, seed, base)
    mask = sim.get("OPPONENT_MASKS").reshape(A, -1)
    no = ~(mask[:, :6] > 0).any(1)
    so = sim.get("SELF_OBSERVATION").reshape(A, -1)
    zy = so[:, 31]
    face = np.abs(zy) < np.float32(0.5)
    acts[no, 4] = _bucket(zy, _YAW_TURN, 6)[no]
    acts[no & face, 0] = 2
    acts[no & face, 1] = 0
    acts[no & ~face, 0] = 0
    acts[(so[:, 24] == 0) & (so[:, 25] == 0), 2] = 2
    return acts


def edge_aimed_rays(verts, n_origins, seed):
    """Rays aimed exactly at every triangle vertex and edge midpoint (shared
    edges/vertices are where two triangles tie) from random origins."""
    rng = np.random.default_rng(seed)
    tris = verts.reshape(-1, 3, 3).astype(np.float64)
    targets = np.concatenate([tris.reshape(-1, 3),
                              0.5 * (tris[:, 0] + tris[:, 1]), 0.5 * (tris[:, 1] + tris[:, 2]),
                              0.5 * (tris[:, 2] + tris[:, 0])])
    o = rng.uniform([-1500, -1500, -50], [1500, 1500, 300], (n_origins, 3))
    oo = np.repeat(o, len(targets), axis=0)
    tt = np.tile(targets, (n_origins, 1))
    d = tt - oo
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return oo.astype(np.float32), d.astype(np.float32)
