"""DESIGN.md §2 definition 13: the ray-box slab products of
MeshBVH::traceRay (q * dirQuant + originQuant, mesh_bvh.inl:165-183) are
evaluated fused, as the reference's NVRTC build contracts them
(--fmad=true), in both the engine (geom_dev.h bvhTraceRayT) and the oracle.
The reference's CPU executor, the north star's parity target, is built
without contraction.  This pins the effect of the choice: with the slab
products multiplied and added separately, no closest hit changes -- hit flag
and t are identical on random rays, on rays aimed exactly at every vertex and
edge midpoint (where boxes and triangles touch), and on lidar fans from a
rollout, in slot order and in the lidar's octant order."""
import numpy as np

import mpenv_testlib as T


def _trace(o, org, d, octant):
    n = len(org)
    org = np.ascontiguousarray(org, np.float32)
    d = np.ascontiguousarray(d, np.float32)
    t = np.zeros(n, np.float32)
    h = np.zeros(n, np.int32)
    o.lib.oracle_trace_ray_batch(o.h, n, T.fptr(org), T.fptr(d), int(octant), T.fptr(t), h.ctypes.data)
    return t, h


def _lidar_rays(n_worlds=8, steps=(5, 60)):
    import sys, os
    sys.path.insert(0, os.path.join(T.ROOT, "tools"))
    from dump_lidar_rays import rays_for
    o = T.Oracle(n_worlds, 6)
    o.put_ctrl([0, 1, 1])
    o.init()
    out = []
    for s in range(max(steps) + 1):
        o.set_actions(T.mpenv_tape.tape_actions(1234, s, 0, n_worlds * 12))
        o.step()
        if s in steps:
            out.append(rays_for(o.get("DEBUG_AGENT_F32"), o.get("DEBUG_AGENT_I32")))
    o.close()
    r = np.concatenate(out)
    return r[:, :3], r[:, 3:]


def test_unfused_slabs_change_no_closest_hit():
    o = T.Oracle(1, 1)
    _, verts, _ = T.scene_bvh()
    rng = np.random.default_rng(11)
    ro = rng.uniform([-2000, -2000, -150], [2000, 2000, 600], (100000, 3)).astype(np.float32)
    rd = rng.normal(size=(100000, 3))
    rd = (rd / np.linalg.norm(rd, axis=1, keepdims=True)).astype(np.float32)
    eo, ed = T.edge_aimed_rays(verts, 20, 12)
    lo, ld = _lidar_rays()
    try:
        for name, org, d, octant in (("random", ro, rd, 0), ("edge", eo, ed, 0), ("lidar", lo, ld, 1),
                                     ("lidar slot order", lo, ld, 0)):
            o.lib.oracle_set_slab_fma(1)
            t1, h1 = _trace(o, org, d, octant)
            o.lib.oracle_set_slab_fma(0)
            t0, h0 = _trace(o, org, d, octant)
            assert h1.sum() > len(h1) // 4, name  # the sets do hit geometry
            np.testing.assert_array_equal(h0, h1, err_msg=name)
            np.testing.assert_array_equal(t0[h1 == 1], t1[h1 == 1], err_msg=name)
    finally:
        o.lib.oracle_set_slab_fma(1)
        o.close()
