"""Scene fixtures and BVH known-answer tests.

Pins the loaders and the MeshBVH against the reference's only data fixture,
data/simple_map/*.bin (copied to scenes/simple_map; formats per
src/map_importer.cpp:223-567), using an independent numpy parser written
here, plus the facts SURVEY.md §8c records for that map.  The BVH traversal
(mesh_bvh.inl:49-186 traceRay, 734-953 sphereCast restatements in the
oracle) is checked bit-exactly against a brute-force loop over the same
triangle tests, and against float64 closed forms for vertical rays.
"""
import ctypes as C
import os
import struct

import numpy as np
import pytest

import mpenv_testlib as T

SCENE = T.SCENE


def parse_collisions(path):
    """map_importer.cpp:223-256: bounds, materials, meshes -> triangle list."""
    buf = open(path, "rb").read()
    off = 0

    def take(fmt, n=1):
        nonlocal off
        size = struct.calcsize("<" + fmt) * n
        out = np.frombuffer(buf, dtype=np.dtype("<" + fmt), count=n, offset=off)
        off += size
        return out

    bounds = take("f", 6)
    nmat = int(take("Q")[0])
    nname = int(take("Q")[0])
    take("B", nname)
    mflags = take("I", nmat)
    nmesh, nvert, ntri = (int(x) for x in take("Q", 3))
    verts = take("f", 3 * nvert).reshape(-1, 3)
    idx = take("I", 3 * ntri).reshape(-1, 3)
    tmat = take("I", ntri)
    minfo = take("I", 4 * nmesh).reshape(-1, 4)
    assert off == len(buf)
    tris = []
    for voff, _nv, toff, nt in minfo:
        for i in range(toff, toff + nt):
            if tmat[i] < nmat and mflags[tmat[i]] == 1:
                continue  # BulletsOnly
            tris.append(verts[voff + idx[i]])
    return bounds, nmat, nmesh, nvert, ntri, np.array(tris, np.float32)


@pytest.fixture(scope="module")
def scene():
    return parse_collisions(os.path.join(SCENE, "collisions.bin"))


@pytest.fixture(scope="module", params=["collision", "lidar"])
def bvh(request):
    """Both trees the engine builds over the same triangles: the collision
    tree (every query but the lidar) and k_lidar's own (scene.h
    lidarBVHOpts); the oracle's octant / lex lidar rules walk the latter
    (tests/test_lidar_order.py pins them against brute force)."""
    return T.scene_bvh(lidar=request.param == "lidar")


@pytest.fixture(scope="module")
def oracle():
    o = T.Oracle(1, 1)
    yield o
    o.close()


def test_collisions_fixture_facts(scene):
    bounds, nmat, nmesh, nvert, ntri, tris = scene
    np.testing.assert_allclose(bounds, [-2007.875, -2007.875, -163.979, 2007.875, 2007.875, 623.423],
                               atol=1e-3)
    assert (nmat, nmesh, nvert, ntri) == (1, 21, 504, 252)
    assert tris.shape == (252, 3, 3)


def test_spawns_and_zones_fixture_facts():
    raw = open(os.path.join(SCENE, "spawns.bin"), "rb").read()
    off, counts, zs = 0, [], []
    for _ in range(3):
        (n,) = struct.unpack_from("<I", raw, off)
        off += 4
        sp = np.frombuffer(raw, "<f4", count=8 * n, offset=off).reshape(n, 8)
        off += 32 * n
        counts.append(n)
        zs.append(sp[:, [2, 5]])
    assert off == len(raw)
    assert counts == [8, 8, 16]
    for z in zs:
        np.testing.assert_allclose(z, 31.496, atol=1e-3)
    raw = open(os.path.join(SCENE, "zones.bin"), "rb").read()
    (nz,) = struct.unpack_from("<I", raw, 0)
    assert nz == 3 and len(raw) == 4 + nz * 24 + nz * 4
    rot = np.frombuffer(raw, "<f4", count=nz, offset=4 + nz * 24)
    np.testing.assert_array_equal(rot, 0)


def _nodes(raw):
    dt = np.dtype([("min", "<f4", 3), ("exp", "i1", 3), ("internal", "u1"), ("triSize", "u1", 4),
                   ("qmin", "u1", (3, 4)), ("qmax", "u1", (3, 4)), ("children", "<i4", 4),
                   ("parent", "<i4")])
    assert dt.itemsize == 64
    return np.frombuffer(raw.tobytes(), dtype=dt)


def test_bvh_structure(scene, bvh):
    tris = scene[5]
    raw, verts, max_stack = bvh
    nodes = _nodes(raw)
    bvh_tris = verts.reshape(-1, 3, 3)
    # every input triangle appears exactly once in the leaves
    key = lambda a: sorted(map(lambda t: t.tobytes(), a))  # noqa: E731
    assert key(bvh_tris) == key(tris)
    assert 1 <= max_stack <= 16
    seen = np.zeros(len(bvh_tris), int)
    for n in nodes:
        scale = np.ldexp(1.0, n["exp"].astype(int))
        for i in range(4):
            c = int(n["children"][i])
            if c == -1:
                continue
            lo = n["min"].astype(np.float64) + scale * n["qmin"][:, i]
            hi = n["min"].astype(np.float64) + scale * n["qmax"][:, i]
            if c & 0x80000000 or c < 0:
                leaf = c & 0x7FFFFFFF
                nt = int(n["triSize"][i])
                assert 1 <= nt <= 2
                seen[leaf:leaf + nt] += 1
                pts = bvh_tris[leaf:leaf + nt].reshape(-1, 3)
            else:
                assert 0 < c < len(nodes)
                pts = None
            if pts is not None:  # conservative child boxes
                assert (pts >= lo - 1e-6).all() and (pts <= hi + 1e-6).all()
    np.testing.assert_array_equal(seen, 1)


def _rays(n, seed, bounds):
    rng = np.random.default_rng(seed)
    lo, hi = bounds[:3], bounds[3:]
    o = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return o, d.astype(np.float32)


def test_trace_ray_matches_brute_force(oracle, scene):
    o, d = _rays(3000, 0, scene[0])
    lib = oracle.lib
    hits = 0
    for i in range(len(o)):
        t1, t2 = C.c_float(0), C.c_float(0)
        h1 = lib.oracle_trace_ray(oracle.h, T.fptr(o[i]), T.fptr(d[i]), C.byref(t1))
        h2 = lib.oracle_trace_ray_brute(oracle.h, T.fptr(o[i]), T.fptr(d[i]), C.byref(t2))
        assert h1 == h2, i
        if h1:
            hits += 1
            assert t1.value == t2.value, (i, t1.value, t2.value)
    assert hits > 300


def test_sphere_cast_matches_brute_force(oracle, scene):
    o, d = _rays(1500, 1, scene[0])
    lib = oracle.lib
    nrm = np.zeros(3, np.float32)
    hits = 0
    for i in range(len(o)):
        for r in (1.0, 15.0):
            t1 = lib.oracle_sphere_cast(oracle.h, T.fptr(o[i]), T.fptr(d[i]), r, T.fptr(nrm))
            t2 = lib.oracle_sphere_cast_brute(oracle.h, T.fptr(o[i]), T.fptr(d[i]), r)
            assert t1 == t2, (i, r, t1, t2)
            hits += t1 < 3.0e38
    assert hits > 300


def _down_ray_f64(tris, x, y, z0):
    """Exact (float64) first hit of a -z ray from (x, y, z0) against tris."""
    best = np.inf
    for a, b, c in tris.astype(np.float64):
        # barycentric point-in-triangle on xy, then plane height
        v0, v1 = b - a, c - a
        den = v0[0] * v1[1] - v1[0] * v0[1]
        if abs(den) < 1e-12:
            continue
        px, py = x - a[0], y - a[1]
        u = (px * v1[1] - v1[0] * py) / den
        v = (v0[0] * py - px * v0[1]) / den
        if u < 0 or v < 0 or u + v > 1:
            continue
        z = a[2] + u * v0[2] + v * v1[2]
        t = z0 - z
        if 0 < t < best:
            best = t
    return best


def test_vertical_rays_closed_form(oracle, scene):
    tris = scene[5]
    rng = np.random.default_rng(3)
    z0 = 1000.0
    d = np.array([0, 0, -1], np.float32)
    checked = 0
    for _ in range(400):
        x, y = rng.uniform(-1500, 1500, 2)
        o = np.array([x, y, z0], np.float32)
        expect = _down_ray_f64(tris, float(o[0]), float(o[1]), z0)
        t = C.c_float(0)
        hit = oracle.lib.oracle_trace_ray(oracle.h, T.fptr(o), T.fptr(d), C.byref(t))
        if np.isinf(expect):
            continue  # edge-grazing/outside: covered by the brute-force test
        assert hit, (x, y, expect)
        assert t.value == pytest.approx(expect, rel=1e-5, abs=1e-3)
        checked += 1
    assert checked > 100
    # sphere cast straight down onto the same surface stops r earlier for a
    # horizontal floor: t_sphere = t_ray - r
    o = np.array([0.0, 0.0, z0], np.float32)
    expect = _down_ray_f64(tris, 0.0, 0.0, z0)
    nrm = np.zeros(3, np.float32)
    ts = oracle.lib.oracle_sphere_cast(oracle.h, T.fptr(o), T.fptr(d), 5.0, T.fptr(nrm))
    if abs(nrm[2]) > 0.999:
        assert ts == pytest.approx(expect - 5.0, abs=1e-2)


def test_node_bytes_follow_the_documented_quantisation(bvh):
    """Pins the node bytes both sides traverse (the visited sets, and through
    the sphere-cast testVert quirk the casts' results, depend on them)
    independently of the builder's code: every node's origin, exponents and
    quantised child boxes are recomputed here from the triangles below each
    child, by the rule DESIGN.md §2 documents (csrc/scene.cpp): node origin =
    the children's exact float32 lower corner; per axis the smallest e with
    253·2^e >= range (clamped to [-100, 100]); child box = floor / ceil of
    its exact bounds in 2^e units, widened by one quantum each way and
    clamped to [0, 255].  The reference quantises the same 64-byte node
    format (mesh_bvh_builder.cpp:452-474, 513-530: floor / ceil against
    2^ceil(log2(range / 255)), no widening) over Embree's topology, which
    this image cannot build; the widening is this builder's own margin."""
    raw, verts, _ = bvh
    nodes = _nodes(raw)
    tris = verts.reshape(-1, 3, 3).astype(np.float64)
    boxes = {}

    def child_box(n, i):
        c = int(n["children"][i])
        if c & 0x80000000 or c < 0:
            leaf = c & 0x7FFFFFFF
            pts = tris[leaf:leaf + int(n["triSize"][i])].reshape(-1, 3)
            return pts.min(0), pts.max(0)
        return node_box(c)

    def node_box(oid):
        if oid not in boxes:
            n = nodes[oid]
            kids = [child_box(n, i) for i in range(4) if int(n["children"][i]) != -1]
            boxes[oid] = (np.min([k[0] for k in kids], 0), np.max([k[1] for k in kids], 0))
        return boxes[oid]

    for oid in range(len(nodes) - 1, -1, -1):
        n = nodes[oid]
        lo, hi = node_box(oid)
        mn = lo.astype(np.float32)
        assert (mn.astype(np.float64) == lo).all()  # exact: triangle coordinates are float32
        np.testing.assert_array_equal(n["min"], mn)
        exps = []
        for a in range(3):
            rng_ = hi[a] - float(mn[a])
            e = -100
            if rng_ > 0:
                e = int(np.ceil(np.log2(rng_ / 253.0)))
                while np.ldexp(253.0, e) < rng_:
                    e += 1
            exps.append(max(-100, min(100, e)))
        assert list(n["exp"]) == exps, oid
        internal = 0
        for i in range(4):
            c = int(n["children"][i])
            if c == -1:
                assert n["triSize"][i] == 0
                continue
            cl, ch = child_box(n, i)
            for a in range(3):
                s = np.ldexp(1.0, exps[a])
                ql = max(0.0, np.floor((cl[a] - float(mn[a])) / s) - 1.0)
                qh = min(255.0, np.ceil((ch[a] - float(mn[a])) / s) + 1.0)
                assert n["qmin"][a][i] == ql and n["qmax"][a][i] == qh, (oid, i, a)
                # conservative in exact arithmetic: the dequantised box holds every
                # triangle of the child's subtree
                assert float(mn[a]) + s * ql <= cl[a] and float(mn[a]) + s * qh >= ch[a]
            if c & 0x80000000 or c < 0:
                assert 1 <= n["triSize"][i] <= 2
            else:
                assert c > oid and n["triSize"][i] == 0  # DFS pre-order ids
                internal += 1
        assert n["internal"] == internal


def _variant(scene, opts):
    lib = T.lib_mpenv()
    fn = lib.mpenv_scene_bvh_variant
    fn.argtypes = [C.c_char_p, C.c_void_p, C.c_int32, C.c_void_p, C.POINTER(C.c_int32), C.c_void_p,
                   C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
    o = np.asarray(opts, np.int32)
    nn, nv, ms = C.c_int32(0), C.c_int32(0), C.c_int32(0)
    assert fn(scene.encode(), o.ctypes.data, len(o), None, C.byref(nn), None, C.byref(nv), C.byref(ms)) == 0
    nodes = np.zeros(nn.value * 64, np.uint8)
    verts = np.zeros(nv.value * 3, np.float32)
    assert fn(scene.encode(), o.ctypes.data, len(o), nodes.ctypes.data, C.byref(nn), verts.ctypes.data,
              C.byref(nv), C.byref(ms)) == 0
    return nodes, verts


def test_lidar_tree_tuning_file(tmp_path):
    """scene.cpp readLidarTuning: k_lidar's tree is lidarBVHOpts() plus the
    split ranks of the scene's lidar_tree.txt (tools/trav_stats.cpp
    TRAV_TUNE), applied only to the collisions.bin whose FNV-1a 64 it names;
    without the file, or for another collisions.bin, the untuned tree."""
    import shutil
    base = [2, 12, 1, 400, 10]  # scene.h lidarBVHOpts
    path = os.path.join(SCENE, "lidar_tree.txt")
    assert os.path.exists(path), "the shipped scene carries its tuned lidar tree"
    pairs, want = [], None
    for line in open(path):
        f = line.split()
        if not f or f[0].startswith("#"):
            continue
        if f[0] == "collisions_fnv1a64":
            want = int(f[1], 16)
        else:
            assert f[0] == "split" and len(f) == 3
            pairs += [int(f[1]), int(f[2])]
    h = 1469598103934665603
    for b in open(os.path.join(SCENE, "collisions.bin"), "rb").read():
        h = ((h ^ b) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    assert want == h
    tuned_nodes, tuned_verts, _ = T.scene_bvh(lidar=True)
    n, v = _variant(SCENE, base + pairs)
    assert np.array_equal(n, tuned_nodes) and np.array_equal(v, tuned_verts)
    un, uv = _variant(SCENE, base)
    assert not np.array_equal(un, tuned_nodes) or un.size != tuned_nodes.size
    # a copy without the file, and one whose file names another hash
    for name, text in (("none", None), ("stale", open(path).read().replace(f"{want:016x}", f"{want ^ 1:016x}"))):
        d = tmp_path / name
        d.mkdir()
        for f in ("collisions.bin", "navmesh.bin", "spawns.bin", "zones.bin"):
            shutil.copy(os.path.join(SCENE, f), d)
        if text is not None:
            (d / "lidar_tree.txt").write_text(text)
        ln, lv, _ = T.scene_bvh(str(d), lidar=True)
        assert np.array_equal(ln, un) and np.array_equal(lv, uv), name


def test_split_rank_overrides():
    """BVHBuildOpts::splitRank (scene.cpp Builder::build): rank 0 is the SAH
    choice itself, a heap index the tree does not have changes nothing, and
    a real override changes the tree while keeping every triangle once."""
    base = [2, 12, 1, 400, 10]
    n0, v0 = _variant(SCENE, base)
    n1, v1 = _variant(SCENE, base + [1, 0, 3, 0])
    assert np.array_equal(n0, n1) and np.array_equal(v0, v1)
    n2, v2 = _variant(SCENE, base + [(1 << 30) + 5, 3])
    assert np.array_equal(n0, n2) and np.array_equal(v0, v2)
    n3, v3 = _variant(SCENE, base + [3, 1])
    assert not (n3.size == n0.size and np.array_equal(n3, n0))
    # the same multiset of triangles (simple_map repeats some)
    assert sorted(map(tuple, v3.reshape(-1, 9).tolist())) == sorted(map(tuple, v0.reshape(-1, 9).tolist()))
