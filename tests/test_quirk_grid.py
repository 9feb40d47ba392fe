"""The guard that lets k_move bound its sphere casts (DESIGN.md §2,
"Distance-bounded sphere casts"): the reference's vertex test
(mesh_bvh.inl:1073-1104) returns t = 0 for any visited triangle with a vertex
within the cast radius of 2·origin, so a bounded cast is only exact where no
vertex lies that close.  k_move reads the grid below with the same float
arithmetic as castQuirkFreeD (kernels.hip); this checks, on CPU, that every
point the guard calls clear is farther than the radius (plus slack) from
every vertex in xy -- and so in 3-D -- including points hugging vertices and
cell edges."""
import ctypes as C

import numpy as np

import mpenv_testlib as T

R = 15.0  # consts::agentRadius, the only sphere-cast radius


def quirk_grid(scene=T.SCENE):
    lib = T.lib_mpenv()
    lib.mpenv_scene_quirk_grid.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_int32)]
    n = C.c_int32(0)
    hdr = np.zeros(5, dtype=np.int32)
    assert lib.mpenv_scene_quirk_grid(scene.encode(), hdr.ctypes.data, None, C.byref(n)) == 0
    bits = np.zeros(max(n.value, 1), dtype=np.uint32)
    assert lib.mpenv_scene_quirk_grid(scene.encode(), hdr.ctypes.data, bits.ctypes.data, C.byref(n)) == 0
    min_x, min_y, cell = hdr[:3].view(np.float32)
    return np.float32(min_x), np.float32(min_y), np.float32(cell), int(hdr[3]), int(hdr[4]), bits


def guard_clear(q, px, py):
    """castQuirkFreeD on float32 points (px, py) = 2·origin."""
    min_x, min_y, cell, w, h, bits = q
    inv = np.float32(1.0) / cell
    fx = (px.astype(np.float32) - min_x) * inv
    fy = (py.astype(np.float32) - min_y) * inv
    inside = (fx >= 0) & (fx < np.float32(w)) & (fy >= 0) & (fy < np.float32(h))
    ix = np.where(inside, fx, 0).astype(np.int64)
    iy = np.where(inside, fy, 0).astype(np.int64)
    bit = iy * w + ix
    marked = (bits[bit >> 5] >> (bit & 31).astype(np.uint32)) & 1
    return ~inside | (marked == 0)


def min_xy_dist(verts, px, py, chunk=4096):
    out = np.empty(len(px), dtype=np.float64)
    vx, vy = verts[:, 0].astype(np.float64), verts[:, 1].astype(np.float64)
    for s in range(0, len(px), chunk):
        dx = px[s:s + chunk, None].astype(np.float64) - vx[None, :]
        dy = py[s:s + chunk, None].astype(np.float64) - vy[None, :]
        out[s:s + chunk] = np.sqrt((dx * dx + dy * dy).min(axis=1))
    return out


def test_quirk_guard_is_conservative():
    q = quirk_grid()
    _, verts, _ = T.scene_bvh()
    verts = verts.reshape(-1, 3)
    rng = np.random.default_rng(7)
    lo, hi = verts[:, :2].min(axis=0) - 200.0, verts[:, :2].max(axis=0) + 200.0
    # uniform over the map and its surroundings
    pu = rng.uniform(lo, hi, size=(60000, 2))
    # near vertices: within 25 units of a random vertex
    vi = rng.integers(0, len(verts), size=60000)
    ang = rng.uniform(0, 2 * np.pi, size=60000)
    rad = rng.uniform(0, 25.0, size=60000)
    pv = verts[vi, :2] + np.stack([rad * np.cos(ang), rad * np.sin(ang)], axis=1)
    # on cell edges near vertices (the float cell index may round either way)
    min_x, min_y, cell = q[0], q[1], q[2]
    pe = pv.copy()
    pe[:, 0] = min_x + np.round((pe[:, 0] - min_x) / cell) * cell
    pts = np.concatenate([pu, pv, pe]).astype(np.float32)
    clear = guard_clear(q, pts[:, 0], pts[:, 1])
    d = min_xy_dist(verts, pts[:, 0], pts[:, 1])
    # every clear point is beyond the radius with slack (the quirk needs
    # |2o - v| <= r up to rounding of v - o, ~1e-3 on this map)
    assert np.all(d[clear] > R + 1.0), d[clear].min()
    # and the guard is not vacuous: most points near vertices are marked,
    # most points far from everything are clear
    assert (~clear[d <= R]).all()
    assert clear[d > R + 2.0 + 2 * 16 * 1.5].mean() > 0.99


def test_quirk_grid_covers_every_vertex_neighbourhood():
    q = quirk_grid()
    _, verts, _ = T.scene_bvh()
    verts = verts.reshape(-1, 3)
    # the vertices themselves (2o == v) are never clear
    assert not guard_clear(q, verts[:, 0], verts[:, 1]).any()
