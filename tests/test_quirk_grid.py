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


# --------------------------------------------------------------------------
# Bounded vs full sphere casts (the exactness claim itself, not only the grid)

KFLT_MAX = np.float32(np.finfo(np.float32).max)
BUFFER = np.float32(0.05 * 15.0)
CAST_SLACK = np.float32(4.0)  # kernels.hip kCastSlack


def guard_path_clear(q, px, py, qx, qy):
    """castPathQuirkFreeD: every cell of the xy box of 2o .. 2o + B·d clear
    (px, py = 2o; qx, qy = 2o + B·d, float32 as the kernel forms them)."""
    min_x, min_y, cell, w, h, bits = q
    inv = np.float32(1.0) / cell
    x0 = np.maximum(np.floor((np.minimum(px, qx) - min_x) * inv).astype(np.int64), 0)
    x1 = np.minimum(np.floor((np.maximum(px, qx) - min_x) * inv).astype(np.int64), w - 1)
    y0 = np.maximum(np.floor((np.minimum(py, qy) - min_y) * inv).astype(np.int64), 0)
    y1 = np.minimum(np.floor((np.maximum(py, qy) - min_y) * inv).astype(np.int64), h - 1)
    clear = np.ones(len(px), bool)
    span = int(max((x1 - x0).max(initial=0), (y1 - y0).max(initial=0))) + 1
    for dy in range(span):
        for dx in range(span):
            x, y = x0 + dx, y0 + dy
            live = (x <= x1) & (y <= y1)
            bit = np.where(live, y * w + x, 0)
            marked = ((bits[bit >> 5] >> (bit & 31).astype(np.uint32)) & 1) == 1
            clear &= ~(live & marked)
    return clear


def casts(o, origins, dirs, t_max=None):
    lib = o.lib
    n = len(origins)
    org = np.ascontiguousarray(origins, np.float32)
    d = np.ascontiguousarray(dirs, np.float32)
    t = np.zeros(n, np.float32)
    nrm = np.zeros((n, 3), np.float32)
    tm = None if t_max is None else T.fptr(np.ascontiguousarray(t_max, np.float32))
    lib.oracle_sphere_cast_batch(o.h, n, T.fptr(org), T.fptr(d), np.float32(R), tm, T.fptr(t), T.fptr(nrm))
    return t, nrm


def k_move_origins(n, rng):
    """Cast origins like applyVelocity's: agent positions from an oracle
    rollout raised by the pose heights, and origins whose 2o lands near a
    vertex (where the testVert quirk lives)."""
    o = T.Oracle(8, 6)
    o.put_ctrl([0, 1, 1])
    o.init()
    pos = []
    for s in range(120):
        o.set_actions(T.mpenv_tape.tape_actions(4321, s, 0, 8 * 12))
        o.step()
        if s % 6 == 5:
            pos.append(o.get("DEBUG_AGENT_F32")[:, :3].copy())
    pos = np.concatenate(pos).astype(np.float32)
    _, verts, _ = T.scene_bvh()
    verts = verts.reshape(-1, 3)
    z_off = np.array([9.0, 50.0, 35.0, 9.75], np.float32)  # low_check / top (stand, crouch, prone)
    a = pos[rng.integers(0, len(pos), n)] + np.stack(
        [rng.uniform(-40, 40, n), rng.uniform(-40, 40, n), z_off[rng.integers(0, 4, n)]], 1)
    # 2o within ~60 units of a vertex, z from the rollout
    vi = rng.integers(0, len(verts), n)
    b = np.stack([(verts[vi, 0] + rng.uniform(-60, 60, n)) * 0.5, (verts[vi, 1] + rng.uniform(-60, 60, n)) * 0.5,
                  pos[rng.integers(0, len(pos), n), 2] + z_off[rng.integers(0, 4, n)]], 1)
    return o, np.concatenate([a, b]).astype(np.float32)


def test_bounded_sphere_casts_equal_full_casts_where_guard_is_clear():
    """castNearD (kernels.hip) returns the bounded cast's hit when the path
    guard is clear: its (t, normal) must equal the full cast's whenever
    either is nearer than the bound, and both must read "no hit" otherwise.
    Horizontal casts with the bounds k_move uses (forward: move_dist + buffer
    + slack, move_dist in [0, 20]; slide: the same with max_move); origins
    from an oracle rollout and origins whose 2o sits near vertices."""
    rng = np.random.default_rng(11)
    o, org = k_move_origins(40000, rng)
    n = len(org)
    ang = rng.uniform(0, 2 * np.pi, n)
    d = np.stack([np.sin(ang), np.cos(ang), np.zeros(n)], 1).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
    move = rng.uniform(0, 20.0, n).astype(np.float32)
    B = (move + BUFFER) + CAST_SLACK
    q = quirk_grid()
    px, py = org[:, 0] + org[:, 0], org[:, 1] + org[:, 1]
    clear = guard_path_clear(q, px, py, px + d[:, 0] * B, py + d[:, 1] * B)
    t_full, n_full = casts(o, org, d)
    t_b, n_b = casts(o, org, d, B)
    near_full = t_full < B
    near_b = t_b < B
    c = clear
    assert c.mean() > 0.3, c.mean()  # the guard is not vacuous
    assert (near_full[c] == near_b[c]).all()
    both = c & near_b
    assert both.sum() > 1000, both.sum()  # many bounded hits compared
    assert np.array_equal(t_full[both], t_b[both])
    assert np.array_equal(n_full[both], n_b[both])
    # the single-cell guard (round 2) was not enough for horizontal casts:
    # report how often it would have taken a bounded cast that differs
    old_clear = guard_clear(q, px, py)
    old_b = (move + BUFFER) * 2 + 10
    t_ob, _ = casts(o, org, d, old_b)
    bad = old_clear & ((t_full < old_b) != (t_ob < old_b))
    bad |= old_clear & (t_full < old_b) & (t_ob < old_b) & (t_full != t_ob)
    print(f"\n{n} casts: path guard clear {c.mean():.3f}, bounded hits compared {both.sum()}, "
          f"single-cell guard clear {old_clear.mean():.3f} with {bad.sum()} differing bounded casts")
    o.close()


def test_bounded_ground_casts_equal_full_casts_where_cell_is_clear():
    """castFirstNearD (vertical casts): where the cell of 2o is clear, a hit
    found within the bound equals the full cast's t."""
    rng = np.random.default_rng(12)
    o, org = k_move_origins(20000, rng)
    n = len(org)
    d = np.tile(np.array([0, 0, -1], np.float32), (n, 1))
    B = np.full(n, 2 * 50.0 + 10, np.float32)  # 2·top + 10 (stand)
    q = quirk_grid()
    clear = guard_clear(q, org[:, 0] + org[:, 0], org[:, 1] + org[:, 1])
    t_full, n_full = casts(o, org, d)
    t_b, n_b = casts(o, org, d, B)
    sel = clear & (t_b < B)
    assert sel.sum() > 1000, sel.sum()
    assert np.array_equal(t_full[sel], t_b[sel])
    assert np.array_equal(n_full[sel], n_b[sel])
    assert ((t_full < B) == (t_b < B))[clear].all()
    o.close()


def test_path_guard_covers_quirk_hits_ahead_of_2o():
    """Casts aimed so that the ray 2o + t·d passes a vertex at t in (r, r + 50):
    the cell of 2o can be clear while the testVert quirk still fires before
    the bound (the round-2 single-cell guard with its old bounds
    takes bounded casts that differ from the full cast here).  The path guard
    must never do so."""
    rng = np.random.default_rng(3)
    o = T.Oracle(1, 1)
    _, verts, _ = T.scene_bvh()
    verts = verts.reshape(-1, 3)
    q = quirk_grid()
    n = 150000
    vi = rng.integers(0, len(verts), n)
    ang = rng.uniform(0, 2 * np.pi, n)
    d = np.stack([np.sin(ang), np.cos(ang), np.zeros(n)], 1).astype(np.float32)
    P = verts[vi, :2] - d[:, :2] * (R + rng.uniform(2, 50, n))[:, None]
    org = np.stack([P[:, 0] / 2, P[:, 1] / 2, rng.uniform(-150, 600, n)], 1).astype(np.float32)
    move = rng.uniform(0, 20, n).astype(np.float32)
    px, py = org[:, 0] + org[:, 0], org[:, 1] + org[:, 1]
    t_full, _ = casts(o, org, d)

    def differing(clear, B):
        t_b, _ = casts(o, org, d, B)
        nf, nb = t_full < B, t_b < B
        return clear & ((nf != nb) | (nf & nb & (t_full != t_b)))

    old_b = (move + BUFFER) * 2 + 10
    old_bad = differing(guard_clear(q, px, py), old_b)
    B = (move + BUFFER) + CAST_SLACK
    clear = guard_path_clear(q, px, py, px + d[:, 0] * B, py + d[:, 1] * B)
    new_bad = differing(clear, B)
    print(f"\nsingle-cell guard: {old_bad.sum()} differing of {n}; path guard clear {clear.mean():.3f}, "
          f"{new_bad.sum()} differing")
    assert old_bad.sum() > 0  # the construction does reach the quirk
    assert clear.sum() > n // 4 and new_bad.sum() == 0
    o.close()
