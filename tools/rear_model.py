"""Work model for rear-fan candidate lists (development tool, CPU): the
oracle steps a batch (tape or combat actions), then for every rear sheet
(agent x height, 8 rays over [0, -pi] in the body frame) counts the
triangles a per-wave list would keep (front side, within the band of the
sheet plane, in the rear half-plane) and, per ray, the triangles it hits
(any t > 0, front side) -- the candidates a lane would test.

  python tools/rear_model.py [tape|combat] [steps] [worlds]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import mpenv_testlib as T  # noqa: E402

R_AG, STAND, CROUCH, PRONE = 15.0, 65.0, 47.0, 30.0


def qrot(q, v):
    w, x, y, z = q[..., 0:1], q[..., 1:2], q[..., 2:3], q[..., 3:4]
    p = np.concatenate([x, y, z], -1)
    t = 2.0 * np.cross(p, v)
    return v + w * t + np.cross(p, t)


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "tape"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 150
    W = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    ts = 6
    A = W * 2 * ts
    o = T.Oracle(W, ts)
    o.put_ctrl([0, 1, 1])
    o.init()
    ring = T.mpenv_tape.tape_ring(1234, 0, A, 64)
    for s in range(steps):
        acts = T.seek_combat_actions(o, s, base=ring[s % 64]) if mode == "combat" else np.ascontiguousarray(ring[s % 64])
        o.lib.oracle_run_threaded(o.h, 1, T.usable_cpus(), acts.ctypes.data, 1)
    af = o.get("DEBUG_AGENT_F32").reshape(A, -1)
    ai = o.get("DEBUG_AGENT_I32").reshape(A, -1)
    pos, rot, pose = af[:, 0:3].astype(np.float64), af[:, 6:10].astype(np.float64), ai[:, 0]
    print("body rotations with x = y = 0 exactly:", float(np.mean((af[:, 7] == 0) & (af[:, 8] == 0))))
    _, verts, _ = T.scene_bvh()
    tri = verts.reshape(-1, 3, 3).astype(np.float64)
    nt = len(tri)
    a, b, c = tri[:, 0], tri[:, 1], tri[:, 2]
    n = np.cross(b - a, c - a)
    n /= np.linalg.norm(n, axis=1, keepdims=True)
    zmin, zmax = tri[:, :, 2].min(1), tri[:, :, 2].max(1)
    theta = -np.pi * np.arange(8) / 7.0
    rng = np.random.default_rng(0)
    agents = rng.choice(A, min(A, 4096), replace=False)
    agents = agents[(agents // 4) * 4 == agents] if False else agents
    Ls, cands, hits = [], [], []
    wave_L = {}
    for g in agents:
        top = {0: STAND, 1: CROUCH}.get(int(pose[g]), PRONE) - R_AG + R_AG
        Rv = qrot(rot[g], np.array([1.0, 0, 0]))
        Fv = qrot(rot[g], np.array([0, 1.0, 0]))
        for h in (0, 1):
            O = pos[g].copy()
            O[2] += R_AG + (top - 2 * R_AG) * h
            front = ((O - a) * n).sum(1) >= -0.05
            band = (zmin <= O[2] + 0.05) & (zmax >= O[2] - 0.05)
            rear = (tri - O) @ Fv
            half = rear.min(1) <= 0.01
            keep = front & band & half
            d = (-np.cos(theta))[:, None] * Rv[None] + np.sin(theta)[:, None] * Fv[None]
            d /= np.linalg.norm(d, axis=1, keepdims=True)
            # Moller-Trumbore against every kept triangle, all 8 rays
            e1, e2 = (b - a)[keep], (c - a)[keep]
            p = np.cross(d[:, None, :], e2[None])
            det = (e1[None] * p).sum(-1)
            inv = 1.0 / np.where(np.abs(det) < 1e-12, 1e-12, det)
            tv = O[None, None, :] - a[keep][None]
            u = (tv * p).sum(-1) * inv
            q = np.cross(tv, e1[None])
            v = (d[:, None, :] * q).sum(-1) * inv
            t = (e2[None] * q).sum(-1) * inv
            hit = (u >= -1e-3) & (v >= -1e-3) & (u + v <= 1 + 1e-3) & (t > 0)
            L = int(hit.any(0).sum())
            Ls.append(L)
            wave_L.setdefault(g // 4, []).append(L)
            cands.extend(hit.sum(1).tolist())
    Ls, cands = np.array(Ls), np.array(cands)
    wl = np.array([max(v) for v in wave_L.values()])
    print(f"{mode}, {steps} steps, {W} worlds: triangles {nt}; per rear sheet: list length mean {Ls.mean():.1f} "
          f"p90 {np.percentile(Ls, 90):.0f} max {Ls.max()}; per ray candidates mean {cands.mean():.2f} "
          f"p90 {np.percentile(cands, 90):.0f} max {cands.max()}; per 4-agent wave (sampled agents) longest list "
          f"mean {wl.mean():.1f}")


if __name__ == "__main__":
    main()
