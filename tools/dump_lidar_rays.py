"""Record lidar rays (origins + directions, f32 [n][6]) in k_lidar's wave
order -- per 4-agent unit: each agent's 64 forward rays, then the 4 agents'
16 rear rays -- from an oracle rollout (analysis input for
tools/trav_stats.cpp; sim.cpp:3324-3506 ray construction, float32 numpy).

    python tools/dump_lidar_rays.py OUT.f32 [worlds] [step ...]
    DUMP_ACTIONS=combat ...   the zone-seeking aim-bot over the tape (bench.py
                              --actions combat; mpenv_testlib.seek_combat_actions)
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import mpenv_testlib as T  # noqa: E402


def qrot(q, v):
    w, x, y, z = q[:, 0:1], q[:, 1:2], q[:, 2:3], q[:, 3:4]
    p = np.concatenate([x, y, z], 1)
    t = 2.0 * np.cross(p, v)
    return (v + w * t + np.cross(p, t)).astype(np.float32)


def rays_for(af, ai):
    A = len(af)
    pos = af[:, 0:3]
    rot = af[:, 6:10]
    aim = af[:, 12:16]
    pose = ai[:, 0]
    top = np.where(pose == 0, 65.0, np.where(pose == 1, 47.0, 30.0)).astype(np.float32)
    out = []
    for u in range(0, A - A % 4, 4):
        for a in range(u, u + 4):
            q = aim[a:a + 1]
            f = qrot(q, np.array([[0, 1, 0]], np.float32))
            r = qrot(q, np.array([[1, 0, 0]], np.float32))
            for h in range(2):
                o = pos[a].copy()
                o[2] += 15.0 + (top[a] - 30.0) * h
                for x in range(32):
                    th = 0.75 * np.pi * x / 31 + 0.125 * np.pi
                    d = -np.cos(th) * r[0] + np.sin(th) * f[0]
                    d = d / np.linalg.norm(d)
                    out.append(np.concatenate([o, d]))
        for a in range(u, u + 4):
            q = rot[a:a + 1]
            f = qrot(q, np.array([[0, 1, 0]], np.float32))
            r = qrot(q, np.array([[1, 0, 0]], np.float32))
            for h in range(2):
                o = pos[a].copy()
                o[2] += 15.0 + (top[a] - 30.0) * h
                for x in range(8):
                    th = -np.pi * x / 7
                    d = -np.cos(th) * r[0] + np.sin(th) * f[0]
                    d = d / np.linalg.norm(d)
                    out.append(np.concatenate([o, d]))
    return np.asarray(out, np.float32)


if __name__ == "__main__":
    path = sys.argv[1]
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    steps = [int(s) for s in sys.argv[3:]] or [5]
    o = T.Oracle(W, 6)
    o.put_ctrl([0, 1, 1])
    o.init()
    allr = []
    for s in range(max(steps) + 1):
        if os.environ.get("DUMP_ACTIONS") == "combat":
            o.set_actions(T.seek_combat_actions(o, s))
        else:
            o.set_actions(T.mpenv_tape.tape_actions(1234, s, 0, W * 12))
        o.step()
        if s in steps:
            allr.append(rays_for(o.get("DEBUG_AGENT_F32"), o.get("DEBUG_AGENT_I32")))
    np.concatenate(allr).tofile(path)
    print(path, sum(len(r) for r in allr), "rays")
