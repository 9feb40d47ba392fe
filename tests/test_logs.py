"""Record / replay / event-log wire formats.

CPU: struct layouts against the reference's types.hpp definitions, and a
record -> replay round trip in the oracle (replaying a recorded match
reproduces its positions, aims, hp and lidar).  The GPU side
(tests/test_parity_gpu.py::test_logs_*) checks the engine's files byte for
byte against the oracle's buffers.
"""
import ctypes as C

import numpy as np
import pytest

import mpenv_testlib as T

# numpy views of the wire structs (include/mpenv.h)
AGENT_LOG = np.dtype([("position", "<f4", 3), ("aim_yaw", "<f4"), ("aim_pitch", "<f4"),
                      ("aim_rot", "<f4", 4), ("hp", "<f4"), ("mag", "<i4", 2), ("stand", "<i4", 3),
                      ("shot_agent_idx", "<i4"), ("fired_shot_t", "<f4"), ("was_killed", "u1"),
                      ("successful_kill", "u1"), ("pad", "u1", 2)])
STEP_LOG = np.dtype([("agents", AGENT_LOG, 12), ("cur_step", "<i4")])
GAME_EVENT = np.dtype([("type", "<u4"), ("pad", "<u4"), ("match_id", "<u8"), ("step", "<u4"),
                       ("a", "u1"), ("b", "u1"), ("c16", "<u2")])
PLAYER = np.dtype([("pos", "<i2", 3), ("yaw", "<i2"), ("pitch", "<i2"), ("mag", "u1"), ("reloading", "u1"),
                   ("hp", "u1"), ("flags", "u1")])
SNAPSHOT = np.dtype([("num_events", "<u4"), ("event_mask", "<u4"), ("match_id", "<u8"), ("step", "<u2"),
                     ("cur_zone", "u1"), ("controller", "i1"), ("zone_steps_remaining", "<u2"),
                     ("steps_until_point", "<u2"), ("players", PLAYER, 12)])


def test_wire_struct_sizes_match_reference_layouts():
    # types.hpp:574-589 (AgentLogData 72 B, StepLog 868 B), 729-760 (GameEvent
    # 24 B), 596-639 (PackedStepSnapshot 192 B)
    assert AGENT_LOG.itemsize == 72
    assert STEP_LOG.itemsize == 868
    assert GAME_EVENT.itemsize == 24
    assert PLAYER.itemsize == 14
    assert SNAPSHOT.itemsize == 192


def compact_events(ev_slots):
    """events.bin bytes for one step: per world, the non-empty slots in order
    (manager.cpp postStep)."""
    rows = ev_slots.reshape(-1, 6)
    keep = rows[:, 0] != 0
    return rows[keep].astype("<i4").tobytes()


def record_run(W, ts, steps, flags, ctrl, policy="combat"):
    o = T.Oracle(W, ts, sim_flags=flags)
    o.lib.oracle_set_log_modes(o.h, 1, 0, 1)
    o.put_ctrl(ctrl)
    o.init()
    logs, states, events, snaps = [], [], [], []
    for s in range(steps):
        acts = T.combat_actions(o, s) if policy == "combat" else T.mpenv_tape.tape_actions(1234, s, 0, W * 2 * ts)
        o.set_actions(acts)
        o.step()
        logs.append(o.get("RECORD_LOG").copy())
        states.append({n: o.get(n) for n in ("SELF_POSITION", "FWD_LIDAR", "HP", "MAGAZINE")})
        events.append(o.get("EVENT_LOG"))
        snaps.append((o.get("PACKED_STEP_SNAPSHOT"), o.get("SNAPSHOT_WRITTEN").ravel()))
    o.close()
    return logs, states, events, snaps


def test_oracle_record_replay_round_trip():
    W, ts, steps = 4, 3, 150
    logs, states, events, _ = record_run(W, ts, steps, 1, [0, 0, 0])
    assert sum(int((e[:, :, 0] != 0).sum()) for e in events) > 10
    r = T.Oracle(W, ts, sim_flags=1)
    r.lib.oracle_set_log_modes(r.h, 0, 1, 0)
    r.put_ctrl([0, 0, 0])
    r.init()
    for s in range(steps):
        r.view("REPLAY_LOG")[:] = logs[s]
        r.set_actions(np.zeros((W * 2 * ts, 6), np.int32))
        r.step()
        for n, v in states[s].items():
            np.testing.assert_array_equal(r.get(n), v, err_msg=f"{n} @ {s}")
    r.close()


def test_event_stream_contents():
    """Events carry the match id (world << 32 | episode), the pre-increment
    step and valid player ids; snapshots flag steps with events."""
    W, ts, steps = 3, 3, 200
    _, _, events, snaps = record_run(W, ts, steps, 1, [0, 1, 1])
    seen = 0
    for s in range(steps):
        ev = events[s].view(GAME_EVENT).reshape(W, 2 * 2 * ts + 1)
        sn = snaps[s][0].view(SNAPSHOT).reshape(W)
        written = snaps[s][1]
        for w in range(W):
            e = ev[w][ev[w]["type"] != 0]
            seen += len(e)
            assert np.all((e["match_id"] >> 32) == w)
            assert set(e["type"]) <= {1, 2, 4, 8}
            for x in e[e["type"] != 1]:
                assert x["a"] % 6 < ts and x["a"] // 6 < 2
            if written[w]:
                assert sn[w]["match_id"] >> 32 == w
                if len(e):
                    assert sn[w]["num_events"] == 1
                    assert sn[w]["event_mask"] & np.bitwise_or.reduce(e["type"]) == np.bitwise_or.reduce(e["type"])
    assert seen > 10
