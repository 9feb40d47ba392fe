"""The lidar's two device paths give the same bytes (DESIGN.md §4 k_lidar):
forward fans through per-wave candidate lists (k_lidar_fan + k_lidar_rear,
the default on scenes of <= 255 triangles) and every fan through the BVH
(k_lidar, MPENV_LIDAR_FAN=0 -- the path of larger scenes).  Both implement
the smallest-t closest-hit rule (§2 definition 12, pinned by
tests/test_lidar_order.py); the live and golden cases compare the default
path with the oracle, this test the other path with the default, on a
full-size batch in the combat regime (many agents, capsule hits, aim
pitch) and on the tape."""
import os
import time

import numpy as np
import pytest

import mpenv_testlib as T

pytestmark = pytest.mark.gpu

RING = 64
SEED = 1234


def _engine(W, ts, fan):
    old = os.environ.get("MPENV_LIDAR_FAN")
    os.environ["MPENV_LIDAR_FAN"] = "1" if fan else "0"
    try:
        e = T.Engine(W, ts)
    finally:
        if old is None:
            del os.environ["MPENV_LIDAR_FAN"]
        else:
            os.environ["MPENV_LIDAR_FAN"] = old
    e.put_ctrl([0, 1, 1])
    e.init()
    return e


@pytest.mark.parametrize("combat", [True, False], ids=["combat", "tape"])
def test_fan_lists_and_bvh_give_the_same_lidar(combat):
    ts, W, steps = 6, 8192, 120
    A = W * 2 * ts
    t0 = time.time()
    a, b = _engine(W, ts, True), _engine(W, ts, False)
    ring = a.mem.upload(T.mpenv_tape.tape_ring(SEED, 0, A, RING))
    for s in range(steps):
        for e in (a, b):
            if combat:
                e.combat_actions(ring + (s % RING) * A * 24, None, 1)
            else:
                e.copy_actions(ring + (s % RING) * A * 24)
            e.step()
        if s % 20 == 19 or s == steps - 1:
            a.mem.hip.hipDeviceSynchronize()
            for name in T.STEP_OUTPUTS:
                T.compare(a.get(name), b.get(name), f"{name} (fan lists vs BVH) @ step {s}")
            print(f"  step {s}: equal, {time.time() - t0:.0f} s", flush=True)
    fl = a.get("FWD_LIDAR").reshape(A, -1, 4)
    assert (fl[:, :, 3] > 0).any() or not combat  # opponents in the forward lidar under combat
    a.mem.free(ring)
