"""Synthetic action tape for benchmarks and parity tests.

actions(step, agent) = counter hash h(seed, step, global agent id, field)
(Threefry-2x32-20, the same function as mp::tapeActions in
csrc/mpenv_core.h), so every rank / thread / shard sees the same actions for
the same global agent regardless of how worlds are partitioned:

  moveAmount U{0,1,2}, moveAngle U{0..7},
  fire 0 p=.45 / 1 p=.50 / 2 p=.05, stand 0 p=.90 / 1 p=.07 / 2 p=.03,
  aim yaw U{0..12}, aim pitch U{0..6}.
"""
import numpy as np

_M32 = np.uint64(0xFFFFFFFF)
_ROT = (13, 15, 26, 6, 17, 29, 16, 24)


def _rotl(x, r):
    return ((x << np.uint32(r)) | (x >> np.uint32(32 - r))).astype(np.uint32)


def threefry2x32(k0, k1, c0, c1):
    """Vectorised Threefry-2x32-20 (Random123).  All inputs uint32 arrays."""
    k0 = np.asarray(k0, dtype=np.uint32)
    k1 = np.asarray(k1, dtype=np.uint32)
    ks = [k0, k1, (np.uint32(0x1BD11BDA) ^ k0 ^ k1).astype(np.uint32)]
    with np.errstate(over="ignore"):
        x0 = (np.asarray(c0, dtype=np.uint32) + ks[0]).astype(np.uint32)
        x1 = (np.asarray(c1, dtype=np.uint32) + ks[1]).astype(np.uint32)
        for blk in range(5):
            for j in range(4):
                r = _ROT[(blk % 2) * 4 + j]
                x0 = (x0 + x1).astype(np.uint32)
                x1 = _rotl(x1, r)
                x1 = (x1 ^ x0).astype(np.uint32)
            s = blk + 1
            x0 = (x0 + ks[s % 3]).astype(np.uint32)
            x1 = (x1 + ks[(s + 1) % 3] + np.uint32(s)).astype(np.uint32)
    return x0, x1


def _mulhi(h, n):
    return ((h.astype(np.uint64) * np.uint64(n)) >> np.uint64(32)).astype(np.int32)


def tape_hash(seed, step, agents, field):
    agents = np.asarray(agents, dtype=np.uint32)
    k0 = np.full(agents.shape, seed, dtype=np.uint32)
    k1 = np.full(agents.shape, 0x5EED7A9E, dtype=np.uint32)
    c0 = np.full(agents.shape, step, dtype=np.uint32)
    with np.errstate(over="ignore"):
        c1 = (agents * np.uint32(8) + np.uint32(field)).astype(np.uint32)
    return threefry2x32(k0, k1, c0, c1)[0]


def tape_actions(seed, step, first_agent, num_agents):
    """Returns int32 [num_agents, 6]: 4 discrete + 2 discrete-aim actions."""
    agents = np.arange(first_agent, first_agent + num_agents, dtype=np.uint32)
    out = np.empty((num_agents, 6), dtype=np.int32)
    out[:, 0] = _mulhi(tape_hash(seed, step, agents, 0), 3)
    out[:, 1] = _mulhi(tape_hash(seed, step, agents, 1), 8)
    hf = tape_hash(seed, step, agents, 2)
    out[:, 2] = np.where(hf < np.uint32(1932735283), 0, np.where(hf < np.uint32(4080218931), 1, 2))
    hs = tape_hash(seed, step, agents, 3)
    out[:, 3] = np.where(hs < np.uint32(3865470566), 0, np.where(hs < np.uint32(4166118277), 1, 2))
    out[:, 4] = _mulhi(tape_hash(seed, step, agents, 4), 13)
    out[:, 5] = _mulhi(tape_hash(seed, step, agents, 5), 7)
    return out


def tape_ring(seed, first_agent, num_agents, ring_len):
    """[ring_len, num_agents, 6] int32: steps 0..ring_len-1 of the tape."""
    return np.stack([tape_actions(seed, s, first_agent, num_agents) for s in range(ring_len)])
