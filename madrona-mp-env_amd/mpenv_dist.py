"""World sharding across GPUs.

Worlds never interact, so a multi-GPU job is one process per GPU, each owning
a contiguous range of *global* world ids.  The manager is created with
`world_id_offset` = the first global id, which keys every per-world RNG
stream (sim.cpp:743-746 split_i(initKey, episodeIdx, worldID)), so the union
of the shards is bit-identical to one device running all worlds.  The step
itself needs no collective.  The learner exchange (config C4: every rank's
trainInterface outputs to one learner rank, RCCL over xGMI when the process
group is "nccl") is `LearnerGather`: one flat, preallocated, double-buffered
gather per step that overlaps the next step; `gather_to_learner` is the
simple blocking per-tensor form kept for small runs and tests.

Bytes per step into the learner (C4, 6v6 x 16,384 worlds per rank, the 21
trainInterface outputs of mgr.cpp:2383-2431): 3,924 B per agent of
observations + 8 B reward/done + 120 B per world of episode_results =
773.5 MB per rank, 7 x 773.5 MB = 5.4 GB arriving at the learner over its
7 xGMI links (~153 GB/s each, ~1.07 TB/s ingress): >= 5.1 ms per step, about
2.7x a 1.9 ms simulator step, so a single learner rank caps C4 at ~37% of
the simulators' throughput however well the transfer overlaps; the
learner-replica form (`all_gather`, each rank a learner over the whole
batch) has the same per-rank ingress.  Keeping observations where they are
produced (learner data parallelism: each rank trains on its own shard and
all-reduces gradients) moves only the gradients.
"""
from typing import Dict, List, Sequence, Tuple

# trainInterface outputs never written by the simulator:
# agent_map / unmasked_agent_map, 4 KB per agent each, constant zeros the
# learner already has, so no exchange ships them.
NOT_SHIPPED = ("agent_map", "unmasked_agent_map")


def flat_layout(sources) -> Tuple[list, int]:
    """Segments of one flat byte buffer holding every source tensor:
    [(name, byte offset, nbytes, dtype, shape)], 256-B aligned, and the
    total size.  The learner exchange ships (and the learner reads) this
    layout."""
    layout, off = [], 0
    for n, t in sources.items():
        nb = t.numel() * t.element_size()
        layout.append((n, off, nb, t.dtype, tuple(t.shape)))
        off += (nb + 255) // 256 * 256
    return layout, off


def pack_flat(layout, srcs, buf) -> None:
    """Copy each source into its segment of `buf` (uint8, on the current
    stream)."""
    import torch

    for (n, off, nb, dt, shape), t in zip(layout, srcs):
        buf[off:off + nb].copy_(t.view(-1).view(torch.uint8))


def unpack_flat(layout, recv) -> Dict[str, object]:
    """Zero-copy views {name: [ranks, rows, ...]} of a received
    [ranks, nbytes] buffer; flattening the first two axes gives global world
    order when rank r holds global worlds [r W, (r + 1) W)."""
    ws = recv.shape[0]
    return {n: recv[:, off:off + nb].view(dt).view((ws,) + shape) for n, off, nb, dt, shape in layout}


def shard_worlds(total_worlds: int, rank: int, world_size: int) -> Tuple[int, int]:
    """Contiguous split of [0, total_worlds): returns (world_id_offset, count).
    The first `total_worlds % world_size` ranks get one extra world."""
    if world_size <= 0 or not 0 <= rank < world_size:
        raise ValueError(f"bad rank {rank} / world_size {world_size}")
    base, extra = divmod(total_worlds, world_size)
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


def gather_to_learner(tensors: Sequence, dst: int = 0, group=None) -> List:
    """Gather per-rank step outputs (leading dim = this rank's agents or
    worlds) to `dst`, concatenated in global world order.  Equal shard sizes
    are required (the bench uses total_worlds divisible by world_size).
    Returns the concatenated tensors on `dst` and [] elsewhere."""
    import torch
    import torch.distributed as dist

    ws = dist.get_world_size(group)
    rank = dist.get_rank(group)
    out = []
    for t in tensors:
        t = t.contiguous()
        bufs = [torch.empty_like(t) for _ in range(ws)] if rank == dst else None
        dist.gather(t, bufs, dst=dst, group=group)
        if rank == dst:
            out.append(torch.cat(bufs, 0))
    return out


class LearnerGather:
    """Per-step learner exchange of trainInterface outputs, double-buffered.

    Each step, `submit()` copies this rank's outputs (on the current
    stream, after the step that produced them) into one flat byte buffer of
    a 2-slot ring -- on the learner, its own row of the receive buffer --
    and starts the slot's transfers to rank `dst` (one send per rank,
    batched point-to-point, so the learner does not copy its own segment
    again); they run on the process group's own stream, so they overlap the
    next step, and the engine's output buffers are free for that step as
    soon as the copy is done.  A slot is reused only after its
    previous gather completed (work.wait() orders the current stream after
    it).  Nothing is allocated or concatenated per step.

    On `dst`, `outputs(slot)` returns each output as a zero-copy view of the
    receive buffer with a leading rank axis: [world_size, rows, ...] -- rank
    r holds global worlds [r W, (r + 1) W) (shard_worlds), so flattening the
    first two axes is global world order.

    sources: {name: tensor} (contiguous; same shapes on every rank, checked
    at construction), e.g.
    SimManager.train_interface()["outputs"] as torch tensors, or
    `from_sim(sim)`.

    Construction is a collective call: every rank of `group` must construct
    its LearnerGather at the same point (the layout check is an
    all_gather_object over the group), and with an RCCL group each rank must
    have called torch.cuda.set_device first.
    """

    NOT_SHIPPED = NOT_SHIPPED
    mode = "gather"

    def __init__(self, sources, dst: int = 0, group=None, slots: int = 2, exclude=NOT_SHIPPED):
        import torch
        import torch.distributed as dist

        if hasattr(sources, "train_interface"):
            sources = self.from_sim(sources)
        sources = {n: t for n, t in sources.items() if n not in exclude}
        # the live engine buffers themselves: a .contiguous() copy would be a
        # snapshot that every later submit() ships unchanged
        for n, t in sources.items():
            if not t.is_contiguous():
                raise ValueError(f"LearnerGather source {n!r} is not contiguous")
        self.dist = dist
        self.group = group
        self.dst = dst
        self.rank = dist.get_rank(group)
        self.ws = dist.get_world_size(group)
        self.names = list(sources.keys())
        self.src = [sources[n] for n in self.names]
        dev = self.src[0].device
        self.layout, off = flat_layout(sources)  # (name, byte offset, nbytes, dtype, shape)
        self.nbytes = off
        # The receive buffers and outputs() views assume every rank ships the
        # same layout (equal shards): a gather of unequal buffers errors on
        # gloo and truncates or overruns silently on RCCL, so check up front.
        sig = [(n, nb, str(dt), shape) for n, _, nb, dt, shape in self.layout]
        sigs = [None] * self.ws
        dist.all_gather_object(sigs, sig, group=group)
        for r, other in enumerate(sigs):
            if other != sig:
                raise ValueError(f"LearnerGather: rank {r} ships a different layout than rank {self.rank} "
                                 "(unequal shards? total worlds must be divisible by the world size)")
        # the learner packs its own outputs straight into its row of the
        # receive buffer (no copy of its own segment); the others pack into a
        # flat send buffer
        self.recv = None
        self.flat = None
        if self.rank == dst:
            self.recv = [torch.empty((self.ws, off), dtype=torch.uint8, device=dev) for _ in range(slots)]
        else:
            self.flat = [torch.empty(off, dtype=torch.uint8, device=dev) for _ in range(slots)]
        self.slots = slots
        self.pending = [None] * slots
        self.k = 0
        self.last_slot = None

    @staticmethod
    def from_sim(sim) -> Dict[str, object]:
        """Every trainInterface output of a madrona_mp_env.SimManager
        (mgr.cpp:2383-2431) as torch tensors (zero-copy views)."""
        outs = sim.train_interface()["outputs"]
        return {n: t.to_torch() for n, t in outs.items()}

    def bytes_per_step(self) -> dict:
        """Bytes this rank sends and the learner receives per step."""
        return {"sent_per_rank": self.nbytes, "learner_ingress": self.nbytes * (self.ws - 1)}

    def _wait(self, slot):
        if self.pending[slot] is not None:
            for w in self.pending[slot]:
                w.wait()
            self.pending[slot] = None

    def submit(self, stream_ptr=None):
        """Pack this step's outputs into the next ring slot (on the current
        stream) and start the slot's point-to-point transfers: every other
        rank sends its buffer, the learner receives one row per peer (RCCL
        runs them on its own stream, overlapping the next step)."""
        dist = self.dist
        slot = self.k % self.slots
        self.k += 1
        self._wait(slot)
        if self.rank == self.dst:
            pack_flat(self.layout, self.src, self.recv[slot][self.rank])
            ops = [dist.P2POp(dist.irecv, self.recv[slot][r], dist.get_global_rank(self.group, r)
                              if self.group is not None else r, self.group)
                   for r in range(self.ws) if r != self.dst]
        else:
            pack_flat(self.layout, self.src, self.flat[slot])
            peer = dist.get_global_rank(self.group, self.dst) if self.group is not None else self.dst
            ops = [dist.P2POp(dist.isend, self.flat[slot], peer, self.group)]
        self.pending[slot] = dist.batch_isend_irecv(ops) if ops else None
        self.last_slot = slot
        return slot

    def drain(self):
        for i in range(self.slots):
            self._wait(i)

    def outputs(self, slot=None):
        """{name: [world_size, rows, ...] view} of a completed gather (dst only)."""
        if self.recv is None:
            return {}
        slot = self.last_slot if slot is None else slot
        self._wait(slot)
        return unpack_flat(self.layout, self.recv[slot])

    def close(self):
        self.drain()



class LearnerLocal:
    """Learner-local exchange (data-parallel learner): each rank's learner
    trains on the shard its simulator produced, so observations never leave
    the GPU that made them (`outputs()` are the engine's own zero-copy
    buffers, [1, rows, ...] like LearnerGather's on one rank); what crosses
    xGMI is the gradient all-reduce of the policy update.  Here that is a
    stand-in: every `update_every` steps (jax_train.py --steps-per-update,
    default 50) one asynchronous RCCL all-reduce of a `grad_bytes` f32
    buffer (the policy's parameter count x 4 B), overlapping the next steps;
    the learner's compute itself is out of scope."""

    NOT_SHIPPED = NOT_SHIPPED
    mode = "local"

    def __init__(self, sources, grad_bytes: int = 16 << 20, update_every: int = 50, group=None,
                 exclude=NOT_SHIPPED):
        import torch
        import torch.distributed as dist

        if hasattr(sources, "train_interface"):
            sources = LearnerGather.from_sim(sources)
        self.sources = {n: t for n, t in sources.items() if n not in exclude}
        self.dist = dist
        self.group = group
        self.ws = dist.get_world_size(group)
        self.update_every = max(1, int(update_every))
        dev = next(iter(self.sources.values())).device
        # zeros: a SUM all-reduce keeps them finite however many updates run
        self.grad = torch.zeros(max(1, grad_bytes // 4), dtype=torch.float32, device=dev)
        self.layout, self.nbytes = flat_layout(self.sources)
        self.pending = None
        self.k = 0
        self.updates = 0

    def bytes_per_step(self) -> dict:
        # ring all-reduce: each rank sends and receives 2 (ws - 1) / ws of the buffer
        ar = 2 * (self.ws - 1) * self.grad.numel() * 4 // self.ws
        return {"sent_per_rank": ar / self.update_every, "learner_ingress": ar / self.update_every}

    def submit(self, stream_ptr=None):
        self.k += 1
        if self.k % self.update_every:
            return None
        if self.pending is not None:
            self.pending.wait()
        self.pending = self.dist.all_reduce(self.grad, group=self.group, async_op=True)
        self.updates += 1
        return self.updates

    def drain(self):
        if self.pending is not None:
            self.pending.wait()
            self.pending = None

    def outputs(self, slot=None):
        return {n: t.unsqueeze(0) for n, t in self.sources.items()}

    def close(self):
        self.drain()


class LearnerWire:
    """Per-step learner exchange in the compact wire format (csrc/wire.hip,
    include/mpenv.h mpenv_wire_*): every rank packs one
    message of its step's outputs (~490 B per agent instead of the 3,924 B
    per agent LearnerGather ships) into a 2-slot ring on the step stream and
    sends it to the learner rank `dst`; the learner receives each peer's
    message into its slot and unpacks it into that peer's shadow manager (a
    SimManager of the same configuration and world range), whose own
    observation kernel rebuilds every trainInterface output bit for bit.
    The first message of each sender is a keyframe (it also carries the
    last-known rows).  Unpacking lags one step: `submit()` posts this step's
    transfers and unpacks the previous slot's messages, so the transfers
    overlap a whole step; `drain()` finishes both.

    `dedicated=True`: the learner rank simulates nothing (sim is None there);
    it only receives and unpacks the other ranks' messages, so the senders
    run at their own speed as long as the learner's unpacks keep up (C4 at 8
    GPUs: 7 simulators + one learner).  Otherwise the learner
    also simulates a shard (its own outputs are read directly).

    On `dst`, `outputs()` returns {name: [shards, rows, ...]}: the
    learner's own engine (not dedicated) and the shadows, in rank order
    (global world order, as LearnerGather), after `drain()`.

    pack(dst_ptr, keyframe, stream) / unpack(r, src_ptr, keyframe, stream) /
    nbytes(keyframe) / wire_error(r) default to the SimManager's wire_*
    methods and make_shadow(r) builds the shadow of rank r; the CPU tests
    substitute byte-level stand-ins.  Construction is a collective call (the
    message sizes are checked across the group); with RCCL, set the device
    first.

    One rank (world_size 1, bench.py --exchange wire at N = 1): loopback --
    the rank packs its own message and unpacks it into its own shadow each
    step, so the line carries the per-message pack and unpack cost a learner
    pays for each peer (nothing crosses xGMI).

    On a GPU the learner unpacks on streams of its own (`overlap`, on by
    default; `unpack_streams` of them, peers dealt round-robin, so
    several peers' unpacks fill the GPU together): the unpacks of one slot
    wait on GPU events for that slot's receives (loopback: its pack), the
    next receive / pack into the slot waits on the events its unpacks
    recorded, and nothing blocks the host -- the learner's own step (if any)
    and its peers' unpacks share the GPU.  `drain()` orders the caller's
    stream after every unpack.  submit() takes torch's current stream.

    A shadow that refused a message (wrong configuration or shard, wrong
    kind, values that did not fit the wire) is out of sync until a keyframe;
    `check()` raises then -- every `check_every` submits (default 64), and in
    outputs() and close().  Senders send a keyframe every `keyframe_every`
    messages (default 256; both sides derive the schedule from the message
    count, so no back channel is needed), so a shadow that refused a message
    recovers within that many steps instead of staying frozen.  On a GPU the
    periodic check reads every shadow's error word asynchronously (into
    pinned host memory, on the streams the unpacks run on, no device
    synchronisation) and raises at the next check on what the previous one
    fetched.
    """

    NOT_SHIPPED = NOT_SHIPPED
    mode = "wire"

    def __init__(self, sim, make_shadow=None, dst: int = 0, group=None, slots: int = 2, pack=None, unpack=None,
                 nbytes=None, device=None, overlap: bool = True, check_every: int = 64, wire_error=None,
                 dedicated: bool = False, unpack_streams: int = 1, keyframe_every: int = 256):
        import torch
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.dst = dst
        self.rank = dist.get_rank(group)
        self.ws = dist.get_world_size(group)
        self.sim = sim
        self.dedicated = bool(dedicated)
        if self.dedicated and self.ws < 2:
            raise ValueError("LearnerWire(dedicated=True) needs at least one sender rank")
        self.shadows = {}
        self.loopback = self.ws == 1
        if self.rank == dst and make_shadow is not None:
            self.shadows = {r: make_shadow(r) for r in range(self.ws) if r != dst or self.loopback}
        if self.rank == dst and self.dedicated:
            self.sim = None  # the learner simulates nothing
        sizer = sim if sim is not None else (next(iter(self.shadows.values())) if self.shadows else None)
        self._nbytes = nbytes or (lambda kf: sizer.wire_bytes(kf))
        self._pack = pack or (lambda ptr, kf, st: sim.wire_pack(ptr, kf, st))
        self._unpack = unpack or (lambda r, ptr, kf, st: self.shadows[r].wire_unpack(ptr, kf, st))
        self.nb, self.nk = int(self._nbytes(False)), int(self._nbytes(True))
        sizes = [None] * self.ws
        dist.all_gather_object(sizes, (self.nb, self.nk), group=group)
        if any(x != (self.nb, self.nk) for x in sizes):
            raise ValueError(f"LearnerWire: message sizes differ across ranks: {sizes}")
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.torch = torch
        self.gpu = dev.type == "cuda"
        self._wire_error = wire_error or (lambda r: self.shadows[r].wire_error())
        self.check_every = int(check_every)
        self.keyframe_every = max(0, int(keyframe_every))
        # asynchronous error reads (GPU shadows): pinned words + the events
        # that mark them written
        self._err_async = (wire_error is None and self.gpu and self.rank == dst and bool(self.shadows)
                           and all(hasattr(x, "wire_error_async") for x in self.shadows.values()))
        self._err_host = torch.zeros(self.ws, dtype=torch.int32, pin_memory=True) if self._err_async else None
        self._err_events = None
        self.slots = slots
        if self.rank == dst:
            self.bufs = [[torch.empty(self.nk, dtype=torch.uint8, device=dev) for _ in range(self.ws)]
                         for _ in range(slots)]
        else:
            self.bufs = [[torch.empty(self.nk, dtype=torch.uint8, device=dev)] for _ in range(slots)]
        self.pending = [None] * slots
        self.unpacked = [True] * slots
        self.keyframe = [True] * slots  # the kind of message in each slot
        self.k = 0
        # the learner's unpack streams and, per slot, the events their unpacks end with
        self.ustreams, self.udone = [], None
        if overlap and self.rank == dst and dev.type == "cuda":
            self.ustreams = [torch.cuda.Stream(device=dev) for _ in range(max(1, int(unpack_streams)))]
            self.udone = [[torch.cuda.Event() for _ in self.ustreams] for _ in range(slots)]

    @property
    def ustream(self):
        """The (first) unpack stream, None when unpacking on the caller's stream."""
        return self.ustreams[0] if self.ustreams else None

    def bytes_per_step(self) -> dict:
        return {"sent_per_rank": self.nb, "learner_ingress": self.nb * (self.ws - 1), "keyframe": self.nk}

    def _caller_stream(self, stream_ptr):
        cur = self.torch.cuda.current_stream()
        if stream_ptr and stream_ptr != cur.cuda_stream:
            raise ValueError("LearnerWire: submit() on a stream other than torch's current one")
        return cur

    def _unpack_stream(self, r):
        """The stream rank r's unpacks run on (None: the caller's)."""
        if not self.ustreams:
            return None
        ranks = [q for q in range(self.ws) if q != self.dst or self.loopback]
        return self.ustreams[ranks.index(r) % len(self.ustreams)]

    def _fetch_errors(self):
        """Queue every shadow's error-word read into pinned memory, ordered
        after its unpacks; events mark the words written."""
        cur = self.torch.cuda.current_stream()
        used = []
        for r in sorted(self.shadows):
            us = self._unpack_stream(r) or cur
            self.shadows[r].wire_error_async(self._err_host.data_ptr() + 4 * r, us.cuda_stream)
            if us not in used:
                used.append(us)
        self._err_events = []
        for us in used:
            ev = self.torch.cuda.Event()
            ev.record(us)
            self._err_events.append(ev)

    def _raise_if_bad(self, bad):
        if bad:
            raise RuntimeError(f"LearnerWire: shadow(s) refused wire messages {bad} (error bits: 1 refused, "
                               "2 out of sync until a keyframe); their outputs are stale")

    def check(self, block: bool = True):
        """Raise if any shadow refused a message (learner).  A refused message
        -- wrong configuration or shard, wrong kind, or values the pack
        flagged as not fitting the wire -- leaves that shadow's history
        (last-known rows, episode counters) behind the sender's until a
        keyframe; its outputs are not the sender's.  block=True reads the
        words now (after every queued unpack); block=False (the periodic
        check on a GPU) raises on the words the previous check fetched and
        queues the next read, without synchronising."""
        if self.rank != self.dst:
            return
        if self._err_async:
            if self._err_events is not None:
                for ev in self._err_events:
                    ev.synchronize()  # recorded a check_every ago: long done
                self._err_events = None
                words = self._err_host.tolist()
                self._raise_if_bad({r: words[r] for r in sorted(self.shadows) if words[r]})
            self._fetch_errors()
            if block:
                for ev in self._err_events:
                    ev.synchronize()
                self._err_events = None
                words = self._err_host.tolist()
                self._raise_if_bad({r: words[r] for r in sorted(self.shadows) if words[r]})
            return
        bad = {}
        for r in sorted(self.shadows):
            e = int(self._wire_error(r))
            if e:
                bad[r] = e
        self._raise_if_bad(bad)

    def is_keyframe(self, k: int) -> bool:
        """Whether message k (0-based, per sender) is a keyframe: the first,
        then every keyframe_every-th."""
        return k == 0 or (self.keyframe_every > 0 and k % self.keyframe_every == 0)

    def _unpack_slot(self, slot, ranks, stream_ptr):
        if not self.ustreams:
            for r in ranks:
                self._unpack(r, self.bufs[slot][r].data_ptr(), self.keyframe[slot], stream_ptr or 0)
            return
        for j, r in enumerate(ranks):
            us = self.ustreams[j % len(self.ustreams)]
            self._unpack(r, self.bufs[slot][r].data_ptr(), self.keyframe[slot], us.cuda_stream)
        for us, ev in zip(self.ustreams, self.udone[slot]):
            ev.record(us)

    def _peer(self, r):
        return self.dist.get_global_rank(self.group, r) if self.group is not None else r

    def _finish(self, slot, stream_ptr):
        """Wait for a slot's transfers and (learner) unpack its messages."""
        if self.pending[slot] is not None:
            if self.ustreams:
                # the unpack streams (not the caller's) wait for the receives
                for us in self.ustreams:
                    with self.torch.cuda.stream(us):
                        for w in self.pending[slot]:
                            w.wait()
            else:
                for w in self.pending[slot]:
                    w.wait()
            self.pending[slot] = None
        if self.rank == self.dst and not self.unpacked[slot]:
            self._unpack_slot(slot, [r for r in range(self.ws) if r != self.dst], stream_ptr)
            self.unpacked[slot] = True

    def submit(self, stream_ptr=None):
        dist = self.dist
        if self.loopback and not stream_ptr:
            # pack and unpack must share a stream: 0 would put each on its own
            # manager's internal stream, unordered against each other
            raise ValueError("LearnerWire loopback: submit() needs the step's stream (not 0)")
        if self.gpu and self.rank != self.dst:
            # a sender packs on torch's current stream, the one the RCCL send
            # below is ordered after (0 would be the manager's own stream: the
            # send could ship a half-written buffer, and the next pack into
            # the slot overwrite one still in flight)
            stream_ptr = self._caller_stream(stream_ptr).cuda_stream
        slot = self.k % self.slots
        kf = self.is_keyframe(self.k)
        self.k += 1
        self._finish(slot, stream_ptr)  # the slot's previous round is done before it is reused
        n = self.nk if kf else self.nb
        self.keyframe[slot] = kf
        if self.ustreams:
            # the slot's buffers are rewritten (pack / receive) only after its
            # previous unpacks have read them
            cur = self._caller_stream(stream_ptr)
            for ev in self.udone[slot]:
                cur.wait_event(ev)
        if self.loopback:
            self._pack(self.bufs[slot][0].data_ptr(), kf, stream_ptr or 0)
            for us in self.ustreams:
                us.wait_stream(self._caller_stream(stream_ptr))
            self._unpack_slot(slot, [0], stream_ptr)
            if self.check_every and self.k % self.check_every == 0:
                self.check(block=False)
            return slot
        if self.rank == self.dst:
            ops = [dist.P2POp(dist.irecv, self.bufs[slot][r][:n], self._peer(r), self.group)
                   for r in range(self.ws) if r != self.dst]
            self.unpacked[slot] = False
        else:
            self._pack(self.bufs[slot][0].data_ptr(), kf, stream_ptr or 0)
            ops = [dist.P2POp(dist.isend, self.bufs[slot][0][:n], self._peer(self.dst), self.group)]
        self.pending[slot] = dist.batch_isend_irecv(ops) if ops else None
        # the previous slot's messages have had a whole step to arrive
        prev = (slot - 1) % self.slots
        if self.slots > 1 and self.k > 1:
            self._finish(prev, stream_ptr)
        if self.check_every and self.k % self.check_every == 0:
            self.check(block=False)
        return slot

    def drain(self, stream_ptr=None):
        for i in range(self.slots):
            self._finish((self.k + i) % self.slots, stream_ptr)
        if self.ustreams:
            cur = self._caller_stream(stream_ptr)
            for us in self.ustreams:
                cur.wait_stream(us)

    def outputs(self):
        """{name: [shards, rows, ...]} on dst: own engine (unless dedicated)
        and shadows, in rank order."""
        import torch

        if self.rank != self.dst:
            return {}
        self.drain()
        self.check()
        if self.loopback:  # the shadow's rebuild of the rank's own outputs
            parts = [LearnerGather.from_sim(self.shadows[0])]
        else:
            parts = [LearnerGather.from_sim(self.sim) if r == self.dst else LearnerGather.from_sim(self.shadows[r])
                     for r in range(self.ws) if not (self.dedicated and r == self.dst)]
        return {n: torch.stack([p[n] for p in parts]) for n in parts[0] if n not in NOT_SHIPPED}

    def close(self):
        self.drain()
        self.check()


def make_exchange(mode: str, sim, group=None, **kw):
    """The learner exchange a multi-GPU run names in config.parallelism:
    "none" (simulators only), "gather" (LearnerGather: every shipped output
    to one learner rank each step, as exported), "wire" (LearnerWire: the
    same outputs in the compact wire format, rebuilt on the learner; needs
    make_shadow=) or "local" (LearnerLocal)."""
    if mode == "none":
        return None
    if mode == "gather":
        return LearnerGather(sim, dst=0, group=group)
    if mode == "wire":
        return LearnerWire(sim, dst=0, group=group, **kw)
    if mode == "local":
        return LearnerLocal(sim, group=group, **kw)
    raise ValueError(f"unknown exchange {mode!r}")
