"""shard.Group's RCCL branch (vcf_amd/codec/shard.py) driven through a fake
communicator on the CPU: the per-rank counts and offsets it hands to the
all-gather and the gatherv, for P = 2, 3, 8 ranks and ragged chunks (ranks
with no frames included).  The real RCCL calls (vcf_comm_*) run only where
there are P GPUs -- one RCCL rank per device -- so this is the part of the
P-rank exchange a CPU can check: frame i on rank floor(i*P/N), every
frame's bytes at the right place on rank 0 (src/III.py:77-115, :132-144).
"""
import threading

import numpy as np
import pytest

from vcf_amd.codec import shard


class FakeComm:
    """The Communicator surface shard.Group uses, over threads: every rank
    deposits its operand, a barrier, every rank reads the result."""

    def __init__(self, world):
        self.world = world
        self.bar = threading.Barrier(world, timeout=30)
        self.slots = [None] * world
        self.calls = []

    def view(self, rank):
        return _RankView(self, rank)


class _RankView:
    def __init__(self, shared, rank):
        self.s, self.rank, self.world = shared, rank, shared.world

    def _exchange(self, item):
        self.s.slots[self.rank] = item
        self.s.bar.wait()
        got = list(self.s.slots)
        self.s.bar.wait()
        return got

    def all_gather_i64(self, values):
        a = np.ascontiguousarray(values, np.int64).ravel()
        rows = self._exchange(a.copy())
        assert len({r.size for r in rows}) == 1, "all-gather operands must have one length"
        return np.stack(rows)

    def gatherv(self, data, counts, root=0):
        counts = np.asarray(counts, np.int64)
        mine = np.frombuffer(bytes(data), np.uint8)
        assert mine.size == counts[self.rank], (self.rank, mine.size, counts)
        got = self._exchange((counts.copy(), mine.copy()))
        for c, _ in got:                      # every rank passed the same counts
            assert np.array_equal(c, counts)
        if self.rank != root:
            return None
        return np.concatenate([g[1] for g in got]) if counts.sum() else np.zeros(0, np.uint8)


def _group(comm, rank, world):
    g = object.__new__(shard.Group)
    g.rank, g.world, g.local = rank, world, rank
    g.host, g.comm, g.backend = None, comm, "rccl"
    return g


def _payload(i):
    rng = np.random.Generator(np.random.PCG64(i))
    return rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8).tobytes()


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("n_frames", [1, 5, 11, 256])
def test_rccl_branch_counts_and_offsets(world, n_frames):
    fake = FakeComm(world)
    results = [None] * world
    errors = []

    def rank_main(r):
        try:
            g = _group(fake.view(r), r, world)
            lo, hi = shard.frame_range(n_frames, r, world)
            assert all(shard.owner(i, n_frames, world) == r for i in range(lo, hi))
            mine = [_payload(i) for i in range(lo, hi)]
            sizes = g.all_gather_sizes(n_frames, [len(p) for p in mine])
            results[r] = (sizes, g.gather_payloads(n_frames, mine, sizes))
        except BaseException as e:   # surface the failing rank's error
            errors.append((r, e))
            fake.bar.abort()

    ts = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not errors, errors
    want = [_payload(i) for i in range(n_frames)]
    for r in range(world):
        sizes, got = results[r]
        assert list(sizes) == [len(p) for p in want]
        if r == 0:
            assert got == want
        else:
            assert got is None


def test_chunks_partition_the_frames():
    for world in (1, 2, 3, 7, 8):
        for n in (0, 1, 7, 8, 9, 256):
            seen = []
            for r in range(world):
                lo, hi = shard.frame_range(n, r, world)
                seen.extend(range(lo, hi))
            assert seen == list(range(n))


def test_gather_blobs_over_the_rccl_branch():
    world = 3
    fake = FakeComm(world)
    out = [None] * world

    def rank_main(r):
        out[r] = _group(fake.view(r), r, world).gather_blobs(bytes([r]) * (r + 1))

    ts = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert out[0] == [b"\x00", b"\x01\x01", b"\x02\x02\x02"] and out[1] is None and out[2] is None
