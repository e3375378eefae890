"""III frame sharding on the CPU: partition properties, and a world_size-2
job (host group, no GPU) that codes its chunks, all-gathers the per-frame sizes and gathers
the code-streams on rank 0.  The per-frame codec here is a
stand-in that writes deterministic files -- the GPU codec itself is covered
by tests/test_codec_gpu.py; this checks the driver around it."""
import os

import numpy as np
import pytest

from vcf_amd.codec import shard


@pytest.mark.parametrize("n,p", [(20, 1), (20, 8), (7, 8), (256, 8), (1, 2), (64, 3)])
def test_frame_range_partitions(n, p):
    seen = []
    for r in range(p):
        lo, hi = shard.frame_range(n, r, p)
        assert 0 <= lo <= hi <= n
        seen += list(range(lo, hi))
        assert all(shard.owner(i, n, p) == r for i in range(lo, hi))
    assert seen == list(range(n))


class FakeCodec:
    """encode_fns/decode_fns with the transform codec's signature."""
    file_extension = ".tif"

    def encode_fns(self, pairs, batch=64):
        sizes = []
        for src, out in pairs:
            i = int(out[-4:])
            data = bytes([i % 251]) * (100 + 7 * i)
            with open(out + self.file_extension, "wb") as f:
                f.write(data)
            sizes.append(len(data))
        return sizes

    def decode_fns(self, pairs, batch=64):
        sizes = []
        for src, out in pairs:
            n = os.path.getsize(src + self.file_extension)
            with open(out, "wb") as f:
                f.write(b"x" * (n // 2))
            sizes.append(n // 2)
        return sizes


def _worker(rank, world, tmp, n):
    from vcf_amd.codec import parser as P
    from vcf_amd.codec.iii import CoDec
    g = shard.Group("host")
    args = P.parse(P.iii_parser(), ["encode", "-N", str(n), "-o", os.path.join(tmp, "orig_%04d.png")])
    c = CoDec(args, codec=FakeCodec(), group=g, encode_prefix=os.path.join(tmp, "enc"),
              decode_prefix=os.path.join(tmp, "dec"))
    total = c.encode()
    payloads = c.gather_codestreams()
    dargs = P.parse(P.iii_parser(), ["decode", "-N", str(n)])
    d = CoDec(dargs, codec=FakeCodec(), group=g, encode_prefix=os.path.join(tmp, "enc"),
              decode_prefix=os.path.join(tmp, "dec"))
    g.barrier()
    dtotal = d.decode()
    g.close()
    return (total, list(c.sizes), None if payloads is None else [len(p) for p in payloads],
            None if payloads is None else [p[:1] for p in payloads], dtotal)


def test_iii_two_ranks_host_group(tmp_path):
    from _dist import run_ranks
    n, world = 11, 2
    res = run_ranks(_worker, world, str(tmp_path), n)
    expect = [100 + 7 * i for i in range(n)]
    for rank in range(world):
        total, sizes, plens, heads, dtotal = res[rank]
        assert sizes == expect and total == sum(expect)
        assert dtotal == sum(e // 2 for e in expect)
    assert res[0][2] == expect and res[0][3] == [bytes([i % 251]) for i in range(n)]
    assert res[1][2] is None
    # every frame was written exactly once, by its owner
    for i in range(n):
        assert os.path.getsize(os.path.join(tmp_path, "enc_%04d.tif" % i)) == expect[i]
        assert os.path.exists(os.path.join(tmp_path, "dec_%04d.png" % i))


def _host_group_worker(rank, world):
    from vcf_amd.comm import HostGroup
    g = HostGroup()
    got = g.all_gather_bytes(bytes([rank]) * (rank + 1))
    mx = g.allreduce_max(rank * 1.5)
    sm = g.allreduce_sum(rank + 1)
    b = g.broadcast_bytes(b"root" if rank == 0 else None)
    g.barrier()
    g.close()
    return got, mx, sm, b


def test_host_group_collectives():
    from _dist import run_ranks
    res = run_ranks(_host_group_worker, 3)
    for r in range(3):
        got, mx, sm, b = res[r]
        assert got == [b"\x00", b"\x01\x01", b"\x02\x02\x02"]
        assert mx == 3.0 and sm == 6.0 and b == b"root"
