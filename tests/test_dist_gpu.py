"""The multi-rank drivers with the real GPU codec.

- RCCL through libvcf_amd.so's vcf_comm_* ABI, single rank (a 1-GPU box
  cannot hold two RCCL ranks: RCCL refuses two ranks on one device, so the
  P-rank exchange over xGMI runs only on the driver's 8-GPU node);
- III and IPP at world size 2, both ranks on this box's GPU running the real
  HIP codec, the exchange on the host group: decoded frames equal the
  oracle's, rank 0's gathered code-streams equal every frame's file;
- `bench.py --gpus 2` without a launcher (the parent spawns the ranks) and
  under `torch.distributed.run`, the driver's command for N > 1.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
from PIL import Image

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_rccl_single_rank_collectives():
    from vcf_amd.comm import HostGroup
    from vcf_amd.device import set_device
    from vcf_amd.rccl import MAX, SUM, Communicator
    set_device(0)
    c = Communicator(HostGroup(0, 1))
    v = np.arange(-3, 1000, 7, dtype=np.int64)
    assert np.array_equal(c.all_gather_i64(v), v[None])
    x = np.array([1.5, -2.0, 3e300])
    assert np.array_equal(c.allreduce_f64(x, MAX), x)
    assert np.array_equal(c.allreduce_f64(x, SUM), x)
    blob = np.random.default_rng(3).integers(0, 256, 1 << 20, dtype=np.uint8)
    got = c.gatherv(blob, [blob.size])
    assert np.array_equal(got, blob)
    assert c.gatherv(b"", [0]).size == 0
    with pytest.raises(ValueError):
        c.gatherv(b"abc", [2])
    c.close()


def _frames(n, H, W, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    return [rng.integers(0, 256, (H, W, 3), dtype=np.uint8) for _ in range(n)]


def _iii_worker(rank, world, tmp, n):
    from vcf_amd.codec import parser as P
    from vcf_amd.codec import shard
    from vcf_amd.codec.iii import CoDec
    from vcf_amd.device import set_device
    set_device(0)                           # both ranks share this box's one GPU
    g = shard.Group("host")
    args = P.parse(P.iii_parser(), ["encode", "-N", str(n), "-o", os.path.join(tmp, "original_%04d.png")])
    c = CoDec(args, group=g, encode_prefix=os.path.join(tmp, "enc"), decode_prefix=os.path.join(tmp, "dec"),
              batch=3)
    total = c.encode()
    payloads = c.gather_codestreams()
    g.barrier()
    d = CoDec(P.parse(P.iii_parser(), ["decode", "-N", str(n)]), group=g, encode_prefix=os.path.join(tmp, "enc"),
              decode_prefix=os.path.join(tmp, "dec"), batch=3)
    dtotal = d.decode()
    g.close()
    return total, list(map(int, c.sizes)), payloads, dtotal


def test_iii_two_ranks_real_codec(tmp_path):
    from _dist import run_ranks
    from oracle import oracle as O
    from vcf_amd.codec.tiff import imwrite_bytes
    n, H, W = 9, 40, 56
    frames = _frames(n, H, W, 21)
    for i, f in enumerate(frames):
        Image.fromarray(f).save(str(tmp_path / f"original_{i:04d}.png"))
    res = run_ranks(_iii_worker, 2, str(tmp_path), n)
    total, sizes, payloads, _ = res[0]
    assert res[1][2] is None and res[1][1] == sizes and res[1][0] == total
    for i, f in enumerate(frames):
        k = O.encode_frame(f, 32, 0)
        tif = open(str(tmp_path / f"enc_{i:04d}.tif"), "rb").read()
        assert tif == imwrite_bytes(k)
        assert payloads[i] == tif and sizes[i] == len(tif)
        got = np.asarray(Image.open(str(tmp_path / f"dec_{i:04d}.png")))
        assert np.array_equal(got, O.decode_frame(k, H, W, 32, 0)), f"frame {i}"


def _ipp_worker(rank, world, pat, prefix):
    from vcf_amd.codec import parser as P
    from vcf_amd.codec import shard
    from vcf_amd.codec.ipp import CoDec
    from vcf_amd.device import set_device
    set_device(0)
    g = shard.Group("host")
    c = CoDec(P.parse(P.ipp_parser(), ["encode", "-i", pat, "-O", prefix, "-N", "8", "-G", "3", "-M", "16",
                                       "-S", "8"]), group=g)
    total = c.encode()
    g.close()
    return total


def test_ipp_two_ranks_real_codec(tmp_path):
    from _dist import run_ranks
    from test_ipp_gpu import _ipp_loop, _moving, _write_seq
    from vcf_amd.codec import parser as P
    from vcf_amd.codec.ipp import CoDec
    frames = _moving(64, 96, 8, 5)
    pat = _write_seq(str(tmp_path), frames)
    res = run_ranks(_ipp_worker, 2, pat, str(tmp_path / "enc" / "v"))
    assert res[1] is None and res[0] > 0
    meta = json.load(open(str(tmp_path / "enc" / "v_meta.json")))
    assert len(meta["I_info"]) == 3 and len(meta["P_info"]) == 5
    dec = str(tmp_path / "dec" / "v")
    assert CoDec(P.parse(P.ipp_parser(), ["decode", "-i", str(tmp_path / "enc" / "v"), "-O", dec,
                                          "-M", "16"])).decode() == 8
    want, want_mv = _ipp_loop(frames, 3, 16, 8, False, 32)
    with np.load(str(tmp_path / "enc" / "v_mv.npz"), allow_pickle=False) as z:
        assert np.array_equal(z["mv_f32"], np.stack(want_mv))
    for i in range(8):
        got = np.asarray(Image.open(f"{dec}_{i:04d}.png").convert("RGB"))
        assert np.array_equal(got, want[i]), f"frame {i}"


def test_bench_two_ranks_without_launcher():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--frames", "4",
                        "--steps", "3", "--warmup", "1", "--settle-max-s", "0", "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 8 and line["value"] > 0
    _check_c4_blocks(line)


def test_bench_two_ranks_under_torchrun():
    """The driver's own N>1 command: torch.distributed.run starts the ranks (the launcher
    process never touches the GPU), bench.py takes RANK/WORLD_SIZE/MASTER_* from it and
    keeps its host group off torchrun's store port."""
    from vcf_amd.comm import free_port
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "VCF_STORE_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
                        os.path.join(ROOT, "bench.py"), "--gpus", "2", "--frames", "4", "--steps", "3",
                        "--warmup", "1", "--settle-max-s", "0", "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.strip().splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 8 and line["value"] > 0
    _check_c4_blocks(line)


def _check_c4_blocks(line):
    """At world 2 the C4 blocks either ran on two GPUs (times, every stage's
    maximum over ranks, every frame verified) or -- two ranks on this box's one
    GPU -- say explicitly that they were skipped; never an RCCL error string."""
    from vcf_amd.device import device_count
    for key in ("c4_e2e_with_gather", "c4_tiff_e2e_with_gather", "c5_e2e_with_gather"):
        b = line[key]
        assert "error" not in b, b
        if device_count() < 2:
            assert b["skipped"].startswith("ranks share a device"), b
        elif key.startswith("c4"):
            assert b["ms"] > 0 and b["verified"].startswith("ok"), b
            assert b["frames_per_rank"] == [128, 128] and set(b["stages_ms_max"]) == set(b["slowest_rank"])
        else:
            assert b["ms"] > 0 and b["stages_ms_max"], b


def test_device_iii_single_rank_rccl():
    """The C4 data path (vcf_amd/codec/iii_device.py) on one rank with a real
    single-rank RCCL communicator: every gathered container equals the frame
    coded on its own by the TCBAACP codec, and decodes to its indices."""
    from oracle import oracle as O
    from vcf_amd import tcbaac as T
    from vcf_amd.codec.iii_device import DeviceIII
    from vcf_amd.comm import HostGroup
    from vcf_amd.device import DeviceBuffer, set_device
    from vcf_amd.rccl import Communicator
    set_device(0)
    n, H, W = 7, 61, 77                      # n_sym % 4 != 0: unaligned frame starts too
    frames = _frames(n, H, W, 31)
    rgb = DeviceBuffer.from_array(np.stack(frames))
    comm = Communicator(HostGroup(0, 1), timeout_s=60)
    job = DeviceIII(comm, 0, 1, n, H, W, 32, seg_len=1024, streams=3)
    stages = {}
    sizes, got = job.run(rgb, stages)
    assert set(stages) == {"dct_dz", "entropy", "pack", "sizes_allgather", "gatherv", "d2h_rank0"}
    codec = T.TiledCBAACCodec(order=0, seg_len=1024, prior=True, nclass=T.PRIOR_CLASSES)   # DeviceIII default
    for i, f in enumerate(frames):
        k = O.encode_frame(f, 32, 0)
        want = codec.compress(k).getvalue()
        assert got[i] == want and sizes[i] == len(want), i
        assert np.array_equal(codec.decompress(bytes(got[i])), k), i
    # reusable: same bytes again.  run() returns memoryviews into one reused
    # page-locked buffer (valid until the next run), so copy before re-running
    first = [bytes(g) for g in got]
    sizes2, got2 = job.run(rgb)
    assert [bytes(g) for g in got2] == first and list(sizes2) == list(sizes)
    comm.close()


def test_bench_c4_block_small():
    """bench.py's C4 block at a small frame count: it runs, times, and rank 0's
    self-check passes."""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--frames", "2", "--steps", "2",
                        "--warmup", "1", "--settle-max-s", "0", "--no-cpu-baseline", "--c4-frames", "6"],
                       env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    for key in ("c4_e2e_with_gather", "c4_tiff_e2e_with_gather"):
        c4 = line[key]
        assert "error" not in c4 and c4["value"] > 0 and c4["verified"].startswith("ok"), c4
