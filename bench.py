#!/usr/bin/env python3
"""Headline benchmark: Mpixels/s of the fused DCT(B=8)+deadzone encode at 4K.

BASELINE.json metric: "Mpixels/s encode (DCT+deadzone) at 4K; % HBM roofline;
1/2/4/8-GPU scaling".  One step = one launch of the encode kernel over a batch
of 4K RGB frames already resident in HBM (the hot path of src/2D-DCT.py
encode_fn :276-361 for every frame of the batch).  Frames shard across ranks
with no data-path collective (frames are independent units), so scaling is
weak: every rank encodes its own batch; value = all ranks' pixels / the
slowest rank's wall time.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Either launch works: without a launcher, `--gpus N` starts N rank processes
itself.  No PyTorch anywhere: device work goes through libvcf_amd.so's C ABI,
the barrier and the max over ranks through a small TCP group on the host
(vcf_amd/comm.py).

Rank 0 prints one JSON line.  The roofline block is measured live with HIP
events on the stream the kernel runs on; the cpu_baseline block times the
reference's CPU path restated in numpy (oracle/ref_numpy.py) on a bounded
sample of the same frames, beside the C port of the oracle.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)
ALG_BYTES_PER_PIXEL = 6  # 3 B RGB read + 3 B index write

# the configs' synthetic frames (shared with the tests and scripts)
from vcf_amd.synthetic import c4_frame, c5_frame, synth_frame  # noqa: E402,F401


def spawn_ranks(ngpus: int) -> int:
    """`python bench.py --gpus N` without a launcher: start N rank processes.

    This parent never touches the GPU (no HIP call, no library load): it
    only picks the rendezvous ports, starts one child per GPU with
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set -- the environment
    torch.distributed.run would give them -- forwards rank 0's JSON line and
    exits non-zero if any rank fails.
    """
    import subprocess
    from vcf_amd.comm import free_port
    env = dict(os.environ)
    env.update(WORLD_SIZE=str(ngpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()),
               VCF_STORE_PORT=str(free_port()))
    procs = []
    for r in range(ngpus):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=e,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out = procs[0].communicate()[0]
    rcs = [procs[0].returncode] + [p.wait() for p in procs[1:]]
    sys.stdout.write(out.decode())
    sys.stdout.flush()
    bad = [(r, rc) for r, rc in enumerate(rcs) if rc != 0]
    if bad:
        print(f"bench: rank(s) failed: {bad}", file=sys.stderr, flush=True)
        return 1
    return 0


def dist_setup(ngpus: int):
    """(world, rank, local_rank, host group); the group carries the barrier and
    the max/sum over ranks on the host (no data-path collective)."""
    from vcf_amd.comm import HostGroup, env_world
    rank, world, local = env_world()
    if world != ngpus:
        raise SystemExit(f"WORLD_SIZE={world} does not match --gpus {ngpus}")
    return world, rank, local, HostGroup(rank, world)


def settle(step, stream, Event, min_s: float, max_s: float, chunk: int = 16, tol: float = 0.02):
    """Keep launching until the launch time is stable (clock / power ramp).

    The per-launch trace (profiles/r01_encode4k_kernel_trace.csv) shows the
    first ~30 launches of a fresh run at 0.77-1.06 ms before the kernel
    settles near 0.71 ms: the board's power management, not the kernel.  So
    after the fixed --warmup steps the bench goes on warming up, in chunks of
    `chunk` launches timed with events, until at least `min_s` seconds have
    passed and the last four chunk averages agree within `tol` (or `max_s`).
    Returns (seconds, launches, last chunk's ms per launch)."""
    e0, e1 = Event(), Event()
    hist, n, t0 = [], 0, time.perf_counter()
    el = 0.0
    while max_s > 0:
        e0.record(stream)
        for _ in range(chunk):
            step()
        e1.record(stream)
        e1.synchronize()
        hist.append(e0.elapsed_ms(e1) / chunk)
        n += chunk
        el = time.perf_counter() - t0
        if el >= max_s:
            break
        if el >= min_s and len(hist) >= 4 and max(hist[-4:]) / min(hist[-4:]) - 1 < tol:
            break
    return el, n, (hist[-1] if hist else None)


def host_desc():
    model = platform.processor() or ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    return model, os.cpu_count(), avail


def cpu_baseline(frame: np.ndarray, Q: int, budget_s: float):
    """The reference's CPU path timed on this host (rank 0, N=1 only).

    Three legs, each on a bounded sample of the same 4K S-smooth frame:
    - `value` (kind "port" of the reference itself): oracle/ref_numpy.py's
      reference-faithful restatement of 2D-DCT.py encode_fn :276-361, the
      per-block scipy.fftpack loop of assumption A1, 1 core;
    - `vectorized`: the same arithmetic as one scipy.fft call per axis over
      the whole frame with workers = the cores this process may use;
    - `c_port`: the C restatement (oracle/vcf_oracle.c), 1 thread.
    All three must return the same indices (checked against each other).
    """
    from oracle import oracle as O       # test infrastructure: the checker, timed as the CPU baseline
    from oracle import ref_numpy as R
    model, ncpu, avail = host_desc()
    # the box's CPU share: OMP_NUM_THREADS is set to it there (os.cpu_count()
    # shows the whole machine)
    avail = min(avail, int(os.environ.get("OMP_NUM_THREADS", avail) or avail))
    H, W = frame.shape[:2]
    res = {}

    # (i) reference-faithful: the per-block loop over successive 64-row strips
    # of the frame (blocks are independent, so a strip costs its share of the
    # frame) until ~45 % of the budget is spent
    rows, t0 = 0, time.perf_counter()
    while True:
        R.encode_frame_loop(np.ascontiguousarray(frame[rows % H:rows % H + 64]), Q)
        rows += 64
        el_loop = time.perf_counter() - t0
        if el_loop >= budget_s * 0.45 or rows >= 4 * H:
            break
    res["loop"] = (rows * W / el_loop / 1e6, el_loop, rows)

    # (ii) vectorised scipy.fft, all available cores
    n, t0 = 0, time.perf_counter()
    while True:
        k_vec = R.encode_frame(frame, Q, workers=avail)
        n += 1
        el_vec = time.perf_counter() - t0
        if el_vec >= budget_s * 0.3 or n >= 32:
            break
    res["vec"] = (n * H * W / el_vec / 1e6, el_vec, n)

    # (iii) the C port, 1 thread
    O.lib()
    n, t0 = 0, time.perf_counter()
    while True:
        k_c = O.encode_frame(frame, Q)
        n += 1
        el_c = time.perf_counter() - t0
        if el_c >= budget_s * 0.25 or n >= 64:
            break
    res["c"] = (n * H * W / el_c / 1e6, el_c, n)

    strip = np.ascontiguousarray(frame[:64])
    agree = bool(np.array_equal(k_vec, k_c) and np.array_equal(R.encode_frame_loop(strip, Q),
                                                                R.encode_frame(strip, Q)))
    host = f"{model}; os.cpu_count()={ncpu}, usable={avail}"
    out = dict(
        value=round(res["loop"][0], 3), unit="Mpixels/s", cores=1, kind="port",
        sample=(f"{rows // 64} strips of 64x3840 px from a 2160x3840 S-smooth frame ({rows * W / 1e6:.2f} Mpix), "
                f"oracle/ref_numpy.py encode_frame_loop: 2D-DCT.py encode_fn restated with the per-block "
                f"scipy.fftpack dct loop (A1), 1 core, {res['loop'][1]:.1f} s"),
        host=host,
        vectorized={"value": round(res["vec"][0], 2), "unit": "Mpixels/s", "cores": avail,
                    "sample": f"{res['vec'][2]} x 2160x3840 frame(s), scipy.fft over the whole frame, "
                              f"workers={avail}, {res['vec'][1]:.1f} s"},
        c_port={"value": round(res["c"][0], 2), "unit": "Mpixels/s", "cores": 1,
                "sample": f"{res['c'][2]} x 2160x3840 frame(s), oracle/vcf_oracle.c (gcc -O2, "
                          f"-ffp-contract=off), 1 thread, {res['c'][1]:.1f} s"},
        legs_agree=agree,
    )
    return out, k_c


def _run_serial(fn, *a):
    """fn(*a) on a worker thread: the host TIFF writer deflates a frame's strips
    serially there (on the main thread it fans them out over a pool), so a
    1-core leg really uses one core."""
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(1) as ex:
        return ex.submit(fn, *a).result()


def c4_cpu_baseline(budget_s: float, Q: int, files=None) -> dict:
    """C4's reference path on host cores (checker leg, rank 0, N = 1): per frame
    of the C4 sequence the oracle's C DCT + deadzone (oracle/vcf_oracle.c,
    2D-DCT.py:276-361 restated) and the host TIFF writer (system zlib level 6,
    TIFF.py:23-31), as III.py:77-115 runs 2D-DCT encode_fn per frame -- on 1
    core, then with frames on a 16-thread pool; each leg stops after about half
    the budget.  The first frames' files are compared with the GPU block's."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle as O
    from vcf_amd.codec.tiff import imwrite_bytes
    H, W = 1080, 1920
    bases = [synth_frame(H, W, seed=100 + s) for s in range(4)]
    code = lambda i: imwrite_bytes(O.encode_frame(c4_frame(bases, i), Q))   # noqa: E731
    model, ncpu, avail = host_desc()
    threads = min(16, avail, int(os.environ.get("OMP_NUM_THREADS", avail) or avail))

    def one_core():
        out, t0 = {}, time.perf_counter()
        i = 0
        while True:
            out[i] = code(i)
            i += 1
            if time.perf_counter() - t0 >= budget_s / 2 or i >= 256:
                return out, time.perf_counter() - t0
    got1, el1 = _run_serial(one_core)
    n_par = max(threads, min(256, int(round(len(got1) * threads * 0.8))))
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(code, range(n_par)))
    elp = time.perf_counter() - t0
    agree = None if not files else all(got1[i] == f for i, f in files.items() if i in got1)
    return {"value": round(len(got1) * H * W / el1 / 1e6, 3), "unit": "Mpixels/s", "cores": 1, "kind": "port",
            "sample": (f"frames 0..{len(got1) - 1} of the C4 sequence (1080p): oracle/vcf_oracle.c DCT+deadzone "
                       f"then the host TIFF writer (system zlib level 6), one frame after the other on 1 core, "
                       f"{el1:.1f} s"),
            "threads": {"value": round(n_par * H * W / elp / 1e6, 2), "unit": "Mpixels/s", "cores": threads,
                        "sample": f"{n_par} frames of the sequence on a {threads}-thread pool, {elp:.1f} s"},
            "host": f"{model}; {threads} threads used (os.cpu_count()={ncpu})",
            "files_equal_gpu": agree}


def c5_cpu_baseline(budget_s: float, Q: int, base, H: int, W: int, G: int, files=None) -> dict:
    """C5's reference path on host cores (checker leg, rank 0, N = 1): the IPP
    GOP loop (IPP_DCT.py:397-575) restated by the C oracle -- I-frame DCT +
    deadzone and its decode; per P-frame the full search (bs 16, S 8) against
    the previous reconstruction, compensation, residual + 128, DCT + deadzone,
    decode and reconstruction -- with every frame's indices written by the host
    TIFF writer (system zlib level 6).  1 core: GOP 0 from its first frame
    until half the budget is spent; then the first frames of every GOP on a
    thread pool (GOPs are independent).  Files compared with the GPU block's."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle as O
    from vcf_amd.codec.tiff import imwrite_bytes

    def gop(g: int, n: int, deadline=None):
        out, ref = {}, None
        for j in range(n):
            i = g * G + j
            cur = c5_frame(base, i, H, W)
            if ref is None:
                k = O.encode_frame(cur, Q)
                ref = O.decode_frame(k, H, W, Q)
            else:
                comp = O.ipp_motion_compensate(ref, O.ipp_block_matching(ref, cur, 16, 8, False), 16)
                k = O.encode_frame(O.ipp_residual(cur, comp), Q)
                ref = O.ipp_reconstruct(comp, O.decode_frame(k, H, W, Q))
            out[i] = imwrite_bytes(k)
            if deadline is not None and time.perf_counter() >= deadline:
                break
        return out
    model, ncpu, avail = host_desc()
    threads = min(16, avail, int(os.environ.get("OMP_NUM_THREADS", avail) or avail))
    t0 = time.perf_counter()
    got1 = _run_serial(gop, 0, G, t0 + budget_s / 2)
    el1 = time.perf_counter() - t0
    n_gops = max(1, (64 + G - 1) // G)
    per = 2
    t0 = time.perf_counter()
    with ThreadPoolExecutor(min(threads, n_gops)) as ex:
        outs = list(ex.map(lambda g: gop(g, per), range(n_gops)))
    elp = time.perf_counter() - t0
    n_par = sum(len(o) for o in outs)
    agree = None if not files else all(got1[i] == f for i, f in files.items() if i in got1)
    return {"value": round(len(got1) * H * W / el1 / 1e6, 3), "unit": "Mpixels/s", "cores": 1, "kind": "port",
            "sample": (f"frames 0..{len(got1) - 1} of GOP 0 (4K; I then P frames): the C oracle's IPP GOP loop "
                       f"(full search bs 16 / S 8, compensation, residual, DCT+deadzone, decode, reconstruction) "
                       f"and the host TIFF writer (system zlib level 6), 1 core, {el1:.1f} s"),
            "threads": {"value": round(n_par * H * W / elp / 1e6, 2), "unit": "Mpixels/s",
                        "cores": min(threads, n_gops),
                        "sample": (f"the first {per} frames of each of the {n_gops} GOPs, one GOP per thread "
                                   f"(GOPs are independent; frames in a GOP are serial), {elp:.1f} s")},
            "host": f"{model}; {min(threads, n_gops)} threads used (os.cpu_count()={ncpu})",
            "files_equal_gpu": agree}


C4_STAGES = ("dct_dz", "entropy", "pack", "sizes_allgather", "gatherv", "d2h_rank0")


def c4_stage_table(rows, frames_per_rank) -> dict:
    """Per-stage seconds of every rank (rows[s][r], NaN where a rank has no
    figure) -> the C4 block's stage report: the maximum over ranks (which rank
    bounds each stage), rank 0's own figures and the frames each rank coded."""
    out = {"frames_per_rank": [int(f) for f in frames_per_rank], "stages_ms_max": {}, "slowest_rank": {},
           "stages_ms_rank0": {}}
    for name, row in zip(C4_STAGES, rows):
        r = np.asarray(row, np.float64)
        if r.size == 0 or not np.isfinite(r).any():
            continue
        j = int(np.nanargmax(r))
        out["stages_ms_max"][name] = round(float(r[j]) * 1e3, 3)
        out["slowest_rank"][name] = j
        if np.isfinite(r[0]):
            out["stages_ms_rank0"][name] = round(float(r[0]) * 1e3, 3)
    return out


def c4_block(args, world: int, rank: int, group, entropy: str = "TCBAACP"):
    """Config C4 of BASELINE.json: III over a 256-frame 1080p sequence,
    frame-sharded across the ranks, end to end on the GPU with the exchange
    (vcf_amd/codec/iii_device.py): DCT+deadzone, the GPU entropy stage
    (-c TCBAACP, or with entropy="TIFF" the reference's default -c TIFF: every
    strip deflated on the GPU exactly as zlib), per-frame sizes all-gathered and the code-streams gathered
    to rank 0 over RCCL (device to device).  Timed like the headline:
    barrier + device sync on both sides, max over ranks.  Rank 0 checks what
    it gathered: every frame's container equals that frame coded on its own
    (TiledCBAACCodec.compress_device of the DCT indices) -- all frames when
    P > 1 (rank 0 re-codes the other ranks' frames), and at P = 1 the
    gathered bytes equal the coder's own output, and two frames decode back
    to their indices.  Returns (block dict, error or None); never raises."""
    from vcf_amd import tcbaac as T
    from vcf_amd.codec.iii_device import DeviceIII
    from vcf_amd.codec.shard import frame_range
    from vcf_amd.comm import HostGroup
    from vcf_amd.device import DeviceBuffer, synchronize
    from vcf_amd.rccl import Communicator
    N, H, W, Q = args.c4_frames, 1080, 1920, args.QSS
    lo, hi = frame_range(N, rank, world)
    ent = (f"-c TCBAACP, {T.CLASS_SEG}-symbol segments, {T.PRIOR_CLASSES} prior classes" if entropy == "TCBAACP"
           else "-c TIFF, the reference's default: every ~64 KB strip deflated on the GPU byte-exact with zlib level 6")
    info = {"workload": (f"III C4: {N} x 1080p frames, DCT+deadzone Q={Q} + GPU entropy ({ent}), frame i on rank "
                         f"floor(i*P/N), sizes all-gather + "
                         f"code-stream gatherv to rank 0 over RCCL (device to device), rank 0 copies them to host"),
            "frames": N, "frame": [H, W, 3], "n_ranks": world, "frames_this_rank0": hi - lo if rank == 0 else None}
    from vcf_amd.device import device_count
    if world > 1 and device_count() < world:
        # every rank sees the same device count, so every rank returns here (no collective is left half-done)
        info["skipped"] = (f"ranks share a device ({world} ranks on {device_count()} GPU(s)): RCCL refuses two "
                           "ranks on one GPU, so the C4 exchange runs only with one GPU per rank")
        return info
    err, comm, t_rank = None, None, float("nan")
    stages = {}
    try:
        bases = [synth_frame(H, W, seed=100 + s) for s in range(4)]
        rgb = DeviceBuffer(max((hi - lo) * H * W * 3, 1))
        for j, i in enumerate(range(lo, hi)):
            rgb.upload(c4_frame(bases, i), offset=j * H * W * 3)
        comm = Communicator(group if world > 1 else HostGroup(0, 1), timeout_s=args.c4_timeout)
        info["backend"] = "rccl" if world > 1 else "rccl (single rank: the root's device copy)"
        job = DeviceIII(comm, rank, world, N, H, W, Q, entropy=entropy)
        for _ in range(args.c4_warmup):
            job.run(rgb)
        group.barrier()
        synchronize()
        t0 = time.perf_counter()
        for _ in range(args.c4_steps):
            sizes, got = job.run(rgb)
        synchronize()
        t_rank = (time.perf_counter() - t0) / args.c4_steps
        job.run(rgb, stages)
        if rank == 0:
            info["code_bytes"] = int(sizes.sum())
            info["bits_per_symbol"] = round(8 * int(sizes.sum()) / (N * job.n_sym), 5)
            info["verified"] = c4_verify(got, bases, job, N, H, W, Q, world, entropy)
            if entropy == "TIFF":   # for the checker leg's CPU baseline: its files against these
                info["_files"] = {i: bytes(got[i]) for i in range(min(N, 4))}
    except Exception as e:   # reported in the block; the headline line still prints
        err = f"{type(e).__name__}: {e}"
    finally:
        if comm is not None:
            try:
                comm.close()
            except Exception:
                pass
    times = group.all_gather_f64(t_rank) if world > 1 else [t_rank]
    # each stage's maximum over ranks (a synchronised run per rank after the timed steps)
    vals = [stages.get(k, float("nan")) for k in C4_STAGES]
    rows = [group.all_gather_f64(v) for v in vals] if world > 1 else [[v] for v in vals]
    info.update(c4_stage_table(rows, [frame_range(N, r, world)[1] - frame_range(N, r, world)[0]
                                      for r in range(world)]))
    if err is None and all(np.isfinite(times)):
        tmax = max(times)
        info.update(ms=round(tmax * 1e3, 3), steps=args.c4_steps, warmup=args.c4_warmup,
                    value=round(N * H * W / tmax / 1e6, 1), unit="Mpixels/s",
                    frames_per_s=round(N / tmax, 1))
    else:
        info["error"] = err or "another rank failed"
    return info


def c4_verify(got, bases, job, N, H, W, Q, world, entropy="TCBAACP") -> str:
    """Rank 0: the gathered containers against per-frame coding on this GPU
    (TIFF: against the host TIFF writer, system zlib, of the frame's indices)."""
    from vcf_amd import dct as D
    from vcf_amd import tcbaac as T
    from vcf_amd.device import DeviceBuffer
    if entropy == "TIFF":
        from vcf_amd.codec.tiff import imread_bytes, imwrite_bytes
        frames = range(N) if world > 1 else sorted({0, N // 2, N - 1})
        for i in frames:
            k = D.encode(c4_frame(bases, i), Q)
            if got[i] != imwrite_bytes(k):
                return f"MISMATCH at frame {i}"
            if i in (0, N - 1) and not np.array_equal(imread_bytes(bytes(got[i])), k):
                return f"decode MISMATCH at frame {i}"
        what = "every frame" if world > 1 else f"frames {list(frames)}"
        return (f"ok: {what} equal to the host TIFF writer's file (system zlib) of the frame's indices; "
                f"frames 0 and {N - 1} read back to them")
    codec = T.TiledCBAACCodec(order=0, seg_len=T.CLASS_SEG, prior=True, nclass=T.PRIOR_CLASSES)
    frames = range(N) if world > 1 else sorted({0, N // 2, N - 1})
    Hp, Wp = D.padded_shape(H, W)
    for i in frames:
        rgb = c4_frame(bases, i)
        din = DeviceBuffer.from_array(rgb)
        k = DeviceBuffer(Hp * Wp * 3)
        D.encode_device(din, 1, H, W, Q, 0, out=k, stream=codec.coder.stream)
        want = codec.compress_device(k, (Hp, Wp, 3)).getvalue()
        if got[i] != want:
            return f"MISMATCH at frame {i}"
        if i in (0, N - 1):
            kh = np.empty((Hp, Wp, 3), np.uint8)
            k.download(kh)
            if not np.array_equal(codec.decompress(bytes(got[i])), kh):
                return f"decode MISMATCH at frame {i}"
    what = "every frame" if world > 1 else f"frames {list(frames)}"
    return f"ok: {what} equal to the frame coded alone; frames 0 and {N - 1} decode to their indices"


def c5_block(args, world: int, rank: int, group):
    """Config C5 of BASELINE.json: IPP_DCT over a 64-frame 4K sequence, GOP 10,
    full search bs 16 / S 8, 2D-DCT + deadzone + the default -c TIFF, GOPs
    sharded across the ranks, end to end on the GPU
    (vcf_amd/codec/ipp_device.py: the rank's GOPs in lock step, batched DCT,
    GPU TIFF deflate and DCT decode per step, files gathered to rank 0 over
    RCCL).  Timed like the headline (barrier + device sync, max over ranks).
    Returns the block dict; never raises."""
    from vcf_amd.codec.ipp_device import DeviceIPP
    from vcf_amd.comm import HostGroup
    from vcf_amd.device import DeviceBuffer, device_count, synchronize
    from vcf_amd.rccl import Communicator
    N, H, W, Q, G = args.c5_frames, 2160, 3840, args.QSS, 10
    info = {"workload": (f"IPP_DCT C5: {N} x 4K frames (panning S-smooth), GOP {G}, full search bs 16 / S 8, "
                         f"residual 2D-DCT + deadzone Q={Q} + -c TIFF (GPU deflate, zlib level 6), GOP g on rank "
                         "floor(g*P/G), the rank's GOPs in lock step, files gathered to rank 0 over RCCL"),
            "frames": N, "frame": [H, W, 3], "gop": G, "n_ranks": world}
    if world > 1 and device_count() < world:
        info["skipped"] = (f"ranks share a device ({world} ranks on {device_count()} GPU(s)): RCCL refuses two "
                           "ranks on one GPU, so the C5 exchange runs only with one GPU per rank")
        return info
    err, comm, t_rank, stages, job = None, None, float("nan"), {}, None
    try:
        base = synth_frame(H + 48, W + 64, seed=500)
        comm = Communicator(group if world > 1 else HostGroup(0, 1), timeout_s=args.c4_timeout)
        job = DeviceIPP(comm, rank, world, N, H, W, Q, G, 16, 8, False)
        rgb = DeviceBuffer(max(job.n_local * H * W * 3, 1))
        for j, i in enumerate(range(job.lo, job.hi)):
            rgb.upload(c5_frame(base, i, H, W), offset=j * H * W * 3)
        for _ in range(args.c5_warmup):
            job.run(rgb)
        group.barrier()
        synchronize()
        t0 = time.perf_counter()
        for _ in range(args.c5_steps):
            sizes, got, mvs = job.run(rgb)
        synchronize()
        t_rank = (time.perf_counter() - t0) / args.c5_steps
        job.run(rgb, stages)
        info["frames_this_rank0"] = job.n_local if rank == 0 else None
        if rank == 0:
            info["code_bytes"] = int(sizes.sum())
            info["bits_per_pixel"] = round(8 * int(sizes.sum()) / (N * H * W), 5)
            info["_check"] = (got, mvs, base)   # verified after the timed regions (rank 0, N = 1)
    except Exception as e:   # reported in the block; the headline line still prints
        err = f"{type(e).__name__}: {e}"
    finally:
        if comm is not None:
            try:
                comm.close()
            except Exception:
                pass
    times = group.all_gather_f64(t_rank) if world > 1 else [t_rank]
    keys = ("gop_loop", "sizes_d2h", "pack", "sizes_allgather", "gatherv", "d2h_rank0")
    rows = [group.all_gather_f64(stages.get(k, float("nan"))) if world > 1 else [stages.get(k, float("nan"))]
            for k in keys]
    info["stages_ms_max"] = {k: round(float(np.nanmax(r)) * 1e3, 3) for k, r in zip(keys, rows)
                             if np.isfinite(r).any()}
    if err is None and all(np.isfinite(times)):
        tmax = max(times)
        info.update(ms=round(tmax * 1e3, 3), steps=args.c5_steps, warmup=args.c5_warmup,
                    value=round(N * H * W / tmax / 1e6, 1), unit="Mpixels/s", frames_per_s=round(N / tmax, 1))
    else:
        info["error"] = err or "another rank failed"
    return info


def c5_check(info, Q: int, budget_s: float = 0.0) -> None:
    """The checker leg (rank 0, N = 1, beside cpu_baseline): frames 0 and 1 of the
    C5 block's first GOP against the reference's GOP loop restated by the C oracle
    (IPP_DCT.py:397-575: the I-frame's indices; the P-frame's full-search motion
    field, compensation, residual and indices), files compared byte for byte with
    the host TIFF writer's.  Replaces the block's private _check entry."""
    chk = info.pop("_check", None) if info else None
    if chk is None:
        return
    from oracle import oracle as O
    from vcf_amd.codec.tiff import imwrite_bytes
    got, mvs, base = chk
    H, W = info["frame"][:2]
    f0, f1 = c5_frame(base, 0, H, W), c5_frame(base, 1, H, W)
    k0 = O.encode_frame(f0, Q)
    ref = O.decode_frame(k0, H, W, Q)
    mv = O.ipp_block_matching(ref, f1, 16, 8, False)
    k1 = O.encode_frame(O.ipp_residual(f1, O.ipp_motion_compensate(ref, mv, 16)), Q)
    w0, w1 = imwrite_bytes(k0), imwrite_bytes(k1)
    parts = {"file0": bytes(got[0]) == w0, "file1": bytes(got[1]) == w1,
             "motion1": np.array_equal(np.asarray(mvs[0]), np.asarray(mv))}
    ok = all(parts.values())
    info["verified"] = ("ok: frames 0 (I) and 1 (P) equal the host TIFF writer's files of the reference GOP "
                        "loop's indices (C oracle), frame 1's motion field equal" if ok else
                        "MISMATCH: " + ", ".join(f"{k} {'ok' if v else 'differs'}" for k, v in parts.items()) +
                        f" (file sizes {len(got[0])}/{len(w0)}, {len(got[1])}/{len(w1)})")
    if budget_s > 0:
        info["cpu_baseline"] = c5_cpu_baseline(budget_s, Q, base, H, W, info.get("gop", 10),
                                               {i: bytes(got[i]) for i in range(min(len(got), 4))})


# config C3 (BASELINE.json configs[2]): 2D-DWT l=5 CDF-9/7 (pywt's bior4.4) + deadzone at 4K
C3_FRAMES, C3_LEVELS, C3_WAVELET = 8, 5, "bior4.4"
# bior4.4's nonzero taps: decomposition low/high 9 / 7 of 10, reconstruction 7 / 9 of 10
# (pywt 1.1.1's filter bank, vcf_amd/csrc/vcf_wavelets.h; zero taps are skipped bit-exactly,
# DESIGN.md §4.5)
C3_TAPS_NZ = (9, 7)
FP64_ISSUE_TOPS = 34.0   # measured fp64 VALU lane-ops/s of gfx950 (scripts/micro/f64_rate.hip)


def c3_fp64_ops_per_pixel(levels: int = C3_LEVELS, taps=C3_TAPS_NZ) -> float:
    """Float64 multiplies + adds per RGB pixel of the C3 encode (the decode is
    the same count with the reconstruction filters): per level and channel
    each of the two separable passes makes one low and one high output per
    input pair, with nz multiplies and nz - 1 adds each (pywt's sums start at
    the first product), over a plane 1/4 the previous level's."""
    per_pair = sum(2 * nz - 1 for nz in taps)           # 30 for bior4.4
    per_plane_px = 2 * per_pair / 2                      # two passes, one output pair per 2 inputs
    return 3 * per_plane_px * sum(0.25 ** l for l in range(levels))


def c3_block(args, world: int, rank: int, group, frames):
    """Config C3 of BASELINE.json: 2D-DWT l=5 (CDF-9/7 = pywt bior4.4, 'per'
    mode, float64 in pywt's own tap order) + per-subband deadzone Q=32, 8 x 4K
    frames resident in HBM per rank (weak scaling, no exchange):
    vcf_dwt_dz_encode (2D-DWT.py:57-78 + quantize_decom_fn :113-136 + the
    subband files' +128/dtype :162-200) and vcf_dwt_dz_decode (:80-101,
    :138-160, :202-228), each timed like the headline (settle, barrier + sync
    on both sides, max over ranks; HIP events on the launch stream for the
    per-launch figure).  Roofline: HBM (RGB in + subband bytes out) and the
    float64 issue rate the transforms are actually bound by.  Never raises."""
    import vcf_amd.dwt as DW
    from vcf_amd.device import DeviceBuffer, Event, Stream, synchronize
    H, W, F, Lv, Q = 2160, 3840, C3_FRAMES, C3_LEVELS, args.QSS
    info = {"workload": (f"2D-DWT C3: {F} x 4K frames per rank resident in HBM, l={Lv} {C3_WAVELET} (CDF-9/7, "
                         f"pywt 'per' mode, float64), per-subband deadzone Q={Q}, packed 3l+1 subbands"),
            "frames": F, "frame": [H, W, 3], "levels": Lv, "wavelet": C3_WAVELET, "n_ranks": world}
    try:
        w = DW.wavelet_index(C3_WAVELET)
        shapes, pb, wb = DW.layout(H, W, Lv)
        Ho, Wo = 2 * shapes[0][0], 2 * shapes[0][1]
        din = DeviceBuffer(F * H * W * 3)
        for f in range(F):
            din.upload(frames[f % len(frames)], offset=f * H * W * 3)
        dpk, dws, dout = DeviceBuffer(F * pb), DeviceBuffer(F * wb), DeviceBuffer(F * Ho * Wo * 3)
        st = Stream()
        enc = lambda: DW.encode_device(din, F, H, W, w, Lv, Q, dpk, dws, st)   # noqa: E731
        dec = lambda: DW.decode_device(dpk, F, H, W, w, Lv, Q, dout, dws, st)  # noqa: E731
        res = {}
        for name, fn in (("encode", enc), ("decode", dec)):
            for _ in range(3):
                fn()
            settle(fn, st, Event, 0.5, 3.0, chunk=8)
            e0, e1 = Event(), Event()
            group.barrier()
            synchronize()
            t0 = time.perf_counter()
            e0.record(st)
            for _ in range(args.c3_steps):
                fn()
            e1.record(st)
            st.synchronize()
            wall = (time.perf_counter() - t0) / args.c3_steps
            res[name] = (group.allreduce_max(wall) if world > 1 else wall, e0.elapsed_ms(e1) / args.c3_steps)
        ops = c3_fp64_ops_per_pixel() * F * H * W
        for name, alg in (("encode", F * (H * W * 3 + pb)), ("decode", F * (pb + Ho * Wo * 3))):
            wall, kms = res[name]
            info[name] = {
                "ms": round(wall * 1e3, 4), "value": round(world * F * H * W / wall / 1e6, 1), "unit": "Mpixels/s",
                "launch_ms_events": round(kms, 4), "steps": args.c3_steps,
                "roofline_hbm": {"achieved": round(alg / (kms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": round(alg / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                 "alg_bytes_per_launch": int(alg)},
                "roofline_fp64_issue": {"achieved": round(ops / (kms * 1e-3) / 1e12, 2), "peak": FP64_ISSUE_TOPS,
                                        "unit": "T fp64 lane-ops/s",
                                        "frac": round(ops / (kms * 1e-3) / 1e12 / FP64_ISSUE_TOPS, 4),
                                        "fp64_ops_per_launch": int(ops),
                                        "ops_per_pixel": round(c3_fp64_ops_per_pixel(), 2)}}
        # the opt-in lifting form (vcf_dwt_dz_*_lift, not bit-exact): the same
        # timing, and its frame-0 output against the bit-exact path's
        dpk_l, dout_l = DeviceBuffer(F * pb), DeviceBuffer(F * Ho * Wo * 3)
        enc_l = lambda: DW.encode_device(din, F, H, W, w, Lv, Q, dpk_l, dws, st, lifting=True)   # noqa: E731
        dec_l = lambda: DW.decode_device(dpk, F, H, W, w, Lv, Q, dout_l, dws, st, lifting=True)  # noqa: E731
        lift = {"entry_points": "vcf_dwt_dz_encode_lift / vcf_dwt_dz_decode_lift (opt-in, +-1 tolerance)"}
        for name, fn in (("encode", enc_l), ("decode", dec_l)):
            for _ in range(3):
                fn()
            settle(fn, st, Event, 0.5, 3.0, chunk=8)
            e0, e1 = Event(), Event()
            group.barrier()
            synchronize()
            t0 = time.perf_counter()
            e0.record(st)
            for _ in range(args.c3_steps):
                fn()
            e1.record(st)
            st.synchronize()
            wall = (time.perf_counter() - t0) / args.c3_steps
            wall = group.allreduce_max(wall) if world > 1 else wall
            lift[name] = {"ms": round(wall * 1e3, 4), "value": round(world * F * H * W / wall / 1e6, 1),
                          "unit": "Mpixels/s", "launch_ms_events": round(e0.elapsed_ms(e1) / args.c3_steps, 4)}
        enc()   # the bit-exact subbands back in dpk, decoded into dout; dout_l = lifting decode of them
        dec()
        dec_l()
        st.synchronize()
        ex = DW.unpack(dpk.download(np.empty(pb, np.uint8)), H, W, Lv)
        enc_l()
        st.synchronize()
        li = DW.unpack(dpk_l.download(np.empty(pb, np.uint8)), H, W, Lv)
        bad = tot = worst = 0
        for nm, v in ex.items():
            d = v.astype(np.int64) - li[nm].astype(np.int64)
            if not nm.startswith("LL"):
                d = (d + 128) % 256 - 128
            bad += int(np.count_nonzero(d))
            tot += d.size
            worst = max(worst, int(np.abs(d).max()))
        ye = dout.download(np.empty((Ho, Wo, 3), np.uint8)).astype(np.int64)
        yl = dout_l.download(np.empty((Ho, Wo, 3), np.uint8)).astype(np.int64)
        lift["vs_bit_exact_frame0"] = {"indices_differing": bad, "indices": tot, "max_index_diff": worst,
                                       "decoded_bytes_differing": int(np.count_nonzero(ye - yl)),
                                       "max_byte_diff": int(np.abs(ye - yl).max())}
        st.synchronize()
        enc()   # leave the bit-exact subbands for the checker
        dec()
        st.synchronize()
        info["lifting"] = lift
        if rank == 0:
            info["_check"] = (dpk, dout, pb, Ho, Wo)
    except Exception as e:   # reported in the block; the headline line still prints
        info["error"] = f"{type(e).__name__}: {e}"
    return info


def c3_check(info, frames, Q: int) -> None:
    """The checker leg (rank 0, N = 1): frame 0's packed subbands and its
    reconstruction against the oracle (oracle/vcf_dwt_oracle.cpp: pywt 1.1.1's
    'per' dwt/idwt restated with 2D-DWT.py's glue), and the oracle timed on
    one frame, 1 thread, as the block's cpu_baseline."""
    chk = info.pop("_check", None) if info else None
    if chk is None:
        return
    import vcf_amd.dwt as DW
    from oracle import oracle as O
    dpk, dout, pb, Ho, Wo = chk
    H, W = info["frame"][:2]
    pk = np.empty(pb, np.uint8)
    dpk.download(pk)
    rec = np.empty((Ho, Wo, 3), np.uint8)
    dout.download(rec)
    t0 = time.perf_counter()
    sb = O.dwt_encode_frame(frames[0], C3_WAVELET, C3_LEVELS, Q)
    t_enc = time.perf_counter() - t0
    t0 = time.perf_counter()
    want_rec = O.dwt_decode_frame(sb, H, W, C3_WAVELET, C3_LEVELS, Q)
    t_dec = time.perf_counter() - t0
    ok_enc = np.array_equal(pk, DW.pack(sb, H, W, C3_LEVELS))
    ok_dec = np.array_equal(rec, want_rec)
    info["verified"] = ("ok: frame 0's subbands and reconstruction bit-exact vs the oracle" if ok_enc and ok_dec else
                        f"MISMATCH: subbands {'ok' if ok_enc else 'differ'}, reconstruction "
                        f"{'ok' if ok_dec else 'differs'}")
    info["cpu_baseline"] = {
        "encode": {"value": round(H * W / t_enc / 1e6, 3), "unit": "Mpixels/s", "cores": 1, "kind": "port",
                   "sample": f"one 4K frame, oracle/vcf_dwt_oracle.cpp (pywt 1.1.1 'per' restated), {t_enc:.2f} s"},
        "decode": {"value": round(H * W / t_dec / 1e6, 3), "unit": "Mpixels/s", "cores": 1, "kind": "port",
                   "sample": f"one 4K frame's subbands, oracle/vcf_dwt_oracle.cpp, {t_dec:.2f} s"}}


def c2_block(args, world: int, rank: int, group):
    """Config C2 of BASELINE.json: one 1080p frame, YCoCg + 2D-DCT B=8 +
    deadzone + CBAAC, through the drop-in CoDec's own encode_fn / decode_fn
    (files on disk: PNG in, code-stream + _shape.bin out, and back to PNG;
    2D-DCT.py:268-468 with -c CBAAC, CBAAC.py:81-150).  Two entropy stages:
    -c CBAAC, the reference's own .adpt_arith format (its serial adaptive
    arithmetic coder, on the host), and -c TCBAACP (the tiled, prior-seeded
    coder on the GPU: the indices never leave HBM).  Every rank codes its own
    frame (replicas); per-call medians, max over ranks.  Never raises."""
    import tempfile

    from PIL import Image

    from vcf_amd.codec import parser as P
    from vcf_amd.codec.dct2d import CoDec
    H, W = 1080, 1920
    info = {"workload": ("C2: one 1080p PNG per rank through dct2d.CoDec.encode_fn / decode_fn (files), YCoCg + "
                         f"2D-DCT B=8 + deadzone Q={args.QSS} + CBAAC (-c CBAAC: the reference's .adpt_arith, serial "
                         "host coder; -c TCBAACP: tiled prior-seeded coder on the GPU)"),
            "frame": [H, W, 3], "n_ranks": world, "reps": args.c2_reps}
    try:
        with tempfile.TemporaryDirectory() as d:
            src = os.path.join(d, "f.png")
            img = synth_frame(H, W, seed=7 + rank)
            Image.fromarray(img).save(src)
            for ec in ("CBAAC", "TCBAACP"):
                enc = CoDec(P.parse(P.dct_parser(), ["encode", "-c", ec, "-q", str(args.QSS)]))
                dec = CoDec(P.parse(P.dct_parser(), ["decode", "-c", ec, "-q", str(args.QSS)]))
                out, rec = os.path.join(d, "e_" + ec), os.path.join(d, "d_" + ec + ".png")
                te, td = [], []
                nbytes = enc.encode_fn(src, out)
                dec.decode_fn(out, rec)
                group.barrier()
                for _ in range(args.c2_reps):
                    t0 = time.perf_counter()
                    nbytes = enc.encode_fn(src, out)
                    t1 = time.perf_counter()
                    dec.decode_fn(out, rec)
                    t2 = time.perf_counter()
                    te.append(t1 - t0)
                    td.append(t2 - t1)
                e_ms, d_ms = float(np.median(te)), float(np.median(td))
                if world > 1:
                    e_ms, d_ms = group.allreduce_max(e_ms), group.allreduce_max(d_ms)
                blk = {"encode_fn_ms": round(e_ms * 1e3, 3), "decode_fn_ms": round(d_ms * 1e3, 3),
                       "encode_value": round(world * H * W / e_ms / 1e6, 2),
                       "decode_value": round(world * H * W / d_ms / 1e6, 2), "unit": "Mpixels/s",
                       "code_bytes": int(nbytes), "bits_per_pixel": round(8 * nbytes / (H * W), 4)}
                if rank == 0:
                    with open(out + enc.file_extension, "rb") as f:
                        cs = f.read()
                    blk["_check"] = (img, dec.decompress(cs), np.asarray(Image.open(rec)))
                info[ec] = blk
            enc.bye()
    except Exception as e:   # reported in the block; the headline line still prints
        info["error"] = f"{type(e).__name__}: {e}"
    return info


def c2_check(info, Q: int) -> None:
    """Checker leg (rank 0, N = 1): each codec's file decodes to the oracle's
    indices of the frame and decode_fn's PNG equals the oracle's reconstruction;
    the CPU baseline is the same C2 encode on one host core: the oracle's C DCT
    (oracle/vcf_oracle.c) then the serial CBAAC coder restated in C++
    (vcf_cbaac_encode, the reference's AdaptiveModel + A8 coder)."""
    if not info or "error" in info:
        return
    from oracle import oracle as O
    from vcf_amd import cbaac as CB
    img = None
    for ec in ("CBAAC", "TCBAACP"):
        blk = info.get(ec)
        if not blk or "_check" not in blk:
            continue
        img, k_got, rec = blk.pop("_check")
        k_ref = O.encode_frame(img, Q)
        ok_k = np.array_equal(np.asarray(k_got).reshape(k_ref.shape), k_ref)
        ok_r = np.array_equal(rec, O.decode_frame(k_ref, img.shape[0], img.shape[1], Q))
        blk["verified"] = ("ok: the file decodes to the oracle's indices, decode_fn's PNG equals the oracle's "
                           "reconstruction" if ok_k and ok_r else
                           f"MISMATCH: indices {'ok' if ok_k else 'differ'}, PNG {'ok' if ok_r else 'differs'}")
    if img is None:
        return
    n, t0 = 0, time.perf_counter()
    while True:
        k = O.encode_frame(img, Q)
        CB.CBAACCodec(order=0).compress(k)
        n += 1
        el = time.perf_counter() - t0
        if el >= 3.0:
            break
    info["cpu_baseline"] = {"value": round(n * img.shape[0] * img.shape[1] / el / 1e6, 3), "unit": "Mpixels/s",
                            "cores": 1, "kind": "port",
                            "sample": (f"{n} x the 1080p frame: oracle/vcf_oracle.c DCT+deadzone, then the serial "
                                       f"CBAAC coder (C++ restatement of CBAAC.py's model + coder), 1 thread, "
                                       f"{el:.1f} s; no file I/O")}


def load_traffic(workload: str):
    """HBM bytes per launch from the committed rocprofv3 --pmc pass (if it matches)."""
    p = os.path.join(ROOT, "profiles", "pmc_encode_4k.json")
    try:
        d = json.load(open(p))
    except Exception:
        return None, None
    if d.get("workload") != workload:
        return None, None
    return d.get("hbm_bytes_per_launch"), os.path.relpath(p, ROOT)


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=50, help="untimed steps before the settle phase")
    ap.add_argument("--settle-min-s", type=float, default=1.5,
                    help="after --warmup, keep warming up at least this long and until launch times are "
                         "stable (0 with --settle-max-s 0 disables)")
    ap.add_argument("--settle-max-s", type=float, default=8.0)
    ap.add_argument("--frames", type=int, default=64, help="4K frames per step per GPU")
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("-q", "--QSS", type=int, default=32)
    ap.add_argument("--cpu-budget", type=float, default=20.0,
                    help="seconds of CPU time for cpu_baseline (rank 0, N=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget-configs", type=float, default=8.0,
                    help="seconds of CPU time for each of the C4 / C5 blocks' cpu_baseline (rank 0, N=1)")
    ap.add_argument("--variant", type=int, default=0, help="encode kernel (0 = automatic)")
    ap.add_argument("--c4-frames", type=int, default=256, help="frames of the C4 block (0 disables it)")
    ap.add_argument("--c4-steps", type=int, default=2)
    ap.add_argument("--no-c4-tiff", action="store_true", help="skip the C4 block with -c TIFF (GPU deflate)")
    ap.add_argument("--c4-warmup", type=int, default=1)
    ap.add_argument("--c4-timeout", type=float, default=90.0, help="seconds before an RCCL call is aborted")
    ap.add_argument("--c5-frames", type=int, default=64, help="4K frames of the C5 block (0 disables it)")
    ap.add_argument("--c5-steps", type=int, default=2)
    ap.add_argument("--c5-warmup", type=int, default=1)
    ap.add_argument("--c3-steps", type=int, default=20, help="timed launches of the C3 block (0 disables it)")
    ap.add_argument("--c2-reps", type=int, default=5, help="encode_fn/decode_fn calls per codec of the C2 block "
                                                        "(0 disables it)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))

    world, rank, local, group = dist_setup(args.gpus)
    import vcf_amd.dct as D
    from vcf_amd.device import DeviceBuffer, Event, Stream, device_count, set_device, synchronize

    ndev = device_count()
    if 0 < ndev < world and rank == 0:
        print(f"warning: {world} ranks on {ndev} GPU(s): ranks share devices (a rehearsal of the N-rank path, "
              "not a scaling measurement)", file=sys.stderr, flush=True)
    set_device(local % ndev if ndev > 0 else local)
    H, W, F, Q = args.height, args.width, args.frames, args.QSS
    Hp, Wp = D.padded_shape(H, W)
    frame_bytes = H * W * 3
    distinct = [synth_frame(H, W, seed=rank * 1000 + s) for s in range(4)]
    din = DeviceBuffer(F * frame_bytes)
    for f in range(F):
        din.upload(distinct[f % len(distinct)], offset=f * frame_bytes)
    dout = DeviceBuffer(F * Hp * Wp * 3)
    stream = Stream()

    def step():
        D.encode_device(din, F, H, W, Q, 0, out=dout, stream=stream, variant=args.variant)

    t_w0 = time.perf_counter()
    for _ in range(args.warmup):
        step()
    stream.synchronize()
    settle_s, settle_n, settle_ms = settle(step, stream, Event, args.settle_min_s, args.settle_max_s)
    warmup_s = time.perf_counter() - t_w0

    e0, e1 = Event(), Event()
    group.barrier()
    synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        step()
    e1.record(stream)
    stream.synchronize()
    synchronize()
    t1 = time.perf_counter()
    group.barrier()
    wall = t1 - t0
    kernel_ms = e0.elapsed_ms(e1) / args.steps   # average launch duration (event-timed)

    wall_max = group.allreduce_max(wall)
    pixels = group.allreduce_sum(float(args.steps * F * H * W))
    value = pixels / wall_max / 1e6

    # C4 (III, 256 x 1080p, frame-sharded, with the RCCL exchange): after the
    # headline's timed region, reported in its own block
    c4 = c4_block(args, world, rank, group) if args.c4_frames > 0 else None
    # the same with the reference's default entropy codec, -c TIFF (GPU deflate)
    c4t = c4_block(args, world, rank, group, "TIFF") if args.c4_frames > 0 and not args.no_c4_tiff else None
    # C5 (IPP_DCT, 64 x 4K, GOP 10, full search, -c TIFF on the GPU deflate, GOP-sharded)
    c5 = c5_block(args, world, rank, group) if args.c5_frames > 0 else None
    # C3 (2D-DWT l=5 bior4.4 + deadzone, 8 x 4K per rank, HBM-resident) and C2
    # (one 1080p PNG through encode_fn/decode_fn with -c CBAAC and -c TCBAACP)
    c3 = c3_block(args, world, rank, group, distinct) if args.c3_steps > 0 else None
    c2 = c2_block(args, world, rank, group) if args.c2_reps > 0 else None

    # after the timed region (an idle GPU during seconds of CPU work would start
    # the timed steps at low clocks): parity spot check of the timed kernel's
    # output, frame 0 vs the C oracle, and the CPU baseline
    parity = None
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, k_ref = cpu_baseline(distinct[0], Q, args.cpu_budget)
        k_gpu = dout.download(np.empty((Hp, Wp, 3), np.uint8))
        parity = "bit-exact vs oracle (frame 0)" if np.array_equal(k_gpu, k_ref) else "MISMATCH"
        c5_check(c5, Q, args.cpu_budget_configs)
        if c4t is not None and "_files" in c4t:
            c4t["cpu_baseline"] = c4_cpu_baseline(args.cpu_budget_configs, Q, c4t.pop("_files"))
        c3_check(c3, distinct, Q)
        c2_check(c2, Q)
    else:
        for blk in (c5, c3):
            if blk is not None:
                blk.pop("_check", None)
        if c4t is not None:
            c4t.pop("_files", None)
        for ec in ("CBAAC", "TCBAACP"):
            if c2 is not None and isinstance(c2.get(ec), dict):
                c2[ec].pop("_check", None)

    workload = (f"dct_dz_encode {H}x{W}x3 u8 RGB frames (4K), B=8, YCoCg, deadzone Q={Q}, "
                f"subband layout, {F} frames/step/GPU resident in HBM")
    alg_bytes = F * H * W * 3 + F * Hp * Wp * 3
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    traffic, tsrc = load_traffic(workload)
    if rank == 0:
        out = {
            "metric": "Mpixels/s encode (DCT+deadzone) at 4K",
            "value": round(value, 1),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (S-smooth 4K RGB, seeded)",
            "config": {"workload": workload, "global_batch": F * world, "frame": [H, W, 3],
                       "block_size": 8, "QSS": Q, "parallelism": f"frame-sharded x{world}"},
            "warmup_s": round(warmup_s, 3),
            "settle": {"launches": settle_n, "seconds": round(settle_s, 3),
                       "last_chunk_ms_per_launch": None if settle_ms is None else round(settle_ms, 4)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "kernel_ms_per_launch": round(kernel_ms, 4),
                         "alg_bytes_per_launch": alg_bytes,
                         "traffic_source": tsrc,
                         # the north star's "HBM-read" view: input bytes only; with one
                         # byte written per byte read, reads can use at most half the peak
                         "read_bytes_per_launch": F * H * W * 3,
                         "read_GBps": round(F * H * W * 3 / (kernel_ms * 1e-3) / 1e9, 1),
                         "read_frac_of_peak": round(F * H * W * 3 / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "cpu_baseline": cpu,
            "parity": parity,
            "c4_e2e_with_gather": c4,
            "c4_tiff_e2e_with_gather": c4t,
            "c5_e2e_with_gather": c5,
            "c3_dwt": c3,
            "c2_encode_decode_fn": c2,
        }
        print(json.dumps(out), flush=True)
    group.close()


if __name__ == "__main__":
    main()
