"""Run a function in `world` spawned rank processes (one process per rank,
the environment a launcher would give them) and collect what each returns.
Used by the world_size-2 driver tests; no PyTorch."""
import multiprocessing as mp
import os
import traceback


def _entry(fn, rank, world, port, store_port, args, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), VCF_STORE_PORT=str(store_port))
    try:
        q.put((rank, "ok", fn(rank, world, *args)))
    except BaseException:
        q.put((rank, "error", traceback.format_exc()))


def run_ranks(fn, world, *args, timeout=180):
    from vcf_amd.comm import free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port, store = free_port(), free_port()
    procs = [ctx.Process(target=_entry, args=(fn, r, world, port, store, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict((r[0], r) for r in (q.get(timeout=timeout) for _ in range(world)))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = [r[2] for r in res.values() if r[1] != "ok"]
    assert not errs, "\n".join(errs)
    return {r: res[r][2] for r in res}
