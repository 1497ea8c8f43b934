"""World-size-2 run of the multi-GPU hand-off on CPU (gloo): rank 0 broadcasts the job table,
every rank parses its own synthetic stream with the product host parser (trace capture; no GPU
needed), and the per-rank counters are all-gathered — the same code bench.py runs over RCCL."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import m2dec_amd
    import m2dec_amd.dist as md
    from tests.gen_check import generate

    seeds = md.job_table(dist, world, rank, "cpu", first_seed=5)
    out = f"/tmp/m2dec_gloo_{os.getpid()}.264"
    generate("cov_cabac", out, seed=seeds[rank], extra=("frames=6",))
    tr = m2dec_amd.Trace(open(out, "rb").read())
    os.unlink(out)
    total, mx, per = md.gather_counters(dist, world, tr.npics, 0.5 + rank, "cpu")
    both = md.all_ranks(dist, world, True, "cpu")
    one = md.all_ranks(dist, world, rank == 0, "cpu")
    q.put((rank, seeds, tr.npics, total, mx, per, both, one))
    dist.destroy_process_group()


def test_job_table_and_counters_world2(built):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, seeds, npics, total, mx, per, both, one in res:
        assert both and not one
        assert seeds == [5, 6]
        assert npics == 6
        assert total == 12
        assert mx == pytest.approx(1.5)
        assert [p[0] for p in per] == [6, 6]
