"""World-size-2 runs of the multi-GPU work queue on CPU (gloo): the same m2dec_amd/dist.py functions
bench.py runs over RCCL (broadcast_jobs, plan, run_queue, timed_steps, gather_counters, all_ranks).  A
job = one synthetic stream parsed by the product host parser (trace capture; no GPU needed), 5 jobs
over 2 ranks.  Unmeasured on hardware: the driver's 8-GPU node runs bench.py at N = 2/4/8."""
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


def _stream(seed, frames):
    from tests.gen_check import generate

    out = f"/tmp/m2dec_gloo_{os.getpid()}_{seed}.264"
    generate("cov_cabac", out, seed=seed, extra=(f"frames={frames}",))
    data = open(out, "rb").read()
    os.unlink(out)
    return data


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import m2dec_amd
    import m2dec_amd.dist as md

    # rank 0's job list: 5 streams of unequal length (cost = pictures); the others receive it
    jobs = md.broadcast_jobs(dist, world, rank, [(0, 5, 6), (1, 6, 4), (2, 7, 6), (3, 8, 3), (4, 9, 5)]
                             if rank == 0 else None, "cpu")
    ran = []
    fail_once = {2}

    def work(job):
        jid, seed, cost = job
        ran.append(jid)
        if jid in fail_once and rank == md.plan(jobs, world).index(
                next(p for p in md.plan(jobs, world) if any(j[0] == jid for j in p))):
            fail_once.discard(jid)
            raise RuntimeError("injected failure")
        tr = m2dec_amd.Trace(_stream(seed, cost))
        n = tr.npics
        tr.close()
        return n, 0.25 * n, n == cost

    q1 = md.run_queue(dist, world, rank, jobs, work, "cpu")
    ran_first = list(ran)
    # a clean queue: warmup pass + 2 timed passes, every job once per pass
    ran.clear()
    res = md.timed_steps(dist, world, rank, jobs, lambda j: (j[2], 0.1 * j[2], True), 2, 1, "cpu")
    total, mx, per = md.gather_counters(dist, world, 7 * (rank + 1), 0.5 + rank, "cpu")
    both = md.all_ranks(dist, world, True, "cpu")
    one = md.all_ranks(dist, world, rank == 0, "cpu")
    seeds = md.job_table(dist, world, rank, "cpu", first_seed=5)
    q.put((rank, jobs, q1, ran_first, res, total, mx, per, both, one, seeds))
    dist.destroy_process_group()


def test_work_queue_world2(built):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    qu = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, qu)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((qu.get(timeout=180) for _ in range(world)), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import m2dec_amd.dist as md

    jobs = res[0][1]
    plan = md.plan(jobs, world)
    # LPT over costs 6,6,5,4,3: {0: 6+4+?, ...} balanced within one job's cost
    loads = [sum(j[2] for j in p) for p in plan]
    assert sorted(j for p in plan for j in p) == sorted(jobs) and max(loads) - min(loads) <= 6
    for rank, jb, q1, ran_first, r, total, mx, per, both, one, seeds in res:
        assert jb == jobs
        # every job completed exactly once, bit-exact; job 2 failed once and was dealt again in round 2
        assert q1.all_ok and q1.rounds == 2
        assert q1.attempts == [1, 1, 2, 1, 1]
        assert q1.frames == [6, 4, 6, 3, 5] and q1.total_frames == 24
        assert sorted(ran_first) == sorted([j[0] for j in plan[rank]] + ([2] if rank == 0 else []))
        assert all(0 <= o < world for o in q1.owner)
        # identical results on both ranks
        assert q1 == res[0][2]
        # timed passes: frames of both passes, max over ranks of the decode seconds, bit-exact
        assert r["ok"] and r["frames"] == 2 * 24 and r["rounds"] == 1
        assert r["max_seconds"] == pytest.approx(2 * 0.1 * max(loads))
        assert r["owners"] == [next(k for k, p in enumerate(plan) if j in p) for j in jobs]
        assert total == 7 + 14 and mx == pytest.approx(1.5) and [p[0] for p in per] == [7, 14]
        assert both and not one
        assert sorted(seeds) == [5, 6]
