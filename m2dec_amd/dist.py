"""Multi-GPU work queue: independent streams sharded over the ranks of one node.

One process per GPU.  The data path has no collective; the only exchanges are the work-queue
hand-off below, over torch.distributed — backend "nccl" (= RCCL over xGMI) with device tensors on
the GPU box, "gloo" with CPU tensors in the CPU tests:

  * rank 0 owns the job list (stream id, seed, cost in pictures) and broadcasts it (`broadcast_jobs`);
  * every rank derives the same assignment from it (`plan`: longest-processing-time first onto the
    least loaded rank, so S >= N streams of unequal length balance), runs its jobs, and then
  * a completion round all-gathers one row per job from every rank (`run_queue`): done, bit-exact,
    frames, seconds.  Each job must be completed by exactly one rank; a job that failed or that no
    rank completed is dealt again, round robin, in the next round (bounded rounds);
  * counters are all-gathered at the end (`gather_counters`), and the per-rank parity results
    all-reduced (`all_ranks`).

bench.py's multi-rank orchestration is `timed_steps` (warmup, barrier + device sync, K timed steps,
barrier, max-over-ranks time) over `run_queue`; tests/test_dist_gloo.py runs the same functions at
world size 2 over 5 jobs on the CPU."""
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence, Tuple

Job = Tuple[int, int, int]  # (job id, stream seed, cost: pictures)


def make_jobs(n: int, first_seed: int = 1, cost: int = 60) -> List[Job]:
    """Rank 0's job list: n independent streams, seeds first_seed.. (bench: C4 = one c3 stream per seed)."""
    return [(i, first_seed + i, cost) for i in range(n)]


def broadcast_jobs(dist, world: int, rank: int, jobs: Optional[Sequence[Job]], device: str) -> List[Job]:
    """Rank 0's job list to every rank (two broadcasts: the count, then the table).  Other ranks pass None."""
    if dist is None or world == 1:
        return [tuple(int(x) for x in j) for j in jobs]
    import torch

    n = torch.tensor([len(jobs) if rank == 0 else 0], dtype=torch.int64, device=device)
    dist.broadcast(n, 0)
    t = torch.zeros((int(n.item()), 3), dtype=torch.int64, device=device)
    if rank == 0:
        t.copy_(torch.tensor([list(j) for j in jobs], dtype=torch.int64))
    dist.broadcast(t, 0)
    return [tuple(int(x) for x in row) for row in t.tolist()]


def plan(jobs: Sequence[Job], world: int) -> List[List[Job]]:
    """Longest-processing-time assignment: jobs by cost (descending, then id), each onto the rank with the
    least cost so far (lowest rank on ties).  Deterministic, so every rank computes the same plan."""
    load = [0] * world
    out: List[List[Job]] = [[] for _ in range(world)]
    for j in sorted(jobs, key=lambda j: (-j[2], j[0])):
        r = min(range(world), key=lambda k: (load[k], k))
        out[r].append(j)
        load[r] += j[2]
    for o in out:
        o.sort(key=lambda j: j[0])
    return out


@dataclass
class QueueResult:
    owner: List[int]                # job -> rank that completed it (-1: never)
    frames: List[int]               # job -> frames delivered
    seconds: List[float]            # job -> seconds its decode took
    ok: List[bool]                  # job -> bit-exact
    rank_seconds: List[float]       # rank -> sum of its jobs' seconds
    rounds: int
    attempts: List[int] = field(default_factory=list)  # job -> times it was run

    @property
    def total_frames(self) -> int:
        return sum(self.frames)

    @property
    def all_ok(self) -> bool:
        return all(self.ok) and all(o >= 0 for o in self.owner)


def run_queue(dist, world: int, rank: int, jobs: Sequence[Job],
              work: Callable[[Job], Tuple[int, float, bool]], device: str, max_rounds: int = 3) -> QueueResult:
    """Run the job list over the ranks: round 0 follows `plan`; after each round a completion round
    all-gathers one row (done, ok, frames, seconds) per job and rank; jobs left undone or not bit-exact are
    dealt round robin in the next round.  `work(job)` -> (frames, seconds, bit-exact); an exception counts
    as a failed attempt.  Every rank returns the same QueueResult."""
    S = len(jobs)
    idx = {j[0]: i for i, j in enumerate(jobs)}
    owner, frames, secs, ok = [-1] * S, [0] * S, [0.0] * S, [False] * S
    attempts = [0] * S
    mine = plan(jobs, world)[rank]
    rounds = 0
    while rounds < max_rounds:
        rounds += 1
        row = [[0.0] * 4 for _ in range(S)]
        for j in mine:
            try:
                f, s, good = work(j)
            except Exception:  # noqa: BLE001 - a failed attempt; dealt again next round
                f, s, good = 0, 0.0, False
            row[idx[j[0]]] = [1.0, 1.0 if good else 0.0, float(f), float(s)]
        if dist is None or world == 1:
            rows = [row]
        else:
            import torch

            r = torch.tensor(row, dtype=torch.float64, device=device)
            rr = [torch.zeros_like(r) for _ in range(world)]
            dist.all_gather(rr, r)
            rows = [x.cpu().tolist() for x in rr]
        for k, rr in enumerate(rows):
            for i in range(S):
                if rr[i][0] > 0:
                    attempts[i] += 1
                    if rr[i][1] > 0 and not ok[i]:
                        owner[i], ok[i], frames[i], secs[i] = k, True, int(rr[i][2]), float(rr[i][3])
        left = [jobs[i] for i in range(S) if not ok[i]]
        if not left:
            break
        mine = [j for n, j in enumerate(left) if n % world == rank]
    rank_seconds = [0.0] * world
    for i in range(S):
        if owner[i] >= 0:
            rank_seconds[owner[i]] += secs[i]
    return QueueResult(owner, frames, secs, ok, rank_seconds, rounds, attempts)


def timed_steps(dist, world: int, rank: int, jobs: Sequence[Job], work: Callable[[Job], Tuple[int, float, bool]],
                steps: int, warmup: int, device: str, sync: Callable[[], None] = lambda: None,
                before_timed: Callable[[], None] = lambda: None) -> dict:
    """bench.py's multi-rank leg: `warmup` untimed passes over the job list, then exactly `steps` timed
    passes, each bracketed by a barrier and a device sync on both sides.  A pass = run_queue over the job
    list.  Returns frames of all ranks, the max-over-ranks sum of decode seconds (each rank's own step
    intervals), the wall time of the timed region, bit-exactness and the per-rank counters."""
    import time

    for _ in range(warmup):
        if not run_queue(dist, world, rank, jobs, work, device).all_ok:
            raise RuntimeError("warmup pass not bit-exact")
    before_timed()
    if dist is not None and world > 1:
        dist.barrier()
    sync()
    w0 = time.perf_counter()
    tot_frames, ok, per_rank = 0, True, [0.0] * world
    results = []
    for _ in range(steps):
        q = run_queue(dist, world, rank, jobs, work, device)
        results.append(q)
        ok &= q.all_ok and all(n == 1 for n in q.attempts)  # (a timed job run twice had failed once)
        tot_frames += q.total_frames
        per_rank = [a + b for a, b in zip(per_rank, q.rank_seconds)]
    sync()
    if dist is not None and world > 1:
        dist.barrier()
    wall = time.perf_counter() - w0
    _, max_wall, _ = gather_counters(dist, world, 0, wall, device)
    return {"frames": tot_frames, "max_seconds": max(per_rank) if per_rank else 0.0, "wall": max_wall,
            "ok": ok, "per_rank_seconds": per_rank, "owners": results[-1].owner if results else [],
            "rounds": max((q.rounds for q in results), default=0)}


def job_table(dist, world: int, rank: int, device: str, first_seed: int = 1) -> List[int]:
    """One stream seed per rank (the single-stream-per-GPU case of the queue): the broadcast job list's
    seeds in plan order."""
    jobs = broadcast_jobs(dist, world, rank, make_jobs(world, first_seed) if rank == 0 else None, device)
    return [p[0][1] for p in plan(jobs, world)]


def gather_counters(dist, world: int, frames: int, seconds: float, device: str) -> Tuple[int, float, List[Tuple[int, float]]]:
    """Returns (total frames over ranks, max seconds over ranks, per-rank list)."""
    if dist is None or world == 1:
        return frames, seconds, [(frames, seconds)]
    import torch

    c = torch.tensor([float(frames), float(seconds)], dtype=torch.float64, device=device)
    outs = [torch.zeros_like(c) for _ in range(world)]
    dist.all_gather(outs, c)
    per = [(int(o[0].item()), float(o[1].item())) for o in outs]
    return sum(p[0] for p in per), max(p[1] for p in per), per


def all_ranks(dist, world: int, ok: bool, device: str) -> bool:
    """True iff `ok` holds on every rank (all-reduce MIN of one int); used for the per-rank parity gate."""
    if dist is None or world == 1:
        return bool(ok)
    import torch

    t = torch.tensor([1 if ok else 0], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


# ---- host CPUs per rank.  Each rank's decode is host-bound (~8 CPU-ms per 1080p frame:
# CABAC parse 5, MD5 2, the rest ~1), so at N GPUs per node the ranks must not share cores: each rank gets a
# disjoint slice of its GPU's NUMA node's CPUs (∩ the job's affinity), the slices of one node equal in size.  The
# library then sizes its parse pool and MD5 helpers from that slice ∩ the cgroup quota ÷ the node's ranks
# (cpushare.c), and numa.c keeps its threads on it.  Unmeasured on an 8-GPU node (no scaling run was available).

def parse_cpulist(s: str) -> List[int]:
    out: List[int] = []
    for part in s.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def node_cpus(sysfs_root: str = "") -> dict:
    """{NUMA node: its CPUs} from <root>/sys/devices/system/node/node<n>/cpulist."""
    import os
    base = os.path.join(sysfs_root or "/", "sys", "devices", "system", "node")
    out = {}
    try:
        names = os.listdir(base)
    except OSError:
        return out
    for n in names:
        if n.startswith("node") and n[4:].isdigit():
            try:
                out[int(n[4:])] = parse_cpulist(open(os.path.join(base, n, "cpulist")).read())
            except (OSError, ValueError):
                pass
    return out


def gpu_numa_node(bus_id: str, sysfs_root: str = "") -> int:
    """The NUMA node of a PCI device (<root>/sys/bus/pci/devices/<bus id>/numa_node), -1 if unknown."""
    import os
    try:
        return int(open(os.path.join(sysfs_root or "/", "sys", "bus", "pci", "devices", bus_id.lower(),
                                     "numa_node")).read())
    except (OSError, ValueError):
        return -1


def cpu_plan(nodes: Sequence[int], cpus_of_node: dict, allowed) -> List[List[int]]:
    """Disjoint CPU slices per rank: rank r's GPU sits on NUMA node nodes[r]; the ranks of one node split that
    node's allowed CPUs into equal contiguous slices (rank order).  When some rank's node is unknown or holds
    none of the allowed CPUs, all allowed CPUs are split among all ranks instead.  A rank gets at least one CPU
    (slices then overlap only when there are fewer CPUs than ranks)."""
    allowed = sorted(set(allowed))
    world = len(nodes)

    def split(pool: List[int], ranks: List[int], out: List[List[int]]):
        k = len(ranks)
        for i, r in enumerate(ranks):
            lo, hi = len(pool) * i // k, len(pool) * (i + 1) // k
            out[r] = pool[lo:hi] if len(pool) >= k else [pool[i % len(pool)]]

    out: List[List[int]] = [[] for _ in range(world)]
    pools = {n: sorted(set(cpus_of_node.get(n, [])) & set(allowed)) for n in set(nodes)}
    if any(n < 0 or not pools[n] for n in nodes):
        split(allowed, list(range(world)), out)
        return out
    for n in sorted(set(nodes)):
        split(pools[n], [r for r in range(world) if nodes[r] == n], out)
    return out


def place_rank(dist, world: int, rank: int, bus_id: Optional[str], device: str, sysfs_root: str = "") -> Optional[List[int]]:
    """All-gather every rank's GPU NUMA node, take this rank's slice of cpu_plan and bind the calling thread to
    it (the library's threads, created later by it, inherit the mask).  Returns the slice (None at world 1)."""
    import os
    if dist is None or world == 1:
        return None
    import torch

    node = gpu_numa_node(bus_id, sysfs_root) if bus_id else -1
    t = torch.tensor([node], dtype=torch.int64, device=device)
    outs = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    nodes = [int(o.item()) for o in outs]
    mine = cpu_plan(nodes, node_cpus(sysfs_root), os.sched_getaffinity(0))[rank]
    if mine:
        os.sched_setaffinity(0, mine)
    return mine
