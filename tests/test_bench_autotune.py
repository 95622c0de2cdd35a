"""bench.autotune_exchange on the CPU (gloo, two ranks): every rank sees the same verdict on
each exchange candidate. A candidate that misses its host deadline on ONE rank is dropped on
every rank; for the library's own communicator ("native") every rank aborts it exactly once
and skips its remaining candidates; a candidate that raises on one rank is dropped too; the
survivors carry the max-over-ranks time and the run continues on the fastest of them."""
import multiprocessing as mp

import pytest
import torch

from tests.rendezvous import HeldStore, init_group

CANDS = [("torch", "reduce", 1), ("torch", "reduce", 2), ("torch", "all_reduce", 1),
         ("native", "reduce", 1), ("native", "reduce", 4), ("native", "all_reduce", 1)]


def _worker(rank, world, port, scenario, q):
    import torch.distributed as dist
    import bench
    init_group("gloo", rank, world, port)
    aborts = []

    def measure(cand):
        eng, col, b = cand
        if scenario == "native_hang" and eng == "native" and b == 4 and rank == 1:
            return None  # this rank's step did not complete within its deadline
        if scenario == "torch_raises" and cand == ("torch", "reduce", 2) and rank == 0:
            raise RuntimeError("simulated RCCL error")
        return 1.0 + 0.25 * rank + {1: 0.5, 2: 0.2, 4: 0.1}[b] + (0.05 if col == "all_reduce" else 0.0)

    tune, dropped = bench.autotune_exchange(CANDS, measure, lambda: aborts.append(1), torch.device("cpu"), rank)
    q.put((rank, tune, dropped, len(aborts)))
    dist.destroy_process_group()


def _run(scenario, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    held = HeldStore(world)
    ps = [ctx.Process(target=_worker, args=(r, world, held.port, scenario, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


def test_native_deadline_on_one_rank_drops_it_everywhere():
    got = _run("native_hang")
    tunes = [g[1] for g in got]
    drops = [g[2] for g in got]
    assert tunes[0] == tunes[1] and drops[0] == drops[1]  # one verdict on every rank
    assert drops[0] == {("native", "reduce", 4): "dropped: missed the deadline",
                        ("native", "all_reduce", 1): "skipped: communicator aborted"}
    assert [g[3] for g in got] == [1, 1]  # both ranks aborted the communicator, once
    # survivors: every torch candidate and the native one measured before the hang, max over ranks
    assert set(tunes[0]) == {c for c in CANDS if c not in drops[0]}
    assert tunes[0][("torch", "reduce", 2)] == pytest.approx(1.0 + 0.25 + 0.2)
    assert min(tunes[0], key=tunes[0].get) == ("torch", "reduce", 2)


def test_candidate_raising_on_one_rank_is_dropped_without_abort():
    got = _run("torch_raises")
    assert got[0][2] == got[1][2] == {("torch", "reduce", 2): "dropped: raised"}
    assert [g[3] for g in got] == [0, 0]
    assert len(got[0][1]) == len(CANDS) - 1
    assert min(got[0][1], key=got[0][1].get) == ("native", "reduce", 4)
