"""bench.py's rank launcher (CPU): a bare ``python bench.py --gpus N`` spawns N ranks
through a ``torch.distributed.run`` child and forwards rank 0's single JSON line.

The rank script here stands in for bench.py's GPU body: it joins a world-size-N gloo
group (the same rendezvous the real ranks use), all-reduces its rank, and rank 0
prints the JSON line; the launcher logic under test is bench.spawn_ranks itself."""
import json
import os
import textwrap

import pytest

import bench

RANK_SCRIPT = textwrap.dedent("""
    import json, os, sys
    import torch, torch.distributed as dist
    fail_rank = int(sys.argv[1])
    dist.init_process_group("gloo")
    r, n = dist.get_rank(), dist.get_world_size()
    t = torch.tensor([float(r)])
    dist.all_reduce(t)
    print(f"rank {r} banner on stdout")  # native libraries print banners; only JSON is forwarded
    if r == fail_rank:
        sys.exit(3)
    if r == 0:
        print(json.dumps({"n_gpus": n, "ranksum": t.item(),
                          "launcher": os.environ.get("FJ_BENCH_LAUNCHER")}))
    dist.destroy_process_group()
""")


@pytest.fixture()
def rank_script(tmp_path):
    p = tmp_path / "rank.py"
    p.write_text(RANK_SCRIPT)
    return str(p)


@pytest.mark.parametrize("n", [2, 3])
def test_spawn_forwards_rank0_json(rank_script, capfd, n):
    rc = bench.spawn_ranks(n, ["-1"], script=rank_script, timeout=180)
    cap = capfd.readouterr()
    out = cap.out
    assert rc == 0, cap.err  # spawn_ranks names the branch that returned non-zero on stderr
    lines = [ln for ln in out.splitlines() if ln.strip()]
    assert len(lines) == 1, out
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["ranksum"] == sum(range(n))
    assert d["launcher"].startswith("bench.py")


def test_spawn_finds_json_after_unterminated_banner(tmp_path, capfd):
    """The ranks share one stdout pipe: a banner written without a newline can precede
    rank 0's JSON on the same line; the launcher still forwards exactly the JSON."""
    p = tmp_path / "rank.py"
    p.write_text("import json, sys\nsys.stdout.write('banner without newline ')\n"
                 "print(json.dumps({'n_gpus': 1}))\n")
    rc = bench.spawn_ranks(1, [], script=str(p), timeout=120)
    out = capfd.readouterr().out
    assert rc == 0
    assert out.strip() == '{"n_gpus": 1}'


def test_spawn_propagates_rank_failure(rank_script, capfd):
    rc = bench.spawn_ranks(2, ["1"], script=rank_script, timeout=180)
    assert rc != 0
    assert capfd.readouterr().out.strip() == ""


def test_spawn_takes_rank0_line_from_its_file(tmp_path, capfd):
    """Rank 0 writes its line to FJ_BENCH_JSON (bench.emit_json): a line longer than
    PIPE_BUF comes back whole while every rank writes to the shared stdout."""
    p = tmp_path / "rank.py"
    p.write_text(textwrap.dedent("""
        import json, os, sys
        sys.path.insert(0, %r)
        import bench
        r = int(os.environ["RANK"])
        for _ in range(200):
            sys.stdout.write(f"rank {r} noise " * 20 + "\\n")
        if r == 0:
            bench.emit_json(os.dup(1), {"n_gpus": 2, "blob": "x" * 20000})
        sys.stdout.flush()
    """ % bench.ROOT))
    rc = bench.spawn_ranks(2, [], script=str(p), timeout=180)
    out = capfd.readouterr().out
    assert rc == 0
    d = json.loads(out)
    assert d["n_gpus"] == 2 and d["blob"] == "x" * 20000


def test_bare_bench_refuses_nccl_without_gpus():
    """--gpus 2 on a box without 2 GPUs and the RCCL backend: the ranks (not the parent,
    which never touches the GPU runtime) stop with a clear error."""
    import subprocess
    import sys

    if bench.torch.cuda.device_count() >= 2:
        pytest.skip("this host has the GPUs")
    p = subprocess.run([sys.executable, os.path.join(bench.ROOT, "bench.py"), "--gpus", "2"],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0
    assert "visible GPUs" in p.stderr


def test_spawn_timeout_names_the_stalled_rank(tmp_path, capfd):
    """A rank that stalls (here: rank 1 sleeps past the limit after its last phase line)
    makes spawn_ranks kill the launcher's process group, return 124 within the timeout
    (+ the 10 s grace), and name that rank with the phase it stopped in."""
    import time

    p = tmp_path / "rank.py"
    p.write_text(textwrap.dedent("""
        import os, sys, time
        sys.path.insert(0, %r)
        import bench
        r = int(os.environ["RANK"])
        bench.phase(r, "native RCCL communicator init")
        if r == 1:
            bench.phase(r, "auto-tune candidate native/reduce/1")
            time.sleep(600)
        bench.phase(r, "done")
    """ % bench.ROOT))
    t0 = time.monotonic()
    rc = bench.spawn_ranks(2, [], script=str(p), timeout=15)
    took = time.monotonic() - t0
    err = capfd.readouterr().err
    assert rc == 124
    assert took < 15 + 25, took
    assert "ranks [1] had not finished" in err, err
    assert "auto-tune candidate native/reduce/1" in err


def test_rank_timeout_scales_with_the_workload():
    import argparse

    a = argparse.Namespace(workload="c3", clients=0, gpus=8, warmup=5, steps=20, candidate_deadline=60.0)
    c5 = argparse.Namespace(workload="c5", clients=0, gpus=8, warmup=5, steps=20, candidate_deadline=60.0)
    # configs[3]: 2.1 GB per rank, plus one missed auto-tune deadline (2 x 60 s) and the abort's 70 s
    assert 300 + 190 < bench.rank_timeout(a) < 400 + 190
    assert bench.rank_timeout(c5) > bench.rank_timeout(a) + 300  # configs[4]: 256 GB per rank


def test_rank_watchdog_ends_a_stalled_rank_under_an_outer_launcher(tmp_path):
    """Under the driver's own torch.distributed.run there is no spawn_ranks parent: each
    rank's watchdog (bench.start_rank_watchdog) ends a rank that has not reached "done"
    within the limit with status 124 and names its phase, and the launcher then tears the
    job down instead of waiting on the stuck rank."""
    import subprocess
    import sys
    import time

    p = tmp_path / "rank.py"
    p.write_text(textwrap.dedent("""
        import os, sys, time
        sys.path.insert(0, %r)
        import bench
        r = int(os.environ["RANK"])
        w = bench.start_rank_watchdog(r, 5.0)
        bench.phase(r, "init process group (gloo, world 2)")
        if r == 1:
            bench.phase(r, "timed loop")
            time.sleep(600)
        bench.phase(r, "done")
        w.cancel()
    """ % bench.ROOT))
    env = {k: v for k, v in os.environ.items() if k != "FJ_BENCH_PHASES"}
    t0 = time.monotonic()
    proc = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--standalone", "--nnodes=1",
                           "--nproc-per-node=2", "--local-addr=127.0.0.1", str(p)],
                          capture_output=True, text=True, timeout=120, env=env)
    took = time.monotonic() - t0
    assert proc.returncode != 0
    assert took < 60, took
    assert "[bench rank 1] watchdog: not done within 5 s, stuck in phase 'timed loop'" in proc.stderr, proc.stderr
    assert "[bench rank 0] done" in proc.stderr
