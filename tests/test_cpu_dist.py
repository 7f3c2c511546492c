"""Multi-process (gloo, world_size 2, CPU) tests of bench.py's distributed
contract: the path is embarrassingly parallel (one replica per GPU, no data-path
collective); the only cross-rank traffic is the barrier pair and the MAX
all-reduce of the timed region."""
import os
import socket
import sys
import time

import numpy as np
import torch.multiprocessing as mp

from conftest import ROOT

sys.path.insert(0, ROOT)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []
    step_s = 0.02 * (rank + 1)                       # rank 1 is the straggler

    def step():
        calls.append(1)
        time.sleep(step_s)

    el = bench.timed_steps(step, 5, lambda: None, dist, "cpu")
    r, w, lr = bench.dist_env()
    q.put((rank, el, len(calls), (r, w, lr)))
    dist.barrier()
    dist.destroy_process_group()


def test_timed_steps_max_over_ranks_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    els = [r[1] for r in res]
    assert els[0] == els[1]                       # every rank reports the same (max) time
    assert els[0] >= 5 * 0.04 * 0.95              # at least the straggler's work
    assert all(r[2] == 5 for r in res)            # exactly K timed steps per rank
    assert [r[3] for r in res] == [(0, 2, 0), (1, 2, 1)]


def test_timed_steps_single_process():
    import bench
    n = []
    el = bench.timed_steps(lambda: n.append(0), 7, lambda: None, None)
    assert len(n) == 7 and el >= 0


def test_rank_shards_are_distinct():
    """Each rank encodes its own shard (weak scaling): seeds differ per rank."""
    import bertpy
    a = bertpy.synthetic_ids(4, 16, 30522, seed=7 + 0)
    b = bertpy.synthetic_ids(4, 16, 30522, seed=7 + 1)
    assert not all(np.array_equal(x, y) for x, y in zip(a, b))
    assert all(x[0] == 101 and x[-1] == 102 for x in a + b)


def test_algorithmic_bytes_bge_base_q4_0():
    """Compulsory HBM bytes per batch (DESIGN.md "Roofline"): weights at 4.5 bits
    plus one gathered word-embedding row per token; activations not counted."""
    import bench
    import bertpy
    b = bench.algorithmic_bytes(bertpy.ARCHS["bge-base-en-v1.5"], "q4_0", 64, 512)
    w = 12 * (4 * 768 * 768 + 2 * 768 * 3072) * 0.5625
    rows = 64 * 512 * 768 * 0.5625
    assert w + rows < b < (w + rows) * 1.05


def test_pmc_passes_skip_under_a_profiler(monkeypatch):
    """bench.py never starts rocprofv3 from under a profiler: with a
    rocprofv3 preload or its ROCPROF* variables in the environment, pmc_live reports
    'skipped' and starts no process."""
    import subprocess
    import bench
    assert not bench.under_profiler({"LD_PRELOAD": "", "PATH": "/usr/bin"})
    assert bench.under_profiler({"LD_PRELOAD": "/opt/rocm/lib/rocprofiler-sdk/librocprofiler-sdk-tool.so"})
    assert bench.under_profiler({"ROCPROF_KERNEL_TRACE": "1"})
    assert bench.under_profiler({"ROCPROFILER_LIBRARY_CTOR": "1"})
    monkeypatch.setenv("ROCPROF_OUTPUT_PATH", "/tmp/x")

    def refuse(*a, **k):
        raise AssertionError("a process was started under the profiler")

    monkeypatch.setattr(subprocess, "run", refuse)
    r = bench.pmc_live("/nonexistent.bin", 1, 32)
    assert "skipped" in r and "bytes_per_forward" not in r


def test_bench_gpus_2_starts_two_ranks():
    """`python bench.py --gpus 2` with no torchrun environment starts its two rank
    processes itself -- here with the --dry-step CPU stub on
    gloo: exactly one JSON line, n_gpus 2, one per-rank entry per rank, and the
    value is the whole job's rate (both ranks' sentences over the max time)."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-step", "--steps", "4",
                        "--warmup", "1"], cwd="/tmp", env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       timeout=300)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    lines = [x for x in r.stdout.decode().splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout.decode()
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["global_batch"] == 128
    assert [p["rank"] for p in res["per_rank"]] == [0, 1]
    t_max = max(p["ms_per_step"] for p in res["per_rank"])
    assert abs(res["ms_per_step"] - t_max) < 1e-3
    assert abs(res["value"] - 128 * 1e3 / res["ms_per_step"]) / res["value"] < 1e-3


def test_bench_refuses_world_mismatch():
    """A rank whose WORLD_SIZE disagrees with --gpus stops before any work."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-step"], cwd="/tmp",
                       env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)
    assert r.returncode != 0 and b"WORLD_SIZE 1" in r.stderr


def _agree_worker(rank, world, port, q):
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    both = bench.all_ranks_ok(True, dist, "cpu")
    one_fails = bench.all_ranks_ok(rank != 1, dist, "cpu")   # rank 1's preparation failed
    q.put((rank, both, one_fails))
    dist.barrier()
    dist.destroy_process_group()


def test_optional_leg_agreement_gloo():
    """an optional bench leg (the encode path) prepares rank-locally, then
    every rank agrees (bench.all_ranks_ok, a MIN all-reduce) before the leg's
    collectives, so one rank's failure skips the leg everywhere instead of leaving
    the other ranks blocked in its barrier."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_agree_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == [(0, True, False), (1, True, False)]
