"""The N > 1 path on CPU: world_size-2 gloo process groups (127.0.0.1), each rank one static
shard with replicated tables.  Per-shard processing sums to the whole batch's counters and
rule_stats (those do not depend on the per-worker L1 caches), and the max / sum reductions the
bench uses behave.  The per-shard checker is the oracle (no GPU here); on the GPU box the same
shards go through libupe_gpu (bench.py --gpus N)."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from upe_amd import shard, synth


# B and the flow-derived C are the batches bench.py's strong-scaling leg splits into contiguous
# shards (one batch over N ranks); seed-3-style C the round-1-4 IMIX draw
WORKLOADS = {"B": lambda: synth.config_b(n=20000, seed=31),
             "C": lambda: synth.config_c(n=12000, seed=32),
             "CF": lambda: synth.config_c_flows(n=12000, seed=34)}


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, case, q):
    import torch.distributed as dist

    import oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        wl = WORKLOADS[case]()
        sh = shard.shard_workload(wl, rank, world)
        r = oracle.run_restated(sh)
        counters = shard.sum_over_ranks([int(x) for x in r.counters[0].tolist()], dist)
        stats = shard.sum_over_ranks(r.rule_stats.view(np.uint64).reshape(-1).astype(np.int64),
                                     dist)
        slowest = shard.max_over_ranks(1.0 + rank, dist)
        total = shard.sum_over_ranks([sh.n], dist)
        if rank == 0:
            q.put((counters.tolist(), stats.tolist(), slowest, int(total[0])))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", ["B", "C", "CF"])
def test_two_rank_shards_sum_to_whole_batch(case):
    import oracle

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    counters, stats, slowest, total = q.get(timeout=10)

    wl = WORKLOADS[case]()
    whole = oracle.run_restated(wl)
    assert total == wl.n
    assert slowest == 2.0
    assert counters == [int(x) for x in whole.counters[0].tolist()]
    assert stats == whole.rule_stats.view(np.uint64).reshape(-1).astype(np.int64).tolist()


def test_shard_ranges_cover_the_batch():
    for n in (0, 1, 7, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            spans = [shard.shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def test_shard_workload_frames_rebased():
    wl = synth.config_c(n=3000, seed=33)
    for r in range(3):
        sh = shard.shard_workload(wl, r, 3)
        s, e = shard.shard_range(wl.n, r, 3)
        from upe_amd.layout import desc_lens, desc_offsets

        for i in (0, sh.n // 2, sh.n - 1):
            o, ln = int(desc_offsets(sh.desc)[i]), int(desc_lens(sh.desc)[i])
            go = int(desc_offsets(wl.desc)[s + i])
            assert np.array_equal(sh.frames[o:o + ln], wl.frames[go:go + ln])


def test_bench_launcher_command():
    """`python bench.py --gpus N` (no WORLD_SIZE) starts N ranks under torch.distributed.run on
    127.0.0.1 with the same arguments; a rank refuses a --gpus that disagrees with WORLD_SIZE.
    Neither needs torch or a GPU in the launching process."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench

    cmd = bench.launch_cmd(8, ["--gpus", "8", "--steps", "20"], 29500)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd
    assert "--master-port=29500" in cmd and cmd[-4:] == ["--gpus", "8", "--steps", "20"]
    assert cmd[-5].endswith("bench.py")
    assert bench.world_check(None, {}) == 1
    assert bench.world_check(1, {}) == 1
    assert bench.world_check(None, {"WORLD_SIZE": "4"}) == 4
    assert bench.world_check(4, {"WORLD_SIZE": "4"}) == 4
    with pytest.raises(SystemExit):
        bench.world_check(4, {"WORLD_SIZE": "2"})
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--steps", "1"], cwd=root,
                       env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE=2 but --gpus 4" in p.stderr
