"""Config E on the HIP path: static shards over a world of 2 ranks (BASELINE
configs[4]), the reference's one worker_t per RSS shard (src/main.c:444-456, src/rx_pcap.c:71-77).

Two spawned processes share the one GPU of the test box (device round robin, as bench.py maps
ranks), joined by a gloo process group on 127.0.0.1 (RCCL cannot put two ranks on one device).
Each rank takes its contiguous shard (upe_amd.shard.shard_workload), runs it through GpuWorker
(in place and emit mode) and checks its verdicts, frames or records and final L1 state against
the oracle on that shard; the per-rank counters and rule_stats are summed with the same
shard.sum_over_ranks bench.py uses and compared with the REFERENCE worker over the whole batch
(neither depends on the per-worker L1 caches).  A second test runs bench.py itself as two ranks."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle
from upe_amd import shard, synth

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = {"B": lambda: synth.config_b(n=300_000, seed=41),
         "C": lambda: synth.config_c(n=200_000, seed=42),
         "CF": lambda: synth.config_c_flows(n=200_000, seed=43)}


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, case, emit, q):
    import torch.distributed as dist

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_gpu_parity import _assert_same
    from upe_amd import gpu

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        wl = CASES[case]()
        sh = shard.shard_workload(wl, rank, world)
        r = oracle.run_restated(sh)
        device = rank % max(1, gpu.device_count())   # bench.py's mapping of ranks to GPUs
        w = gpu.GpuWorker(device, sh.capacity)
        try:
            w.configure(sh)
            got = gpu.run_workload(sh, worker=w, emit=emit)
        finally:
            w.close()
        _assert_same(got, {"verdict": r.verdict, "frames": r.frames, "counters": r.counters,
                           "rule_stats": r.rule_stats, "l1": r.l1}, f"rank {rank} {case}")
        counters, stats = got[2], got[3]
        tot_c = shard.sum_over_ranks([int(x) for x in counters[0].tolist()], dist)
        tot_s = shard.sum_over_ranks(stats.view(np.uint64).reshape(-1).astype(np.int64), dist)
        total = shard.sum_over_ranks([sh.n], dist)
        slowest = shard.max_over_ranks(float(rank), dist)
        if rank == 0:
            q.put(("ok", tot_c.tolist(), tot_s.tolist(), int(total[0]), slowest))
    except Exception as e:   # the parent reports it
        q.put(("error", f"rank {rank}: {type(e).__name__}: {e}"))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("emit", [False, True])
@pytest.mark.parametrize("case", ["B", "C", "CF"])
def test_two_rank_static_shards_on_gpu(case, emit):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, case, emit, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    msg = q.get(timeout=10)
    assert msg[0] == "ok", msg
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    _, counters, stats, total, slowest = msg
    wl = CASES[case]()
    ref = oracle.run_reference(wl) if oracle.ref_available() else oracle.run_restated(wl)
    assert total == wl.n and slowest == 1.0
    assert counters == [int(x) for x in ref.counters[0].tolist()]
    assert stats == ref.rule_stats.view(np.uint64).reshape(-1).astype(np.int64).tolist()


def test_bench_two_ranks():
    """bench.py's N > 1 path end to end, started the way the driver starts N = 1: plain
    `python bench.py --gpus 2`, which launches its two ranks itself (here on the one GPU, gloo
    for the barrier and the max / sum over ranks, as UPE_BENCH_DIST_BACKEND allows on a one-GPU
    box): config B plus the IMIX leg, each rank its own shard (weak scaling), the strong-scaling
    leg (one B and one C batch split into the two ranks' contiguous shards) and rank 0's CPU
    baseline after the timed regions."""
    env = dict(os.environ, UPE_BENCH_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "bench.py", "--gpus", "2",
           "--steps", "20", "--warmup", "5", "--no-hbm-probe", "--cpu-threads", "2",
           "--dropin-seconds", "0", "--max-copies", "24", "--imix-copies", "8",
           "--imix-v6fwd", "0"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    # stdout carries the JSON line and nothing else (gloo's connection lines go to stderr)
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert d["value"] > 0 and d["imix"]["value"] > 0
    assert "x2" in d["config"]["parallelism"]
    for k in ("B", "C"):
        st = d["strong"][k]
        assert st["scaling"] == "strong" and st["value"] > 0
        assert st["packets_per_step"] == 1 << 20 and st["packets_this_rank"] == 1 << 19
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and "ranks_note" in cb
    print(json.dumps({k: d[k] for k in ("value", "ms_per_step", "n_gpus")}))

