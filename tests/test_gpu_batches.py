"""GPU parity of the native batch loop the bench measures (include/upe_gpu.h
upe_gpu_process_batches / upe_gpu_process_batches_emit: a ring of resident batches queued back
to back from native code).  K batches through one call must equal K upe_gpu_process calls, i.e.
the reference worker running the K bursts in order: per-batch frames (in place) or records (emit),
the last batch's verdict words (the batches share the verdict / record arrays), and the worker's
counters, rule_stats and L1 state carried across all of them (oracle restatement, pinned by the
reference's golden vectors)."""
from __future__ import annotations

import dataclasses

import numpy as np
import pytest

import oracle
from upe_amd import gpu, synth

pytestmark = pytest.mark.gpu


def _batches(k, n):
    """k config-B batches of the same descriptor layout (64-byte stride) and different packets,
    classified against the first batch's tables (one worker, one table snapshot)."""
    wls = [synth.config_b(n=n, seed=90 + j) for j in range(k)]
    for j in range(1, k):
        assert np.array_equal(wls[j].desc, wls[0].desc)
        wls[j] = dataclasses.replace(wls[j], rules=wls[0].rules, capacity=wls[0].capacity,
                                     arp=wls[0].arp, ndp=wls[0].ndp)
    return wls


def _oracle_chain(wls):
    """The restatement over the batches in order, carrying L1, counters and rule_stats."""
    l1 = counters = stats = None
    outs = []
    for wl in wls:
        r = oracle.run_restated(wl, l1=l1, counters=counters, rule_stats=stats)
        l1, counters, stats = r.l1, r.counters, r.rule_stats
        outs.append(r)
    return outs


@pytest.mark.parametrize("emit", [False, True])
@pytest.mark.parametrize("k,n", [(4, 50_000), (3, 1000), (2, 64 * 1024 + 17)])
def test_process_batches_chain(gpu_worker_factory, k, n, emit):
    wls = _batches(k, n)
    ref = _oracle_chain(wls)
    w = gpu_worker_factory(wls[0].capacity)
    try:
        w.configure(wls[0])
        bufs = [w.malloc(wl.frames.nbytes) for wl in wls]
        for b, wl in zip(bufs, wls):
            w.h2d(b, np.ascontiguousarray(wl.frames))
        desc = w.malloc(wls[0].desc.nbytes)
        w.h2d(desc, np.ascontiguousarray(wls[0].desc))
        verdict = w.malloc(4 * n)
        hdr = w.malloc(16 * n)
        w.sync()
        if emit:
            w.process_batches_emit(bufs, desc, verdict, hdr, n)
        else:
            w.process_batches(bufs, desc, verdict, n)
        w.sync()
        got_v = np.empty(n, np.uint32)
        w.d2h(got_v, verdict)
        rec = np.empty((n, 16), np.uint8)
        w.d2h(rec, hdr)
        frames = []
        for b, wl in zip(bufs, wls):
            f = np.empty(wl.frames.nbytes, np.uint8)
            w.d2h(f, b)
            frames.append(f)
        w.sync()
        counters, stats = w.get_stats()
        l1 = w.get_l1()
    finally:
        w.close()
    last = ref[-1]
    bad = np.nonzero(got_v != last.verdict)[0]
    assert bad.size == 0, f"last batch: {bad.size} verdicts differ, first {bad[:8].tolist()}"
    if emit:
        # frames are only read; the last batch's records rebuild its rewritten frames
        for f, wl in zip(frames, wls):
            assert np.array_equal(f, wl.frames), "emit mode wrote a frame"
        rec = gpu.expand_records(rec, got_v)   # (compacted per 64-packet group)
        assert np.array_equal(gpu.hdr_apply(wls[-1].frames, wls[-1].desc, rec), last.frames)
    else:
        for j, (f, r) in enumerate(zip(frames, ref)):
            assert np.array_equal(f, r.frames), f"batch {j}: rewritten frames differ"
    assert counters.tobytes() == np.asarray(last.counters).tobytes()
    assert np.array_equal(stats, last.rule_stats)
    assert l1.tobytes() == np.asarray(last.l1).tobytes()
