"""GPU: the worker loop queued from native code (upe_gpu_process_queue_emit, one launch per
batch) gives exactly what the same batches give as one upe_gpu_process_emit() call after
another: every verdict word (UPE_VF_L1_INIT included: both are per batch), record, counter,
rule_stat and the final L1 state, on ragged batches (an empty one among them), look-back-live
batches and beside a second context's concurrent queue; a batch without records is refused
before anything is queued.  The worker state carried from batch to batch is the reference's
(src/worker.c:255-307 over src/worker.c:186-195, 218-225)."""
from __future__ import annotations

import threading

import numpy as np
import pytest

import oracle
from test_gpu_parity import _assert_same
from upe_amd import gpu, synth
from upe_amd.layout import desc_offsets

pytestmark = pytest.mark.gpu


def _run(w, wl, bounds, queue: bool):
    """The workload's batches [bounds[i], bounds[i+1]) as one queue or one call each; returns
    (frames, verdict, records) of the whole stream."""
    b = gpu.DeviceBatch(w, wl.frames, wl.desc)
    b.hdr = w.malloc(16 * max(wl.n, 1))
    parts = [(b.frames, b.desc + 8 * s, b.verdict + 4 * s, b.hdr + 16 * s, e - s)
             for s, e in zip(bounds[:-1], bounds[1:])]
    if queue:
        w.process_queue_emit(parts)
    else:
        for p in parts:
            w.process_emit(*p)
    frames, verdict = b.fetch()
    raw = b.fetch_hdr(raw=True)
    b.free()
    # each batch's records are compacted per 64-packet group counted from its own first packet
    rec = np.zeros_like(raw)
    for s, e in zip(bounds[:-1], bounds[1:]):
        rec[s:e] = gpu.expand_records(raw[s:e], verdict[s:e])
    return frames, verdict, rec


def _both(factory, wl, bounds):
    out = []
    for queue in (True, False):
        w = factory(wl.capacity)
        try:
            w.configure(wl)
            before = w.launch_info()["launches"]
            frames, verdict, rec = _run(w, wl, bounds, queue)
            counters, stats = w.get_stats()
            out.append(dict(frames=frames, verdict=verdict, rec=rec, counters=counters,
                            stats=stats, l1=w.get_l1(),
                            launches=w.launch_info()["launches"] - before))
        finally:
            w.close()
    return out


def _check(q, s, wl, what):
    assert np.array_equal(q["frames"], wl.frames), f"{what}: the queue wrote into the frames"
    bad = np.nonzero(q["verdict"] != s["verdict"])[0]
    assert bad.size == 0, (f"{what}: {bad.size} verdicts differ from sequential launches, first "
                           f"{bad[:8].tolist()}")
    assert np.array_equal(q["rec"], s["rec"]), f"{what}: records differ"
    assert q["counters"].tobytes() == s["counters"].tobytes(), f"{what}: counters differ"
    assert np.array_equal(q["stats"], s["stats"]), f"{what}: rule_stats differ"
    assert q["l1"].tobytes() == s["l1"].tobytes(), f"{what}: L1 state differs"


def _against_oracle(q, wl, what):
    """The whole stream through the restated worker: the verdicts (L1_INIT aside: it is defined
    per batch), the records applied to the frames, counters, rule_stats and L1 state."""
    r = oracle.run_restated(wl)
    applied = gpu.hdr_apply(q["frames"], wl.desc, q["rec"])
    _assert_same((applied, q["verdict"], q["counters"], q["stats"], q["l1"]),
                 {"verdict": r.verdict, "frames": r.frames, "counters": r.counters,
                  "rule_stats": r.rule_stats, "l1": r.l1}, what, batch_relative=True)


@pytest.mark.parametrize("config,n,cuts", [
    ("B", 600_000, [262_144, 262_209, 400_000, 400_001]),
    ("C", 500_000, [1, 64, 100_000, 100_000, 300_000, 300_063]),   # an empty batch in the middle
    ("B", 40_000, list(range(1000, 40_000, 1000))),
    ("C", 48_000, list(range(3000, 48_000, 3000))),
])
def test_queue_equals_sequential(gpu_worker_factory, config, n, cuts):
    make = synth.config_b if config == "B" else synth.config_c
    wl = make(n=n, seed=71 + len(cuts))
    bounds = [0] + cuts + [n]
    q, s = _both(gpu_worker_factory, wl, bounds)
    what = f"queue {config} {n} in {len(bounds) - 1}"
    _check(q, s, wl, what)
    assert q["launches"] == s["launches"], (q["launches"], s["launches"])
    _against_oracle(q, wl, what)


@pytest.mark.parametrize("first_hit", [None, 5, 150_001, 299_999])
def test_queue_lookback_live(gpu_worker_factory, first_hit):
    """Batches that start from an ARP entry disagreeing with the table, every packet aimed at it
    (the look-back live in every launch until a packet misses the entry and hits the table):
    the state each batch hands the next decides every NEIGH_HIT and MAC."""
    n = 300_000
    wl = synth.config_b(n=n, seed=12)
    ip0 = 0x0A800007
    l1 = synth.l1_zero()
    l1["last_arp_ip"] = ip0
    l1["last_arp_mac"] = np.frombuffer(bytes.fromhex("0badc0ffee01"), np.uint8)
    wl.l1 = l1
    offs = desc_offsets(wl.desc)
    dst = np.frombuffer(ip0.to_bytes(4, "big"), np.uint8)
    wl.frames[(offs[:, None] + np.arange(30, 34)[None, :]).ravel()] = np.tile(dst, wl.n)
    if first_hit is not None:
        other = np.frombuffer((0x0A800000 + int(wl.arp["ip"][wl.arp["valid"] == 1][0] & 0xFF))
                              .to_bytes(4, "big"), np.uint8)
        wl.frames[offs[first_hit] + 30:offs[first_hit] + 34] = other
        wl.frames[offs[first_hit] + 22] = 64
        wl.frames[offs[first_hit] + 36:offs[first_hit] + 38] = [0, 53]
    bounds = [0, 100_000, 150_000, 150_002, 220_000, n]
    q, s = _both(gpu_worker_factory, wl, bounds)
    _check(q, s, wl, f"look-back queue first_hit={first_hit}")
    _against_oracle(q, wl, f"look-back queue first_hit={first_hit}")


def test_queue_shared_outputs(gpu_worker_factory):
    """upe_gpu_process_batches_emit: distinct frame copies sharing one descriptor, verdict and
    record array — every batch's stores land after the previous batch's, so the arrays end
    holding the last batch's outputs, and the counters are those of all batches."""
    n = 262_144
    wls = [synth.config_b(n=n, seed=s) for s in (5, 6, 7)]
    assert all(np.array_equal(x.desc, wls[0].desc) for x in wls)
    res = []
    for queue in (True, False):
        w = gpu_worker_factory(wls[0].capacity)
        try:
            w.configure(wls[0])
            bs = [gpu.DeviceBatch(w, x.frames, x.desc) for x in wls]
            hdr = w.malloc(16 * n)
            if queue:
                w.process_batches_emit([b.frames for b in bs], bs[0].desc, bs[0].verdict, hdr, n)
            else:
                for b in bs:
                    w.process_emit(b.frames, bs[0].desc, bs[0].verdict, hdr, n)
            _, verdict = bs[0].fetch()
            rec = np.empty((n, 16), np.uint8)
            w.d2h(rec, hdr)
            w.sync()
            rec = gpu.expand_records(rec, verdict)   # (compacted per 64-packet group)
            counters, stats = w.get_stats()
            res.append((verdict, rec, counters.tobytes(), stats.copy(), w.get_l1().tobytes()))
            w.free(hdr)
            for b in bs:
                b.free()
        finally:
            w.close()
    (vq, rq, cq, sq, lq), (vs, rs, cs, ss, ls) = res
    assert np.array_equal(vq, vs) and np.array_equal(rq, rs)
    assert cq == cs and np.array_equal(sq, ss) and lq == ls


def test_queue_two_contexts_concurrently(gpu_worker_factory):
    """Two contexts' queues at the same time from two host threads (their launches compete for
    the CUs): each equals its own sequential run."""
    wls = [synth.config_c(n=400_000, seed=31), synth.config_b(n=500_000, seed=32)]
    bounds = [[0, 50_000, 150_000, 151_000, 300_000, 400_000],
              [0, 1, 100_000, 262_144, 262_145, 500_000]]
    ws = [gpu_worker_factory(x.capacity) for x in wls]
    got = [None, None]
    errs = []
    try:
        for w, x in zip(ws, wls):
            w.configure(x)

        def go(i):
            try:
                got[i] = _run(ws[i], wls[i], bounds[i], True)
            except Exception as e:   # reported below
                errs.append(e)

        ts = [threading.Thread(target=go, args=(i,)) for i in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=120)
        assert not errs, errs
        stats = [w.get_stats() for w in ws]
        l1s = [w.get_l1() for w in ws]
    finally:
        for w in ws:
            w.close()
    for i in range(2):
        frames, verdict, rec = got[i]
        q = dict(frames=frames, verdict=verdict, rec=rec, counters=stats[i][0],
                 stats=stats[i][1], l1=l1s[i])
        _against_oracle(q, wls[i], f"concurrent queue {i}")


def test_queue_large_tables(gpu_worker_factory):
    """Tables over 4096 rules (rule_stats by a group-by launch after each classify)."""
    wl = synth.config_d(n=40_000)
    bounds = [0, 10_000, 10_001, 25_000, 40_000]
    q, s = _both(gpu_worker_factory, wl, bounds)
    _check(q, s, wl, "queue D")
    _against_oracle(q, wl, "queue D")


def test_queue_rejects_missing_records(gpu_worker_factory):
    """A batch of n > 0 packets without records: the call fails and queues nothing."""
    wl = synth.config_b(n=4096, seed=3)
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        b = gpu.DeviceBatch(w, wl.frames, wl.desc)
        b.hdr = w.malloc(16 * wl.n)
        before = w.launch_info()["launches"]
        with pytest.raises(gpu.UpeGpuError):
            w.process_queue_emit([(b.frames, b.desc, b.verdict, b.hdr, 2048),
                                  (b.frames, b.desc, b.verdict, 0, 2048)])
        assert w.launch_info()["launches"] == before
        b.free()
    finally:
        w.close()
