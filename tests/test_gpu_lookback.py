"""GPU: the L1-cache emulation when a batch starts from an entry that disagrees with its table
(reference src/worker.c:186-195, 218-225) — the bounded look-back, its
deferral to the launch's last workgroup (forward progress without co-residency), concurrent
contexts on one GPU, and the switch to (and back from) the kernels without look-back.

UPE_GPU_LB_SPIN=0 makes every wave that finds an unpublished earlier chunk defer at once, so the
repair path answers a large share of the candidates; UPE_GPU_LB_SYNC=1 makes the switch to the
kernel without look-back happen at a known launch (the host waits for each launch's report)."""
from __future__ import annotations

import numpy as np
import pytest

import golden_io
import oracle
from test_gpu_parity import _assert_same, _force_dst, _run
from upe_amd import gpu, synth
from upe_amd.layout import desc_offsets

pytestmark = pytest.mark.gpu


def _expect(wl):
    r = oracle.run_restated(wl)
    return {"verdict": r.verdict, "frames": r.frames, "counters": r.counters,
            "rule_stats": r.rule_stats, "l1": r.l1}


def _aimed_b(n, first_hit, seed=12, ip0=0x0A800007):
    """Config B with a starting ARP entry that disagrees with the table and every packet sent to
    it, except one miss-then-hit packet at `first_hit` (None: none)."""
    wl = synth.config_b(n=n, seed=seed)
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
    return wl


@pytest.mark.parametrize("emit", [False, True])
@pytest.mark.parametrize("n,first_hit", [(300_000, None), (300_000, 150_001), (800_000, 777),
                                         (800_000, 799_000), (2_000_000, 1_500_000)])
def test_deferred_lookback_repaired(gpu_worker_factory, monkeypatch, n, first_hit, emit):
    """Every look-back that meets an unpublished chunk defers (spin 0): the last workgroup's
    repair must give exactly the reference's answers, and it must have had work to do."""
    monkeypatch.setenv("UPE_GPU_LB_SPIN", "0")
    wl = _aimed_b(n, first_hit)
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        got = gpu.run_workload(wl, worker=w, emit=emit)
        info = w.launch_info()
    finally:
        w.close()
    _assert_same(got, _expect(wl), f"n={n} first_hit={first_hit}")
    assert not info["variant"] & gpu.VAR_NOLB
    assert info["deferred"] > 0, info


@pytest.mark.parametrize("emit", [False, True])
def test_deferred_random_l1_starts(gpu_worker_factory, monkeypatch, emit):
    """Config C (IPv4 + IPv6, both families' entries disagreeing or absent) with spin 0."""
    monkeypatch.setenv("UPE_GPU_LB_SPIN", "0")
    rng = np.random.default_rng(17)
    base = synth.config_c(n=300_000, seed=19)
    for trial in range(4):
        wl = base.copy()
        l1 = synth.l1_zero()
        a = wl.arp[rng.choice(np.nonzero(wl.arp["valid"])[0])]
        nd = wl.ndp[rng.choice(np.nonzero(wl.ndp["valid"])[0])]
        l1["last_arp_ip"] = a["ip"]
        l1["last_arp_mac"] = rng.integers(0, 256, 6)
        l1["last_ndp_ip"] = nd["ip"]
        l1["last_ndp_mac"] = rng.integers(0, 256, 6) if trial % 2 else nd["mac"]
        wl.l1 = l1
        _force_dst(wl, 3000 + 5000 * trial, int(l1["last_arp_ip"][0]), l1["last_ndp_ip"][0])
        _assert_same(_run(gpu_worker_factory, wl, emit=emit), _expect(wl), f"trial {trial}")


def test_edge_inconsistent_deferred(gpu_worker_factory, monkeypatch):
    monkeypatch.setenv("UPE_GPU_LB_SPIN", "0")
    wl, _ = golden_io.load("edge_inconsistent")
    r = oracle.run_restated(wl, apply_control=False)
    _assert_same(_run(gpu_worker_factory, wl), {"verdict": r.verdict, "frames": r.frames,
                                                "counters": r.counters,
                                                "rule_stats": r.rule_stats, "l1": r.l1})


@pytest.mark.parametrize("spin", ["0", "5000"])
def test_two_contexts_concurrent(gpu_worker_factory, monkeypatch, spin):
    """Two worker contexts on one GPU, each on its own stream, running look-back-live batches at
    the same time (config C, whose calloc'd NDP entry never agrees with its table, and config B
    started from a disagreeing ARP entry with every packet aimed at it), queued behind a third
    context's stream of 4M-packet launches that holds every CU: neither look-back grid is wholly
    resident when it starts, its workgroups are dispatched into the gaps the other launches
    leave.  Each context's results equal the oracle's."""
    monkeypatch.setenv("UPE_GPU_LB_SPIN", spin)
    wc = synth.config_c(n=1 << 20, seed=23)
    wb = _aimed_b(800_000, 600_000, seed=24)
    wh = synth.config_b(n=1 << 22, seed=25)
    want_c, want_b = _expect(wc), _expect(wb)
    hog = gpu_worker_factory(wh.capacity)
    hog.configure(wh)
    hb = gpu.DeviceBatch(hog, wh.frames, wh.desc)
    deferred = []
    try:
        for rep in range(3):
            workers = [gpu_worker_factory(wc.capacity), gpu_worker_factory(wb.capacity)]
            try:
                batches = []
                for w, wl in zip(workers, (wc, wb)):
                    w.configure(wl)
                    batches.append(gpu.DeviceBatch(w, wl.frames, wl.desc))
                hog.process_batches([hb.frames] * 12, hb.desc, hb.verdict, hb.n)
                for b in batches:   # each context's own stream
                    b.run_emit() if rep % 2 else b.run()
                for w, b, wl, want in zip(workers, batches, (wc, wb), (want_c, want_b)):
                    frames, verdict = b.fetch()
                    if rep % 2:
                        frames = gpu.hdr_apply(frames, wl.desc, b.fetch_hdr())
                    b.free()
                    counters, stats = w.get_stats()
                    _assert_same((frames, verdict, counters, stats, w.get_l1()), want,
                                 f"{wl.name} rep {rep} spin {spin}")
                    deferred.append(w.launch_info()["deferred"])
            finally:
                for w in workers:
                    w.close()
        hog.sync()
    finally:
        hb.free()
        hog.close()
    print("deferred look-back entries per launch:", deferred)


def test_no_lookback_switch_with_empty_index(gpu_worker_factory, monkeypatch):
    """ARP entry disagreeing with an EMPTY ARP table: once a launch has reported, the kernel
    without look-back runs, and it answers the packets aimed at the entry from the entry itself
    (no packet can hit the empty table first) — checked against the oracle over three batches."""
    monkeypatch.setenv("UPE_GPU_LB_SYNC", "1")
    wl = synth.config_b(n=90_000, seed=31)
    wl.arp = np.zeros_like(wl.arp)
    l1 = synth.l1_zero()
    l1["last_arp_ip"] = 0x0A800009
    l1["last_arp_mac"] = np.frombuffer(bytes.fromhex("020406080a0c"), np.uint8)
    wl.l1 = l1
    _force_dst(wl, 40_000, 0x0A800009)
    want = _expect(wl)
    variants = []
    got = _run_batches(gpu_worker_factory, wl, 3, variants)
    _assert_same(got, want, "empty ARP index", batch_relative=True)
    assert not variants[0] & gpu.VAR_NOLB and variants[1] & gpu.VAR_NOLB and variants[2] & gpu.VAR_NOLB, variants


def test_lookback_returns_after_set_l1_and_load_neigh(gpu_worker_factory, monkeypatch):
    """Agreement reached (kernel without look-back), then set_l1 to a disagreeing entry: the
    next launch runs the look-back again; then load_neigh does the same.  Exact throughout."""
    monkeypatch.setenv("UPE_GPU_LB_SYNC", "1")
    wl = synth.config_b(n=200_000, seed=32)
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        r = oracle.run_restated(wl)
        variants = []
        for k in range(3):
            frames, verdict, _, _, _ = _one(w, wl)
            variants.append(w.launch_info()["variant"])
        assert variants[-1] & gpu.VAR_NOLB, variants
        # a disagreeing entry aimed at by the next batch
        l1 = w.get_l1()
        l1["last_arp_mac"] = np.frombuffer(bytes.fromhex("0e0e0e0e0e0e"), np.uint8)
        wl2 = wl.copy()
        wl2.l1 = l1.copy()
        _force_dst(wl2, 30_000, int(l1["last_arp_ip"][0]))
        w.set_l1(l1)
        w.reset_stats()
        frames, verdict, _, _, _ = _one(w, wl2)
        assert not w.launch_info()["variant"] & gpu.VAR_NOLB
        r2 = oracle.run_restated(wl2)
        assert np.array_equal(verdict, r2.verdict)
        assert np.array_equal(frames, r2.frames)
        assert w.get_l1().tobytes() == r2.l1.tobytes()
        # reach agreement again, then a table change
        for k in range(2):
            _one(w, wl)
        assert w.launch_info()["variant"] & gpu.VAR_NOLB
        w.load_neigh(wl.arp, wl.ndp)
        _one(w, wl)
        assert not w.launch_info()["variant"] & gpu.VAR_NOLB
    finally:
        w.close()
    assert r.verdict.size == wl.n


def _one(w, wl):
    b = gpu.DeviceBatch(w, wl.frames, wl.desc)
    b.run()
    frames, verdict = b.fetch()
    b.free()
    return frames, verdict, None, None, None


def _run_batches(worker_factory, wl, batches, variants):
    w = worker_factory(wl.capacity)
    try:
        w.configure(wl)
        frames = wl.frames.copy()
        verdict = np.zeros(wl.n, np.uint32)
        bounds = np.linspace(0, wl.n, batches + 1).astype(int)
        for s, e in zip(bounds[:-1], bounds[1:]):
            b = gpu.DeviceBatch(w, frames, wl.desc[s:e])
            b.run()
            frames, verdict[s:e] = b.fetch()
            b.free()
            variants.append(w.launch_info()["variant"])
        counters, stats = w.get_stats()
        return frames, verdict, counters, stats, w.get_l1()
    finally:
        w.close()
