"""upe_gpu_process_segmented: control packets (ARP learn / reply, NDP NS / NA) inside a device
batch with the reference's sequential table-write semantics (src/worker.c:23-104 within the burst
loop), against the reference's edge goldens and against the
reference worker (oracle/_ref, or the C restatement with control replay) on synthetic streams
where the learned entries change how later packets are forwarded."""
from __future__ import annotations

import numpy as np
import pytest

import golden_io
import oracle
from test_gpu_parity import _assert_same
from upe_amd import gpu, synth
from upe_amd.layout import desc_lens, desc_offsets

pytestmark = pytest.mark.gpu

KEEP = ["ip", "mac", "valid"]


def _segmented(worker_factory, wl):
    w = worker_factory(wl.capacity)
    try:
        w.configure(wl)
        arp, ndp = wl.arp.copy(), wl.ndp.copy()
        b = gpu.DeviceBatch(w, wl.frames, wl.desc)
        writes = w.process_segmented(b.frames, b.desc, b.verdict, b.n, arp, ndp, now=1234)
        frames, verdict = b.fetch()
        b.free()
        counters, stats = w.get_stats()
        l1 = w.get_l1()
    finally:
        w.close()
    return (frames, verdict, counters, stats, l1), arp, ndp, writes


@pytest.mark.parametrize("case", ["edge_zero", "edge_consistent", "edge_inconsistent",
                                  "ndp_walk"])
def test_edge_goldens_native_segmented(gpu_worker_factory, case):
    """ndp_walk: NS / NA frames up to 400 bytes whose option walk crosses the uint8_t opt_len
    wrap of src/worker.c:73 (length bytes 32, 33, 64), each followed by packets to the address
    it may teach."""
    wl, ref = golden_io.load(case)
    got, arp, ndp, writes = _segmented(gpu_worker_factory, wl)
    _assert_same(got, ref, case, batch_relative=True)
    assert np.array_equal(arp[KEEP], ref["arp"][KEEP])
    assert np.array_equal(ndp[KEEP], ref["ndp"][KEEP])
    assert writes > 0
    # every table write the reference made carries the caller's timestamp
    changed = (arp["valid"] != 0) & (wl.arp["mac"] != arp["mac"]).any(axis=1)
    assert np.all(arp["update_at"][changed] == 1234)
    if case == "ndp_walk":
        # the wrap decides what is learned: length byte 32 / 64 teaches nothing, 33 the option
        # 8 bytes on (MAC 0a:..), never the one 264 bytes on (MAC 0b:..)
        learned = {bytes(e["ip"])[-1]: bytes(e["mac"]) for e in ndp[ndp["valid"] != 0]}
        assert 0x00 not in learned and 0x02 not in learned and 0x06 not in learned
        assert learned[0x01][0] == 0x0A and learned[0x04][0] == 0x0A


def _rows(wl):
    """First 128 bytes of every frame (zero past len) and the lengths."""
    offs, lens = desc_offsets(wl.desc), desc_lens(wl.desc)
    h = np.zeros((wl.n, 128), np.uint8)
    for i in range(wl.n):
        k = int(min(lens[i], 128))
        h[i, :k] = wl.frames[offs[i]:offs[i] + k]
    return h, lens.astype(np.int64)


def with_control(wl, k, seed):
    """wl with k control packets inserted at random positions.  ARP packets teach the MACs of
    IPv4 destinations that later packets go to (new entries and changed ones), some ask for the
    port address (in-place reply); NS / NA teach IPv6 destinations; a few carry no usable
    address (wrong hlen, no option) and must leave the tables alone."""
    rng = np.random.default_rng(seed)
    h, lens = _rows(wl)
    et = (h[:, 12].astype(np.int64) << 8) | h[:, 13]
    v4 = np.nonzero(et == 0x0800)[0]
    v6 = np.nonzero(et == 0x86DD)[0]
    ctrl = []
    for j in range(k):
        mac = bytes(rng.integers(0, 256, 6, dtype=np.uint8))
        kind = rng.integers(0, 6)
        if kind <= 1 and len(v4):
            dst = int.from_bytes(bytes(h[rng.choice(v4), 30:34]), "big")
            tpa = synth.PORT_IP4 if kind == 1 else 0x0A800001
            f = synth._frame(synth._eth(0x0806, dst=b"\xff" * 6),
                             synth._arp(1, mac, dst, bytes(6), tpa))
        elif kind == 2 and len(v4):
            dst = int.from_bytes(bytes(h[rng.choice(v4), 30:34]), "big")
            f = synth._frame(synth._eth(0x0806), synth._arp(1, mac, dst, bytes(6), 0, hlen=8))
        elif kind == 3 and len(v6):
            dst = bytes(h[rng.choice(v6), 38:54])
            f = synth._frame(synth._eth(0x86DD), synth._ip6(58, dst, bytes(16)),
                             bytes([135, 0, 0, 0, 0, 0, 0, 0]) + bytes(16), bytes([1, 1]) + mac)
        elif kind == 4 and len(v6):
            dst = bytes(h[rng.choice(v6), 38:54])
            f = synth._frame(synth._eth(0x86DD), synth._ip6(58, bytes(16), dst),
                             bytes([136, 0, 0, 0, 0x60, 0, 0, 0]) + dst,
                             bytes([5, 1]) + bytes(6) + bytes([2, 1]) + mac)
        else:
            f = synth._frame(synth._eth(0x86DD), synth._ip6(58, bytes(16), bytes(16)),
                             bytes([135, 0, 0, 0, 0, 0, 0, 0]) + bytes(16))
        ctrl.append(f)
    pos = np.sort(rng.integers(0, wl.n + 1, k))
    rows, lns = [], []
    src = 0
    for p, f in zip(pos, ctrl):
        rows.append(h[src:p])
        lns.append(lens[src:p])
        r = np.zeros((1, 128), np.uint8)
        r[0, :len(f)] = np.frombuffer(f, np.uint8)
        rows.append(r)
        lns.append(np.array([len(f)], np.int64))
        src = p
    rows.append(h[src:])
    lns.append(lens[src:])
    frames, desc = synth.pack_frames(np.concatenate(rows), np.concatenate(lns))
    return synth.Workload(wl.name + "+ctrl", frames, desc, wl.rules, wl.capacity, wl.arp.copy(),
                          wl.ndp.copy(), wl.eth_addr, wl.ip4_addr, wl.l1.copy())


def _expected(wl):
    if oracle.ref_available():
        return oracle.run_reference(wl)
    return oracle.run_restated(wl, apply_control=True)


@pytest.mark.parametrize("seed,n,k", [(31, 4000, 40), (32, 20000, 200), (33, 60000, 7)])
def test_learned_entries_change_forwarding(gpu_worker_factory, seed, n, k):
    wl = with_control(synth.config_c(n=n, seed=seed), k, seed)
    r = _expected(wl)
    got, arp, ndp, writes = _segmented(gpu_worker_factory, wl)
    ref = {"verdict": r.verdict, "frames": r.frames, "counters": r.counters,
           "rule_stats": r.rule_stats, "l1": r.l1}
    _assert_same(got, ref, f"seed {seed}", batch_relative=True)
    assert np.array_equal(arp[KEEP], r.arp[KEEP])
    assert np.array_equal(ndp[KEEP], r.ndp[KEEP])
    assert 0 < writes <= k
    # the learning mattered: a run with the tables frozen forwards differently
    frozen = oracle.run_restated(wl, apply_control=False)
    assert not np.array_equal(frozen.frames, r.frames)


def test_no_control_packets_is_one_batch(gpu_worker_factory):
    wl = synth.config_b(n=50000, seed=8)
    got, arp, ndp, writes = _segmented(gpu_worker_factory, wl)
    r = oracle.run_restated(wl)
    _assert_same(got, {"verdict": r.verdict, "frames": r.frames, "counters": r.counters,
                       "rule_stats": r.rule_stats, "l1": r.l1}, "config B")
    assert writes == 0
    assert np.array_equal(arp, wl.arp) and np.array_equal(ndp, wl.ndp)


def test_empty_batch(gpu_worker_factory):
    wl = synth.config_b(n=16, seed=8)
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        dev = w.malloc(256)
        assert w.process_segmented(dev, dev, dev, 0, wl.arp.copy(), wl.ndp.copy()) == 0
        w.free(dev)
    finally:
        w.close()
