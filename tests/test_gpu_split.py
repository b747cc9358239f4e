"""GPU parity of the header-split batch (upe_gpu_process_split_emit): each packet's first 64
bytes in a dense row of their own (as a NIC's header-data split lays them out), the full frames
beside them; the kernel reads bytes 0..63 from the rows and the rest from the frames.  Every
verdict bit, record, counter, rule_stats word and the L1 state must equal the reference worker's
(goldens, full-size digests) and the oracle's (edge sets in one segment, ragged sizes)."""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

import golden_io
import oracle
from test_gpu_parity import _assert_same
from upe_amd import gpu, synth

pytestmark = pytest.mark.gpu

VAR_SPLIT = gpu.VAR_SPLIT


def _split_run(w, wl):
    """(frames as the reference leaves them, verdict, counters, stats, l1) of one split call."""
    rows = synth.header_rows(wl)
    b = gpu.DeviceBatch(w, wl.frames, wl.desc)
    d_rows = w.malloc(rows.nbytes)
    w.h2d(d_rows, rows)
    b.hdr = w.malloc(max(16 * wl.n, 16))
    try:
        w.process_split_emit(d_rows, b.frames, b.desc, b.verdict, b.hdr, wl.n)
        w.sync()
        if wl.n:
            assert w.launch_info()["variant"] & VAR_SPLIT, "not the header-split kernel"
        frames, verdict = b.fetch()
        frames = gpu.hdr_apply(frames, wl.desc, b.fetch_hdr())
    finally:
        w.free(d_rows)
        b.free()
    counters, stats = w.get_stats()
    return frames, verdict, counters, stats, w.get_l1()


def _with(gpu_worker_factory, wl):
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        return _split_run(w, wl)
    finally:
        w.close()


def _oracle_ref(wl, apply_control=True):
    r = oracle.run_restated(wl, apply_control=apply_control)
    return {"verdict": r.verdict, "frames": r.frames, "counters": r.counters,
            "rule_stats": r.rule_stats, "l1": r.l1}


@pytest.mark.parametrize("case", ["config_a", "config_b_small", "config_c_small",
                                  "config_d_small"])
def test_split_golden(gpu_worker_factory, case):
    wl, ref = golden_io.load(case)
    _assert_same(_with(gpu_worker_factory, wl), ref, f"split {case}")


@pytest.mark.parametrize("case", ["edge_zero", "edge_consistent", "edge_inconsistent"])
def test_split_edges_vs_oracle(gpu_worker_factory, case):
    """Every parse gate, truncation (rows zero past len), IHL options reaching past byte 64, ARP
    request / reply (rewritten in its frame) and NS / NA in one batch."""
    wl, _ = golden_io.load(case)
    _assert_same(_with(gpu_worker_factory, wl), _oracle_ref(wl, apply_control=False), case)


@pytest.mark.parametrize("n", [1, 63, 65, 1000, 16385])
def test_split_ragged_sizes(gpu_worker_factory, n):
    wl = synth.config_c(n=n, seed=1900 + n)
    _assert_same(_with(gpu_worker_factory, wl), _oracle_ref(wl), f"split n={n}")


def _sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


@pytest.mark.parametrize("key,make", [("B_1M", lambda: synth.config_b()),
                                      ("C_1M", lambda: synth.config_c()),
                                      ("D_256k_64k_rules", lambda: synth.config_d(n=1 << 18))])
def test_split_full_size_digest(gpu_worker_factory, key, make):
    dg = golden_io.digests()[key]
    wl = make()
    assert _sha(wl.frames, wl.desc, wl.rules, wl.arp, wl.ndp) == dg["inputs"]
    frames, verdict, counters, stats, l1 = _with(gpu_worker_factory, wl)
    assert [int(x) for x in counters[0].tolist()] == dg["counters"]
    assert _sha(verdict) == dg["verdict"]
    assert _sha(frames) == dg["frames"]
    assert _sha(stats) == dg["rule_stats"]
    assert _sha(l1) == dg["l1"]


def test_split_then_packed_carry(gpu_worker_factory):
    """A split batch then an ordinary one on the same worker: the state carries as between any
    two batches."""
    wl = synth.config_c(n=120_000, seed=77)
    half = 50_000
    first = synth.Workload(wl.name, wl.frames, wl.desc[:half].copy(), wl.rules, wl.capacity,
                           wl.arp, wl.ndp, wl.eth_addr, wl.ip4_addr, wl.l1)
    w = gpu_worker_factory(wl.capacity)
    ref_w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        ref_w.configure(wl)
        _split_run(w, first)
        b = gpu.DeviceBatch(w, wl.frames, wl.desc[half:])
        b.run_emit()
        _, v2 = b.fetch()
        r2h = b.fetch_hdr()
        b.free()
        r1 = gpu.DeviceBatch(ref_w, wl.frames, wl.desc[:half])
        r1.run_emit()
        r2 = gpu.DeviceBatch(ref_w, wl.frames, wl.desc[half:])
        r2.run_emit()
        _, rv2 = r2.fetch()
        rr2h = r2.fetch_hdr()
        r1.free()
        r2.free()
        assert np.array_equal(v2, rv2) and np.array_equal(r2h, rr2h)
        c1, s1 = w.get_stats()
        c2, s2 = ref_w.get_stats()
        assert c1.tobytes() == c2.tobytes() and np.array_equal(s1, s2)
        assert w.get_l1().tobytes() == ref_w.get_l1().tobytes()
    finally:
        w.close()
        ref_w.close()
