"""GPU: the ring launch (upe_gpu_process_ring_emit) — `count` resident batches classified by one
persistent launch — gives exactly what back-to-back batches give (every verdict code, record,
counter, rule_stat and the final L1 state; UPE_VF_L1_INIT relative to the ring's start), and
stamps each batch's completion."""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from test_emit_records import records_from_reference
from test_gpu_parity import _assert_same
from upe_amd import gpu, synth

pytestmark = pytest.mark.gpu


def _ring(w, wl, per, count):
    b = gpu.DeviceBatch(w, wl.frames, wl.desc)
    b.hdr = w.malloc(16 * wl.n)
    done = w.malloc(8 * count)
    w.process_ring_emit(b.frames, b.desc, b.verdict, b.hdr, per, count, done)
    frames, verdict = b.fetch()
    rec = b.fetch_hdr()
    stamps = np.zeros(count, np.uint64)
    w.d2h(stamps, done)
    w.sync()
    w.free(done)
    b.free()
    return frames, verdict, rec, stamps


@pytest.mark.parametrize("config,per,count", [("B", 262144, 4), ("C", 262144, 3),
                                              ("B", 1024, 9), ("C", 8192, 5)])
def test_ring_equals_one_stream(gpu_worker_factory, config, per, count):
    make = synth.config_b if config == "B" else synth.config_c
    wl = make(n=per * count, seed=90 + count)
    r = oracle.run_restated(wl)
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        frames, verdict, rec, stamps = _ring(w, wl, per, count)
        counters, stats = w.get_stats()
        l1 = w.get_l1()
        info = w.launch_info()
    finally:
        w.close()
    assert np.array_equal(frames, wl.frames), "the ring wrote into the frames"
    want = records_from_reference(wl.frames, r.frames, wl.desc, r.verdict)
    assert np.array_equal(rec, want), "records differ from the reference's rewritten frames"
    applied = gpu.hdr_apply(frames, wl.desc, rec)
    _assert_same((applied, verdict, counters, stats, l1),
                 {"verdict": r.verdict, "frames": r.frames, "counters": r.counters,
                  "rule_stats": r.rule_stats, "l1": r.l1}, f"ring {config} {per}x{count}")
    if per >= 262144:   # at least one tile of every batch per persistent workgroup: stamped
        assert info["variant"] & gpu.VAR_RING, info
        assert np.all(stamps > 0), stamps
        assert stamps[-1] >= stamps[0]
    else:
        assert np.all(stamps == 0), stamps


def test_ring_equals_batches(gpu_worker_factory):
    """The same packets as `count` separate upe_gpu_process_emit calls: verdicts (L1_INIT aside),
    records, counters and rule_stats identical."""
    per, count = 262144, 4
    wl = synth.config_b(n=per * count, seed=97)
    w1, w2 = gpu_worker_factory(wl.capacity), gpu_worker_factory(wl.capacity)
    try:
        w1.configure(wl)
        w2.configure(wl)
        _, v_ring, rec_ring, _ = _ring(w1, wl, per, count)
        v_b = np.zeros(wl.n, np.uint32)
        rec_b = np.zeros((wl.n, 16), np.uint8)
        for k in range(count):
            sub = wl.desc[k * per:(k + 1) * per]
            b = gpu.DeviceBatch(w2, wl.frames, sub)
            b.run_emit()
            _, v_b[k * per:(k + 1) * per] = b.fetch()
            rec_b[k * per:(k + 1) * per] = b.fetch_hdr()
            b.free()
        assert np.array_equal(v_ring & ~np.uint32(0x80), v_b & ~np.uint32(0x80))
        assert np.array_equal(rec_ring, rec_b)
        c1, s1 = w1.get_stats()
        c2, s2 = w2.get_stats()
        assert c1.tobytes() == c2.tobytes() and np.array_equal(s1, s2)
        assert w1.get_l1().tobytes() == w2.get_l1().tobytes()
    finally:
        w1.close()
        w2.close()


def test_ring_rejects_bad_shapes(gpu_worker_factory):
    wl = synth.config_b(n=4096, seed=3)
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        b = gpu.DeviceBatch(w, wl.frames, wl.desc)
        b.hdr = w.malloc(16 * wl.n)
        with pytest.raises(gpu.UpeGpuError):
            w.process_ring_emit(b.frames, b.desc, b.verdict, b.hdr, 1000, 4)   # not 1024-aligned
        with pytest.raises(gpu.UpeGpuError):
            w.process_ring_emit(b.frames, b.desc, b.verdict, b.hdr, 1 << 22, 8)  # over 2^24
        b.free()
    finally:
        w.close()
