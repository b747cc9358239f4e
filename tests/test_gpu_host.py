"""GPU parity of the host round trip (upe_gpu_process_host: host batch -> H2D -> classify ->
D2H of verdicts and rewritten header bytes, pipelined in chunks), against the reference's golden
vectors and the oracle.  Chunked processing must equal back-to-back batches, i.e. the reference
worker's sequential result (only UPE_VF_L1_INIT is relative to each chunk's start)."""
from __future__ import annotations

import numpy as np
import pytest

import golden_io
import oracle
from upe_amd import gpu, synth
from upe_amd.layout import REWRITE_EXTENT, desc_lens, desc_offsets

pytestmark = pytest.mark.gpu

L1_INIT = np.uint32(0x80)


def _check(w, wl, frames, verdict, ref, what):
    bad = np.nonzero((verdict & ~L1_INIT) != (ref["verdict"] & ~L1_INIT))[0]
    assert bad.size == 0, f"{what}: {bad.size} verdicts differ, first {bad[:8].tolist()}"
    assert np.array_equal(frames, ref["frames"]), f"{what}: frames differ"
    counters, stats = w.get_stats()
    assert counters.tobytes() == np.asarray(ref["counters"]).tobytes(), what
    assert np.array_equal(stats, ref["rule_stats"]), what
    assert w.get_l1().tobytes() == np.asarray(ref["l1"]).tobytes(), what


@pytest.mark.parametrize("case", ["config_b_small", "config_c_small", "config_d_small"])
@pytest.mark.parametrize("chunk,pinned", [(1000, True), (333, False), (0, True)])
def test_host_roundtrip_golden(gpu_worker_factory, case, chunk, pinned):
    wl, ref = golden_io.load(case)
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        if pinned:
            pf = gpu.PinnedArray(wl.frames.shape, np.uint8)
            pd = gpu.PinnedArray(wl.desc.shape, np.uint64)
            pv = gpu.PinnedArray((wl.n,), np.uint32)
            frames, desc, verdict = pf.array, pd.array, pv.array
        else:
            frames, desc, verdict = np.empty_like(wl.frames), np.empty_like(wl.desc), \
                np.zeros(wl.n, np.uint32)
        frames[:] = wl.frames
        desc[:] = wl.desc
        w.process_host(frames, desc, verdict, chunk)
        _check(w, wl, frames, verdict, ref, f"{case} chunk={chunk} pinned={pinned}")
        if pinned:
            for x in (pf, pd, pv):
                x.free()
    finally:
        w.close()


def test_host_roundtrip_header_windows(gpu_worker_factory):
    """IMIX shipped as 96-byte header windows: same verdicts, counters and rule_stats as the full
    frames, and the written-back window bytes equal the reference's rewritten frame bytes."""
    wl, ref = golden_io.load("config_c_small")
    hw = synth.header_windows(wl)
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        frames = hw.frames.copy()
        verdict = np.zeros(wl.n, np.uint32)
        w.process_host(frames, hw.desc, verdict, 1500)
        assert np.array_equal(verdict & ~L1_INIT, ref["verdict"] & ~L1_INIT)
        counters, stats = w.get_stats()
        assert counters.tobytes() == np.asarray(ref["counters"]).tobytes()
        assert np.array_equal(stats, ref["rule_stats"])
        offs, woffs, lens = desc_offsets(wl.desc), desc_offsets(hw.desc), desc_lens(wl.desc)
        for i in range(wl.n):
            k = int(min(lens[i], REWRITE_EXTENT))
            assert np.array_equal(frames[woffs[i]:woffs[i] + k], ref["frames"][offs[i]:offs[i] + k])
    finally:
        w.close()


def test_host_roundtrip_full_size_b(gpu_worker_factory):
    """Config B at 1M through the host path: equals the oracle's sequential run."""
    wl = synth.config_b()
    r = oracle.run_restated(wl)
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        frames = wl.frames.copy()
        verdict = np.zeros(wl.n, np.uint32)
        w.process_host(frames, wl.desc, verdict)
        _check(w, wl, frames, verdict, {"verdict": r.verdict, "frames": r.frames,
                                        "counters": r.counters, "rule_stats": r.rule_stats,
                                        "l1": r.l1}, "B 1M host")
    finally:
        w.close()


def test_host_roundtrip_rejects_short_buffer(gpu_worker_factory):
    wl, _ = golden_io.load("config_b_small")
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        verdict = np.zeros(wl.n, np.uint32)
        with pytest.raises(gpu.UpeGpuError):
            w.process_host(wl.frames[: int(desc_offsets(wl.desc)[-1]) + 8].copy(), wl.desc, verdict)
    finally:
        w.close()


@pytest.mark.parametrize("chunk", [257, 4096])
def test_host_roundtrip_permuted_descriptors(gpu_worker_factory, chunk):
    """Descriptors in pool order, not address order (include/upe_gpu.h allows any order): every
    chunk's byte span interleaves with its neighbours', so a chunk's copy-back also rewrites
    frames of the chunks before and after it.  The round trip must wait for those and end with
    exactly the oracle's bytes for every frame."""
    import dataclasses

    base = synth.config_c(n=60_000, seed=71)
    perm = np.random.default_rng(71).permutation(base.n)
    wl = dataclasses.replace(base, desc=np.ascontiguousarray(base.desc[perm]))
    r = oracle.run_restated(wl)
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        frames = wl.frames.copy()
        verdict = np.zeros(wl.n, np.uint32)
        w.process_host(frames, wl.desc, verdict, chunk)
        _check(w, wl, frames, verdict, {"verdict": r.verdict, "frames": r.frames,
                                        "counters": r.counters, "rule_stats": r.rule_stats,
                                        "l1": r.l1}, f"permuted chunk={chunk}")
    finally:
        w.close()


@pytest.mark.parametrize("case", ["edge_zero", "edge_consistent"])
@pytest.mark.parametrize("chunk", [100, 0])
def test_host_roundtrip_edge_frames(gpu_worker_factory, case, chunk):
    """Edge frames (ARP requests for the port answered in place, NS / NA, every parse gate)
    through the host round trip: equals the oracle with table writes deferred (the snapshot
    semantics of upe_gpu_process, as test_gpu_parity's one-segment edge case)."""
    wl, _ = golden_io.load(case)
    r = oracle.run_restated(wl, apply_control=False)
    assert np.count_nonzero(r.verdict & np.uint32(0x40)) > 0, "no ARP reply in the fixture"
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        if case == "edge_consistent":
            w.set_l1(wl.l1)
        frames = wl.frames.copy()
        verdict = np.zeros(wl.n, np.uint32)
        w.process_host(frames, wl.desc, verdict, chunk)
        _check(w, wl, frames, verdict, {"verdict": r.verdict, "frames": r.frames,
                                        "counters": r.counters, "rule_stats": r.rule_stats,
                                        "l1": r.l1}, f"{case} chunk={chunk}")
    finally:
        w.close()


@pytest.mark.parametrize("case", ["config_b_small", "config_c_small", "config_d_small",
                                  "edge_zero"])
@pytest.mark.parametrize("chunk,apply", [(1000, 3), (333, 0), (0, 2), (1000, -1), (333, -1)])
def test_host_emit_roundtrip(gpu_worker_factory, case, chunk, apply):
    """upe_gpu_process_host_emit: only verdicts and records come back.  With the records applied
    on the host (apply >= 0) the frames equal the reference worker's; with apply = -1 they stay
    as they were (answered ARP requests aside) and the records equal the ones the reference's
    rewritten frames define."""
    from test_emit_records import records_from_reference

    wl, ref = golden_io.load(case)
    if case.startswith("edge"):
        # control packets' table writes apply after the batch (snapshot semantics): compare with
        # the oracle run as one constant-table segment; chunks are consecutive batches of it
        # (UPE_VF_L1_INIT, relative to each chunk's start, is masked by _check)
        r = oracle.run_restated(wl, apply_control=False)
        ref = {"verdict": r.verdict, "frames": r.frames, "counters": r.counters,
               "rule_stats": r.rule_stats, "l1": r.l1}
    w = gpu_worker_factory(wl.capacity)
    pf = gpu.PinnedArray(wl.frames.shape, np.uint8)
    pd = gpu.PinnedArray(wl.desc.shape, np.uint64)
    pv = gpu.PinnedArray((wl.n,), np.uint32)
    ph = gpu.PinnedArray((wl.n, 16), np.uint8)
    try:
        w.configure(wl)
        pf.array[:] = wl.frames
        pd.array[:] = wl.desc
        w.process_host_emit(pf.array, pd.array, pv.array, ph.array, chunk, apply)
        want_rec = records_from_reference(wl.frames, ref["frames"], wl.desc, ref["verdict"])
        got_rec = gpu.expand_records(ph.array, pv.array)   # (compacted per 64-packet group)
        bad = np.nonzero((got_rec != want_rec).any(axis=1))[0]
        assert bad.size == 0, f"{bad.size} records differ, first {bad[:8].tolist()}"
        if apply >= 0:
            _check(w, wl, pf.array.copy(), pv.array.copy(), ref, f"{case} chunk={chunk}")
        else:
            replied = (pv.array & 0x40) != 0
            keep = np.ones(wl.frames.size, bool)
            for o in desc_offsets(wl.desc)[replied]:
                keep[o:o + REWRITE_EXTENT] = False
            assert np.array_equal(pf.array[keep], wl.frames[keep]), "frames were written"
            assert np.array_equal(pf.array[~keep], ref["frames"][~keep]), "ARP replies differ"
    finally:
        for x in (pf, pd, pv, ph):
            x.free()
        w.close()


def test_host_emit_full_size_b(gpu_worker_factory):
    """Config B at 1M through the emit round trip with 8 apply threads, against the digest."""
    import hashlib

    dg = golden_io.digests()["B_1M"]
    wl = synth.config_b()
    w = gpu_worker_factory(wl.capacity)
    pf = gpu.PinnedArray(wl.frames.shape, np.uint8)
    pd = gpu.PinnedArray(wl.desc.shape, np.uint64)
    pv = gpu.PinnedArray((wl.n,), np.uint32)
    ph = gpu.PinnedArray((wl.n, 16), np.uint8)
    try:
        w.configure(wl)
        pf.array[:] = wl.frames
        pd.array[:] = wl.desc
        w.process_host_emit(pf.array, pd.array, pv.array, ph.array, 1 << 18, 8)
        assert hashlib.sha256(pf.array.tobytes()).hexdigest() == dg["frames"]
        counters, _ = w.get_stats()
        assert [int(x) for x in counters[0].tolist()] == dg["counters"]
    finally:
        for x in (pf, pd, pv, ph):
            x.free()
        w.close()
