"""GPU parity of the mapped host path (upe_gpu_process_mapped[_emit]): the kernel classifies a
batch where it lies in pinned host memory — descriptors and header windows read, verdicts and the
rewritten header bytes (or records) written, over the link, with no DMA copy — against the
reference's golden vectors and full-size digests.  One launch over the whole batch, so every
verdict bit (UPE_VF_L1_INIT included) is the reference worker's.  Also: an existing host buffer
made GPU-visible by upe_gpu_host_register (the reference's pktbuf pool, src/pktbuf.c), and the
loud failure on memory the GPU cannot reach."""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

import golden_io
import oracle
from test_gpu_parity import _assert_same
from upe_amd import gpu, synth

pytestmark = pytest.mark.gpu


def _mapped_run(w, wl, emit: bool, registered: bool = False):
    """(frames as the reference leaves them, verdict, counters, stats, l1) of one mapped call."""
    if registered:
        hold = [gpu.RegisteredArray(wl.frames.copy()), gpu.RegisteredArray(wl.desc.copy()),
                gpu.RegisteredArray(np.zeros(max(wl.n, 1), np.uint32)),
                gpu.RegisteredArray(np.zeros((max(wl.n, 1), 16), np.uint8))]
    else:
        hold = [gpu.PinnedArray(wl.frames.shape, np.uint8),
                gpu.PinnedArray(wl.desc.shape, np.uint64),
                gpu.PinnedArray((max(wl.n, 1),), np.uint32),
                gpu.PinnedArray((max(wl.n, 1), 16), np.uint8)]
        hold[0].array[:] = wl.frames
        hold[1].array[:] = wl.desc
        hold[2].array[:] = 0
        hold[3].array[:] = 0xEE
    f, d, v, h = (x.array for x in hold)
    v = v[:wl.n]
    h = h[:wl.n]
    try:
        if emit:
            w.process_mapped_emit(f, d, v, h)
        else:
            w.process_mapped(f, d, v)
        w.sync()
        if wl.n:
            assert w.launch_info()["variant"] & gpu.VAR_HOST, "not the host-path kernel"
        frames = f.copy()
        verdict = v.copy()
        if emit:
            # emit mode leaves the frames as they were, except the answered ARP requests, which
            # are rewritten into replies in place (as upe_gpu_process_emit does)
            from upe_amd.layout import desc_offsets

            changed = np.zeros(frames.shape[0], bool)
            changed[frames != wl.frames] = True
            offs = desc_offsets(wl.desc)
            replies = np.zeros(frames.shape[0], bool)
            for i in np.nonzero(verdict & np.uint32(0x40))[0]:
                replies[offs[i]:offs[i] + 96] = True
            assert not (changed & ~replies).any(), "emit mode wrote into non-reply frames"
            frames = gpu.hdr_apply(frames, wl.desc, gpu.expand_records(h.copy(), verdict))
        counters, stats = w.get_stats()
        return frames, verdict, counters, stats, w.get_l1()
    finally:
        for x in hold:
            x.free()


@pytest.mark.parametrize("emit", [False, True])
@pytest.mark.parametrize("case", ["config_a", "config_b_small", "config_c_small",
                                  "config_d_small"])
def test_mapped_golden(gpu_worker_factory, case, emit):
    wl, ref = golden_io.load(case)
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        _assert_same(_mapped_run(w, wl, emit), ref, f"mapped {case} emit={emit}")
    finally:
        w.close()


@pytest.mark.parametrize("emit", [False, True])
@pytest.mark.parametrize("case", ["edge_zero", "edge_consistent", "edge_inconsistent"])
def test_mapped_edges_vs_oracle(gpu_worker_factory, case, emit):
    """Every parse gate, truncation, TTL edge, ARP request / reply and NS / NA as ONE mapped
    batch (control writes deferred, as upe_gpu_process does): equals the oracle with control
    replay off; the ARP reply is rewritten in place in host memory."""
    wl, _ = golden_io.load(case)
    r = oracle.run_restated(wl, apply_control=False)
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        _assert_same(_mapped_run(w, wl, emit), {"verdict": r.verdict, "frames": r.frames,
                                                 "counters": r.counters,
                                                 "rule_stats": r.rule_stats, "l1": r.l1}, case)
    finally:
        w.close()


@pytest.mark.parametrize("emit", [False, True])
def test_mapped_registered_buffer(gpu_worker_factory, emit):
    """Plain numpy buffers page-locked and mapped in place (as a caller would register the
    reference's pktbuf pool) give the same answers."""
    wl, ref = golden_io.load("config_c_small")
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        _assert_same(_mapped_run(w, wl, emit, registered=True), ref, f"registered emit={emit}")
    finally:
        w.close()


def _sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


@pytest.mark.parametrize("key,make,emit", [
    ("B_1M", lambda: synth.config_b(), False),
    ("B_1M", lambda: synth.config_b(), True),
    ("C_1M", lambda: synth.config_c(), False),
    ("C_1M", lambda: synth.config_c(), True),
])
def test_mapped_full_size_digest(gpu_worker_factory, key, make, emit):
    """BASELINE.json full sizes (full IMIX frames in host memory for C) against the reference
    worker's output digests."""
    dg = golden_io.digests()[key]
    wl = make()
    assert _sha(wl.frames, wl.desc, wl.rules, wl.arp, wl.ndp) == dg["inputs"]
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        frames, verdict, counters, stats, l1 = _mapped_run(w, wl, emit)
    finally:
        w.close()
    assert [int(x) for x in counters[0].tolist()] == dg["counters"]
    assert _sha(verdict) == dg["verdict"]
    assert _sha(frames) == dg["frames"]
    assert _sha(stats) == dg["rule_stats"]
    assert _sha(l1) == dg["l1"]


def test_mapped_rejects_unmapped_memory(gpu_worker_factory):
    """Ordinary pageable memory is refused before any launch (a kernel never touches it)."""
    wl, _ = golden_io.load("config_b_small")
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        v = np.zeros(wl.n, np.uint32)
        with pytest.raises(gpu.UpeGpuError, match="not pinned"):
            w.process_mapped(wl.frames.copy(), wl.desc.copy(), v)
        assert w.launch_info()["launches"] == 0
    finally:
        w.close()


def test_mapped_then_resident_carry(gpu_worker_factory):
    """A mapped batch and a device-resident batch on one context: the L1 state and counters
    carry across them as across any two batches of the worker (src/worker.c:255-307)."""
    wl = synth.config_b(n=200_000, seed=44)
    a = synth.config_b(n=200_000, seed=44)
    w = gpu_worker_factory(wl.capacity)
    ref_w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        ref_w.configure(wl)
        half = 100_000
        first = synth.Workload(wl.name, wl.frames, wl.desc[:half].copy(), wl.rules, wl.capacity,
                               wl.arp, wl.ndp, wl.eth_addr, wl.ip4_addr, wl.l1)
        _mapped_run(w, first, emit=False)
        b = gpu.DeviceBatch(w, wl.frames, wl.desc[half:])
        b.run()
        _, v2 = b.fetch()
        b.free()
        c1, s1 = w.get_stats()
        l1 = w.get_l1()
        # the same two batches, both device-resident
        r1 = gpu.DeviceBatch(ref_w, a.frames, a.desc[:half])
        r1.run()
        r2 = gpu.DeviceBatch(ref_w, a.frames, a.desc[half:])
        r2.run()
        _, rv2 = r2.fetch()
        r1.free()
        r2.free()
        c2, s2 = ref_w.get_stats()
        assert np.array_equal(v2, rv2)
        assert c1.tobytes() == c2.tobytes() and np.array_equal(s1, s2)
        assert l1.tobytes() == ref_w.get_l1().tobytes()
    finally:
        w.close()
        ref_w.close()


@pytest.mark.parametrize("emit", [False, True])
@pytest.mark.parametrize("n", [1, 63, 65, 1000, 16385])
def test_mapped_ragged_sizes(gpu_worker_factory, n, emit):
    """Batch sizes at every edge of the work split (one packet, part of a chunk, a chunk and one,
    a tile and one), IMIX frames in host memory, against the oracle."""
    wl = synth.config_c(n=n, seed=900 + n)
    r = oracle.run_restated(wl)
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        _assert_same(_mapped_run(w, wl, emit), {"verdict": r.verdict, "frames": r.frames,
                                                 "counters": r.counters,
                                                 "rule_stats": r.rule_stats, "l1": r.l1},
                     f"mapped n={n} emit={emit}")
    finally:
        w.close()
