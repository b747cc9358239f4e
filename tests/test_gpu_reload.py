"""GPU parity of the SIGHUP rule reload (upe_gpu_reload_rules) against the REFERENCE worker
with the stats thread's swap (reference src/main.c:216-282, driven by oracle/ref_harness.c's
upe_refh_process_reload inside one reference worker_t): part of a stream runs with table A,
the table is reloaded — renumbered rule_ids, changed priorities and actions, a rule gone, a new
one, a new capacity — and the stream continues.  Every verdict word (L1_INIT aside: it is
defined against each batch's starting entry), every rewritten frame byte or record, the worker
counters, the OLD rule_stats handed back at the swap, the NEW rule_stats and the final L1 state
must equal the reference's, in place and in emit mode, for the three ways the kernel keeps
rule_stats (small tables in LDS accumulators, 1k-rule tables in per-index replicas, 8k-rule
tables through the group-by)."""
from __future__ import annotations

import numpy as np
import pytest

import oracle
import reload_util
from test_gpu_parity import _assert_same
from upe_amd import gpu, synth

pytestmark = pytest.mark.gpu


def _gpu_reload(w, wl, rules_b_sorted, cap_b, at, emit, sync_before, image=False):
    """Batch [0, at) with the loaded table, reload, batch [at, n); the reload is issued while
    the first batch may still be running unless sync_before.  image: the new table compiled
    beforehand (upe_rules_compile, while the first batch runs) and installed by
    upe_gpu_reload_image."""
    b1 = gpu.DeviceBatch(w, wl.frames, wl.desc[:at])
    (b1.run_emit if emit else b1.run)()
    if sync_before:
        w.sync()
    if image:
        im = gpu.RuleImage(rules_b_sorted, cap_b)
        old = w.reload_image(im)
        im.free()
    else:
        old = w.reload_rules(rules_b_sorted, cap_b)
    frames1, v1 = b1.fetch()
    if emit:
        frames1 = gpu.hdr_apply(frames1, wl.desc[:at], b1.fetch_hdr())
    b1.free()
    b2 = gpu.DeviceBatch(w, frames1, wl.desc[at:])
    (b2.run_emit if emit else b2.run)()
    frames, v2 = b2.fetch()
    if emit:
        frames = gpu.hdr_apply(frames, wl.desc[at:], b2.fetch_hdr())
    b2.free()
    counters, stats = w.get_stats()
    return frames, np.concatenate([v1, v2]), counters, stats, w.get_l1(), old


@pytest.mark.parametrize("image", [False, True], ids=["rules", "image"])
@pytest.mark.parametrize("emit", [False, True])
@pytest.mark.parametrize("name", ["B", "C", "D"])
def test_reload_equals_reference(gpu_worker_factory, name, emit, image):
    wl, rules_b, at, cap_b = reload_util.case(name)
    ref, old_ref = oracle.run_reference_reload(wl, rules_b, cap_b, at)
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        frames, verdict, counters, stats, l1, old = _gpu_reload(
            w, wl, ref.rules_sorted, cap_b, at, emit, sync_before=name == "C", image=image)
        assert w.capacity == cap_b and stats.shape[0] == cap_b
    finally:
        w.close()
    assert np.array_equal(old, old_ref), f"{name}: rule_stats handed back at the swap differ"
    _assert_same((frames, verdict, counters, stats, l1),
                 {"verdict": ref.verdict, "frames": ref.frames, "counters": ref.counters,
                  "rule_stats": ref.rule_stats, "l1": ref.l1}, f"reload {name} emit={emit}",
                 batch_relative=True)


def test_reload_keeps_counters_and_l1_unlike_reset(gpu_worker_factory):
    """A reload to the SAME table (as a SIGHUP with an unchanged file): counters and the L1 entry
    carry on, rule_stats restart at zero — the whole stream's counters equal one uninterrupted
    run's, and the new rule_stats equal the second part's alone."""
    wl = synth.config_b(n=200_000, seed=44)
    at = 70_000
    whole = oracle.run_restated(wl)
    import dataclasses

    tail = oracle.run_restated(dataclasses.replace(wl, desc=wl.desc[at:]),
                               l1=oracle.run_restated(dataclasses.replace(
                                   wl, desc=wl.desc[:at])).l1)
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        _, verdict, counters, stats, l1, old = _gpu_reload(w, wl, wl.rules_sorted, wl.capacity,
                                                           at, True, sync_before=False)
    finally:
        w.close()
    assert counters.tobytes() == whole.counters.tobytes()
    assert l1.tobytes() == whole.l1.tobytes()
    assert np.array_equal(verdict & ~np.uint32(0x80), whole.verdict & ~np.uint32(0x80))
    assert np.array_equal(stats, tail.rule_stats)
    assert np.array_equal(old["packets"] + stats["packets"], whole.rule_stats["packets"])


def test_reload_rejects_bad_tables_and_keeps_the_old(gpu_worker_factory):
    """A table the new capacity cannot index is refused before anything changes (the reference
    keeps the old rules when the new file fails to load, src/main.c:229-235)."""
    wl = synth.config_b(n=50_000, seed=45)
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        bad = wl.rules_sorted.copy()
        bad["rule_id"][0] = 5000
        with pytest.raises(gpu.UpeGpuError):
            w.reload_rules(bad, 1024)
        with pytest.raises(gpu.UpeGpuError):
            w.reload_rules(wl.rules_sorted, len(wl.rules) - 1)
        assert w.capacity == wl.capacity
        frames, verdict, counters, stats, l1 = gpu.run_workload(wl, worker=w)
    finally:
        w.close()
    r = oracle.run_restated(wl)
    _assert_same((frames, verdict, counters, stats, l1),
                 {"verdict": r.verdict, "frames": r.frames, "counters": r.counters,
                  "rule_stats": r.rule_stats, "l1": r.l1}, "after refused reloads")


@pytest.mark.parametrize("host", [False, True], ids=["device", "host-emit"])
def test_reload_in_a_stream_of_batches(gpu_worker_factory, host):
    """Many small batches before and after the reload (the kernel without look-back is in use by
    then), device-resident or through the emit-mode host round trip."""
    import dataclasses

    wl, rules_b, at, cap_b = reload_util.case("B")
    wl = dataclasses.replace(wl, desc=wl.desc[:40_000])
    at = 20_480
    ref, old_ref = oracle.run_reference_reload(wl, rules_b, cap_b, at)
    w = gpu_worker_factory(wl.capacity)
    verdict = np.zeros(wl.n, np.uint32)
    frames = wl.frames.copy()
    try:
        w.configure(wl)
        bounds = list(range(0, wl.n, 1024)) + [wl.n]
        for s, e in zip(bounds[:-1], bounds[1:]):
            if s == at:
                old = w.reload_rules(ref.rules_sorted, cap_b)
            if host:
                rec = np.zeros((e - s, 16), np.uint8)
                v = np.zeros(e - s, np.uint32)
                w.process_host_emit(frames, wl.desc[s:e].copy(), v, rec, 0, 0)
                verdict[s:e] = v
            else:
                b = gpu.DeviceBatch(w, frames, wl.desc[s:e])
                b.run()
                frames, verdict[s:e] = b.fetch()
                b.free()
        counters, stats = w.get_stats()
        l1 = w.get_l1()
    finally:
        w.close()
    assert np.array_equal(old, old_ref)
    _assert_same((frames, verdict, counters, stats, l1),
                 {"verdict": ref.verdict, "frames": ref.frames, "counters": ref.counters,
                  "rule_stats": ref.rule_stats, "l1": ref.l1}, f"stream reload host={host}",
                 batch_relative=True)


def test_reload_returns_to_lookback(gpu_worker_factory, monkeypatch):
    """A family that no reachable rule forwards never consults its L1 entry, so a disagreeing
    entry of that family does not keep the look-back kernel (config C's table: IPv6 all dropped at
    rule 0).  A reload that lets that family forward must bring the look-back back: here the
    starting NDP entry holds a wrong MAC for the destination of the first IPv6 packet the new
    table forwards, which must take the entry's MAC as in the reference worker."""
    from upe_amd.layout import V_FWD, desc_offsets

    monkeypatch.setenv("UPE_GPU_LB_SYNC", "1")
    n, at = 60_000, 30_000
    wa = synth.config_c(n=n, seed=3)
    w6 = synth.config_c(n=n, seed=3, v6_forwarding=True)
    part2 = w6.copy()
    part2.desc = w6.desc[at:]
    r2 = oracle.run_restated(part2)
    offs = desc_offsets(part2.desc)
    is6 = part2.frames[offs + 12] == 0x86
    k = int(np.nonzero(is6 & ((r2.verdict & 0xF) == V_FWD))[0][0])
    l1 = synth.l1_zero()
    l1["last_ndp_ip"] = part2.frames[offs[k] + 38: offs[k] + 54]
    l1["last_ndp_mac"] = [2, 0, 0, 0, 0, 1]
    wa.l1 = l1
    ref, _ = oracle.run_reference_reload(wa, w6.rules, w6.capacity, at)
    w = gpu_worker_factory(wa.capacity)
    variants = []
    try:
        w.configure(wa)
        frames = wa.frames
        verdicts = []
        for s, e in ((0, 10_000), (10_000, 20_000), (20_000, at), (at, n)):
            if s == at:
                w.reload_rules(ref.rules_sorted, w6.capacity)
            b = gpu.DeviceBatch(w, frames, wa.desc[s:e])
            b.run()
            frames, v = b.fetch()
            b.free()
            verdicts.append(v)
            variants.append(w.launch_info()["variant"])
        counters, stats = w.get_stats()
        l1_out = w.get_l1()
    finally:
        w.close()
    assert variants[2] & gpu.VAR_NOLB, variants             # IPv6 cannot forward under table A
    assert not variants[3] & gpu.VAR_NOLB, variants         # ... and can under table B
    verdict = np.concatenate(verdicts)
    _assert_same((frames, verdict, counters, stats, l1_out),
                 {"verdict": ref.verdict, "frames": ref.frames, "counters": ref.counters,
                  "rule_stats": ref.rule_stats, "l1": ref.l1}, "reload to IPv6 forwarding",
                 batch_relative=True)
    hit = ref.verdict[at + k]
    assert (hit & 0xF) == V_FWD and hit & 0x10, "the aimed packet is forwarded with a MAC"
