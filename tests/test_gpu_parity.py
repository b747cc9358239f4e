"""GPU parity: the HIP path (through the C ABI) against the reference's golden vectors and the
oracle, bit-exact on verdict words, rewritten frames, counters, rule_stats and L1 state.

Sizes: the golden fixtures (reference outputs, tests/golden/) at small sizes; BASELINE.json's
full sizes against reference digests (B 1M, C 1M, D 256k x 64k rules) and, for D at 16M,
size-independent properties, a random-chunk comparison against the oracle and every packet
classified by two independent indexes (tuple space, decision tree) that must agree.
"""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

import golden_io
import oracle
import stream
from upe_amd import gpu, synth
from upe_amd.layout import COUNTERS_DTYPE, L1_DTYPE, V_CONSUMED, V_FWD

pytestmark = pytest.mark.gpu


def _run(worker_factory, wl, batches=1, emit=False):
    """emit: the batch runs in emit mode and the frames come back with upe_hdr_apply applied."""
    w = worker_factory(wl.capacity)
    try:
        w.configure(wl)
        if batches == 1:
            frames, verdict, counters, stats, l1 = gpu.run_workload(wl, worker=w, emit=emit)
        else:
            frames = wl.frames.copy()
            verdict = np.zeros(wl.n, np.uint32)
            bounds = np.linspace(0, wl.n, batches + 1).astype(int)
            for s, e in zip(bounds[:-1], bounds[1:]):
                b = gpu.DeviceBatch(w, frames, wl.desc[s:e])
                if emit:
                    b.run_emit()
                    frames, verdict[s:e] = b.fetch()
                    frames = gpu.hdr_apply(frames, wl.desc[s:e], b.fetch_hdr())
                else:
                    b.run()
                    frames, verdict[s:e] = b.fetch()
                b.free()
            counters, stats = w.get_stats()
            l1 = w.get_l1()
        return frames, verdict, counters, stats, l1
    finally:
        w.close()


def _assert_same(got, ref, what="", batch_relative=False):
    """batch_relative: the run was cut into several batches, so UPE_VF_L1_INIT (defined against
    the L1 entry each batch starts with) is compared only through its effect on the frames."""
    frames, verdict, counters, stats, l1 = got
    rv = ref["verdict"]
    if batch_relative:
        verdict = verdict & ~np.uint32(0x80)
        rv = rv & ~np.uint32(0x80)
    bad = np.nonzero(verdict != rv)[0]
    assert bad.size == 0, (f"{what}: {bad.size} verdicts differ, first {bad[:8].tolist()}: "
                           f"gpu {[hex(x) for x in verdict[bad[:8]]]} "
                           f"ref {[hex(x) for x in rv[bad[:8]]]}")
    assert np.array_equal(frames, ref["frames"]), f"{what}: rewritten frames differ"
    assert counters.tobytes() == np.asarray(ref["counters"]).tobytes(), \
        f"{what}: counters {counters} vs {ref['counters']}"
    assert np.array_equal(stats, ref["rule_stats"]), f"{what}: rule_stats differ"
    assert l1.tobytes() == np.asarray(ref["l1"]).tobytes(), f"{what}: L1 state differs"


@pytest.mark.parametrize("emit", [False, True])
@pytest.mark.parametrize("case", ["config_a", "config_b_small", "config_c_small",
                                  "config_cf_small", "config_d_small"])
def test_golden_no_control(gpu_worker_factory, case, emit):
    wl, ref = golden_io.load(case)
    _assert_same(_run(gpu_worker_factory, wl, emit=emit), ref, f"{case} emit={emit}")


@pytest.mark.parametrize("case", ["config_b_small", "config_c_small", "config_d_small",
                                  "edge_inconsistent"])
def test_emit_records_exact(gpu_worker_factory, case):
    """Emit mode: every record equals the one the reference's rewritten frame defines (zero for
    packets not forwarded), and the frames stay as they were (ARP replies aside)."""
    from test_emit_records import records_from_reference

    wl, ref = golden_io.load(case)
    if case.startswith("edge"):
        r = oracle.run_restated(wl, apply_control=False)
        ref = {"verdict": r.verdict, "frames": r.frames}
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        b = gpu.DeviceBatch(w, wl.frames, wl.desc)
        b.run_emit()
        frames, verdict = b.fetch()
        rec = b.fetch_hdr()
        b.free()
    finally:
        w.close()
    assert np.array_equal(verdict, ref["verdict"])
    want = records_from_reference(wl.frames, ref["frames"], wl.desc, ref["verdict"])
    bad = np.nonzero((rec != want).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} records differ, first {bad[:8].tolist()}"
    replied = (verdict & 0x40) != 0
    from upe_amd.layout import desc_offsets

    offs = desc_offsets(wl.desc)
    keep = np.ones(len(frames), bool)
    for o in offs[replied]:
        keep[o:o + 48] = False
    assert np.array_equal(frames[keep], wl.frames[keep]), "emit mode wrote into the frames"


@pytest.mark.parametrize("case", ["edge_zero", "edge_consistent", "edge_inconsistent"])
def test_golden_edge_segmented(gpu_worker_factory, case):
    """Edge frames incl. ARP/NDP control packets: segmented stream == reference worker."""
    wl, ref = golden_io.load(case)
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        frames, verdict, arp, ndp = stream.run_stream(w, wl)
        counters, stats = w.get_stats()
        l1 = w.get_l1()
    finally:
        w.close()
    _assert_same((frames, verdict, counters, stats, l1), ref, case, batch_relative=True)
    keep = ["ip", "mac", "valid"]
    assert np.array_equal(arp[keep], ref["arp"][keep])
    assert np.array_equal(ndp[keep], ref["ndp"][keep])


@pytest.mark.parametrize("emit", [False, True])
@pytest.mark.parametrize("case", ["edge_zero", "edge_consistent", "edge_inconsistent"])
def test_edge_one_segment_vs_oracle(gpu_worker_factory, case, emit):
    """The same frames as ONE batch (control writes deferred): equals the oracle run with
    control replay off — exercises the L1 repair path with control packets in the batch."""
    wl, _ = golden_io.load(case)
    r = oracle.run_restated(wl, apply_control=False)
    got = _run(gpu_worker_factory, wl, emit=emit)
    _assert_same(got, {"verdict": r.verdict, "frames": r.frames, "counters": r.counters,
                       "rule_stats": r.rule_stats, "l1": r.l1}, case)


@pytest.mark.parametrize("emit", [False, True])
@pytest.mark.parametrize("batches", [2, 7, 33])
def test_multi_batch_l1_carry(gpu_worker_factory, batches, emit):
    """L1 caches, counters and rule_stats carry across batches exactly as across bursts."""
    wl, ref = golden_io.load("config_c_small")
    _assert_same(_run(gpu_worker_factory, wl, batches=batches, emit=emit), ref,
                 f"{batches} batches", batch_relative=True)


def _force_dst(wl, count, v4_ip=None, v6_ip=None):
    """Point the destination of the first `count` IPv4 / IPv6 packets at the given addresses."""
    from upe_amd.layout import desc_offsets

    offs = desc_offsets(wl.desc)
    fr = wl.frames
    et = (fr[offs + 12].astype(np.int64) << 8) | fr[offs + 13]
    if v4_ip is not None:
        for o in offs[et == 0x0800][:count]:
            fr[o + 30:o + 34] = np.frombuffer(int(v4_ip).to_bytes(4, "big"), np.uint8)
    if v6_ip is not None:
        for o in offs[et == 0x86DD][:count]:
            fr[o + 38:o + 54] = v6_ip


@pytest.mark.parametrize("emit", [False, True])
def test_random_l1_starts(gpu_worker_factory, emit):
    """Starting L1 entries that agree / disagree with the tables (or are absent from them), with
    the first packets of the batch sent to those destinations so the repair path runs."""
    rng = np.random.default_rng(11)
    base = synth.config_c(n=20000, seed=9)
    for trial in range(8):
        wl = base.copy()
        l1 = synth.l1_zero()
        arp_valid = np.nonzero(wl.arp["valid"])[0]
        ndp_valid = np.nonzero(wl.ndp["valid"])[0]
        a = wl.arp[rng.choice(arp_valid)]
        nd = wl.ndp[rng.choice(ndp_valid)]
        l1["last_arp_ip"] = a["ip"] if trial < 6 else 0xAC10FFFF  # last: not in the table
        l1["last_arp_mac"] = a["mac"] if trial % 2 == 0 else rng.integers(0, 256, 6)
        l1["last_ndp_ip"] = nd["ip"] if trial < 4 else (0 if trial < 6 else 0x55)
        l1["last_ndp_mac"] = nd["mac"] if trial % 3 == 0 else rng.integers(0, 256, 6)
        wl.l1 = l1
        _force_dst(wl, 40 + 10 * trial, int(l1["last_arp_ip"][0]), l1["last_ndp_ip"][0])
        r = oracle.run_restated(wl)
        got = _run(gpu_worker_factory, wl, emit=emit)
        _assert_same(got, {"verdict": r.verdict, "frames": r.frames, "counters": r.counters,
                           "rule_stats": r.rule_stats, "l1": r.l1}, f"trial {trial}")
        assert np.count_nonzero(r.verdict & 0x80) > 0


@pytest.mark.parametrize("emit", [False, True])
@pytest.mark.parametrize("config", ["B", "C"])
def test_ragged_batch_sizes(gpu_worker_factory, config, emit):
    """Batch sizes around every boundary of the work split: a single packet, a partial first
    chunk, one chunk plus one packet, batches too small to give every resident workgroup a
    full tile (narrow tiles), a partial last tile and a partial last chunk of a large batch —
    each against the oracle, so the chunk claims, late claims and the window prefetch of the
    next chunk are exact at every edge."""
    make = synth.config_b if config == "B" else synth.config_c
    for n in (1, 63, 65, 1000, 16385, 262145):
        wl = make(n=n, seed=70 + n % 97)
        r = oracle.run_restated(wl)
        got = _run(gpu_worker_factory, wl, emit=emit)
        _assert_same(got, {"verdict": r.verdict, "frames": r.frames, "counters": r.counters,
                           "rule_stats": r.rule_stats, "l1": r.l1}, f"{config} n={n}")


@pytest.mark.parametrize("emit", [False, True])
def test_line_aligned_layout(gpu_worker_factory, monkeypatch, emit):
    """Config C at 1M with every header window inside one 128-byte line (frames of up to 64
    bytes on 64-byte boundaries, longer ones on 128-byte boundaries): the layout changes only
    where frames sit, so the results equal the oracle's on the same batch."""
    monkeypatch.setenv("UPE_SYNTH_LAYOUT", "line")
    wl = synth.config_c()
    r = oracle.run_restated(wl)
    got = _run(gpu_worker_factory, wl, emit=emit)
    _assert_same(got, {"verdict": r.verdict, "frames": r.frames, "counters": r.counters,
                       "rule_stats": r.rule_stats, "l1": r.l1}, "C line-aligned")


def test_empty_batch(gpu_worker_factory):
    wl, _ = golden_io.load("config_b_small")
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        dev = w.malloc(256)
        w.process(dev, dev, dev, 0)
        info = w.batch_info()
        assert int(info["counters"]["pkts_in"][0]) == 0
        assert int(info["first_ctrl"][0]) == 2**64 - 1
        c, s = w.get_stats()
        assert c.tobytes() == np.zeros(1, COUNTERS_DTYPE).tobytes()
        assert w.get_l1().tobytes() == np.zeros(1, L1_DTYPE).tobytes()
        w.free(dev)
    finally:
        w.close()


def test_batch_info_control(gpu_worker_factory):
    wl, _ = golden_io.load("edge_zero")
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        b = gpu.DeviceBatch(w, wl.frames, wl.desc)
        b.run()
        _, verdict = b.fetch()
        info = w.batch_info()
        ctrl = np.nonzero(((verdict & 0xF) == V_CONSUMED) | ((verdict & 0x20) != 0))[0]
        assert int(info["n_ctrl"][0]) == ctrl.size
        assert int(info["first_ctrl"][0]) == ctrl.min()
        assert int(info["counters"]["pkts_forwarded"][0]) == np.count_nonzero((verdict & 0xF) == V_FWD)
        b.free()
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
    ("D_256k_64k_rules", lambda: synth.config_d(n=1 << 18), False),
    ("D_256k_64k_rules", lambda: synth.config_d(n=1 << 18), True),
    ("CF_1M", lambda: synth.config_c_flows(), False),
    ("CF_1M", lambda: synth.config_c_flows(), True),
    ("C6_1M", lambda: synth.config_c(v6_forwarding=True), False),
    ("C6_1M", lambda: synth.config_c(v6_forwarding=True), True),
])
def test_full_size_digest(gpu_worker_factory, key, make, emit):
    """BASELINE.json full sizes against SHA-256 digests of the reference worker's outputs."""
    dg = golden_io.digests()[key]
    wl = make()
    assert _sha(wl.frames, wl.desc, wl.rules, wl.arp, wl.ndp) == dg["inputs"], \
        "synthetic generator drifted (inputs differ from the ones the digest was made from)"
    frames, verdict, counters, stats, l1 = _run(gpu_worker_factory, wl, emit=emit)
    assert np.bincount(verdict & 0xF, minlength=7).tolist() == dg["codes"]
    assert [int(x) for x in counters[0].tolist()] == dg["counters"]
    assert _sha(verdict) == dg["verdict"]
    assert _sha(frames) == dg["frames"]
    assert _sha(stats) == dg["rule_stats"]
    assert _sha(l1) == dg["l1"]


_D_CACHE: dict = {}


@pytest.mark.parametrize("emit", [False, True])
def test_config_d_full_properties(gpu_worker_factory, emit):
    """16M packets x 64k rules: size-independent checks (counter identities, stats sums,
    parse-fail and TTL invariants), the first 64k packets (from the calloc'd L1 state the batch
    starts with) exactly — every verdict bit and every output byte, rewritten in place or
    through the records — and random 4k-packet chunks against the oracle."""
    from upe_amd.layout import desc_lens, desc_offsets

    wl = synth.config_d()
    frames, verdict, counters, stats, l1 = _run(gpu_worker_factory, wl, emit=emit)
    c = counters[0]
    codes = np.bincount(verdict & 0xF, minlength=7)
    assert int(c["pkts_in"]) == wl.n
    assert int(c["pkts_forwarded"]) == codes[V_FWD]
    assert int(c["pkts_dropped"]) + int(c["pkts_forwarded"]) + int(c["pkts_consumed"]) == wl.n
    assert int(stats["packets"].sum()) == int(c["pkts_matched"])
    assert int(c["pkts_parsed"]) == int(c["pkts_matched"])  # catch-all rule
    rs = wl.rules_sorted
    pre = wl.copy()
    pre.desc = wl.desc[:1 << 16]
    if "d_prefix" not in _D_CACHE:   # ~20 s of oracle work, shared by both modes
        _D_CACHE["d_prefix"] = oracle.run_restated(pre, rules_sorted=rs)
    r = _D_CACHE["d_prefix"]
    bad = np.nonzero(verdict[:1 << 16] != r.verdict)[0]
    assert bad.size == 0, f"prefix verdicts differ at {bad[:8].tolist()}"
    offs, lens = desc_offsets(pre.desc).astype(np.int64), desc_lens(pre.desc).astype(np.int64)
    mine = np.repeat(offs, lens) + (np.arange(int(lens.sum())) - np.repeat(np.cumsum(lens) - lens, lens))
    assert np.array_equal(frames[mine], r.frames[mine]), "prefix output bytes differ"
    assert not np.array_equal(frames[mine], wl.frames[mine])   # the prefix forwards packets
    rng = np.random.default_rng(7)
    for start in rng.integers(0, wl.n - 4096, size=4):
        sub = wl.copy()
        sub.desc = wl.desc[start:start + 4096]
        r = oracle.run_restated(sub, rules_sorted=rs)
        v = verdict[start:start + 4096]
        # verdict code, rule index and the TTL/checksum rewrite do not depend on L1 history
        assert np.array_equal(v & 0xFFFFFF0F, r.verdict & 0xFFFFFF0F)


def test_config_d_full_two_indexes_agree(gpu_worker_factory, monkeypatch):
    """16M packets x 64k rules, every packet: the tuple-space index (D's default) and the
    decision tree over the family lists (forced, image read from memory) are two independent
    first-match classifiers of the same table (src/rule_table.c:163-176); each is pinned to the
    reference on the fixtures (test_rule_index_kinds_agree).  Over the whole batch they must give
    the same verdict word, rewritten bytes, counters, rule_stats and L1 state — a size-independent
    check of every packet the random-chunk comparison above does not reach."""
    wl = synth.config_d()
    got = {}
    for mode in ("tss", "tree"):
        monkeypatch.setenv("UPE_GPU_TSS", "1" if mode == "tss" else "0")
        monkeypatch.setenv("UPE_GPU_TREE", "1")
        w = gpu_worker_factory(wl.capacity)
        try:
            w.configure(wl)
            assert w.rule_index_kind() == (1 if mode == "tss" else 2)
            got[mode] = gpu.run_workload(wl, worker=w, emit=True)
        finally:
            w.close()
    frames, verdict, counters, stats, l1 = got["tree"]
    _assert_same(got["tss"], {"verdict": verdict, "frames": frames, "counters": counters,
                              "rule_stats": stats, "l1": l1}, "D 16M tuple space vs tree")
    codes = np.bincount(verdict & 0xF, minlength=7)
    assert codes[V_FWD] > 0 and int(counters[0]["pkts_in"]) == wl.n


@pytest.mark.parametrize("emit", [False, True])
@pytest.mark.parametrize("n,first_hit", [(300_000, None), (300_000, 0), (300_000, 777),
                                         (300_000, 150_001), (300_000, 299_999),
                                         (800_000, None), (800_000, 400_000),
                                         (800_000, 799_000)])
def test_lookback_far_first_hit(gpu_worker_factory, n, first_hit, emit):
    """A starting ARP entry that disagrees with the table and a batch aimed at it: every packet
    before the first miss-then-hit packet (placed far into the batch, or absent) must take the
    entry's MAC — the decoupled look-back across ~1200 tiles (and, at 800k packets, across
    workgroups that own several tiles each)."""
    from upe_amd.layout import desc_offsets

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
        wl.frames[offs[first_hit] + 22] = 64     # TTL alive
        wl.frames[offs[first_hit] + 36:offs[first_hit] + 38] = [0, 53]  # dport 53 -> FWD rule
    r = oracle.run_restated(wl)
    got = _run(gpu_worker_factory, wl, emit=emit)
    _assert_same(got, {"verdict": r.verdict, "frames": r.frames, "counters": r.counters,
                       "rule_stats": r.rule_stats, "l1": r.l1}, f"first_hit={first_hit}")


@pytest.mark.parametrize("name,kind", [("B", 0), ("C3", 0), ("CF", 2), ("C6", 2), ("D", 1)])
def test_default_rule_index(gpu_worker_factory, monkeypatch, name, kind):
    """The index load_rules picks with no override: B's 8 rules and
    seed-3 C (every list reaches its family catch-all within 64 entries) keep the scan, the
    flow-derived C and C6 get the decision tree, D's 64k exact flows the tuple-space index."""
    for k in ("UPE_GPU_TREE", "UPE_GPU_TSS"):
        monkeypatch.delenv(k, raising=False)
    wl = {"B": lambda: synth.config_b(n=4096), "C3": lambda: synth.config_c(n=4096),
          "CF": lambda: synth.config_c_flows(n=4096),
          "C6": lambda: synth.config_c(n=4096, v6_forwarding=True),
          "D": lambda: synth.config_d(n=4096)}[name]()
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        assert w.rule_index_kind() == kind
    finally:
        w.close()


@pytest.mark.parametrize("mode", ["scan", "tree", "tree-memory", "tss", "tss-unstaged"])
@pytest.mark.parametrize("case", ["config_a", "config_b_small", "config_c_small",
                                  "config_cf_small", "config_d_small", "edge_inconsistent"])
def test_rule_index_kinds_agree(gpu_worker_factory, monkeypatch, case, mode):
    """Every classifier — the linear first-match scan, the decision tree over the family lists
    (its image staged in LDS, or read from memory) and the tuple-space index (small groups'
    fingerprints in LDS, or none staged) — forced on every fixture (version-0 rules, mixed v4/v6
    masks, wildcard fields, catch-alls) gives the reference's first match."""
    monkeypatch.setenv("UPE_GPU_TSS", "1" if mode.startswith("tss") else "0")
    monkeypatch.setenv("UPE_GPU_TREE", "0" if mode == "scan" else "1")
    monkeypatch.setenv("UPE_GPU_TREE_LDS", "0" if mode == "tree-memory" else "1")
    monkeypatch.setenv("UPE_GPU_FP_STAGE", "0" if mode.endswith("unstaged") else "1")
    wl, ref = golden_io.load(case)
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        big = len(wl.rules) > 64
        assert w.rule_index_kind() == (1 if mode.startswith("tss") else
                                       2 if mode.startswith("tree") and big else 0)
        frames, verdict, counters, stats, l1 = gpu.run_workload(wl, worker=w)
        if mode.startswith("tree") and big:
            assert w.launch_info()["variant"] & gpu.VAR_SCAN == gpu.VAR_TREE
    finally:
        w.close()
    if case.startswith("edge"):
        # one segment (control writes deferred): compare with the oracle run the same way
        r = oracle.run_restated(wl, apply_control=False)
        ref = {"verdict": r.verdict, "frames": r.frames, "counters": r.counters,
               "rule_stats": r.rule_stats, "l1": r.l1}
    _assert_same((frames, verdict, counters, stats, l1), ref, f"{case} {mode}")


def test_config_d_uses_tuple_space(gpu_worker_factory):
    wl, _ = golden_io.load("config_d_small")
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        assert w.rule_index_kind() == 1
    finally:
        w.close()


def test_config_a_pcap_replay(gpu_worker_factory, tmp_path):
    """BASELINE config A end to end through this repo's own ingress: the 10k-packet capture
    (reference smoke-test pcap format) read by upe_pcap_read, rules.example loaded by
    upe_rules_load_ini, classified on the GPU: equal to the reference worker's golden outputs."""
    import os

    from test_host_builders import _frames_of, write_pcap

    wl, ref = golden_io.load("config_a")
    p = tmp_path / "a.pcap"
    write_pcap(p, _frames_of(wl))
    frames, desc, info = gpu.pcap_read(str(p))
    rules = gpu.rules_load_ini(os.path.join(os.path.dirname(__file__), "golden", "rules.example"))
    w = gpu_worker_factory(1024)
    try:
        w.load_rules(rules)
        w.load_neigh(wl.arp, wl.ndp)
        w.set_port(wl.eth_addr, wl.ip4_addr)
        w.set_l1(wl.l1)
        b = gpu.DeviceBatch(w, frames, desc)
        b.run()
        out_frames, verdict = b.fetch()
        b.free()
        counters, stats = w.get_stats()
    finally:
        w.close()
    assert np.array_equal(verdict, ref["verdict"])
    assert counters.tobytes() == np.asarray(ref["counters"]).tobytes()
    assert np.array_equal(stats, ref["rule_stats"])
    from upe_amd.layout import desc_lens, desc_offsets

    for o, go, ln in zip(desc_offsets(desc), desc_offsets(wl.desc), desc_lens(desc)):
        assert np.array_equal(out_frames[o:o + ln], ref["frames"][go:go + ln])


@pytest.mark.parametrize("emit", [False, True])
@pytest.mark.parametrize("n_rules", [4100, 65536, 65540, 1 << 17])
def test_group_by_key_forms(gpu_worker_factory, n_rules, emit):
    """rule_stats of tables past the LDS histogram: up to 64k rules the group-by reads one
    4-byte key per packet (rule << 16 | length) the classify pass leaves; past that the verdict
    word and a 2-byte length — both forms, and the boundary between them, against the oracle."""
    wl = synth.config_d(n=20_000, seed=91, n_rules=n_rules)
    frames, verdict, counters, stats, l1 = _run(gpu_worker_factory, wl, emit=emit)
    key = ("group_by", n_rules)
    if key not in _D_CACHE:   # up to ~12 s of oracle scans, shared by both modes
        _D_CACHE[key] = oracle.run_restated(wl)
    r = _D_CACHE[key]
    assert np.array_equal(verdict, r.verdict)
    assert np.array_equal(stats, r.rule_stats)
    assert counters.tobytes() == r.counters.tobytes()
    assert np.array_equal(frames, r.frames)


@pytest.mark.parametrize("emit", [False, True])
def test_config_c_ipv6_forwarding(gpu_worker_factory, emit):
    """Config C with its family-wide wildcards moved last (synth.config_c(v6_forwarding=True)):
    IPv6 packets now reach the NDP lookup and are forwarded with the hop-limit rewrite, and match
    at spread-out positions of the 1k-rule table (deep linear scans) — against the reference
    worker itself (oracle/_ref) on the same batch: verdicts, bytes, counters, rule_stats, L1."""
    from upe_amd.layout import desc_offsets

    wl = synth.config_c(n=60_000, seed=3, v6_forwarding=True)
    got = _run(gpu_worker_factory, wl, emit=emit)
    key = ("c6", 60_000)
    if key not in _D_CACHE:
        _D_CACHE[key] = oracle.run_reference(wl) if oracle.ref_available() else oracle.run_restated(wl)
    ref = _D_CACHE[key]
    frames, verdict, counters, stats, l1 = got
    assert np.array_equal(verdict, ref.verdict)
    assert np.array_equal(frames, ref.frames)
    assert counters.tobytes() == ref.counters.tobytes()
    assert np.array_equal(stats, ref.rule_stats)
    assert l1.tobytes() == ref.l1.tobytes()
    offs = desc_offsets(wl.desc)
    is6 = wl.frames[offs + 12] == 0x86
    fwd6 = ((verdict & 0xF) == V_FWD) & is6 & ((verdict & 0x10) != 0)
    assert fwd6.sum() > 1000, "IPv6 packets must be forwarded through the NDP table"


@pytest.mark.parametrize("tree", [False, True])
@pytest.mark.parametrize("kind", ["C", "C6", "CF", "big_linear"])
def test_linear_scan_flavours(gpu_worker_factory, monkeypatch, kind, tree):
    """The ways a linear table past 64 rules is matched, each against the oracle.  Without the
    tree (UPE_GPU_TREE=0): seed-3 config C (its IPv6 list is one catch-all: the whole table
    through the scalar unit), C6 and the flow-derived C (per-family lists, the IPv6 one in LDS,
    sorted indexes carried in the rule words) and a 16k-rule table with the tuple-space index
    switched off (per-family lists, sorted indexes from the index array).  With it (the default):
    every one through the decision tree."""
    monkeypatch.setenv("UPE_GPU_TREE", "1" if tree else "0")
    if kind == "big_linear":
        monkeypatch.setenv("UPE_GPU_TSS", "0")
        wl = synth.config_d(n=30_000, seed=93, n_rules=1 << 14)
        want = gpu.VAR_FAM
    elif kind == "CF":
        wl = synth.config_c_flows(n=40_000, seed=5)
        want = gpu.VAR_FAM
    else:
        wl = synth.config_c(n=40_000, seed=3, v6_forwarding=kind == "C6")   # seed 3: C's rules
        want = gpu.VAR_GLB if kind == "C" else gpu.VAR_FAM
    if tree:
        want = gpu.VAR_TREE
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        frames, verdict, counters, stats, l1 = gpu.run_workload(wl, worker=w)
        info = w.launch_info()
    finally:
        w.close()
    assert info["variant"] & gpu.VAR_SCAN == want
    r = oracle.run_restated(wl)
    assert np.array_equal(verdict, r.verdict)
    assert np.array_equal(frames, r.frames)
    assert counters.tobytes() == r.counters.tobytes()
    assert np.array_equal(stats, r.rule_stats)
    assert l1.tobytes() == r.l1.tobytes()


def _mixed_table(n_rules: int, seed: int):
    return synth.mixed_table(n_rules, seed)


@pytest.mark.parametrize("emit", [False, True])
@pytest.mark.parametrize("table", ["mixed_64k", "flows_16k"])
def test_large_linear_tables(gpu_worker_factory, table, emit):
    """Tables with many mask signatures past the LDS (the tuple-space index declines them), so
    the decision tree is read from memory: a 64k-rule config-C-style random table over config C's
    traffic (early first matches), and a 16k-rule flow-derived table whose first matches spread
    over the whole table (deep scans for the reference) — against the oracle on 20k packets."""
    if table == "mixed_64k":
        wl = synth.config_c(n=20_000, seed=61)
        wl.rules = _mixed_table(1 << 16, 61)
        wl.capacity = 1 << 16
    else:
        wl = synth.config_c_flows(n=20_000, seed=62, n_rules=1 << 14, max_cover=2.0 ** -18)
    key = ("large", table)
    if key not in _D_CACHE:
        _D_CACHE[key] = oracle.run_restated(wl)
    r = _D_CACHE[key]
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        assert w.rule_index_kind() == 2
        frames, verdict, counters, stats, l1 = _run(gpu_worker_factory, wl, emit=emit)
    finally:
        w.close()
    assert np.array_equal(verdict, r.verdict)
    assert np.array_equal(frames, r.frames)
    assert counters.tobytes() == r.counters.tobytes()
    assert np.array_equal(stats, r.rule_stats)
    assert l1.tobytes() == r.l1.tobytes()
