"""GPU parity of both neighbour-lookup paths.  Indexes of up to 2048 slots per family are staged
in LDS and looked up there; larger ones are read from memory (upe_gpu.hip `a.arp_lds` /
`a.ndp_lds`).  The benchmark configurations all fit in LDS, so these cases enlarge the ARP and/or
NDP table of a config-C stream (IMIX, v4 + v6, 1k rules) past 2048 slots — extra reachable
entries that no packet is aimed at — and compare every output with the oracle: one table in
memory and the other in LDS, both in memory, and with a starting L1 state that disagrees with
the table (the look-back path), in both output modes."""
from __future__ import annotations

import dataclasses

import numpy as np
import pytest

import oracle
from upe_amd import gpu, synth
from upe_amd.layout import L1_DTYPE

pytestmark = pytest.mark.gpu


def _grow(wl, arp_extra: int, ndp_extra: int, seed: int):
    """The same workload with `arp_extra` / `ndp_extra` more valid entries in tables of 8192
    slots (reachable entries at load factor 0.4 need > 2048 cuckoo slots past ~820 entries)."""
    rng = np.random.default_rng(seed)
    arp, ndp = wl.arp, wl.ndp
    if arp_extra:
        ents = [(int(e["ip"]), bytes(e["mac"])) for e in arp if e["valid"]]
        used = {ip for ip, _ in ents}
        want = len(ents) + arp_extra
        while len(ents) < want:
            ip = int(rng.integers(0x0B000000, 0x0BFFFFFF))
            if ip not in used:
                used.add(ip)
                ents.append((ip, rng.integers(0, 256, 6, dtype=np.uint8).tobytes()))
        arp = synth.arp_table(8192, ents)
    if ndp_extra:
        ents = [(bytes(e["ip"]), bytes(e["mac"])) for e in ndp if e["valid"]]
        base = len(ents)
        for _ in range(ndp_extra):
            ip = bytes.fromhex("20010db9") + rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
            ents.append((ip, rng.integers(0, 256, 6, dtype=np.uint8).tobytes()))
        assert len(ents) == base + ndp_extra
        ndp = synth.ndp_table(8192, ents)
    return dataclasses.replace(wl, arp=arp, ndp=ndp)


def _check(worker_factory, wl, emit, l1=None, what=""):
    r = oracle.run_restated(wl, l1=l1)
    w = worker_factory(wl.capacity)
    try:
        w.configure(wl)
        if l1 is not None:
            w.set_l1(l1)
        frames, verdict, counters, stats, got_l1 = gpu.run_workload(wl, worker=w, emit=emit)
    finally:
        w.close()
    bad = np.nonzero(verdict != r.verdict)[0]
    assert bad.size == 0, f"{what}: {bad.size} verdicts differ, first {bad[:8].tolist()}"
    assert np.array_equal(frames, r.frames), f"{what}: frames differ"
    assert counters.tobytes() == np.asarray(r.counters).tobytes(), what
    assert np.array_equal(stats, r.rule_stats), what
    assert got_l1.tobytes() == np.asarray(r.l1).tobytes(), what


@pytest.mark.parametrize("emit", [False, True])
@pytest.mark.parametrize("arp_extra,ndp_extra", [(1500, 0), (0, 1500), (1500, 1500)],
                         ids=["arp-memory", "ndp-memory", "both-memory"])
def test_neighbour_index_in_memory(gpu_worker_factory, arp_extra, ndp_extra, emit):
    wl = _grow(synth.config_c(n=120_000, seed=81), arp_extra, ndp_extra, 81)
    _check(gpu_worker_factory, wl, emit, what=f"arp+{arp_extra} ndp+{ndp_extra} emit={emit}")


@pytest.mark.parametrize("emit", [False, True])
def test_neighbour_index_in_memory_inconsistent_l1(gpu_worker_factory, emit):
    """A starting L1 state whose entries disagree with the tables: the packets aimed at them take
    the stale MAC until the first miss-then-hit (look-back), with lookups from memory."""
    wl = _grow(synth.config_c(n=120_000, seed=82), 1500, 1500, 82)
    offs = wl.desc >> np.uint64(16)
    fr = wl.frames
    i4 = next(i for i in range(wl.n) if fr[offs[i] + 12] == 0x08 and fr[offs[i] + 13] == 0x00)
    i6 = next(i for i in range(wl.n) if fr[offs[i] + 12] == 0x86 and fr[offs[i] + 13] == 0xDD)
    l1 = np.zeros(1, L1_DTYPE)
    o4, o6 = int(offs[i4]), int(offs[i6])
    l1["last_arp_ip"] = int.from_bytes(bytes(fr[o4 + 30:o4 + 34]), "big")
    l1["last_arp_mac"] = np.frombuffer(bytes.fromhex("02deadbeef01"), np.uint8)
    l1["last_ndp_ip"] = np.frombuffer(bytes(fr[o6 + 38:o6 + 54]), np.uint8)
    l1["last_ndp_mac"] = np.frombuffer(bytes.fromhex("02deadbeef02"), np.uint8)
    _check(gpu_worker_factory, wl, emit, l1=l1, what=f"inconsistent L1 emit={emit}")
