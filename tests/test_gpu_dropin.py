"""The drop-in claim, tested: the REFERENCE pipeline (RX-like producer -> reference SPSC ring ->
reference worker_t, built from the reference's sources by oracle/Makefile) running this repo's
GPU worker loop (upe_gpu_worker_run, upe_amd/csrc/upe_worker.c, through the binding
oracle/dropin_worker.c that INTEGRATION.md shows) ends with the same worker counters, rule_stats,
packet bytes and neighbour tables as the reference's own src/worker.c on the same packets — also
when ARP / NS / NA packets inside the stream teach entries that later packets are forwarded with,
and when the stats thread reloads the rules in the middle of the stream (src/main.c:216-282) —
and makes exactly the TX calls the reference's worker_main makes for the bursts it popped: one
tx_send_batch per burst with forwarded packets, holding them in packet order
(src/worker.c:240-243, 287-303), and a tx_send per answered ARP request (src/worker.c:52)."""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

import oracle
from upe_amd import synth
from upe_amd.layout import RULE_DTYPE, RULE_STAT_DTYPE, V_FWD, desc_lens, desc_offsets

pytestmark = pytest.mark.gpu

SO = os.path.join(os.path.dirname(oracle.__file__), "_ref", "libupe_dropin.so")


def _lib():
    if not os.path.exists(SO):
        pytest.fail(f"{SO} not built (make -C oracle where the reference sources exist)")
    lib = ctypes.CDLL(SO)
    P, SZ = ctypes.c_void_p, ctypes.c_size_t
    lib.upe_dropin_run.restype = ctypes.c_int
    lib.upe_dropin_run.argtypes = [P, SZ, SZ, P, SZ, P, SZ, P, ctypes.c_uint32, P, P, SZ,
                                   ctypes.c_int, P, P, P, P, P,
                                   P, SZ, SZ, SZ, P, SZ, P, P, P, P, P]
    lib.upe_dropin_set_mapped.argtypes = [ctypes.c_int]
    lib.upe_dropin_set_mapped.restype = None
    return lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _with_control(n, seed):
    from test_gpu_control import with_control

    return with_control(synth.config_c(n=n, seed=seed), 60, seed)


def _dropin(wl, mapped, reload=None):
    """The stream through the pipeline; reload = (rules_b in insertion order, cap_b, at).
    Returns (counters[5], rule_stats, frames, arp, ndp, stats_a, log) with log = (pops, tx call
    sizes, tx packet indexes, reply packet indexes)."""
    lib = _lib()
    lib.upe_dropin_set_mapped(1 if mapped else 0)
    rules = np.ascontiguousarray(wl.rules, dtype=RULE_DTYPE)
    eth = np.frombuffer(bytes(wl.eth_addr), np.uint8).copy()
    counters = np.zeros(5, np.uint64)
    cap_out = reload[1] if reload else wl.capacity
    stats = np.zeros(cap_out, RULE_STAT_DTYPE)
    stats_a = np.zeros(wl.capacity, RULE_STAT_DTYPE)
    frames = wl.frames.copy()
    arp, ndp = wl.arp.copy(), wl.ndp.copy()
    cap = wl.n + 16
    pops, sizes, tx, replies = (np.zeros(cap, np.uint32) for _ in range(4))
    log_n = np.zeros(4, np.uint64)
    rb = np.ascontiguousarray(reload[0], dtype=RULE_DTYPE) if reload else None
    rc = lib.upe_dropin_run(_p(rules), len(rules), wl.capacity, _p(wl.arp), len(wl.arp),
                            _p(wl.ndp), len(wl.ndp), _p(eth), wl.ip4_addr, _p(wl.frames),
                            _p(wl.desc), wl.n, 0, _p(counters), _p(stats), _p(frames), _p(arp),
                            _p(ndp), _p(rb) if reload else None, len(rb) if reload else 0,
                            reload[1] if reload else 0, reload[2] if reload else 0,
                            _p(stats_a), cap, _p(pops), _p(sizes), _p(tx), _p(replies),
                            _p(log_n))
    assert rc == 0
    k = [int(x) for x in log_n]
    return counters, stats, frames, arp, ndp, stats_a, (pops[:k[0]], sizes[:k[1]], tx[:k[2]],
                                                       replies[:k[3]])


def _check_tx(log, verdict, n):
    """The TX calls worker_main makes for the popped bursts (src/worker.c:240-243, 287-303)."""
    pops, sizes, tx, replies = log
    assert int(pops.sum()) == n, "the worker did not pop every packet"
    fwd = (verdict & 0xF) == V_FWD
    want_sizes, want_tx = [], []
    s = 0
    for k in pops.tolist():
        idx = np.nonzero(fwd[s:s + k])[0] + s
        if idx.size:
            want_sizes.append(idx.size)
            want_tx.extend(idx.tolist())
        s += k
    assert sizes.tolist() == want_sizes, "tx_send_batch calls differ from the reference's"
    assert tx.tolist() == want_tx, "frames handed to tx_send_batch differ from the reference's"
    assert replies.tolist() == np.nonzero(verdict & 0x40)[0].tolist(), "ARP replies differ"


def _check_bytes_tables(wl, frames, arp, ndp, ref):
    offs, lens = desc_offsets(wl.desc), desc_lens(wl.desc)
    bad = [i for i, (o, ln) in enumerate(zip(offs, lens))
           if not np.array_equal(frames[o:o + ln], ref.frames[o:o + ln])]
    assert not bad, f"{len(bad)} packets differ from the reference worker's bytes, first {bad[:5]}"
    keep = ["ip", "mac", "valid"]
    assert np.array_equal(arp[keep], ref.arp[keep]), "ARP table differs"
    assert np.array_equal(ndp[keep], ref.ndp[keep]), "NDP table differs"


@pytest.mark.parametrize("make", [lambda: synth.config_b(n=150_000, seed=61),
                                  lambda: synth.config_c(n=150_000, seed=62),
                                  lambda: _with_control(60_000, 63),
                                  lambda: synth.config_ndp_walk(repeat=20)],
                         ids=["B", "C", "C+control", "NS/NA opt_len wrap"])
@pytest.mark.parametrize("mapped", [False, True], ids=["windows", "mapped-pool"])
def test_reference_pipeline_with_gpu_worker(make, mapped):
    """mapped-pool: the reference's pktbuf pool registered with upe_gpu_host_register and each
    batch classified where its pktbufs lie (upe_gpu_process_mapped), frames rewritten in the pool
    itself."""
    wl = make()
    counters, stats, frames, arp, ndp, _, log = _dropin(wl, mapped)
    ref = oracle.run_reference(wl)
    want = [int(x) for x in ref.counters[0].tolist()[:5]]
    assert [int(x) for x in counters] == want
    assert np.array_equal(stats, ref.rule_stats)
    _check_bytes_tables(wl, frames, arp, ndp, ref)
    _check_tx(log, ref.verdict, wl.n)


@pytest.mark.parametrize("name", ["B", "C"])
@pytest.mark.parametrize("mapped", [False, True], ids=["windows", "mapped-pool"])
def test_reference_pipeline_rule_reload(name, mapped):
    """The stats thread's SIGHUP reload (src/main.c:237-265: new table, fresh rule_stats, both
    swapped into the worker_t) after the first part of the stream: the binding sees the swap
    between two bursts and reloads the context (upe_gpu_reload_rules).  Counters, the new and
    the old rule_stats arrays, bytes and TX calls equal the reference worker's with the same
    swap (oracle/ref_harness.c upe_refh_process_reload)."""
    import reload_util

    wl, rules_b, at, cap_b = reload_util.case(name)
    counters, stats, frames, arp, ndp, stats_a, log = _dropin(wl, mapped, (rules_b, cap_b, at))
    ref, old_ref = oracle.run_reference_reload(wl, rules_b, cap_b, at)
    want = [int(x) for x in ref.counters[0].tolist()[:5]]
    assert [int(x) for x in counters] == want
    assert np.array_equal(stats_a, old_ref), "the rule_stats swapped out differ"
    assert np.array_equal(stats, ref.rule_stats), "the new rule_stats differ"
    _check_bytes_tables(wl, frames, arp, ndp, ref)
    _check_tx(log, ref.verdict, wl.n)
