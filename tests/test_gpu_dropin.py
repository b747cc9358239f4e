"""The drop-in claim, tested: the REFERENCE pipeline (RX-like producer -> reference SPSC ring ->
reference worker_t, built from the reference's sources by oracle/Makefile) running this repo's
GPU worker loop (oracle/dropin_worker.c, the loop INTEGRATION.md shows) ends with the same
worker counters, rule_stats, packet bytes and neighbour tables as the reference's own
src/worker.c on the same packets — also when ARP / NS / NA packets inside the stream teach
entries that later packets are forwarded with."""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

import oracle
from upe_amd import synth
from upe_amd.layout import RULE_STAT_DTYPE, desc_lens, desc_offsets

pytestmark = pytest.mark.gpu

SO = os.path.join(os.path.dirname(oracle.__file__), "_ref", "libupe_dropin.so")


def _lib():
    if not os.path.exists(SO):
        pytest.fail(f"{SO} not built (make -C oracle where the reference sources exist)")
    lib = ctypes.CDLL(SO)
    P, SZ = ctypes.c_void_p, ctypes.c_size_t
    lib.upe_dropin_run.restype = ctypes.c_int
    lib.upe_dropin_run.argtypes = [P, SZ, SZ, P, SZ, P, SZ, P, ctypes.c_uint32, P, P, SZ,
                                   ctypes.c_int, P, P, P, P, P]
    lib.upe_dropin_set_mapped.argtypes = [ctypes.c_int]
    lib.upe_dropin_set_mapped.restype = None
    return lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _with_control(n, seed):
    from test_gpu_control import with_control

    return with_control(synth.config_c(n=n, seed=seed), 60, seed)


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
    lib = _lib()
    lib.upe_dropin_set_mapped(1 if mapped else 0)
    rules = np.ascontiguousarray(wl.rules)
    eth = np.frombuffer(bytes(wl.eth_addr), np.uint8).copy()
    counters = np.zeros(5, np.uint64)
    stats = np.zeros(wl.capacity, RULE_STAT_DTYPE)
    frames = wl.frames.copy()
    arp, ndp = wl.arp.copy(), wl.ndp.copy()
    rc = lib.upe_dropin_run(_p(rules), len(rules), wl.capacity, _p(wl.arp), len(wl.arp),
                            _p(wl.ndp), len(wl.ndp), _p(eth), wl.ip4_addr, _p(wl.frames),
                            _p(wl.desc), wl.n, 0, _p(counters), _p(stats), _p(frames), _p(arp),
                            _p(ndp))
    assert rc == 0
    ref = oracle.run_reference(wl)
    want = [int(x) for x in ref.counters[0].tolist()[:5]]
    assert [int(x) for x in counters] == want
    assert np.array_equal(stats, ref.rule_stats)
    offs, lens = desc_offsets(wl.desc), desc_lens(wl.desc)
    bad = [i for i, (o, ln) in enumerate(zip(offs, lens))
           if not np.array_equal(frames[o:o + ln], ref.frames[o:o + ln])]
    assert not bad, f"{len(bad)} packets differ from the reference worker's bytes, first {bad[:5]}"
    keep = ["ip", "mac", "valid"]
    assert np.array_equal(arp[keep], ref.arp[keep]), "ARP table differs"
    assert np.array_equal(ndp[keep], ref.ndp[keep]), "NDP table differs"
