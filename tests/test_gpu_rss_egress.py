"""GPU: software RSS in the classify pass (flow_hash, reference src/parser.c:113-135 as the RX
thread applies it, src/rx_pcap.c:71-72) and the ordered egress list (the frames process_packet
queues for tx_send_batch, src/worker.c:240-243), against the oracle."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

import golden_io
import oracle
from upe_amd import gpu, synth
from upe_amd.layout import V_FWD, V_DROP_RULE, desc_lens, desc_offsets

pytestmark = pytest.mark.gpu


def _expected_hashes(wl):
    lib = oracle.oracle_lib()
    offs, lens = desc_offsets(wl.desc), desc_lens(wl.desc)
    out = np.zeros(wl.n, np.uint32)
    for i in range(wl.n):
        fr = bytes(wl.frames[offs[i]:offs[i] + min(int(lens[i]), 2048)])
        rc, key = oracle.parse(fr, int(lens[i]))
        if rc == 0:
            out[i] = lib.upe_ref_flow_hash(key.ctypes.data_as(ctypes.c_void_p))
    return out


@pytest.mark.parametrize("case", ["config_b_small", "config_c_small", "config_d_small",
                                  "edge_zero"])
def test_flow_hash_in_pass(gpu_worker_factory, case):
    wl, ref = golden_io.load(case)
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        b = gpu.DeviceBatch(w, wl.frames, wl.desc)
        fh = w.malloc(4 * wl.n)
        w.process_rss(b.frames, b.desc, b.verdict, fh, wl.n)
        got = np.zeros(wl.n, np.uint32)
        w.d2h(got, fh)
        _, v = b.fetch()
        w.free(fh)
        b.free()
    finally:
        w.close()
    assert np.array_equal(got, _expected_hashes(wl))
    if not case.startswith("edge"):
        assert np.array_equal(v, ref["verdict"])


@pytest.mark.parametrize("n", [0, 1, 4095, 4096, 4097, 1 << 20])
@pytest.mark.parametrize("code", [V_FWD, V_DROP_RULE])
def test_egress_list_in_order(gpu_worker_factory, n, code):
    wl = synth.config_b(n=max(n, 1), seed=51)
    if n == 0:
        wl.desc = wl.desc[:0]
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        b = gpu.DeviceBatch(w, wl.frames, wl.desc)
        b.run()
        index = w.malloc(4 * max(n, 1))
        count = w.malloc(8)
        w.compact(b.verdict, n, code, index, count)
        k_arr = np.zeros(1, np.uint64)
        w.d2h(k_arr, count)
        w.sync()
        k = int(k_arr[0])
        got = np.zeros(max(k, 1), np.uint32)
        if k:
            w.d2h(got, index)
        _, v = b.fetch()
        w.free(index)
        w.free(count)
        b.free()
    finally:
        w.close()
    want = np.nonzero((v & 0xF) == code)[0]
    assert k == want.size
    assert np.array_equal(got[:k], want.astype(np.uint32))
