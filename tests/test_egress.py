"""Egress (upe_tx_flush, include/upe_gpu.h) against the reference worker's own TX calls: the
forwarded frames of a classified batch, in packet order, handed to tx_send_batch once per input
burst of WORKER_BURST_SIZE packets (reference src/worker.c:240-243, 287-303; sendmmsg cap of 64,
src/tx_afpacket.c:82-84).  The reference side is the harness's log of every tx_send_batch call of
src/worker.c itself (oracle/_ref, built from the reference sources); the verdicts fed to
upe_tx_flush are the golden (reference) verdicts, so these tests need no GPU — the GPU side is
tests/test_gpu_rss_egress.py."""
from __future__ import annotations

import numpy as np
import pytest

import golden_io
import oracle
from upe_amd import gpu
from upe_amd.layout import desc_lens, desc_offsets

WORKER_BURST_SIZE = 32   # reference include/worker.h


def _need_ref():
    if not oracle.ref_available():
        pytest.skip("oracle/_ref not built (needs the reference sources)")


@pytest.mark.parametrize("case", ["config_a", "config_b_small", "config_c_small",
                                  "config_d_small"])
def test_tx_batches_equal_reference(case):
    _need_ref()
    wl, ref = golden_io.load(case)
    r = oracle.run_reference(wl)
    assert np.array_equal(r.verdict, ref["verdict"])
    sizes, order = oracle.tx_log()
    batches, fwd, drp = gpu.tx_flush(r.frames, wl.desc, r.verdict, WORKER_BURST_SIZE)
    assert [len(b[0]) for b in batches] == sizes.tolist(), "TX call sizes differ"
    got = np.concatenate([b[0] for b in batches]) if batches else np.zeros(0, np.int64)
    assert np.array_equal(got, order.astype(np.int64)), "TX frame order differs"
    # the bytes each call hands to sendmmsg: the reference's rewritten frames
    offs, lens = desc_offsets(wl.desc), desc_lens(wl.desc)
    for idx, data in batches:
        for i, d in zip(idx, data):
            assert d == bytes(r.frames[offs[i]:offs[i] + lens[i]])
    assert fwd == int(r.counters["pkts_forwarded"][0]) and drp == 0


def test_tx_partial_sends_counted_as_the_worker_counts():
    """sendmmsg sending fewer than asked: forwarded += sent, dropped += count - sent
    (src/worker.c:288-294)."""
    wl, ref = golden_io.load("config_b_small")
    batches, fwd, drp = gpu.tx_flush(ref["frames"], wl.desc, ref["verdict"], WORKER_BURST_SIZE,
                                     sent_of=lambda c: c // 2)
    total = sum(len(b[0]) for b in batches)
    assert fwd == sum(len(b[0]) // 2 for b in batches)
    assert fwd + drp == total == int(np.count_nonzero((ref["verdict"] & 0xF) == 4))
    # a failing call (negative) counts every frame of the batch as dropped
    batches, fwd, drp = gpu.tx_flush(ref["frames"], wl.desc, ref["verdict"], 16,
                                     sent_of=lambda c: -1)
    assert fwd == 0 and drp == total


@pytest.mark.parametrize("burst", [1, 7, 64])
def test_tx_burst_sizes(burst):
    """Other burst sizes: one call per burst that forwarded anything, packet order kept."""
    wl, ref = golden_io.load("config_c_small")
    v = ref["verdict"]
    batches, fwd, _ = gpu.tx_flush(ref["frames"], wl.desc, v, burst)
    fwd_idx = np.nonzero((v & 0xF) == 4)[0]
    assert np.array_equal(np.concatenate([b[0] for b in batches]), fwd_idx)
    want = [int(np.count_nonzero(fwd_idx // burst == k)) for k in np.unique(fwd_idx // burst)]
    assert [len(b[0]) for b in batches] == want
    assert fwd == fwd_idx.size


@pytest.mark.parametrize("burst", [0, 65])
def test_tx_burst_out_of_range(burst):
    wl, ref = golden_io.load("config_b_small")
    with pytest.raises(gpu.UpeGpuError, match="burst"):
        gpu.tx_flush(ref["frames"], wl.desc, ref["verdict"], burst)


def grouped_list(verdict: np.ndarray):
    """The egress list by 64-packet group that upe_gpu_process_emit_tx writes (include/upe_gpu.h):
    group g's forwarded packets at tx[64g ..], their count in tx_count[g]; slots past a count left
    as garbage (0xDEADBEEF here, to catch a reader that looks at them)."""
    n = len(verdict)
    fwd = (verdict & 0xF) == 4
    tx = np.full(max(n, 1), 0xDEADBEEF, np.uint32)
    cnt = np.zeros((n + 63) // 64, np.uint32)
    for g in range(len(cnt)):
        idx = np.nonzero(fwd[64 * g:64 * g + 64])[0] + 64 * g
        tx[64 * g:64 * g + len(idx)] = idx
        cnt[g] = len(idx)
    return tx, cnt


@pytest.mark.parametrize("burst", [32, 7, 64, 1])
@pytest.mark.parametrize("case", ["config_a", "config_b_small", "config_cf_small",
                                  "config_d_small"])
def test_tx_from_grouped_list_equals_reference(case, burst):
    """upe_tx_flush_groups (the TX calls from the in-pass egress list) makes exactly the calls
    upe_tx_flush makes from the verdicts; at the worker's burst of 32 those are the reference
    worker's own tx_send_batch calls."""
    wl, ref = golden_io.load(case)
    v = ref["verdict"]
    want = gpu.tx_flush(ref["frames"], wl.desc, v, burst)
    got = gpu.tx_flush(ref["frames"], wl.desc, None, burst, groups=grouped_list(v))
    assert [b[0].tolist() for b in got[0]] == [b[0].tolist() for b in want[0]]
    assert [b[1] for b in got[0]] == [b[1] for b in want[0]]
    assert got[1:] == want[1:]
    if burst == WORKER_BURST_SIZE and oracle.ref_available():
        oracle.run_reference(wl)
        sizes, order = oracle.tx_log()
        assert [len(b[0]) for b in got[0]] == sizes.tolist()
