"""Fuzzed frames: valid IMIX headers with random byte flips, random truncations and wholly
random frames, so that every parse gate of parse_flow_key (reference src/parser.c:6-111), the
control-packet branches of handle_control_packet (src/worker.c:23-104) and the general path see
inputs no generator was written for.  One batch on the GPU against the C restatement with
control writes deferred (the GPU's one-batch semantics; the restatement is pinned to the
reference worker by tests/test_oracle.py and the golden vectors)."""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from test_gpu_control import _rows
from test_gpu_parity import _assert_same, _run
from upe_amd import synth

pytestmark = pytest.mark.gpu


def fuzzed(seed: int, n: int) -> synth.Workload:
    rng = np.random.default_rng(seed)
    wl = synth.config_c(n=n, seed=seed)
    h, lens = _rows(wl)
    lens = np.minimum(lens, 128)          # header rows carry the first 128 bytes
    k = len(h)
    # byte flips in the header region of 40 % of the frames
    flip = rng.random(k) < 0.4
    for i in np.nonzero(flip)[0]:
        pos = rng.integers(0, 96, rng.integers(1, 4))
        h[i, pos] = rng.integers(0, 256, len(pos), dtype=np.uint8)
    # ethertype / version / protocol / IHL / doff hot spots in another 20 %
    hot = rng.random(k) < 0.2
    spots = np.array([12, 13, 14, 20, 23, 46, 66])
    for i in np.nonzero(hot)[0]:
        s = rng.choice(spots)
        h[i, s] = rng.integers(0, 256, dtype=np.uint8)
    # truncations of 15 %
    cut = rng.random(k) < 0.15
    lens[cut] = rng.integers(0, np.maximum(lens[cut], 1) + 1)
    # wholly random frames (5 %), a third of them with a real ethertype
    rnd = np.nonzero(rng.random(k) < 0.05)[0]
    h[rnd] = rng.integers(0, 256, (len(rnd), 128), dtype=np.uint8)
    et = rng.choice([0x0800, 0x86DD, 0x0806], len(rnd))
    keep = rng.random(len(rnd)) < 0.33
    h[rnd[keep], 12] = (et[keep] >> 8).astype(np.uint8)
    h[rnd[keep], 13] = (et[keep] & 0xFF).astype(np.uint8)
    lens[rnd] = rng.integers(0, 129, len(rnd))
    frames, desc = synth.pack_frames(h, lens)
    return synth.Workload(f"fuzz{seed}", frames, desc, wl.rules, wl.capacity, wl.arp.copy(),
                          wl.ndp.copy(), wl.eth_addr, wl.ip4_addr, wl.l1.copy())


@pytest.mark.parametrize("seed,n", [(51, 20000), (52, 50000), (53, 3000)])
def test_fuzzed_frames_match_oracle(gpu_worker_factory, seed, n):
    wl = fuzzed(seed, n)
    r = oracle.run_restated(wl, apply_control=False)
    if oracle.ref_available():
        # these seeds carry no table-writing control packet, so the reference worker itself
        # agrees with the deferred-write restatement
        ref = oracle.run_reference(wl)
        assert np.array_equal(ref.frames, r.frames)
        assert np.array_equal(ref.verdict & ~np.uint32(0x80), r.verdict & ~np.uint32(0x80))
    got = _run(gpu_worker_factory, wl)
    _assert_same(got, {"verdict": r.verdict, "frames": r.frames, "counters": r.counters,
                       "rule_stats": r.rule_stats, "l1": r.l1}, f"fuzz {seed}")
    # the fuzz reached the slow and failing paths, not only the fast path
    code = r.verdict & 0xF
    assert (code == 0).sum() > n // 20          # parse failures
    assert (code == 4).sum() > n // 10          # still plenty forwarded
