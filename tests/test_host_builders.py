"""Host-side batch builders (upe_amd/csrc/upe_host.c), CPU only:

* upe_rules_load_ini against the REFERENCE rule_config_load (golden outputs made by
  tests/golden/make_golden.py through oracle/_ref; live too where the harness is built): every
  accept / reject branch and quirk in tests/golden/ini_cases.py, rules.example and the file of
  reference tests/test_suite.c:592-633.
* upe_pcap_read on captures in the reference smoke test's format (tests/smoke-test.sh:38-49):
  record order, caplen > 2048 dropped as src/rx_pcap.c:53-57 drops it, BE / nanosecond files.
"""
from __future__ import annotations

import os
import struct
import sys

import numpy as np
import pytest

from upe_amd import gpu, synth
from upe_amd.layout import RULE_DTYPE, desc_lens, desc_offsets

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLDEN)
from ini_cases import cases  # noqa: E402

EXAMPLE = open(os.path.join(GOLDEN, "rules.example")).read()
REF = np.load(os.path.join(GOLDEN, "ini_cases.npz"), allow_pickle=False)


def _load(tmp_path, name, text, cap):
    p = tmp_path / f"{name}.conf"
    p.write_text(text)
    try:
        return 0, gpu.rules_load_ini(str(p), cap)
    except gpu.UpeGpuError as e:
        return -1, str(e)


def _same_rules(a, b):
    assert len(a) == len(b)
    for f in RULE_DTYPE.names:
        assert np.array_equal(a[f], b[f]), f


@pytest.mark.parametrize("name,text,cap", cases(EXAMPLE), ids=[c[0] for c in cases(EXAMPLE)])
def test_ini_matches_reference(tmp_path, name, text, cap):
    rc, got = _load(tmp_path, name, text, cap)
    assert rc == int(REF[f"{name}__rc"]), got
    if rc == 0:
        _same_rules(got, REF[f"{name}__rules"])
    else:
        assert got.startswith("rules:")


def test_rules_example_is_config_a_table(tmp_path):
    """rules.example through the loader == the table config A's golden vectors were made with."""
    rc, got = _load(tmp_path, "ex", EXAMPLE, 1024)
    assert rc == 0
    _same_rules(got, synth.build_rule_table(synth.rules_example()))


def test_ini_live_reference(tmp_path):
    import oracle

    if not oracle.ref_available():
        pytest.skip("reference harness not built here")
    import ctypes

    lib = oracle.ref_lib()
    lib.upe_refh_rules_load.restype = ctypes.c_int
    lib.upe_refh_rules_load.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p,
                                        ctypes.c_void_p]
    for name, text, cap in cases(EXAMPLE):
        p = tmp_path / f"live_{name}.conf"
        p.write_text(text)
        rules = np.zeros(cap, RULE_DTYPE)
        count = np.zeros(1, np.uint64)
        rc = lib.upe_refh_rules_load(str(p).encode(), cap, rules.ctypes.data, count.ctypes.data)
        rc2, got = _load(tmp_path, name, text, cap)
        assert rc == rc2, name
        if rc == 0:
            _same_rules(got, rules[: int(count[0])])


# ---- pcap --------------------------------------------------------------------------------

def write_pcap(path, frames, be=False, nsec=False):
    e = ">" if be else "<"
    magic = 0xA1B23C4D if nsec else 0xA1B2C3D4
    with open(path, "wb") as f:
        f.write(struct.pack(e + "IHHiIII", magic, 2, 4, 0, 0, 65535, 1))
        for i, fr in enumerate(frames):
            f.write(struct.pack(e + "IIII", i, 0, len(fr), len(fr)))
            f.write(fr)


def _frames_of(wl):
    offs, lens = desc_offsets(wl.desc), desc_lens(wl.desc)
    return [bytes(wl.frames[o:o + ln]) for o, ln in zip(offs, lens)]


@pytest.mark.parametrize("be,nsec", [(False, False), (True, False), (False, True)])
def test_pcap_round_trip(tmp_path, be, nsec):
    wl = synth.config_c(n=500, seed=41)
    frs = _frames_of(wl)
    frs.insert(7, bytes(3000))          # caplen > 2048: dropped by RX
    frs.insert(20, b"")                 # empty record: kept (parse fails later)
    p = tmp_path / "c.pcap"
    write_pcap(p, frs, be, nsec)
    frames, desc, info = gpu.pcap_read(str(p))
    assert int(info["records"][0]) == len(frs)
    assert int(info["dropped_oversize"][0]) == 1
    kept = [f for f in frs if len(f) <= 2048]
    assert desc.shape[0] == len(kept)
    offs, lens = desc_offsets(desc), desc_lens(desc)
    assert np.all(offs % 16 == 0)
    for f, o, ln in zip(kept, offs, lens):
        assert ln == len(f) and bytes(frames[o:o + ln]) == f
    assert frames.shape[0] >= int(offs[-1]) + 96


def test_pcap_rejects_bad_files(tmp_path):
    p = tmp_path / "bad.pcap"
    p.write_bytes(b"\x00" * 24)
    with pytest.raises(gpu.UpeGpuError):
        gpu.pcap_read(str(p))
    write_pcap(p, [bytes(64)])
    data = p.read_bytes()
    p.write_bytes(data[:-10])             # truncated record
    with pytest.raises(gpu.UpeGpuError):
        gpu.pcap_read(str(p))


def test_rule_image_compiles_without_a_gpu():
    """upe_rules_compile builds the table on the host alone (no context, no GPU: the stats thread
    can do it while the workers forward), for every index kind; bad arguments fail cleanly."""
    from upe_amd import gpu, synth

    for wl in (synth.config_b(n=64), synth.config_c_flows(n=64), synth.config_d(n=64)):
        im = gpu.RuleImage(wl.rules_sorted, wl.capacity)
        assert im.ptr
        im.free()
        im.free()   # idempotent
    wl = synth.config_b(n=64)
    with pytest.raises(gpu.UpeGpuError, match="capacity"):
        gpu.RuleImage(wl.rules_sorted, 0)
    with pytest.raises(gpu.UpeGpuError, match="exceeds the capacity"):
        gpu.RuleImage(wl.rules_sorted, 2)   # more rules than rule_stats entries
    r = wl.rules_sorted.copy()
    r["rule_id"][0] = 1000
    with pytest.raises(gpu.UpeGpuError, match="rule_id"):
        gpu.RuleImage(r, len(r))            # a rule id past the rule_stats
    gpu.LIB.upe_rules_image_free(None)
