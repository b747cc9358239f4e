"""The C-ABI library: loads, exports every symbol include/upe_gpu.h declares, and the struct
layouts the Python side uses agree with the C header (which static-asserts them against the
reference layouts).  No compute calls: these run without a GPU."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

from upe_amd import layout

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "upe_gpu.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(upe_[a-z0-9_]+)\s*\(", src)))


def test_library_loads_and_exports_every_declared_symbol():
    from upe_amd import gpu

    lib = ctypes.CDLL(gpu.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) >= 18
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, f"declared in upe_gpu.h but not exported: {missing}"
    assert sorted(gpu.EXPORTED) == syms


def test_library_is_gfx950_code_object():
    from upe_amd import gpu

    # the embedded offload bundle names its target triple
    data = open(gpu.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


C_LAYOUT = r"""
#include <stdio.h>
#include <stddef.h>
#include "upe_gpu.h"
#define P(t, f) printf(#t "." #f " %zu\n", offsetof(t, f))
#define S(t) printf(#t " %zu\n", sizeof(t))
int main(void) {
  S(upe_rule_t); P(upe_rule_t, priority); P(upe_rule_t, ip_ver); P(upe_rule_t, src_ip);
  P(upe_rule_t, src_mask); P(upe_rule_t, dst_ip); P(upe_rule_t, dst_mask);
  P(upe_rule_t, src_port); P(upe_rule_t, dst_port); P(upe_rule_t, protocol);
  P(upe_rule_t, action); P(upe_rule_t, rule_id);
  S(upe_arp_entry_t); P(upe_arp_entry_t, mac); P(upe_arp_entry_t, update_at); P(upe_arp_entry_t, valid);
  S(upe_ndp_entry_t); P(upe_ndp_entry_t, mac); P(upe_ndp_entry_t, update_at); P(upe_ndp_entry_t, valid);
  S(upe_l1_state_t); P(upe_l1_state_t, last_arp_mac); P(upe_l1_state_t, last_ndp_ip);
  P(upe_l1_state_t, last_ndp_mac);
  S(upe_counters_t); S(upe_batch_info_t); P(upe_batch_info_t, n_ctrl); P(upe_batch_info_t, first_ctrl);
  S(upe_rule_stat_t);
  S(upe_launch_info_t); P(upe_launch_info_t, deferred); P(upe_launch_info_t, launches);
  S(upe_gpu_batch_t); P(upe_gpu_batch_t, verdict); P(upe_gpu_batch_t, n);
  return 0;
}
"""


def test_struct_layouts_match_numpy_mirrors():
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "l.c")
        exe = os.path.join(d, "l")
        open(src, "w").write(C_LAYOUT)
        subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), src, "-o", exe],
                       check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout
    got = dict(line.rsplit(" ", 1) for line in out.strip().splitlines())
    got = {k: int(v) for k, v in got.items()}
    R = layout.RULE_DTYPE
    assert got["upe_rule_t"] == R.itemsize == 92
    for f in ("priority", "ip_ver", "src_ip", "src_mask", "dst_ip", "dst_mask", "src_port",
              "dst_port", "protocol", "rule_id"):
        assert got[f"upe_rule_t.{f}"] == R.fields[f][1], f
    assert got["upe_rule_t.action"] == R.fields["action"][1]
    for name, dt in (("upe_arp_entry_t", layout.ARP_DTYPE), ("upe_ndp_entry_t", layout.NDP_DTYPE)):
        assert got[name] == dt.itemsize
        for f in ("mac", "update_at", "valid"):
            assert got[f"{name}.{f}"] == dt.fields[f][1]
    L = layout.L1_DTYPE
    assert got["upe_l1_state_t"] == L.itemsize
    for f in ("last_arp_mac", "last_ndp_ip", "last_ndp_mac"):
        assert got[f"upe_l1_state_t.{f}"] == L.fields[f][1]
    assert got["upe_counters_t"] == layout.COUNTERS_DTYPE.itemsize
    assert got["upe_batch_info_t"] == layout.BATCH_INFO_DTYPE.itemsize
    assert got["upe_batch_info_t.n_ctrl"] == layout.BATCH_INFO_DTYPE.fields["n_ctrl"][1]
    assert got["upe_rule_stat_t"] == layout.RULE_STAT_DTYPE.itemsize
    LI = layout.LAUNCH_INFO_DTYPE
    assert got["upe_launch_info_t"] == LI.itemsize
    assert got["upe_launch_info_t.deferred"] == LI.fields["deferred"][1]
    assert got["upe_launch_info_t.launches"] == LI.fields["launches"][1]
    import ctypes

    from upe_amd.gpu import QueueBatch
    assert got["upe_gpu_batch_t"] == ctypes.sizeof(QueueBatch) == 40
    assert got["upe_gpu_batch_t.verdict"] == QueueBatch.verdict.offset
    assert got["upe_gpu_batch_t.n"] == QueueBatch.n.offset


def test_header_compiles_as_c_and_cpp():
    with tempfile.TemporaryDirectory() as d:
        for lang, comp, ext in (("c", "gcc", "c"), ("c++", "g++", "cc")):
            src = os.path.join(d, f"h.{ext}")
            open(src, "w").write('#include "upe_gpu.h"\nint main(void){return 0;}\n')
            subprocess.run([comp, "-Wall", "-Werror", "-pedantic", "-I",
                            os.path.join(ROOT, "include"), src, "-o", os.path.join(d, "h")],
                           check=True)


def test_open_without_gpu_fails_cleanly():
    from upe_amd import gpu

    if gpu.device_count() > 0:
        pytest.skip("a GPU is visible; the GPU suite covers open()")
    with pytest.raises(gpu.UpeGpuError):
        gpu.GpuWorker(0, 16)
    assert gpu.LIB.upe_gpu_last_error()


def test_verdict_helpers():
    v = np.array([layout.V_FWD | layout.VF_NEIGH_HIT | (3 << 8), layout.V_DROP_PARSE],
                 dtype=np.uint32)
    assert layout.verdict_code(v).tolist() == [layout.V_FWD, layout.V_DROP_PARSE]
    assert layout.verdict_rule(v).tolist() == [2, -1]
    d = layout.make_desc(np.array([0, 64]), np.array([64, 1518]))
    assert layout.desc_offsets(d).tolist() == [0, 64]
    assert layout.desc_lens(d).tolist() == [64, 1518]


def test_record_layout_version():
    """the emit-mode record layout changed in round 5 (records compacted per 64-packet
    group); the header names the layout and the library reports the one it was built with."""
    from upe_amd import gpu

    m = re.search(r"#define UPE_HDR_LAYOUT (\d+)", open(HEADER).read())
    assert m and int(m.group(1)) == 2
    assert gpu.LIB.upe_gpu_hdr_layout() == 2
