"""The decision-tree rule index (round 5) against the oracle's first match, on the CPU.

upe_rules_match_host walks the same image the GPU path builds (include/upe_gpu.h; the device's
tree_match is the same walk bit for bit), so these tests pin the index itself — the grouping into
a forest, the splits, the leaf truncation at a covering rule, the key-word order — against
reference rule_table_match semantics (src/rule_table.c:76-91,163-176, restated in
oracle/cpu_ref.c upe_ref_match) on tables of every shape: config C as flow-derived rules, seed-3
config C, C with IPv6 forwarded, config D's exact 5-tuples, the edge rules, and random tables
whose masks are not prefixes (version-agnostic rules, IPv4 views of IPv6 masks), with keys cut
from the traffic, from the rules' own boundaries and at random."""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from upe_amd import gpu, layout, synth
from upe_amd.layout import FLOW_KEY_DTYPE, RULE_DTYPE


def keys_of(wl, n: int = 6000) -> np.ndarray:
    """parse_flow_key of the workload's first n packets (the ones that parse)."""
    m = min(n, wl.n)
    keys = np.zeros(m, FLOW_KEY_DTYPE)
    offs = layout.desc_offsets(wl.desc)
    lens = layout.desc_lens(wl.desc)
    ok = np.zeros(m, bool)
    for i in range(m):
        o, ln = int(offs[i]), int(lens[i])
        rc, k = oracle.parse(bytes(wl.frames[o:o + min(ln, 128)]), ln)
        if rc == 0:
            keys[i:i + 1].view(np.uint8)[:] = k
            ok[i] = True
    return keys[ok]


def ref_match(rules_sorted: np.ndarray, keys: np.ndarray) -> np.ndarray:
    lib = oracle.oracle_lib()
    rs = np.ascontiguousarray(rules_sorted, dtype=RULE_DTYPE)
    keys = np.ascontiguousarray(keys, dtype=FLOW_KEY_DTYPE)   # (concatenate may repack fields)
    out = np.zeros(len(keys), np.int64)
    for i in range(len(keys)):
        out[i] = lib.upe_ref_match(oracle._ptr(rs), len(rs), keys[i:i + 1].ctypes.data_as(oracle._P))
    return out


def boundary_keys(rules_sorted: np.ndarray, rng, n: int) -> np.ndarray:
    """Keys on and just past the rules' own edges: a rule's value with the free bits all zero,
    all one or random, one word nudged by +-1, ports and protocol exact or off by one."""
    keys = np.zeros(n, FLOW_KEY_DTYPE)
    pick = rng.integers(0, len(rules_sorted), size=n)
    for i, j in enumerate(pick):
        r = rules_sorted[j]
        ver = int(r["ip_ver"]) or int(rng.choice([4, 6]))
        keys[i]["ip_ver"] = ver
        for a, m in (("src_ip", "src_mask"), ("dst_ip", "dst_mask")):
            v = r[a].astype(np.uint8)
            mk = r[m].astype(np.uint8)
            mode = rng.integers(0, 3)
            free = (np.zeros(16, np.uint8) if mode == 0 else np.full(16, 255, np.uint8)
                    if mode == 1 else rng.integers(0, 256, 16, dtype=np.uint8))
            k = (v & mk) | (free & ~mk)
            if rng.random() < 0.2:   # nudge one byte across an edge
                b = int(rng.integers(0, 4 if ver == 4 else 16))
                k[b] = (int(k[b]) + int(rng.choice([-1, 1]))) & 0xFF
            keys[i][a] = k
        for f, rf in (("src_port", "src_port"), ("dst_port", "dst_port")):
            v = int(r[rf])
            keys[i][f] = (v + int(rng.choice([0, 0, 0, 1, -1]))) & 0xFFFF if v else \
                int(rng.integers(0, 65536))
        p = int(r["protocol"])
        keys[i]["protocol"] = p if p and rng.random() < 0.8 else int(rng.choice([1, 6, 17]))
    return keys


def random_table(rng, n_rules: int, prefix_masks: bool) -> np.ndarray:
    """Rules with every field kind: versions 0 / 4 / 6, masks that are prefixes or arbitrary
    bit patterns (rule_t takes any mask: the tree's ranges must stay conservative), wildcards,
    and a catch-all at the end only half of the time (keys may then match nothing)."""
    r = np.zeros(n_rules, RULE_DTYPE)
    for i in range(n_rules):
        r[i]["priority"] = int(rng.integers(1, 1 << 20))
        r[i]["ip_ver"] = int(rng.choice([0, 4, 6], p=[0.2, 0.5, 0.3]))
        for a, m in (("src_ip", "src_mask"), ("dst_ip", "dst_mask")):
            if rng.random() < 0.3:
                continue
            if prefix_masks:
                if r[i]["ip_ver"] == 6 or (r[i]["ip_ver"] == 0 and rng.random() < 0.5):
                    mk = np.frombuffer(synth.ipv6_mask(int(rng.integers(0, 129))), np.uint8)
                else:
                    mk = np.zeros(16, np.uint8)
                    mk[:4] = np.frombuffer(np.uint32(synth.ipv4_mask(int(rng.integers(0, 33))))
                                           .astype("<u4").tobytes(), np.uint8)
            else:
                mk = rng.integers(0, 256, 16, dtype=np.uint8) & rng.integers(0, 256, 16,
                                                                              dtype=np.uint8)
            r[i][m] = mk
            r[i][a] = rng.integers(0, 4, 16, dtype=np.uint8) * 64   # few values: overlaps
        if rng.random() < 0.4:
            r[i]["src_port"] = int(rng.choice([53, 80, 443, 1234, 65535]))
        if rng.random() < 0.5:
            r[i]["dst_port"] = int(rng.choice([53, 80, 443, 22, 0x0800]))
        if rng.random() < 0.4:
            r[i]["protocol"] = int(rng.choice([1, 6, 17]))
        r[i]["action"] = int(rng.integers(0, 2))
    if rng.random() < 0.5:
        r[-1] = synth.make_rule(1 << 30, layout.ACT_DROP)
    return synth.build_rule_table(r)


def check(rules_sorted, keys, want_tree=True):
    got, info = gpu.rules_match_host(rules_sorted, keys)
    want = ref_match(rules_sorted, keys)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (f"{bad.size} of {len(keys)} keys differ, first {int(bad[0])}: "
                           f"tree {int(got[bad[0]])} vs oracle {int(want[bad[0]])}")
    if want_tree:
        assert info["nodes"] > 0, "the table got no tree"
    return info, want


WORKLOADS = {
    "C_flows": lambda: synth.config_c_flows(n=6000),
    "C_seed3": lambda: synth.config_c(n=6000),
    "C6": lambda: synth.config_c(n=6000, v6_forwarding=True),
    "D_4k_rules": lambda: synth.config_d(n=6000, n_rules=4096),
    "edge": lambda: synth.config_edge(),
}


@pytest.mark.parametrize("name", list(WORKLOADS))
def test_tree_equals_first_match_on_workloads(name):
    wl = WORKLOADS[name]()
    rs = wl.rules_sorted
    rng = np.random.default_rng(11)
    keys = np.concatenate([keys_of(wl), boundary_keys(rs, rng, 3000)])
    info, want = check(rs, keys, want_tree=len(rs) > 0)
    if name == "C_flows":
        # the flow-derived table's point: first matches spread over the whole table
        m = want[want >= 0]
        assert np.percentile(m, 90) > 0.7 * len(rs) and np.percentile(m, 10) < 0.3 * len(rs)


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
@pytest.mark.parametrize("prefix_masks", [True, False])
def test_tree_equals_first_match_on_random_tables(seed, prefix_masks):
    rng = np.random.default_rng(100 + seed)
    rs = random_table(rng, 300, prefix_masks)
    keys = boundary_keys(rs, rng, 6000)
    check(rs, keys)


def test_tree_shape_of_config_c():
    """Config C's forest fits the classify kernel's LDS beside its neighbour indexes and both family
    lists (the leaf size is the shortest whose image leaves them room: ~48 KB); its five field
    trees (split on their own field's words only) stay shallow, leaves short."""
    rs = synth.config_c_flows(n=16).rules_sorted
    _, info = gpu.rules_match_host(rs, np.zeros(0, FLOW_KEY_DTYPE))
    image = 8 * int(info["nodes"]) + 4 * int(info["leaf_entries"])
    assert 0 < image < 56 * 1024, info
    assert info["depth4"] <= 16 and info["depth6"] <= 16 and info["max_leaf"] <= 16
    assert info["trees"] == 5 | 5 << 16


def test_no_rules_and_foreign_versions():
    keys = np.zeros(3, FLOW_KEY_DTYPE)
    keys["ip_ver"] = [4, 6, 5]
    got, info = gpu.rules_match_host(np.zeros(0, RULE_DTYPE), keys)
    assert got.tolist() == [-1, -1, -1]
    rs = synth.build_rule_table(synth.rules_array([synth.make_rule(1, layout.ACT_FWD)]))
    got, _ = gpu.rules_match_host(rs, keys)
    assert got.tolist() == [0, 0, -1]
