"""Wave-level cost model of the decision-tree walk (round 5 design tool, CPU only).

  python tools/tree_cost.py [--n 65536] [cases...]     cases: CF C6 C3 (config C flows / v6fwd / seed 3)

Per 64-packet wave (the kernel's chunk): the walk's loop iterations (ILP groups of 3 trees, each
as long as the wave's deepest walk in it) and the leaf loop's iterations, tree by tree (as built)
or interleaved over a group's trees, from upe_tree_profile_host (the host walk of the same image:
levels walked and leaf entries read per key and tree).  Environment knobs of the builder
(UPE_GPU_TREE_BINTH) applies."""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def keys_of(wl, n):
    """The flow keys of the first n packets of a well-formed IMIX batch (Ethernet + option-less
    IPv4 / IPv6 + UDP / TCP / ICMP), FLOW_KEY_DTYPE as parse_flow_key leaves it: a design-tool
    parse of config C's traffic (the parity tests check the product's parse)."""
    from upe_amd import layout
    from upe_amd.layout import FLOW_KEY_DTYPE
    m = min(n, wl.n)
    offs = layout.desc_offsets(wl.desc)[:m].astype(np.int64)
    fr = wl.frames
    keys = np.zeros(m, FLOW_KEY_DTYPE)
    et = (fr[offs + 12].astype(np.int64) << 8) | fr[offs + 13]
    v4, v6 = et == 0x0800, et == 0x86DD
    keys["ip_ver"] = np.where(v4, 4, np.where(v6, 6, 0))
    proto = np.where(v4, fr[offs + 23], fr[offs + 20]).astype(np.int64)
    keys["protocol"] = proto
    l4 = np.where(v4, offs + 14 + 4 * (fr[offs + 14] & 0xF).astype(np.int64), offs + 54)
    a = (fr[l4].astype(np.int64) << 8) | fr[l4 + 1]
    b = (fr[l4 + 2].astype(np.int64) << 8) | fr[l4 + 3]
    icmp = proto == 1
    keys["src_port"] = np.where(icmp, (fr[l4 + 4].astype(np.int64) << 8) | fr[l4 + 5], a)
    keys["dst_port"] = np.where(icmp, (fr[l4].astype(np.int64) << 8) | fr[l4 + 1], b)
    for i in range(m):
        o = int(offs[i])
        if v4[i]:
            keys[i]["src_ip"][:4] = np.frombuffer(bytes(fr[o + 26:o + 30])[::-1], np.uint8)
            keys[i]["dst_ip"][:4] = np.frombuffer(bytes(fr[o + 30:o + 34])[::-1], np.uint8)
        elif v6[i]:
            keys[i]["src_ip"] = fr[o + 22:o + 38]
            keys[i]["dst_ip"] = fr[o + 38:o + 54]
    return keys[(v4 | v6)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("cases", nargs="*", default=["CF", "C6", "C3"])
    args = ap.parse_args()
    from upe_amd import gpu, synth
    from upe_amd.layout import RULE_DTYPE, RULE_INDEX_INFO_DTYPE
    lib = gpu.LIB
    lib.upe_tree_profile_host.restype = ctypes.c_int
    makers = {"CF": lambda: synth.config_c_flows(n=args.n), "C3": lambda: synth.config_c(n=args.n),
              "C6": lambda: synth.config_c(n=args.n, v6_forwarding=True),
              "F16k": lambda: synth.config_c_flows(seed=62, n_rules=1 << 14, max_cover=2.0 ** -18)}
    P = ctypes.c_void_p
    for c in args.cases:
        wl = makers[c]()
        keys = keys_of(wl, args.n)
        n = len(keys)
        rs = np.ascontiguousarray(wl.rules_sorted, dtype=RULE_DTYPE)
        out = np.zeros(n, np.int64)
        info = np.zeros(1, RULE_INDEX_INFO_DTYPE)
        dep = np.zeros((n, 16), np.uint8)
        stp = np.zeros((n, 16), np.uint8)
        rc = lib.upe_tree_profile_host(rs.ctypes.data_as(P), ctypes.c_size_t(len(rs)),
                                       keys.ctypes.data_as(P), ctypes.c_size_t(n),
                                       out.ctypes.data_as(P), info.ctypes.data_as(P),
                                       dep.ctypes.data_as(P), stp.ctypes.data_as(P))
        assert rc == 0
        nw = n // 64
        dep = dep[:nw * 64].reshape(nw, 64, 16).astype(np.int32)
        stp = stp[:nw * 64].reshape(nw, 64, 16).astype(np.int32)
        ntw = int(max(info["trees"][0] & 0xFFFF, info["trees"][0] >> 16))
        walk = leaf_seq = leaf_il = 0
        for g0 in range(0, ntw, 3):
            g = slice(g0, min(g0 + 3, ntw))
            walk += dep[:, :, g].max(axis=2).max(axis=1).mean()
            leaf_seq += stp[:, :, g].max(axis=1).sum(axis=1).mean()
            leaf_il += stp[:, :, g].max(axis=2).max(axis=1).mean()
        # the kernel's grouping (tree_match): the deep trees (0 source, 1 destination address,
        # 3 destination port) walked together, then the shallow ones (2 source port, 4 protocol)
        deep = dep[:, :, [0, 1, 3]].max(axis=2).max(axis=1).mean()
        shallow = dep[:, :, [2, 4]].max(axis=2).max(axis=1).mean()
        print(f"{c}: kernel grouping: deep walk {deep:.1f} + shallow walk {shallow:.1f} iterations per wave")
        ilp = []
        for k in range(1, 6):
            it = sum(dep[:, :, g0:min(g0 + k, ntw)].max(axis=2).max(axis=1).mean()
                     for g0 in range(0, ntw, k))
            ilp.append(f"ilp{k}: {it:.1f} it / {it * k:.1f} slots")
        print(f"{c}: walk " + ", ".join(ilp))
        for t in range(2 * 5 if ntw == 5 else 16):
            if stp[:, :, t].any() or dep[:, :, t].any():
                print(f"{c}: tree slot {t}: wave walk {dep[:, :, t].max(axis=1).mean():.1f}, wave leaf "
                      f"{stp[:, :, t].max(axis=1).mean():.1f}, lane leaf {stp[:, :, t].mean():.2f}")
        lane_walk = dep.sum(axis=2).mean()
        lane_steps = stp.sum(axis=2).mean()
        print(f"{c}: index {info[0].tolist()} trees/family {ntw}; per wave: walk iterations "
              f"{walk:.1f}, leaf iterations tree-by-tree {leaf_seq:.1f} / interleaved {leaf_il:.1f}; "
              f"per lane: levels {lane_walk:.1f}, leaf entries read {lane_steps:.2f}")


if __name__ == "__main__":
    main()
