"""Load the golden vectors of tests/golden/ (written by tests/golden/make_golden.py from the
reference worker) back into synth.Workload objects plus the reference's outputs."""
from __future__ import annotations

import json
import os

import numpy as np

from upe_amd import synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

CASES = ("config_a", "config_b_small", "config_c_small", "config_d_small", "edge_zero",
         "edge_consistent", "edge_inconsistent", "ndp_walk")


def flow_hash(name: str):
    """The reference RX thread's flow_hash per packet of a golden case (0 where parse_flow_key
    fails) and whether it parsed (tests/golden/flow_hash.npz)."""
    z = np.load(os.path.join(GOLDEN, "flow_hash.npz"), allow_pickle=False)
    return z[name], z[name + "__ok"]


def load(name: str):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    presorted = bool(z["presorted"])
    rules = z["rules"]
    if presorted:
        # the stored table is already rt->rules; insertion order = sorted order by rule_id
        rules = rules[np.argsort(rules["rule_id"], kind="stable")]
    wl = synth.Workload(name, z["frames"].copy(), z["desc"].copy(), rules, int(z["capacity"]),
                        z["arp"].copy(), z["ndp"].copy(), bytes(z["eth_addr"].tobytes()),
                        int(z["ip4_addr"]), z["l1"].copy())
    ref = {k[4:]: z[k] for k in z.files if k.startswith("out_")}
    return wl, ref


def digests() -> dict:
    with open(os.path.join(GOLDEN, "digests.json")) as f:
        return json.load(f)
