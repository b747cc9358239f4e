"""Rule tables for the SIGHUP-reload tests (reference src/main.c:216-282): the table a stats
thread would load after the one a workload starts with — the same kinds of rules in another
insertion order (so every rule_id is renumbered, src/rule_table.c:138), some priorities and
actions changed, one rule gone and one new one."""
from __future__ import annotations

import numpy as np

from upe_amd import synth
from upe_amd.layout import ACT_DROP, ACT_FWD, RULE_DTYPE

CASES = {
    # name: (workload maker, packets, reload point, rule capacity after the reload)
    "B": (lambda: synth.config_b(n=300_000, seed=41), 300_000, 131_072 + 77, 64),
    "C": (lambda: synth.config_c(n=200_000, seed=42), 200_000, 99_999, 2048),
    "D": (lambda: synth.config_d(n=200_000, seed=43, n_rules=8192), 200_000, 64_001, 8192),
}


def reloaded_rules(rules: np.ndarray, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    r = rules[::-1].copy()                                # new insertion order -> new rule_ids
    k = max(1, len(r) // 4)
    idx = rng.choice(len(r), k, replace=False)
    r["priority"][idx] = rng.integers(0, 20_000, k).astype(r["priority"].dtype)
    flip = rng.choice(len(r), max(1, len(r) // 8), replace=False)
    act = r["action"][flip]
    r["action"][flip] = np.where(act == ACT_FWD, ACT_DROP, ACT_FWD)
    r = np.delete(r, int(rng.integers(0, len(r))))
    extra = np.zeros(1, r.dtype)
    extra[0] = synth.make_rule(1, ACT_FWD, ip_ver=4, proto=17, dport=53)
    # (concatenate drops the structured dtype's padding: back to the 92-byte rule_t layout)
    out = np.ascontiguousarray(np.concatenate([extra, r]).astype(RULE_DTYPE))
    assert out.dtype.itemsize == 92
    return out


def case(name: str):
    make, n, at, cap_b = CASES[name]
    wl = make()
    assert wl.n == n
    return wl, reloaded_rules(wl.rules, 7 + len(name) + n), at, cap_b
