"""Wall time of upe_gpu_load_rules (rule compile + index build + upload) for the large-table
cases (the decision tree is built on the worker thread at a reload).

  python tools/load_time.py [cases...]     cases: C3 CF C6 F16k M64k D (default all)

Median of 3 loads each, on GPU 0; prints one JSON line per case with the index kind chosen."""
from __future__ import annotations

import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    from upe_amd import gpu, synth

    def mixed_64k():
        wl = synth.config_c(seed=61, n=1024)
        wl.rules, wl.capacity = synth.mixed_table(1 << 16, 61), 1 << 16
        return wl

    makers = {"C3": lambda: synth.config_c(n=1024), "CF": lambda: synth.config_c_flows(n=4096),
              "C6": lambda: synth.config_c(n=1024, v6_forwarding=True),
              "F16k": lambda: synth.config_c_flows(seed=62, n=4096, n_rules=1 << 14,
                                                   max_cover=2.0 ** -18),
              "M64k": mixed_64k, "D": lambda: synth.config_d(n=4096)}
    for c in sys.argv[1:] or list(makers):
        wl = makers[c]()
        w = gpu.GpuWorker(0, wl.capacity)
        rs = wl.rules_sorted
        w.load_rules(rs)   # warm-up (allocations)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            w.load_rules(rs)
            ts.append(time.perf_counter() - t0)
        kind = w.rule_index_kind()
        w.close()
        print(json.dumps({"case": c, "rules": int(len(rs)), "load_ms": round(1e3 * statistics.median(ts), 2),
                          "index": {0: "linear scan", 1: "tuple space", 2: "decision tree"}.get(kind, kind)}),
              flush=True)


if __name__ == "__main__":
    main()
