"""Split a rocprofv3 kernel trace of one bench.py run into its legs and summarise each.

A default config-B bench run launches the same classify instantiation for two workloads: the
64 B batches of `value` and, after the other-mode leg, the IMIX batches of the "imix" field.
rocprofv3's --stats table averages them together; this splits the dispatches of each kernel
into legs at gaps longer than --gap-ms (the IMIX leg starts after its batch is generated on the
host, seconds later) and prints count / mean / min / max per leg, so that each leg's mean can
be set beside the bench line's kernel_ms.

Full-batch means: a leg also holds the small launches of the same instantiation (the first
warm-up batch, census probes, the host legs' chunks), which drag rocprof's plain mean down.
Dispatches shorter than --min-frac x the leg's median are dropped from the `full_*` columns
(and counted in `small`), so that full_mean_us is the mean over full-size batches only.

Usage: python tools/kernel_legs.py <p_kernel_trace.csv | run_results.db> [--gap-ms 50]
       [--match upe_] [--min-frac 0.5]
"""
from __future__ import annotations

import argparse
import csv
import statistics


def _rows(path: str, match: str):
    """Kernel dispatches (name, start ns, end ns) from a kernel-trace CSV or, for rocprofv3's
    SQLite output (`*_results.db`, ROCm 7), from its `kernels` view."""
    if path.endswith(".db"):
        import sqlite3
        con = sqlite3.connect(path)
        return [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e}
                for n, s, e in con.execute("select name, start, end from kernels")
                if match in n]
    return [r for r in csv.DictReader(open(path)) if match in r["Kernel_Name"]]


def legs(path: str, gap_ms: float, match: str):
    rows = _rows(path, match)
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    by_name: dict[str, list[list[tuple[int, int]]]] = {}
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        segs = by_name.setdefault(r["Kernel_Name"], [])
        if not segs or s - segs[-1][-1][1] > gap_ms * 1e6:
            segs.append([])
        segs[-1].append((s, e))
    return by_name


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap-ms", type=float, default=50.0)
    ap.add_argument("--match", default="upe_")
    ap.add_argument("--min-frac", type=float, default=0.5)
    a = ap.parse_args()
    print(f"{'kernel':100s} {'leg':>3s} {'calls':>6s} {'mean_us':>9s} {'min_us':>9s} "
          f"{'max_us':>9s} {'small':>6s} {'full_n':>6s} {'full_mean_us':>12s} {'full_min_us':>11s}")
    for name, segs in legs(a.trace, a.gap_ms, a.match).items():
        for i, seg in enumerate(segs):
            d = [(e - s) / 1e3 for s, e in seg]
            cut = a.min_frac * statistics.median(d)
            full = [x for x in d if x >= cut]
            short = name
            if "upe_classify<" in name:   # the instantiation's template arguments
                short = "upe_classify<" + name.split("upe_classify<", 1)[1].split(">", 1)[0] + ">"
            print(f"{short[:100]:100s} {i:3d} {len(d):6d} {statistics.mean(d):9.2f} "
                  f"{min(d):9.2f} {max(d):9.2f} {len(d) - len(full):6d} {len(full):6d} "
                  f"{statistics.mean(full):12.2f} {min(full):11.2f}")


if __name__ == "__main__":
    main()
