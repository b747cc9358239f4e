"""Launch-to-launch timeline of the classify kernels in a rocprofv3 kernel trace (diagnostic for
the overlapped queue, upe_gpu_process_queue_emit): per consecutive pair of classify dispatches,
the step (end to end), the kernel's own duration, and how long the next one started before the
previous one ended (its overlap; negative = a gap).  Medians over the longest run of dispatches
with no gap over --gap-us.

Usage: python tools/overlap_trace.py <p_kernel_trace.csv> [--gap-us 200]
"""
from __future__ import annotations

import argparse
import csv
import statistics


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap-us", type=float, default=200.0)
    a = ap.parse_args()
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
            for r in csv.DictReader(open(a.trace)) if "upe_classify" in r["Kernel_Name"]]
    rows.sort()
    runs, cur = [], []
    for s, e in rows:
        if cur and s - cur[-1][1] > a.gap_us * 1e3:
            runs.append(cur)
            cur = []
        cur.append((s, e))
    runs.append(cur)
    run = max(runs, key=len)[2:]   # skip the first launches of the run
    step = [run[i + 1][1] - run[i][1] for i in range(len(run) - 1)]
    dur = [e - s for s, e in run]
    ovl = [run[i][1] - run[i + 1][0] for i in range(len(run) - 1)]
    med = lambda x: statistics.median(x) / 1e3
    print(f"dispatches {len(run)}: step {med(step):.2f} us, duration {med(dur):.2f} us, "
          f"next starts {med(ovl):.2f} us before the previous ends "
          f"(min {min(ovl) / 1e3:.2f}, max {max(ovl) / 1e3:.2f})")


if __name__ == "__main__":
    main()
