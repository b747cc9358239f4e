"""Per-dispatch averages of the PMC counters tools/pmc_run.sh collected (classify kernel)."""
import csv
import re
import collections
import glob
import sys


def _emit_arg(name: str):
    m = re.search(r"upe_classify<(\w+), (\w+)", name)
    return m.group(2) if m else None


cfg = sys.argv[1] if len(sys.argv) > 1 else "B"
mode = sys.argv[2] if len(sys.argv) > 2 else "emit"
# upe_classify<tss, emit[, lean]>: the second template argument says emit mode
want = "true" if mode == "emit" else "false"
for f in sorted(glob.glob(f"gpurun_out/pmc_{cfg}_{mode}/*/p_counter_collection.csv")):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if _emit_arg(r["Kernel_Name"]) != want:
            continue
        acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for c, per in sorted(acc.items()):
        vals = list(per.values())
        print(f"{f.split('/')[-2]:6s} {c:24s} n={len(vals):3d} avg={sum(vals)/len(vals):.4g}")
