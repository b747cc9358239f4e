"""Per-dispatch averages of the PMC counters tools/pmc_run.sh collected (classify kernel)."""
import csv
import collections
import glob
import sys

cfg = sys.argv[1] if len(sys.argv) > 1 else "B"
mode = sys.argv[2] if len(sys.argv) > 2 else "emit"
tag = "true>" if mode == "emit" else "false>"
for f in sorted(glob.glob(f"gpurun_out/pmc_{cfg}_{mode}/*/p_counter_collection.csv")):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "upe_classify" not in r["Kernel_Name"] or tag not in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for c, per in sorted(acc.items()):
        vals = list(per.values())
        print(f"{f.split('/')[-2]:6s} {c:24s} n={len(vals):3d} avg={sum(vals)/len(vals):.4g}")
