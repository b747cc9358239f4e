"""Summary of tools/pmc_ab.sh: per variant, the median full-batch classify dispatch's FETCH_SIZE
(x 2, the gfx950 correction of MI355X_MICROARCH.md §HBM) and WRITE_SIZE, in bytes per packet."""
import collections
import csv
import glob
import os
import sys

cfg = sys.argv[1]
packets = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
for d in sorted(glob.glob(f"gpurun_out/pmcab/{cfg}/*")):
    out = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(f"{d}/{c}/**/p_counter_collection.csv", recursive=True)
        if not f:
            continue
        rows = [r for r in csv.DictReader(open(f[0])) if "upe_classify" in r["Kernel_Name"]]
        gmax = max(int(r["Grid_Size"]) for r in rows)
        acc = collections.defaultdict(float)
        for r in rows:
            if int(r["Grid_Size"]) == gmax:
                acc[r["Dispatch_Id"]] += float(r["Counter_Value"])
        v = sorted(acc.values())
        out[c] = v[len(v) // 2] * 1024
    rd = 2 * out.get("FETCH_SIZE", float("nan"))
    wr = out.get("WRITE_SIZE", float("nan"))
    print(f"{cfg} {os.path.basename(d):12s} read {rd / packets:7.1f} B/pkt  write {wr / packets:6.1f} "
          f"B/pkt  total {(rd + wr) / 1e6:8.1f} MB/launch")
