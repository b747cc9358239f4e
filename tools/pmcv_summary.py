"""Per-variant SQ counters (per classify dispatch) next to the profiled kernel time."""
import csv
import collections
import glob
import os

for d in sorted(glob.glob("gpurun_out/pmcv/*")):
    v = os.path.basename(d)
    f = glob.glob(f"{d}/**/p_counter_collection.csv", recursive=True)
    if not f:
        continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f[0])):
        if "upe_classify" in r["Kernel_Name"]:
            acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    avg = {c: sum(p.values()) / len(p) for c, p in acc.items()}
    st = glob.glob(f"gpurun_out/var/{v}/**/*kernel_stats.csv", recursive=True)
    us = float("nan")
    if st:
        for r in csv.DictReader(open(st[0])):
            if "upe_classify" in r["Name"]:
                us = float(r["AverageNs"]) / 1e3
    tw = 1048576 / 64   # tile-waves per dispatch
    print(f"{v:8s} us={us:6.1f} VALU/tw={avg.get('SQ_INSTS_VALU',0)/tw:6.1f} SALU/tw={avg.get('SQ_INSTS_SALU',0)/tw:6.1f} "
          f"VMEM_RD/tw={avg.get('SQ_INSTS_VMEM_RD',0)/tw:5.1f} wave_cyc={avg.get('SQ_WAVE_CYCLES',0)/1e6:6.1f}M "
          f"wait={avg.get('SQ_WAIT_ANY',0)/1e6:6.1f}M waitinst={avg.get('SQ_WAIT_INST_ANY',0)/1e6:6.1f}M act={avg.get('SQ_ACTIVE_INST_ANY',0)/1e6:5.1f}M")
