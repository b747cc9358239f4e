"""Summarise tools/variants_run.sh output: bench value and rocprof kernel averages per variant."""
import csv
import glob
import json
import os

for f in sorted(glob.glob("gpurun_out/var_*.json")):
    label = os.path.basename(f)[4:-5]
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(label, "no json", e)
        continue
    stats = glob.glob(f"gpurun_out/var/{label}/**/*kernel_stats.csv", recursive=True)
    ks = {}
    if stats:
        for r in csv.DictReader(open(stats[0])):
            name = r["Name"]
            for k in ("upe_classify", "upe_finalize"):
                if k in name:
                    ks[k] = float(r["AverageNs"]) / 1e3
    print(f"{label:8s} value={d['value']:9.1f} ms/step={d['ms_per_step']*1e3:6.1f}us "
          f"ev_classify={d['roofline']['kernel_ms']*1e3:6.1f} ev_fin={d['roofline']['finalize_ms']*1e3:5.1f} "
          f"prof_classify={ks.get('upe_classify', float('nan')):6.1f} prof_fin={ks.get('upe_finalize', float('nan')):5.1f}")
