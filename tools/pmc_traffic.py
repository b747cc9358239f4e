"""Turn rocprofv3 PMC passes (tools/pmc_run.sh <config> fetch write) into the HBM traffic per
classify launch that bench.py reports as roofline.traffic (profiles/pmc_config<X>.json).

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of a wide
coalesced read, so read bytes = 2 x FETCH_SIZE; WRITE_SIZE is exact for 16-byte stores.
Both counters are in KB per dispatch (summed over the counter instances)."""
import collections
import csv
import re
import glob
import json
import sys


def _emit_arg(name: str):
    m = re.search(r"upe_classify<(\w+), (\w+)", name)
    return m.group(2) if m else None


cfg = sys.argv[1] if len(sys.argv) > 1 else "B"
packets = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
mode = sys.argv[3] if len(sys.argv) > 3 else "emit"      # emit | inplace
# upe_classify<tss, emit[, lean]>: the second template argument says emit mode
want = "true" if mode == "emit" else "false"
vals = {}
for name in ("fetch", "write"):
    f = glob.glob(f"gpurun_out/pmc_{cfg}_{mode}/{name}/p_counter_collection.csv")[0]
    rows = [r for r in csv.DictReader(open(f))
            if _emit_arg(r["Kernel_Name"]) == want]
    # only the full-batch launches (the bench's host leg launches smaller chunks)
    gmax = max(int(r["Grid_Size"]) for r in rows)
    acc = collections.defaultdict(float)
    for r in rows:
        if int(r["Grid_Size"]) == gmax:
            acc[r["Dispatch_Id"]] += float(r["Counter_Value"])
    v = sorted(acc.values())
    vals[name] = v[len(v) // 2]           # median dispatch
read_b = 2 * vals["fetch"] * 1024
write_b = vals["write"] * 1024
out = {"config": cfg, "mode": mode, "packets": packets, "fetch_size_kb": vals["fetch"],
       "write_size_kb": vals["write"], "read_bytes": read_b, "write_bytes": write_b,
       "traffic_bytes_per_launch": read_b + write_b,
       "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                 "bench.py (kernel trace only); read = 2 x FETCH_SIZE (gfx950), median dispatch"}
json.dump(out, open(f"profiles/pmc_config{cfg}{'_emit' if mode == 'emit' else ''}.json", "w"),
          indent=1)
print(json.dumps(out))
