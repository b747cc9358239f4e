#!/bin/bash
# FETCH_SIZE per dispatch of tools/fetch_calib's six access shapes (one rocprofv3 pass, kernel
# trace only), printed beside the bytes each shape asked for / touched.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/calib
timeout -k 10 120 build/fetch_calib > gpurun_out/calib/plain.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib/pmc -o p --output-format csv -- build/fetch_calib > gpurun_out/calib/pmc.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d gpurun_out/calib/pmc2 -o p --output-format csv -- build/fetch_calib > gpurun_out/calib/pmc2.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_32B_sum -d gpurun_out/calib/pmc3 -o p --output-format csv -- build/fetch_calib > gpurun_out/calib/pmc3.txt 2>&1
python - <<'PY'
import csv, glob, collections
per = collections.defaultdict(dict)   # dispatch -> counter -> value
for d in ("pmc", "pmc2", "pmc3"):
    f = glob.glob(f"gpurun_out/calib/{d}/**/p_counter_collection.csv", recursive=True)
    if not f:
        continue
    rows = [r for r in csv.DictReader(open(f[0])) if "gather" in r["Kernel_Name"]]
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})
    for r in rows:
        k = ids.index(int(r["Dispatch_Id"]))
        per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
lines = [l for l in open("gpurun_out/calib/plain.txt") if l.startswith("mode")]
for k, l in enumerate(lines):
    c = per.get(k, {})
    mb = lambda x: f"{x / 1e6:8.1f}"
    print(l.strip())
    print("    FETCH_SIZE x2", mb(2 * c.get("FETCH_SIZE", 0) * 1024), "MB;",
          "RDREQ", int(c.get("TCC_EA0_RDREQ_sum", 0)), "(32B", int(c.get("TCC_EA0_RDREQ_32B_sum", 0)),
          "64B", int(c.get("TCC_EA0_RDREQ_64B_sum", 0)), "128B", int(c.get("TCC_EA0_RDREQ_128B_sum", 0)), ");",
          "DRAM", int(c.get("TCC_EA0_RDREQ_DRAM_sum", 0)), "(32B", int(c.get("TCC_EA0_RDREQ_DRAM_32B_sum", 0)), ")")
PY
