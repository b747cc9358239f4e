"""Summarise the PMC passes of tools/pmc_refresh.sh into profiles/r06/pmc_<label>_<mode>.json,
the files bench.py reads for `roofline.traffic` (and config D's VALU roofline).

Per pass: the classify kernel's full-batch dispatches only (the largest grid; dispatches whose
counter total is below half the median are small launches and are dropped), the median over
them.  gfx950 corrections (MI355X_MICROARCH.md, HBM section): read bytes = 2 x FETCH_SIZE,
WRITE_SIZE exact for 16-byte stores; both counters are KB per dispatch summed over instances.
GRBM_GUI_ACTIVE is summed over the 8 XCDs (/ 8 for kernel cycles).  Every pass's stamp (UTC
time, counters, sha256 of the profiled libupe_gpu.so) is carried into the summary.

Usage: python tools/pmc_r06.py <label> <mode> <packets> [indir] [outdir]
"""
from __future__ import annotations

import collections
import csv
import glob
import json
import os
import re
import statistics
import sys


def classify_median(path: str, want_emit: str) -> tuple[dict, int]:
    rows = [r for r in csv.DictReader(open(path))
            if (m := re.search(r"upe_classify<(\w+), (\w+)", r["Kernel_Name"]))
            and m.group(2) == want_emit]
    gmax = max(int(r["Grid_Size"]) for r in rows)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        if int(r["Grid_Size"]) == gmax:
            per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    out, n = {}, 0
    for c, d in per.items():
        v = list(d.values())
        med = statistics.median(v)
        full = [x for x in v if x >= 0.5 * med] or v
        out[c] = statistics.median(full)
        n = max(n, len(full))
    return out, n


def main() -> None:
    label, mode, packets = sys.argv[1], sys.argv[2], int(sys.argv[3])
    indir = sys.argv[4] if len(sys.argv) > 4 else f"gpurun_out/pmc_r06/{label}_{mode}"
    want = "true" if mode == "emit" else "false"
    vals, stamps, dispatches = {}, {}, {}
    for g in sorted(os.listdir(indir)):
        f = glob.glob(os.path.join(indir, g, "p_counter_collection.csv"))
        if not f:
            continue
        v, n = classify_median(f[0], want)
        vals.update(v)
        dispatches[g] = n
        st = os.path.join(indir, g, "stamp.txt")
        stamps[g] = open(st).read().strip() if os.path.exists(st) else None
    shas = {re.search(r"lib_sha16=(\w+)", s).group(1) for s in stamps.values() if s}
    out = {"label": label, "mode": mode, "packets": packets, "kernel": "upe_classify",
           "passes": stamps, "full_batch_dispatches_per_pass": dispatches,
           "lib_sha16": shas.pop() if len(shas) == 1 else sorted(shas)}
    if "FETCH_SIZE" in vals and "WRITE_SIZE" in vals:
        rb, wb = 2 * vals["FETCH_SIZE"] * 1024, vals["WRITE_SIZE"] * 1024
        out.update({"fetch_size_kb": vals["FETCH_SIZE"], "write_size_kb": vals["WRITE_SIZE"],
                    "read_bytes": rb, "write_bytes": wb, "traffic_bytes_per_launch": rb + wb,
                    "read_bytes_per_packet": round(rb / packets, 2),
                    "write_bytes_per_packet": round(wb / packets, 2),
                    "traffic_bytes_per_packet": round((rb + wb) / packets, 2)})
    if "SQ_WAVE_CYCLES" in vals:
        wc = vals["SQ_WAVE_CYCLES"]
        out["sq"] = {k: vals.get(k) for k in ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
                                              "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                              "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VALU",
                                              "SQ_INSTS_SALU")}
        out["wave_time"] = {"waiting": round(vals["SQ_WAIT_ANY"] / wc, 4),
                            "issue_stalled": round(vals["SQ_WAIT_INST_ANY"] / wc, 4),
                            "issuing": round(vals["SQ_ACTIVE_INST_ANY"] / wc, 4)}
        out["valu_insts_per_64_packets"] = round(vals["SQ_INSTS_VALU"] * 64 / packets, 1)
        out["salu_insts_per_64_packets"] = round(vals["SQ_INSTS_SALU"] * 64 / packets, 1)
    if "GRBM_GUI_ACTIVE" in vals:
        cyc = vals["GRBM_GUI_ACTIVE"] / 8.0
        out["kernel_cycles"] = cyc
        out["kernel_us_at_2p4GHz"] = round(cyc / 2400.0, 2)
        if "SQ_INSTS_VALU" in vals:
            out["valu_frac"] = round(vals["SQ_INSTS_VALU"] * 2 / (1024 * cyc), 4)
    out["method"] = ("rocprofv3 --pmc, one counter group per pass (kernel trace only) over "
                     "bench.py; the classify kernel's full-batch dispatches, median; read = 2 x "
                     "FETCH_SIZE (gfx950), write = WRITE_SIZE; valu_frac = SQ_INSTS_VALU x 2 / "
                     "(1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)")
    outdir = sys.argv[5] if len(sys.argv) > 5 else "profiles/r06"
    os.makedirs(outdir, exist_ok=True)
    dst = f"{outdir}/pmc_{label}_{mode}.json"
    json.dump(out, open(dst, "w"), indent=1)
    print(dst, json.dumps({k: out.get(k) for k in ("traffic_bytes_per_packet", "read_bytes_per_packet",
                                                  "write_bytes_per_packet", "wave_time",
                                                  "valu_frac", "lib_sha16")}))


if __name__ == "__main__":
    main()
