"""Counter table for classify launches from rocprofv3 PMC passes (one counter group per pass):
    python tools/pmc_table.py <out.json> <label>=<dir> [<label>=<dir> ...] [--packets N] [--us label=us ...]
<dir> holds the group subdirectories (fetch, write, sq, sq2, clk) tools/pmc_c.sh / pmc_run.sh
write.  Per label: the median over full-batch emit-mode classify dispatches of every counter,
and the derived figures — read bytes = 2 x FETCH_SIZE (gfx950 correction), write bytes =
WRITE_SIZE (both KB), kernel cycles = GRBM_GUI_ACTIVE / 8 XCDs, VALU issue fraction =
SQ_INSTS_VALU x 2 / (1024 SIMDs x cycles), bytes past L2 / kernel time."""
import collections
import csv
import glob
import json
import re
import statistics
import sys


def rows(path):
    rs = [r for r in csv.DictReader(open(path))
          if (m := re.search(r"upe_classify<(\w+), (\w+)", r["Kernel_Name"])) and m.group(2) == "true"]
    if not rs:
        return {}
    gmax = max(int(r["Grid_Size"]) for r in rs)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rs:
        if int(r["Grid_Size"]) == gmax:
            per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {c: statistics.median(v.values()) for c, v in per.items()}


def main():
    out_path = sys.argv[1]
    args = sys.argv[2:]
    packets = 1 << 20
    us = {}
    labels = []
    i = 0
    while i < len(args):
        if args[i] == "--packets":
            packets = int(args[i + 1]); i += 2; continue
        if args[i] == "--us":
            k, v = args[i + 1].split("="); us[k] = float(v); i += 2; continue
        labels.append(args[i].split("=", 1)); i += 1
    table = {}
    for label, d in labels:
        vals = {}
        for f in sorted(glob.glob(f"{d}/*/p_counter_collection.csv")):
            vals.update(rows(f))
        e = {"counters": vals, "packets": packets}
        if "FETCH_SIZE" in vals:
            e["read_bytes"] = 2 * vals["FETCH_SIZE"] * 1024
            e["read_bytes_per_packet"] = e["read_bytes"] / packets
        if "WRITE_SIZE" in vals:
            e["write_bytes"] = vals["WRITE_SIZE"] * 1024
            e["write_bytes_per_packet"] = e["write_bytes"] / packets
        if "GRBM_GUI_ACTIVE" in vals:
            cyc = vals["GRBM_GUI_ACTIVE"] / 8
            e["kernel_cycles"] = cyc
            if "SQ_INSTS_VALU" in vals:
                e["valu_frac"] = vals["SQ_INSTS_VALU"] * 2 / (1024 * cyc)
                e["valu_wave_insts_per_wave64"] = vals["SQ_INSTS_VALU"] / (packets / 64)
            if "SQ_BUSY_CYCLES" in vals:
                e["sq_busy_frac"] = vals["SQ_BUSY_CYCLES"] / 32 / cyc   # 32 SEs
        if "SQ_WAVE_CYCLES" in vals:
            wc = vals["SQ_WAVE_CYCLES"]
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_SCA", "SQ_INST_CYCLES_VMEM", "SQ_WAIT_INST_LDS"):
                if k in vals:
                    e[k.lower() + "_per_wave_cycle"] = vals[k] / wc
        if label in us:
            e["kernel_us"] = us[label]
            if "read_bytes" in e and "write_bytes" in e:
                e["past_l2_GBps"] = (e["read_bytes"] + e["write_bytes"]) / (us[label] * 1e3)
        table[label] = e
    json.dump(table, open(out_path, "w"), indent=1, sort_keys=True)
    keys = ["kernel_us", "read_bytes_per_packet", "write_bytes_per_packet", "past_l2_GBps",
            "valu_frac", "valu_wave_insts_per_wave64", "sq_wait_inst_any_per_wave_cycle",
            "sq_active_inst_any_per_wave_cycle", "sq_active_inst_valu_per_wave_cycle",
            "sq_inst_cycles_vmem_per_wave_cycle"]
    print(f"{'':26s}" + "".join(f"{l:>12s}" for l, _ in labels))
    for k in keys:
        print(f"{k:26.26s}" + "".join(f"{table[l].get(k, float('nan')):12.3f}" for l, _ in labels))
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
              "SQ_INSTS_LDS", "SQ_WAVES"):
        print(f"{c:26.26s}" + "".join(f"{table[l]['counters'].get(c, float('nan')):12.4g}" for l, _ in labels))


main()
