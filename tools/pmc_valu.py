"""The VALU roofline of a configuration's classify kernel from rocprofv3 PMC passes
(tools/pmc_run.sh <config> <mode> sq clk): per classify dispatch (median over the full-batch
dispatches) the vector-ALU wave-instructions issued (SQ_INSTS_VALU) and the kernel's shader
cycles (GRBM_GUI_ACTIVE, which rocprofv3 sums over the 8 XCDs: / 8).  gfx950 issues one wave64
VALU instruction per SIMD every 2 cycles (MI355X_MICROARCH.md, "Wave scheduling": SIMD-32,
32 lanes/cycle x 2), so the VALU issue roofline is 1024 SIMDs / 2 wave-instructions per cycle:
    valu_frac = SQ_INSTS_VALU * 2 / (1024 * GRBM_GUI_ACTIVE / 8)
Writes profiles/pmc_config<X>[_emit]_valu.json (bench.py reads it for config D's line)."""
import collections
import csv
import glob
import json
import re
import statistics
import sys

cfg = sys.argv[1] if len(sys.argv) > 1 else "D"
packets = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 24
mode = sys.argv[3] if len(sys.argv) > 3 else "emit"
want = "true" if mode == "emit" else "false"


def classify_rows(path):
    rows = [r for r in csv.DictReader(open(path))
            if (m := re.search(r"upe_classify<(\w+), (\w+)", r["Kernel_Name"])) and m.group(2) == want]
    gmax = max(int(r["Grid_Size"]) for r in rows)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        if int(r["Grid_Size"]) == gmax:
            per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {c: statistics.median(v.values()) for c, v in per.items()}


vals = {}
for g in ("sq", "clk"):
    for f in glob.glob(f"gpurun_out/pmc_{cfg}_{mode}/{g}/p_counter_collection.csv"):
        vals.update(classify_rows(f))
cycles = vals["GRBM_GUI_ACTIVE"] / 8.0
out = {"config": cfg, "mode": mode, "packets": packets, "kernel": "upe_classify",
       "sq_insts_valu": vals["SQ_INSTS_VALU"], "sq_insts_salu": vals.get("SQ_INSTS_SALU"),
       "sq_active_inst_valu": vals.get("SQ_ACTIVE_INST_VALU"),
       "sq_busy_cycles": vals.get("SQ_BUSY_CYCLES"), "sq_wave_cycles": vals.get("SQ_WAVE_CYCLES"),
       "sq_wait_inst_any": vals.get("SQ_WAIT_INST_ANY"), "sq_waves": vals.get("SQ_WAVES"),
       "grbm_gui_active": vals["GRBM_GUI_ACTIVE"], "kernel_cycles": cycles,
       "valu_issue_peak_per_cycle": 1024 / 2,
       "valu_frac": vals["SQ_INSTS_VALU"] * 2 / (1024 * cycles),
       "valu_insts_per_packet": vals["SQ_INSTS_VALU"] * 64 / packets,
       "method": "rocprofv3 --pmc (SQ group, GRBM group: separate passes, kernel trace only) over "
                 "bench.py; median full-batch classify dispatch; valu_frac = SQ_INSTS_VALU x 2 / "
                 "(1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)"}
json.dump(out, open(f"profiles/pmc_config{cfg}{'_emit' if mode == 'emit' else ''}_valu.json", "w"),
          indent=1)
print(json.dumps(out))
