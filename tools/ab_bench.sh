#!/bin/bash
# Diagnostic A/B: the product build against variant libraries on B (main), C (imix) and D
# (config_d), alternating: tools/ab_bench.sh <rounds> label=<so or "product"> ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
rounds=$1; shift
for r in $(seq 1 $rounds); do
  for spec in "$@"; do
    label=${spec%%=*}; lib=${spec#*=}
    envs=""; [ "$lib" != "product" ] && envs="UPE_GPU_LIB_DIAG=$lib"
    f=gpurun_out/ab/${label}_$r.json
    timeout -k 10 180 env $envs python bench.py --no-cpu-baseline --no-hbm-probe \
        --ring 0 --host-reps 0 --no-host-emit --no-host-mapped --imix-v6fwd 0 > $f 2> ${f%.json}.err
    rc=$?
    python - "$label" "$f" "$rc" <<'PY'
import json, sys
label, f, rc = sys.argv[1:]
try:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    D = d.get("config_d", {}).get("roofline", {})
    print(f"{label:10s} B {d['roofline']['kernel_ms']*1e3:7.2f} us  C {d['imix']['roofline']['kernel_ms']*1e3:7.2f} us  "
          f"inplace {d['other_mode']['kernel_ms']*1e3:7.2f} us  D classify {D.get('classify_ms', 0)*1e3:7.1f} + group-by {D.get('group_by_ms', 0)*1e3:5.1f} us", flush=True)
except Exception as e:
    print(f"{label:10s} rc={rc} failed: {e}", flush=True)
PY
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
