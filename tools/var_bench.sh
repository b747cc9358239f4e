#!/bin/bash
# Diagnostic: config-B bench (emit mode unless MODE is set) of the product build and variant
# libraries, one line each: tools/var_bench.sh label=[ENV=VALUE,...] ...
#   a label's ENV list may name UPE_GPU_LIB_DIAG=<so> and any other environment variable.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/vb
for spec in "$@"; do
  label=${spec%%=*}; envs=${spec#*=}
  [ "$envs" = "$spec" ] && envs=""
  timeout -k 10 120 env UPE_GPU_VERBOSE=1 ${envs//,/ } python bench.py --no-cpu-baseline --no-hbm-probe --no-other-mode --no-imix \
      --mode ${MODE:-emit} ${BENCH_ARGS:-} > gpurun_out/vb/$label.json 2> gpurun_out/vb/$label.err
  rc=$?
  python - "$label" "$rc" <<'PY'
import json, sys
label, rc = sys.argv[1], sys.argv[2]
try:
    d = json.loads(open(f"gpurun_out/vb/{label}.json").read().strip().splitlines()[-1])
    print(f"{label:14s} value={d['value']:9.1f} Mpps  step={d['ms_per_step']*1e3:6.2f} us  "
          f"kernel={d['roofline']['kernel_ms']*1e3:6.2f} us  frac={d['roofline']['frac']:.4f}")
except Exception as e:
    print(f"{label:14s} rc={rc} failed: {e}")
PY
  [ $rc -ge 124 ] && exit $rc
done
exit 0
