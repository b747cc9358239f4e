#!/bin/bash
# Summarise a variants run: bench value and rocprof mean kernel time per variant, plus C lines.
for f in gpurun_out/var_*.json; do
  v=$(basename $f .json); v=${v#var_}
  python3 -c "
import json,csv
d=json.load(open('$f'))
k=[r for r in csv.DictReader(open('gpurun_out/var/$v/v_kernel_stats.csv')) if 'upe_classify' in r['Name']]
print('%-8s %9.1f Mpps  rocprof %7.2f us' % ('$v', d['value'], float(k[0]['AverageNs'])/1e3 if k else float('nan')))"
done
for f in gpurun_out/C*.log; do echo "$(basename $f .log) $(grep -o '"value": [0-9.]*' $f) $(grep -o '"kernel_ms": [0-9.]*' $f)"; done
