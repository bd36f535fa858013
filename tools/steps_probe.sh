#!/bin/bash
# C1 bench value vs timed-region length (steps) and warmup.
set -o pipefail
for cfg in "20 3" "200 20" "1000 100" "20 3" "200 200"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps $1 --warmup $2 > gpurun_out/steps_$1_$2.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/steps_$1_$2.json')); r=d['roofline']; print('steps=$1 warmup=$2', d['value'], r['kernel_ms'], r['seal_ms'], r['open_ms'])"
done
