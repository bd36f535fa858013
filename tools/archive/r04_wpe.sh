#!/bin/bash
# C2: the half-occupancy k_step grid in the 128-VGPR build (WG_STEP_WPE4=1) vs the 64-VGPR one, alternating.
set -o pipefail
out=gpurun_out/${1:-r04wpe}
mkdir -p $out
for k in 1 2 3; do
  for v in 0 1; do
    WG_STEP_WPE4=$v timeout -k 10 200 python bench.py --workload c2 > $out/c2_w${v}_$k.json 2>>$out/err || exit 1
    python3 -c "
import json; j=json.loads(open('$out/c2_w${v}_$k.json').read().strip().splitlines()[-1]); r=j['roofline']
print('wpe4=$v', j['value'], j['ms_per_step'], r['frac'], j['verified'], j['oracle_sample']['bit_exact'])"
  done
done
