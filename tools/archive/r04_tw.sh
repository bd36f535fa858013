#!/bin/bash
# Workgroup size A/B (waves per workgroup TW = 2 / 4 (product) / 8), C1 default step, alternating.
set -o pipefail
out=gpurun_out/${1:-r04tw}
mkdir -p $out
for k in 1 2; do
  for v in 4 2 8; do
    lib=""; [ $v != 4 ] && lib="build_ab/libwgaead_tw$v.so"
    WG_LIB_PATH=$lib timeout -k 10 200 python bench.py --workload c1 > $out/c1_tw${v}_$k.json 2>>$out/err || exit 1
    python3 -c "
import json; j=json.loads(open('$out/c1_tw${v}_$k.json').read().strip().splitlines()[-1]); r=j['roofline']
print('tw$v', j['value'], j['ms_per_step'], r['frac'], r.get('kernel_ms'), r['step']['frac'], j['oracle_sample']['bit_exact'])"
  done
done
