#!/bin/bash
# Two-chunk Horner step (product build) vs one chunk per reduction (build_ab/libwgaead_h1.so,
# -DWG_HORNER1), C1 (default two streams) and C2, alternating; every line carries the oracle sample.
set -o pipefail
out=gpurun_out/${1:-r04h2}
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_duplex.py tests/test_gpu_parity.py -m gpu > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for k in 1 2 3; do
  for v in h2 h1; do
    lib=""; [ $v = h1 ] && lib="build_ab/libwgaead_h1.so"
    for w in c1 c2; do
      WG_LIB_PATH=$lib timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > $out/${w}_${v}_$k.json 2>>$out/err || exit 1
      python3 -c "
import json; j=json.loads(open('$out/${w}_${v}_$k.json').read().strip().splitlines()[-1]); r=j['roofline']
print('$w $v', j['value'], j['ms_per_step'], r['frac'], r['step']['frac'], j['verified'], j['oracle_sample']['bit_exact'])"
    done
  done
done
