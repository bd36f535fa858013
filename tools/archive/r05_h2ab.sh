#!/bin/bash
# Two chunks per Horner reduction (-DWG_HORNER2, libwgaead_h2.so) against the product, alternating on one box:
# C1 two-stream steps (k_step<8,4>: 68 VGPRs, no spill) and C2 (k_step<8,4>)
set -o pipefail
O=gpurun_out/r05h2; mkdir -p $O
for r in 1 2 3; do
  for v in prod h2; do
    L=wireguard-java_amd/libwgaead.so; [ $v = h2 ] && L=wireguard-java_amd/libwgaead_h2.so
    for w in c1 c2; do
      WG_LIB_PATH=$PWD/$L timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline | sed "s/^{/{\"lib\": \"$v\", /" >> $O/ab.jsonl || { echo "rc $?"; exit 1; }
      tail -1 $O/ab.jsonl | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['lib'], '$w', j['value'], j['roofline']['step']['frac'], j['verified'])"
    done
  done
done
