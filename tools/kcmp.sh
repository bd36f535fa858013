#!/bin/bash
# Compare transport kernel configurations on C1/C2/C3 (bench.py value) and C1 kernel time.
# Usage: bash tools/kcmp.sh "kernel variant wpg" ...
for cfg in "$@"; do
  set -- $cfg
  line="$1 V=$2 G=$3:"
  for w in c1 c2 c3; do
    st=20; [ $w = c3 ] && st=3
    v=$(WG_TRANSPORT_KERNEL=$1 WG_STREAM_VARIANT=$2 WG_WAVE_VARIANT=$2 WG_WAVE_WPG=$3 timeout -k 10 200 python bench.py --no-cpu-baseline --workload $w --steps $st --warmup 2 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'], d['verified'])")
    line="$line  $w $v"
  done
  echo "$line"
done
