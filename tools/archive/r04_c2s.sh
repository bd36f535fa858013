#!/bin/bash
# C2: one stream (default) vs two streams, with and without the progress-based issue priority, alternating.
set -o pipefail
out=gpurun_out/${1:-r04c2s}
mkdir -p $out
for k in 1 2; do
  for cfg in "s1:--streams 1" "s2:--streams 2" "s2p0:--streams 2" "s1p0:--streams 1"; do
    name=${cfg%%:*}; args=${cfg#*:}
    env_=""; [[ $name == *p0 ]] && env_="WG_PRIO=0"
    env $env_ timeout -k 10 200 python bench.py --workload c2 $args > $out/${name}_$k.json 2>>$out/err || exit 1
    python3 -c "
import json; j=json.loads(open('$out/${name}_$k.json').read().strip().splitlines()[-1]); r=j['roofline']
print('$name', j['value'], j['ms_per_step'], r['frac'], r['step']['frac'], j['oracle_sample']['bit_exact'])"
  done
done
