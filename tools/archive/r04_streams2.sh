#!/bin/bash
# C1 on 1..4 streams and C3 on 1..2 streams, alternating, 2 repetitions
O=gpurun_out/${1:-r04s2}
mkdir -p $O
for rep in 1 2; do
  for cfg in "c1 1" "c1 2" "c1 3" "c1 4" "c3 1" "c3 2"; do
    set -- $cfg
    extra=""; [ $1 = c3 ] && extra="--steps 5 --warmup 1"
    timeout -k 10 300 python bench.py --workload $1 --streams $2 --no-cpu-baseline $extra > $O/b.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print(json.dumps({'rep': $rep, 'workload': '$1', 'streams': $2, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'verified': d['verified']}))" | tee -a $O/streams.jsonl
  done
done
