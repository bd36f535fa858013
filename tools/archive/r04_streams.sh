#!/bin/bash
# C1 / C2 step on 1 vs 2 streams (the batch cut into halves, each sealed and opened on its own stream, so
# one half's kernel tail overlaps the other's), alternating, 3 repetitions
O=gpurun_out/${1:-r04s}
mkdir -p $O
for rep in 1 2 3; do
  for w in c1 c2; do
    for k in 1 2; do
      timeout -k 10 200 python bench.py --workload $w --streams $k --no-cpu-baseline > $O/b.json 2>/dev/null || exit 1
      python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print(json.dumps({'rep': $rep, 'workload': '$w', 'streams': $k, 'value': d['value'], 'ms_per_step': d['ms_per_step']}))" | tee -a $O/streams.jsonl
    done
  done
done
