#!/bin/bash
# 1 / 16 / 64 / 128 per-packet callers: default (at most host_cpus() callers poll, the rest sleep) vs every
# caller polling 4096 times first (WG_PP_SPIN_CALLERS=100000, round 4 before the fix), with the cgroup's
# throttling counters before and after each run.
O=gpurun_out/${1:-r04q2}
mkdir -p $O
for T in 1 16 64 128; do
  for pol in "WG_PP_X=0" "WG_PP_SPIN_CALLERS=100000" "WG_PP_X=0" "WG_PP_SPIN_CALLERS=100000"; do
    a=$(grep -E "nr_throttled" /sys/fs/cgroup/cpu.stat | awk '{print $2}')
    env $pol timeout -k 10 120 ./tools/batcher_bench $T $((160000 / T)) 1420 > $O/r.json || exit 1
    b=$(grep -E "nr_throttled" /sys/fs/cgroup/cpu.stat | awk '{print $2}')
    python3 -c "
import json; j=json.load(open('$O/r.json')); l=j['lat_us']
print('T=$T', '$pol', j['payload_gib_s'], 'p50', l['p50'], 'p99', l['p99'], 'p999', l['p999'], 'max', l['max'], 'throttled', $b-$a)" | tee -a $O/summary.txt
    cat $O/r.json >> $O/all.jsonl
  done
done
