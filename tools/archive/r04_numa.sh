#!/bin/bash
# Queue harness on the GPU's NUMA node (default: tools/queue_bench pins its threads, the library its
# dispatchers) vs unpinned (QB_PIN=0 WG_QUEUE_PIN=0), alternating; then the pinned producer sweep.
set -o pipefail
out=gpurun_out/${1:-r04numa}
mkdir -p $out
for k in 1 2 3; do
  timeout -k 10 120 tools/queue_bench 16 100000 1420 >> $out/pin.jsonl 2>>$out/err || exit 1
  QB_PIN=0 WG_QUEUE_PIN=0 timeout -k 10 120 tools/queue_bench 16 100000 1420 >> $out/unpin.jsonl 2>>$out/err || exit 1
done
for a in "12 130000 1420" "8 200000 1420" "4 400000 1420" "1 1000000 1420" "16 100000 0" "16 100000 1420"; do
  timeout -k 10 120 tools/queue_bench $a >> $out/sweep.jsonl 2>>$out/err || exit 1
done
python3 - $out <<'PY'
import json,sys
for f in ('pin','unpin','sweep'):
    for l in open(sys.argv[1]+'/'+f+'.jsonl'):
        j=json.loads(l); print(f, j['producers'], j['len'], j['seal_open_gib_s'], 'seal p50/p99', j['seal_lat_us']['p50'], j['seal_lat_us']['p99'], 'open p50/p99', j['open_lat_us']['p50'], j['open_lat_us']['p99'], 'batch', round(j['seal_mean_batch']), round(j['open_mean_batch']), 'cpus', j['cpus_busy'], 'node', j['pinned_node'], 'bad', j['bad'])
PY
