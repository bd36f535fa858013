#!/bin/bash
# Queue A/B: producers taking free slots from other lanes (WG_QUEUE_STEAL=1, default) or not, alternating.
set -o pipefail
out=gpurun_out/${1:-r04qab}
mkdir -p $out
for k in 1 2 3; do
  for st in 1 0; do
    for a in "16 100000 1420" "1 600000 1420"; do
      echo "{\"steal\": $st, \"args\": \"$a\"}" >> $out/qab.jsonl
      WG_QUEUE_STEAL=$st timeout -k 10 120 tools/queue_bench $a >> $out/qab.jsonl 2>>$out/err || exit 1
    done
  done
done
python3 - $out/qab.jsonl <<'PY'
import json,sys
tag=None
for l in open(sys.argv[1]):
    j=json.loads(l)
    if 'steal' in j: tag=j; continue
    print('steal', tag['steal'], j['producers'], j['seal_open_gib_s'], 'seal p50', j['seal_lat_us']['p50'], 'open p50/p99', j['open_lat_us']['p50'], j['open_lat_us']['p99'], 'batch', round(j['seal_mean_batch']), round(j['open_mean_batch']), 'cpus', j['cpus_busy'], 'thr', j['throttled_periods'], 'bad', j['bad'])
PY
