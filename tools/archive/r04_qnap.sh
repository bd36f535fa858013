#!/bin/bash
# Queue dispatcher naps (default) vs the library before (saved as gpurun-side copy is not possible:
# compare against WG_QUEUE_MIN_BATCH / defaults only) -- runs the harness 4x at 16 producers and 2x at 1.
set -o pipefail
out=gpurun_out/${1:-r04qn}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_queue.py -m gpu > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for a in "16 100000 1420" "1 600000 1420" "16 100000 1420" "16 100000 1420" "1 600000 1420" "16 100000 1420" "16 100000 0"; do
  timeout -k 10 120 tools/queue_bench $a >> $out/q.jsonl 2>>$out/err || exit 1
done
python3 - $out/q.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    j=json.loads(l); print(j['producers'], j['len'], j['seal_open_gib_s'], 'open p50/p99', j['open_lat_us']['p50'], j['open_lat_us']['p99'], 'batch', round(j['seal_mean_batch']), round(j['open_mean_batch']), 'cpus', j['cpus_busy'], 'thr', j['throttled_periods'], 'bad', j['bad'])
PY
