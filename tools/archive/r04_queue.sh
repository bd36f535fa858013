#!/bin/bash
# Queue harness: bit-exact tests, then tools/queue_bench at 16 (x3), 12, 8, 4, 1 producers and mixed sizes.
set -o pipefail
out=gpurun_out/${1:-r04q}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_queue.py -m gpu > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
for a in "16 100000 1420" "16 100000 1420" "16 100000 1420" "12 130000 1420" "8 200000 1420" "4 400000 1420" "1 1000000 1420" "16 100000 0"; do
  timeout -k 10 120 tools/queue_bench $a >> $out/queue.jsonl 2>>$out/err || exit 1
done
python3 - $out/queue.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    j=json.loads(l); print(j['producers'], j['len'], j['seal_open_gib_s'], 'seal p50', j['seal_lat_us']['p50'], 'open p50/p99', j['open_lat_us']['p50'], j['open_lat_us']['p99'], 'batch', round(j['seal_mean_batch']), round(j['open_mean_batch']), 'cpus', j['cpus_busy'], 'thr', j['throttled_periods'], j['throttled_ms'], 'bad', j['bad'])
PY
