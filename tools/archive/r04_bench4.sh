#!/bin/bash
# Round-4 bench lines: c1, c2, c3, c1 with the two-stream step beside the one-stream kernel roofline,
# then the queue harness three times (stability of the 16-producer rate).
set -o pipefail
out=gpurun_out/${1:-r04o}
mkdir -p $out
for w in c1 c2 c3 c1b; do
  wl=${w%b}; extra=""
  [ $wl = c3 ] && extra="--steps 5 --warmup 1"
  timeout -k 10 300 python bench.py --workload $wl $extra > $out/$w.json 2>>$out/err || exit 1
  python3 - $out/$w.json <<'PY' || exit 1
import json,sys
j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=j["roofline"]
print(sys.argv[1], j["value"], j["ms_per_step"], r["frac"], r.get("kernel_ms"), r.get("traffic"), r.get("step"), j.get("verified"), j.get("oracle_sample"), j["cpu_baseline"]["value"])
PY
done
for k in 1 2 3; do
  timeout -k 10 120 tools/queue_bench 16 100000 1420 >> $out/queue.jsonl 2>>$out/err || exit 1
done
timeout -k 10 120 tools/queue_bench 8 200000 1420 >> $out/queue.jsonl 2>>$out/err || exit 1
timeout -k 10 120 tools/queue_bench 1 200000 1420 >> $out/queue.jsonl 2>>$out/err || exit 1
timeout -k 10 120 tools/queue_bench 16 100000 0 >> $out/queue.jsonl 2>>$out/err || exit 1
cat $out/queue.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    j=json.loads(l); print(j['producers'], j['len'], j['seal_open_gib_s'], j['seal_lat_us']['p50'], j['open_lat_us']['p50'], j['open_lat_us']['p99'], j['bad'])
"
