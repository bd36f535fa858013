#!/bin/bash
# Per-packet latency: round-4 library + harness (build_ab/r04) against the current ones, alternating on one box
set -o pipefail
O=gpurun_out/r05ppab; mkdir -p $O
for r in 1 2 3; do
  for v in r04 r05; do
    B=./tools/batcher_bench; [ $v = r04 ] && B=./build_ab/r04/batcher_bench
    for t in 1 16; do
      timeout -k 10 120 $B $t $((t == 1 ? 4000 : 10000)) 1420 | sed "s/^{/{\"build\": \"$v\", /" >> $O/ab.jsonl || { echo "rc $?"; exit 1; }
    done
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r05ppab/ab.jsonl"):
    j = json.loads(l); print(j["build"], j["threads"], j["payload_gib_s"], j["lat_us"], j["throttled_periods"])
PY
