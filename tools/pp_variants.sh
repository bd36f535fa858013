#!/bin/bash
# Per-packet server build variants under build_ab/<V>/ (libwgaead.so + batcher_bench + pp_stamps),
# alternating on one box: usage pp_variants.sh OUT V1 V2 ...
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
for v in "$@"; do
  timeout -k 10 60 ./build_ab/$v/pp_stamps 1420 alt | sed "s/^{/{\"build\": \"$v\", /" >> $O/stamps.jsonl || { echo "stamps rc $?"; exit 1; }
done
for r in 1 2 3; do
  for v in "$@"; do
    for t in 1 16; do
      timeout -k 10 120 ./build_ab/$v/batcher_bench $t $((t == 1 ? 4000 : 10000)) 1420 | sed "s/^{/{\"build\": \"$v\", /" >> $O/ab.jsonl || { echo "rc $?"; exit 1; }
    done
  done
done
python - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for l in open(O + "/stamps.jsonl"):
    j = json.loads(l)
    print(j["build"], j["op"][:4], "host", j["host_p50_us"], "prefix", j["seen->prefix loaded_us"], "ack->seen", j["prev ack->seen_us"])
for l in open(O + "/ab.jsonl"):
    j = json.loads(l); print(j["build"], j["threads"], j["payload_gib_s"], j["lat_us"]["p50"], j["lat_us"]["p99"], j["throttled_periods"])
PY
