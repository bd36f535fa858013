#!/bin/bash
# Per-packet server, in-tree build: batcher tests, stage stamps, then 1..64 callers (tools/batcher_bench)
# Usage: bash tools/pp_round.sh OUT
set -o pipefail
O=gpurun_out/${1:-r05ppf2}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_batcher.py tests/test_keypair.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for a in "1420" "1420 alt" "64" "4000"; do timeout -k 10 60 ./tools/pp_stamps $a >> $O/stamps.jsonl || { echo "stamps rc $?"; exit 1; }; done
for r in 1 2; do
  for t in 1 2 4 8 12 16 24 32 64 128; do
    timeout -k 10 120 ./tools/batcher_bench $t $((t == 1 ? 4000 : 160000 / t)) 1420 >> $O/callers.jsonl || { echo "rc $?"; exit 1; }
  done
done
python3 - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for l in open(O + "/stamps.jsonl"):
    j = json.loads(l); print(j["len"], j["op"], j["host_p50_us"], j["seen->prefix loaded_us"], j["->chacha+xor_us"], j["->poly tag_us"], j["prev ack->seen_us"])
for l in open(O + "/callers.jsonl"):
    j = json.loads(l); print(j["threads"], j["payload_gib_s"], j["lat_us"]["p50"], j["lat_us"]["p99"], j["lat_us"]["p999"], j["throttled_periods"])
PY
