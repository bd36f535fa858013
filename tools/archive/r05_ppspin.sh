#!/bin/bash
# Per-packet callers beyond the CPUs: this build's spin tokens, 16..128 callers, with and without
# stage stamps (stamps=1: more host work per call), batcher tests first
set -o pipefail
O=gpurun_out/${1:-r05ppspin}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_batcher.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for st in 0 1; do
    for t in 16 20 24 32 64 128; do
      timeout -k 10 120 ./tools/batcher_bench $t $((160000 / t)) 1420 stamps=$st | sed "s/^{/{\"stamps\": $st, /" >> $O/ab.jsonl || { echo "rc $?"; exit 1; }
    done
  done
done
python - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for l in open(O + "/ab.jsonl"):
    j = json.loads(l)
    print(j["stamps"], j["threads"], j["payload_gib_s"], j["lat_us"]["p50"], j["lat_us"]["p99"], j["lat_us"]["p999"], j["lat_us"]["max"], j["throttled_periods"])
PY
