#!/bin/bash
# Per-packet callers past the CPU count: WG_PP_WAKERS 1 / 2 / 4 waker threads, 24..128 callers,
# alternating on one box (batcher tests first, with the default)
set -o pipefail
O=gpurun_out/${1:-ppwk}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_batcher.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for w in 1 2 4; do
    for t in 16 24 32 64 128; do
      WG_PP_WAKERS=$w timeout -k 10 120 ./tools/batcher_bench $t $((160000 / t)) 1420 | sed "s/^{/{\"wakers\": $w, /" >> $O/ab.jsonl || { echo "rc $?"; exit 1; }
    done
  done
done
python3 - "$O" <<'PY'
import json, sys
for l in open(sys.argv[1] + "/ab.jsonl"):
    j = json.loads(l)
    print(j["wakers"], j["threads"], j["payload_gib_s"], j["lat_us"]["p50"], j["lat_us"]["p99"], j["lat_us"]["p999"], j["lat_us"]["max"], j["throttled_periods"])
PY
