#!/bin/bash
# tools/batcher_bench for build_ab/<V>/ builds, alternating on one box (1, 8, 16 callers), after the
# batcher tests of the in-tree build: usage pp_ab.sh OUT V1 V2 ...
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_batcher.py tests/test_keypair.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for v in "$@"; do
    for t in 1 8 16; do
      timeout -k 10 120 ./build_ab/$v/batcher_bench $t $((t == 1 ? 4000 : 160000 / t)) 1420 | sed "s/^{/{\"build\": \"$v\", /" >> $O/ab.jsonl || { echo "rc $?"; exit 1; }
    done
  done
done
python3 - "$O" <<'PY'
import json, sys
for l in open(sys.argv[1] + "/ab.jsonl"):
    j = json.loads(l)
    print(j["build"], j["threads"], j["payload_gib_s"], j["lat_us"]["p50"], j["lat_us"]["p99"], j["throttled_periods"])
PY
