#!/bin/bash
# Per-packet calls against the number of callers, with per-call stage stamps (stamps=1: one more PCIe
# write per call) and without
set -o pipefail
O=gpurun_out/${1:-r05pps}; mkdir -p $O
for t in 1 2 4 8 12 16 24 32; do
  timeout -k 10 120 ./tools/batcher_bench $t $((t == 1 ? 4000 : 64000 / t)) 1420 stamps=1 >> $O/stamps.jsonl || { echo "rc $?"; exit 1; }
  timeout -k 10 120 ./tools/batcher_bench $t $((t == 1 ? 4000 : 64000 / t)) 1420 >> $O/plain.jsonl || { echo "rc $?"; exit 1; }
done
python - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for f in ("plain", "stamps"):
    for l in open(f"{O}/{f}.jsonl"):
        j = json.loads(l)
        print(f, j["threads"], j["payload_gib_s"], j["lat_us"]["p50"], j["lat_us"]["p99"], j.get("stage_mean_us"), j["throttled_periods"])
PY
