#!/bin/bash
# 16 per-packet callers with and without a caller held 50 ms, three times each: where do single-call
# outliers of a few ms come from?
set -o pipefail
out=gpurun_out/${1:-r04out}
mkdir -p $out
for k in 1 2 3; do
  timeout -k 10 60 tools/batcher_bench 16 2000 1420 hold_us=50000 >> $out/hold.jsonl || exit 1
  timeout -k 10 60 tools/batcher_bench 16 2000 1420 >> $out/nohold.jsonl || exit 1
done
python3 - $out <<'PY'
import json, sys
for f in ("hold", "nohold"):
    for l in open(sys.argv[1] + "/" + f + ".jsonl"):
        j = json.loads(l)
        print(f, j["lat_us"], j["throttled_periods"], j["launches"])
PY
