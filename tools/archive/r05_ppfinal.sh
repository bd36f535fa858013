#!/bin/bash
# Per-packet server, round-5 rewrite: the GPU suite, stage stamps, then batcher_bench (threads on the
# GPU's NUMA node) for build_ab/r05pp0 (before) and the current build, alternating on one box
set -o pipefail
O=gpurun_out/${1:-r05ppf}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for a in "64" "1420" "4000" "1420 alt"; do
  timeout -k 10 60 ./tools/pp_stamps $a >> $O/stamps.jsonl || { echo "stamps rc $?"; exit 1; }
done
for r in 1 2 3; do
  for v in old new; do
    B=./tools/batcher_bench; [ $v = old ] && B=./build_ab/r05pp0/batcher_bench
    for t in 1 16 64; do
      timeout -k 10 120 $B $t $((t == 1 ? 4000 : 160000 / t)) 1420 | sed "s/^{/{\"build\": \"$v\", /" >> $O/ab.jsonl || { echo "rc $?"; exit 1; }
    done
  done
done
python - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for l in open(O + "/stamps.jsonl"):
    print(l.strip())
for l in open(O + "/ab.jsonl"):
    j = json.loads(l); print(j["build"], j["threads"], j["payload_gib_s"], j["lat_us"], j["throttled_periods"], j.get("pinned_node"))
PY
