#!/bin/bash
# Per-packet server, round-5 rewrite (quad-lane ChaCha20, DPP Poly1305 scan, one-round-trip loads,
# 16-B result stores) against the build before it (build_ab/r05pp0), alternating on one box
set -o pipefail
O=gpurun_out/${1:-r05ppq}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_batcher.py tests/test_keypair.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for v in old new; do
  P=./tools/pp_stamps; [ $v = old ] && P=./build_ab/r05pp0/pp_stamps
  for L in 64 1420 4000; do
    timeout -k 10 60 $P $L | sed "s/^{/{\"build\": \"$v\", /" >> $O/stamps.jsonl || { echo "stamps rc $?"; exit 1; }
  done
done
for r in 1 2 3; do
  for v in old new; do
    B=./tools/batcher_bench; [ $v = old ] && B=./build_ab/r05pp0/batcher_bench
    for t in 1 16; do
      timeout -k 10 120 $B $t $((t == 1 ? 4000 : 10000)) 1420 | sed "s/^{/{\"build\": \"$v\", /" >> $O/ab.jsonl || { echo "rc $?"; exit 1; }
    done
  done
done
python - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for l in open(O + "/stamps.jsonl"):
    print(l.strip())
for l in open(O + "/ab.jsonl"):
    j = json.loads(l); print(j["build"], j["threads"], j["payload_gib_s"], j["lat_us"], j["throttled_periods"])
PY
