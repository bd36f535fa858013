#!/bin/bash
# Queue: prefetch distance of wg_submit_*_n (WG_QUEUE_PREFETCH 0 / 2 / 4), one forwarder submitting per
# reap, 64..1500 B and 1420 B, alternating on one box
set -o pipefail
O=gpurun_out/${1:-qpf}; mkdir -p $O
for r in 1 2 3; do
  for pf in 0 2 4; do
    WG_QUEUE_PREFETCH=$pf timeout -k 10 120 ./tools/queue_bench 16 100000 0 8192 1 1 fwd_batch=1 | sed "s/^{/{\"prefetch\": $pf, /" >> $O/ab.jsonl || { echo "rc $?"; exit 1; }
    WG_QUEUE_PREFETCH=$pf timeout -k 10 120 ./tools/queue_bench 16 100000 1420 8192 1 1 fwd_batch=1 | sed "s/^{/{\"prefetch\": $pf, /" >> $O/ab.jsonl || { echo "rc $?"; exit 1; }
  done
done
python3 - "$O" <<'PY'
import json, sys
for l in open(sys.argv[1] + "/ab.jsonl"):
    j = json.loads(l)
    print(j["prefetch"], j["len"], j["seal_open_gib_s"], j["packets_per_s"], j["bad"], j["throttled_periods"])
PY
