#!/bin/bash
# Queue: batched submits (wg_submit_*_n) — the queue tests, then tools/queue_bench with the forwarder
# submitting per packet (fwd_batch=0) and per reap (fwd_batch=1), alternating on one box
set -o pipefail
O=gpurun_out/${1:-r05qb}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_queue.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for r in 1 2 3 4 5; do
  for b in 0 1; do
    timeout -k 10 120 ./tools/queue_bench 16 100000 0 8192 1 1 fwd_batch=$b >> $O/mixed.jsonl || { echo "rc $?"; exit 1; }
    timeout -k 10 120 ./tools/queue_bench 16 100000 1420 8192 1 1 fwd_batch=$b >> $O/1420.jsonl || { echo "rc $?"; exit 1; }
  done
done
timeout -k 10 300 ./tools/queue_bench 16 100000 0 8192 1 1 fwd_batch=1 cpu_port=oracle/liboracle.so >> $O/mixed_cpu.jsonl || exit 1
python - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for f in ("mixed", "1420", "mixed_cpu"):
    for l in open(f"{O}/{f}.jsonl"):
        j = json.loads(l)
        print(f, j["fwd_batch"], j["seal_open_gib_s"], j["packets_per_s"], j["bad"], j.get("cpu_port_gib_s"), j["throttled_periods"])
PY
