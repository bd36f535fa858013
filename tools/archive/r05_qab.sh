#!/bin/bash
# Queue: round-5 (a) library (build_ab/q1: batched pops, no shared submit counter) against (b) the current
# one (+ cached ring views, asymmetric membarrier fence), alternating on one box; tests first
set -o pipefail
O=gpurun_out/r05qab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_queue.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc $?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3 4; do
  for v in a b; do
    B=./tools/queue_bench; [ $v = a ] && B=./build_ab/q1/queue_bench
    for L in 1420 0; do
      timeout -k 10 120 $B 16 100000 $L 8192 1 1 | sed "s/^{/{\"build\": \"$v\", /" >> $O/ab.jsonl || { echo "qb rc $?"; exit 1; }
    done
  done
done
python -c "
import json, collections
d = collections.defaultdict(list)
for l in open('$O/ab.jsonl'):
    j = json.loads(l); d[(j['build'], j['len'])].append(round(j['seal_open_gib_s'], 2))
    assert j['bad'] == 0
for k, v in sorted(d.items()): print(k, v)"
