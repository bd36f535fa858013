#!/bin/bash
# Round 5, queue + per-packet: the queue / per-packet tests, per-packet A/B against round 4 (stamps now
# opt-in), the queue at 1420 B (10 runs) and on the 64..1500 B mix with the CPU port on the same
# packets in the same process, then the rocprof traces / counters of C1 (one and two streams) and C2.
set -o pipefail
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_queue.py tests/test_batcher.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc $?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in r04 r05; do
    B=./tools/batcher_bench; [ $v = r04 ] && B=./build_ab/r04/batcher_bench
    for t in 1 16; do
      timeout -k 10 120 $B $t $((t == 1 ? 4000 : 10000)) 1420 | sed "s/^{/{\"build\": \"$v\", /" >> $O/ppab.jsonl || { echo "pp rc $?"; exit 1; }
    done
  done
done
python -c "
import json
for l in open('$O/ppab.jsonl'):
    j=json.loads(l); print(j['build'], j['threads'], j['payload_gib_s'], j['lat_us']['p50'], j['lat_us']['p999'])"
for r in 1 2 3 4 5 6 7 8 9 10; do
  timeout -k 10 120 ./tools/queue_bench 16 100000 1420 8192 1 1 $([ $r = 1 ] && echo cpu_port=oracle/liboracle.so) >> $O/queue_1420.jsonl || { echo "qb rc $?"; exit 1; }
done
for r in 1 2 3 4 5; do
  timeout -k 10 120 ./tools/queue_bench 16 100000 0 8192 1 1 cpu_port=oracle/liboracle.so >> $O/queue_mixed.jsonl || { echo "qbm rc $?"; exit 1; }
  timeout -k 10 120 ./tools/queue_bench 16 100000 0 8192 2 2 >> $O/queue_mixed_2x2.jsonl || { echo "qbm2 rc $?"; exit 1; }
done
python -c "
import json
for f in ['queue_1420','queue_mixed','queue_mixed_2x2']:
    v=[json.loads(l) for l in open('$O/'+f+'.jsonl')]
    print(f, sorted(round(j['seal_open_gib_s'],2) for j in v), [j.get('cpu_port_gib_s') for j in v if 'cpu_port_gib_s' in j], sum(j['bad'] for j in v))"
bash tools/gpu_round.sh r05 prof
