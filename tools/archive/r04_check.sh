#!/bin/bash
# Round-4 focused GPU check: the full-size k_step parity tests, the per-packet server and queue tests,
# the C1 / C2 / C3 bench lines (with the oracle sample check) and the per-packet / queue load figures.
set -o pipefail
R=${1:-r04a}
O=gpurun_out/$R
mkdir -p $O
step() { echo "[r04] $1 $(date +%T)"; }
step tests
timeout -k 10 600 python -u -m pytest tests/test_batcher.py tests/test_queue.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
step queue_bench
for a in "16 100000 1420" "16 100000 0" "4 100000 1420" "1 50000 1420"; do timeout -k 10 120 ./tools/queue_bench $a >> $O/queue.jsonl || exit 1; done
cut -c1-420 $O/queue.jsonl
step batcher
for t in 1 16 64 128; do timeout -k 10 120 ./tools/batcher_bench $t $((t == 1 ? 4000 : 160000 / t)) 1420 >> $O/batcher.jsonl || exit 1; done
timeout -k 10 120 ./tools/batcher_bench 1 300 1420 gap_us=2000 >> $O/batcher.jsonl || exit 1
timeout -k 10 120 ./tools/batcher_bench 16 2000 1420 hold_us=50000 >> $O/batcher.jsonl || exit 1
cut -c1-300 $O/batcher.jsonl
step bench_c1
timeout -k 10 300 python bench.py > $O/c1.json 2> $O/bench.err || exit 1
cat $O/c1.json
step bench_c1_graph
timeout -k 10 300 python bench.py --graph --no-cpu-baseline > $O/c1_graph.json 2>> $O/bench.err || exit 1
step bench_c2
timeout -k 10 300 python bench.py --workload c2 > $O/c2.json 2>> $O/bench.err || exit 1
step bench_c3
timeout -k 10 300 python bench.py --workload c3 --steps 5 --warmup 1 > $O/c3.json 2>> $O/bench.err || exit 1
step done
