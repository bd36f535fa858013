# per-packet server check on the GPU box: batcher tests, then the latency/throughput tool
set -o pipefail
O=gpurun_out/${1:-pp}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_batcher.py tests/test_keypair.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for t in 1 16 64; do timeout -k 10 120 ./tools/batcher_bench $t $((t == 1 ? 4000 : 160000 / t)) 1420 >> $O/batcher.jsonl || exit 1; done
timeout -k 10 120 ./tools/batcher_bench 16 10000 0 >> $O/batcher.jsonl
cat $O/batcher.jsonl
