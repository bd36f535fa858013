set -o pipefail
mkdir -p gpurun_out/ppsleep
timeout -k 10 200 python -u -m pytest tests/test_batcher.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ppsleep/tests.log 2>&1 || { tail -30 gpurun_out/ppsleep/tests.log; exit 1; }
tail -1 gpurun_out/ppsleep/tests.log
for t in 1 16 64 128; do timeout -k 10 120 ./tools/batcher_bench $t $((t == 1 ? 4000 : 160000 / t)) 1420 >> gpurun_out/ppsleep/batcher.jsonl || exit 1; done
cat gpurun_out/ppsleep/batcher.jsonl
