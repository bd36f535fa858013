set -o pipefail
mkdir -p gpurun_out/ppsleep
timeout -k 10 200 python -u -m pytest tests/test_batcher.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ppsleep/tests.log 2>&1 || { tail -30 gpurun_out/ppsleep/tests.log; exit 1; }
tail -1 gpurun_out/ppsleep/tests.log
for t in 1 16 64 128; do
  s0=$(date +%s.%N)
  timeout -k 5 60 ./tools/batcher_bench $t $((t == 1 ? 4000 : 80000 / t)) 1420 >> gpurun_out/ppsleep/batcher.jsonl; rc=$?
  echo "callers $t rc $rc seconds $(echo "$(date +%s.%N) - $s0" | bc)"
  [ $rc -eq 0 ] || exit $rc
done
cat gpurun_out/ppsleep/batcher.jsonl
