#!/bin/bash
# Round 5, first box: the whole GPU suite (new: bench self-check, replay skew, queue key snapshot /
# timeout / concurrency), then C1 with the k_step<8,4> build for half-machine grids against k_step<8,8>
# (WG_STEP_WPE4=0), alternating.
set -o pipefail
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc $?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 1 0; do
    WG_STEP_WPE4=$v timeout -k 10 300 python bench.py --no-cpu-baseline >> $O/wpe4_$v.jsonl 2>> $O/bench.err || { echo "bench rc $?"; exit 1; }
    tail -1 $O/wpe4_$v.jsonl | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('wpe4=$v', j['value'], j['roofline']['frac'], j['roofline']['step']['frac'], j['verified'])"
  done
done
# the per-packet outlier: the held-caller shape with per-call stage stamps, 6 runs
for r in 1 2 3 4 5 6; do
  timeout -k 10 120 ./tools/batcher_bench 16 2000 1420 hold_us=50000 stamps=1 >> $O/outlier.jsonl || { echo "batcher rc $?"; exit 1; }
done
python - <<'PY'
import json
for l in open("gpurun_out/r05a/outlier.jsonl"):
    j = json.loads(l); print(j["lat_us"], j["throttled_periods"], j.get("slowest"), j.get("calls_over_1ms"), j.get("calls_over_1ms_preempted"))
PY
