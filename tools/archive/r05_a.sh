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
# per-wave start / end times of one k_step launch (diagnostic build): the C2 tail, and C1 for reference
for w in c2 c1; do
  timeout -k 10 120 python tools/phase_stamps.py --mode step --workload $w $([ $w = c1 ] && echo --keys 1) > $O/stamps_step_$w.json || { echo "stamps rc $?"; exit 1; }
  python -c "import json; j=json.load(open('$O/stamps_step_$w.json')); print('$w', j['kernel_span_us'], j['wave_life_us_mean'], j['wave_end_us'], j['tail_idle_frac'], j['live_waves_over_time'])"
done
# C2: dynamic claims (k_step_claim) against the static snake, with and without the issue-priority schedule
for r in 1 2; do
  for cfg in "WG_CLAIM=0" "WG_CLAIM=1" "WG_CLAIM=1 WG_PRIO=0"; do
    env $cfg timeout -k 10 300 python bench.py --workload c2 --no-cpu-baseline >> $O/c2_claim.jsonl 2>> $O/bench.err || { echo "bench c2 rc $?"; exit 1; }
    tail -1 $O/c2_claim.jsonl | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$cfg', j['value'], j['roofline']['frac'], j['roofline']['kernel_ms'], j['verified'])"
  done
done
