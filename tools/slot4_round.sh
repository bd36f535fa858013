#!/bin/bash
# 4-lane slots (WG_SLOT4) on the GPU box: their parity tests, then IMIX and C2 with the size-based plan
# against WG_SLOT4=0 (the round-4 plan), alternating, and C1 once (its plan is unchanged).
set -o pipefail
R=${1:-r05m}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$R
mkdir -p $O
echo "[slot4] tests"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_duplex.py tests/test_gpu_configs.py -x -v -m gpu -k "4_lane or after_seal_mixed or imix or c2_full" --timeout 120 --timeout-method thread > $O/slot4_tests.log 2>&1 || { echo "[slot4] tests FAILED rc $?"; tail -30 $O/slot4_tests.log; exit 1; }
tail -1 $O/slot4_tests.log
for rep in 1 2; do
  for w in imix; do
    for v in 0 planned all4; do
      case $v in 0) env="WG_SLOT4=0" ;; planned) env="WG_SLOT4_PLANNED=1" ;; all4) env="WG_SLOT4=1" ;; esac
      line=$(env $env timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --steps 100 2>> $O/slot4_ab.err) || { echo "[slot4] bench FAILED $w $v"; exit 1; }
      echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'workload':'$w','slot4':'$v','rep':$rep,'gib_s':d['value'],'kernel_ms':d['roofline']['kernel_ms'],'verified':d['verified']}))" | tee -a $O/slot4_ab.jsonl
    done
  done
done
echo "[slot4] c1"
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c1.json 2>> $O/slot4_ab.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench_c1.json')); print('c1', d['value'], d['verified'])"
