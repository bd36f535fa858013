#!/bin/bash
# Round 6: 2-lane slots for the short-packet split plan's tiny packets (WG_SLOT2=k): the parity tests, then
# IMIX bench lines alternating WG_SLOT2=0 / 1 / 2.
# Usage: bash tools/r06_slot2.sh <tag> [alternations]
set -o pipefail
T=${1:-r06s2}
ALT=${2:-3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$T
mkdir -p $O
cd $ROOT
die() { echo "[slot2] FAILED: $1 (rc $2)"; exit $2; }
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 600 $PYT tests/test_gpu_configs.py -k "two_lane or imix" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; die tests $?; }
tail -1 $O/tests.log
for a in $(seq 1 $ALT); do
  for k in 0 1 2; do
    WG_SLOT2=$k timeout -k 10 300 python bench.py --no-cpu-baseline --workload imix > $O/tmp.json 2>> $O/bench.err || die "bench $k" $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'slot2': $k, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['roofline']['kernel_ms'], 'verified': d['verified']}))" $O/tmp.json >> $O/ab.jsonl
    tail -1 $O/ab.jsonl
  done
done
echo "[slot2] done"
