#!/bin/bash
# Round 6: per-stream plan workspaces (WG_STREAM_WS) for the IMIX step on two streams: the bench's own checks
# on every line, alternating one stream, two streams, and two streams on the shared workspace.
# Usage: bash tools/r06_ws.sh <tag> [alternations]
set -o pipefail
T=${1:-r06ws}
ALT=${2:-3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$T
mkdir -p $O
cd $ROOT
die() { echo "[ws] FAILED: $1 (rc $2)"; exit $2; }
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 600 $PYT tests/test_gpu_configs.py -k "two_lane or imix" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; die tests $?; }
tail -1 $O/tests.log
run() {  # name env... -- args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline --workload imix "$@" > $O/tmp.json 2>> $O/bench.err || die "bench $name" $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'variant': sys.argv[2], 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['roofline']['kernel_ms'], 'verified': d['verified'], 'n_streams': d['config'].get('streams')}))" $O/tmp.json "$name" >> $O/ab.jsonl
  tail -1 $O/ab.jsonl
}
for a in $(seq 1 $ALT); do
  run s1 X=1 -- --streams 1
  run s2 X=1 -- --streams 2
  run s2_shared WG_STREAM_WS=0 -- --streams 2
  run s2_20 X=1 -- --streams 2 --steps 20 --warmup 5
done
echo "[ws] done"
