#!/bin/bash
# Round 6 closing measurements: the driver's command (C1, 20 steps) and 200-step lines, C2, IMIX one stream
# and IMIX captured in a HIP graph, alternated.
# Usage: bash tools/r06_final_ab.sh <tag> [alternations]
set -o pipefail
T=${1:-r06z}
ALT=${2:-2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$T
mkdir -p $O
cd $ROOT
die() { echo "[final] FAILED: $1 (rc $2)"; exit $2; }
run() {  # name -- args
  local name=$1; shift; shift
  timeout -k 10 300 python bench.py "$@" > $O/$name.json 2>> $O/bench.err || die "bench $name" $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'variant': sys.argv[2], 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['roofline']['kernel_ms'], 'frac': d['roofline']['frac'], 'verified': d['verified']}))" $O/$name.json "$name" >> $O/ab.jsonl
  tail -1 $O/ab.jsonl
}
for a in $(seq 1 $ALT); do
  run c1_driver_$a -- --gpus 1 --steps 20 --warmup 5
  run c1_200_$a -- --no-cpu-baseline --steps 200 --warmup 20
  run c2_$a -- --no-cpu-baseline --workload c2
  run imix_$a -- --no-cpu-baseline --workload imix
  run imix_graph_$a -- --no-cpu-baseline --workload imix --graph
done
echo "[final] done"
