#!/bin/bash
# Round 6: C1 (two streams) launched vs captured in a HIP graph, at the driver's 20 steps and at 200.
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${1:-r06g}
mkdir -p $O
die() { echo "[g] FAILED: $1 (rc $2)"; exit $2; }
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/tmp.json 2>> $O/err.log || die "$name" $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'variant': sys.argv[2], 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'host_enqueue_ms_per_step': d['host_enqueue_ms_per_step'], 'verified': d['verified']}))" $O/tmp.json "$name" >> $O/ab.jsonl
  tail -1 $O/ab.jsonl
}
for a in 1 2 3; do
  run c1_20 --steps 20 --warmup 5
  run c1_20_graph --steps 20 --warmup 5 --graph
  run c1_200 --steps 200 --warmup 20
  run c1_200_graph --steps 200 --warmup 20 --graph
  run c2_graph --workload c2 --graph
done
echo "[g] done"
