#!/bin/bash
# Round 6: the workspace event recorded by the step kernel's own completion (hipExtLaunchKernel stop event,
# WG_WS_EXT) instead of a hipEventRecord after it: the GPU suite, then IMIX / C2 / C1 lines alternating.
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${1:-r06e}
mkdir -p $O
die() { echo "[wsext] FAILED: $1 (rc $2)"; exit $2; }
timeout -k 10 700 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; die tests $?; }
tail -1 $O/tests.log
for a in 1 2 3; do
  for w in imix c2; do
    for v in 1 0; do
      WG_WS_EXT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --workload $w > $O/tmp.json 2>> $O/bench.err || die "bench $w $v" $?
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'workload': sys.argv[2], 'ws_ext': int(sys.argv[3]), 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'verified': d['verified']}))" $O/tmp.json $w $v | tee -a $O/ab.jsonl
    done
  done
done
for v in 1 0; do
  WG_WS_EXT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --workload imix --streams 2 > $O/tmp.json 2>> $O/bench.err || die "bench s2 $v" $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'workload': 'imix --streams 2', 'ws_ext': int(sys.argv[2]), 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'verified': d['verified']}))" $O/tmp.json $v | tee -a $O/ab.jsonl
done
echo "[wsext] done"
