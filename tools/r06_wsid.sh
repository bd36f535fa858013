#!/bin/bash
# Round 6: per-stream workspaces without a per-call event (stream-id guard): parity tests, then IMIX launched
# and in a graph, alternated.
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${1:-r06i}
mkdir -p $O
die() { echo "[wsid] FAILED: $1 (rc $2)"; exit $2; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_bench.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; die tests $?; }
tail -1 $O/tests.log
for a in 1 2 3; do
  for g in "" "--graph" "--streams 2"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --workload imix $g > $O/tmp.json 2>> $O/bench.err || die "bench $g" $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'args': sys.argv[2], 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'verified': d['verified']}))" $O/tmp.json "$g" | tee -a $O/ab.jsonl
  done
  timeout -k 10 300 python bench.py --no-cpu-baseline --workload c2 > $O/tmp.json 2>> $O/bench.err || die "bench c2" $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'args': 'c2', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'verified': d['verified']}))" $O/tmp.json | tee -a $O/ab.jsonl
done
echo "[wsid] done"
