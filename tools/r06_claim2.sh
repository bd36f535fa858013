#!/bin/bash
# Round 6: k_step_claim claiming two packets ahead (WG_CLAIM=1): its parity tests, then C2 bench lines
# alternating the static snake (default) and the claims.
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${1:-r06cl}
mkdir -p $O
die() { echo "[claim2] FAILED: $1 (rc $2)"; exit $2; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_configs.py -k "claim or c2" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; die tests $?; }
tail -1 $O/tests.log
for a in 1 2 3; do
  for v in 0 1; do
    WG_CLAIM=$v timeout -k 10 300 python bench.py --no-cpu-baseline --workload c2 > $O/tmp.json 2>> $O/bench.err || die "bench $v" $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'claim': int(sys.argv[2]), 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['roofline']['kernel_ms'], 'verified': d['verified']}))" $O/tmp.json $v | tee -a $O/ab.jsonl
  done
done
echo "[claim2] done"
