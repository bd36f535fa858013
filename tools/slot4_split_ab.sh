#!/bin/bash
# The 16 / 4-lane split's threshold on IMIX (WG_SLOT4=2 with WG_MIXED_SPLIT=R: packets of more than R
# 8-block rounds in 16-lane slots), alternating, two reps; and a 2-stream line of the planned default.
set -o pipefail
R=${1:-r05r}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$R
mkdir -p $O
for rep in 1 2; do
  for v in 1 2 3; do
    line=$(WG_SLOT4=2 WG_MIXED_SPLIT=$v timeout -k 10 200 python bench.py --workload imix --no-cpu-baseline --steps 100 2>> $O/split.err) || { echo "FAILED $v"; exit 1; }
    echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'split':$v,'rep':$rep,'gib_s':d['value'],'kernel_ms':d['roofline']['kernel_ms'],'verified':d['verified']}))" | tee -a $O/split_ab.jsonl
  done
done
line=$(timeout -k 10 200 python bench.py --workload imix --no-cpu-baseline --steps 100 --streams 2 2>> $O/split.err) || exit 1
echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'streams':2,'gib_s':d['value'],'verified':d['verified']}))" | tee -a $O/split_ab.jsonl
