#!/bin/bash
# IMIX-shaped batches of 8,192 to 131,072 packets: the size-based plan (WG_SLOT4 unset) against the 16 / 4
# split forced (WG_SLOT4=2) and the old plans (WG_SLOT4=0), alternating, two reps.
set -o pipefail
R=${1:-r05t}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$R
mkdir -p $O
for rep in 1 2; do
  for n in 8192 16384 32768 131072; do
    for v in 0 planned 2; do
      case $v in 0) env="WG_SLOT4=0" ;; planned) env="WG_SLOT4_PLANNED=1" ;; 2) env="WG_SLOT4=2" ;; esac
      line=$(env $env timeout -k 10 200 python bench.py --workload imix --packets $n --no-cpu-baseline --steps 100 2>> $O/sizes.err) || { echo "FAILED $n $v"; exit 1; }
      echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'packets':$n,'plan':'$v','rep':$rep,'gib_s':d['value'],'verified':d['verified']}))" | tee -a $O/sizes_ab.jsonl
    done
  done
done
