#!/bin/bash
# IMIX plan A/B on one box (run through gpurun from the repo root): the default plan against the
# one-packet-per-slot plans (WG_MIXED_SPLIT) and dynamic claims (WG_CLAIM), alternating, two reps.
set -o pipefail
R=${1:-r05l}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$R
mkdir -p $O
for rep in 1 2; do
  for v in default split1 split2 split4 claim; do
    case $v in
      default) env="" ;; split1) env="WG_MIXED_SPLIT=1" ;; split2) env="WG_MIXED_SPLIT=2" ;;
      split4) env="WG_MIXED_SPLIT=4" ;; claim) env="WG_CLAIM=1" ;;
    esac
    line=$(env $env timeout -k 10 200 python bench.py --workload imix --no-cpu-baseline --steps 100 2>> $O/imix_ab.err) || { echo "FAILED $v rc $?"; exit 1; }
    echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'variant':'$v','rep':$rep,'gib_s':d['value'],'kernel_ms':d['roofline']['kernel_ms'],'verified':d['verified'],'bit_exact':d.get('oracle_sample',{}).get('bit_exact')}))" | tee -a $O/imix_ab.jsonl
  done
done
