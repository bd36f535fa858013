set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05w
mkdir -p $O
for rep in 1 2; do
  for v in default s2 s6 s12; do
    case $v in default) env="WG_SLOT4=0" ;; s2) env="WG_SLOT4=2 WG_MIXED_SPLIT=2" ;; s6) env="WG_SLOT4=2 WG_MIXED_SPLIT=6" ;; s12) env="WG_SLOT4=2 WG_MIXED_SPLIT=12" ;; esac
    line=$(env $env timeout -k 10 200 python bench.py --workload c2 --no-cpu-baseline --steps 100 2>> $O/c2.err) || { echo "FAILED $v"; exit 1; }
    echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'plan':'$v','rep':$rep,'gib_s':d['value'],'verified':d['verified']}))" | tee -a $O/c2_slot4_ab.jsonl
  done
done
