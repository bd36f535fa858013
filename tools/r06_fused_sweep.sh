#!/bin/bash
# Round 6: k_step_mixed_fused's poll kind (WG_FUSED_POLL) and planner count (WG_FUSED_NP) on IMIX: the diagnostic
# build's per-workgroup timing (tools/fused_timing.py), then a bench line of the product build per setting and
# the two-launch plan (WG_LPT_FUSED=0) between them.
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${1:-r06fs}
mkdir -p $O
die() { echo "[sweep] FAILED: $1 (rc $2)"; exit $2; }
for poll in 0 1 2; do
  for np in 64 128 256; do
    WG_FUSED_POLL=$poll WG_FUSED_NP=$np timeout -k 10 120 python tools/fused_timing.py >> $O/timing.jsonl 2>> $O/err.log || die "timing $poll $np" $?
    tail -1 $O/timing.jsonl
    WG_FUSED_POLL=$poll WG_FUSED_NP=$np timeout -k 10 300 python bench.py --no-cpu-baseline --workload imix > $O/tmp.json 2>> $O/err.log || die "bench $poll $np" $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'poll': $poll, 'np': $np, 'ms_per_step': d['ms_per_step'], 'verified': d['verified']}))" $O/tmp.json >> $O/ab.jsonl
    tail -1 $O/ab.jsonl
  done
  WG_LPT_FUSED=0 timeout -k 10 300 python bench.py --no-cpu-baseline --workload imix > $O/tmp.json 2>> $O/err.log || die "bench two-launch" $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'fused': 0, 'ms_per_step': d['ms_per_step'], 'verified': d['verified']}))" $O/tmp.json >> $O/ab.jsonl
  tail -1 $O/ab.jsonl
done
echo "[sweep] done"
