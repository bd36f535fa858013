#!/bin/bash
# Round 6: k_lpt_one's block shape (WG_LPT_VARIANT 0..4) on IMIX in a graph: the planner's own duration from a
# kernel trace, then bench lines alternating the shapes (every line checks every packet).
set -o pipefail
T=${1:-r06v}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
die() { echo "[lptv] FAILED: $1 (rc $2)"; exit $2; }
for v in 0 1 2 3 4; do
  WG_LPT_VARIANT=$v timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 $ROOT/bench.py --workload imix --graph --no-cpu-baseline > $O/prof_bench_$v.json 2> $O/prof_$v.log || die prof_$v $?
  python3 $ROOT/tools/prof_window.py trace $(find $O/prof_$v -name "run_kernel_trace.csv" | head -1) $O/prof_bench_$v.json --out $O/window_$v.json > /dev/null || die window_$v $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'lpt_variant': int(sys.argv[2]), **{k: d.get(k) for k in ('window_span_per_step_us', 'kernel_busy_per_step_us', 'planning_busy_per_step_us', 'gap_per_step_us')}}))" $O/window_$v.json $v | tee -a $O/trace.jsonl
done
cd $ROOT
for a in 1 2; do
  for v in 0 1 2 3 4; do
    WG_LPT_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --workload imix --graph > $O/tmp.json 2>> $O/bench.err || die "bench $v" $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'lpt_variant': int(sys.argv[2]), 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'verified': d['verified']}))" $O/tmp.json $v | tee -a $O/ab.jsonl
  done
done
echo "[lptv] done"
