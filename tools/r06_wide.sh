#!/bin/bash
# Round 6: the one-launch sparse plan for C2's 8-lane longest-first pairs (WG_LPT_WIDE): the whole GPU suite,
# then C2 bench lines alternating it with the two planning launches, and a kernel trace of each.
set -o pipefail
T=${1:-r06x}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$T
mkdir -p $O
cd $ROOT
die() { echo "[wide] FAILED: $1 (rc $2)"; exit $2; }
timeout -k 10 700 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; die tests $?; }
tail -1 $O/tests.log
for a in 1 2 3; do
  for v in 1 0; do
    WG_LPT_WIDE=$v timeout -k 10 300 python bench.py --no-cpu-baseline --workload c2 > $O/tmp.json 2>> $O/bench.err || die "bench $v" $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'lpt_wide': int(sys.argv[2]), 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['roofline']['kernel_ms'], 'verified': d['verified']}))" $O/tmp.json $v | tee -a $O/ab.jsonl
  done
done
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  WG_LPT_WIDE=$v timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 $ROOT/bench.py --workload c2 --no-cpu-baseline > $O/prof_bench_$v.json 2> $O/prof_$v.log || die prof_$v $?
  python3 $ROOT/tools/prof_window.py trace $(find $O/prof_$v -name "run_kernel_trace.csv" | head -1) $O/prof_bench_$v.json --out $O/window_$v.json > /dev/null || die window_$v $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'lpt_wide': int(sys.argv[2]), **{k: d.get(k) for k in ('window_span_per_step_us', 'kernel_busy_per_step_us', 'planning_busy_per_step_us', 'gap_per_step_us')}}))" $O/window_$v.json $v | tee -a $O/trace.jsonl
done
echo "[wide] done"
