#!/bin/bash
# Round 6: k_lpt_one with one parallel LDS atomic per wave and pass: parity tests, the planner's duration
# (kernel trace, IMIX in a graph) for block shapes 0 and 4, bench lines.
set -o pipefail
T=${1:-r06w}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$T
mkdir -p $O
cd $ROOT
die() { echo "[lptw] FAILED: $1 (rc $2)"; exit $2; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_duplex.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; die tests $?; }
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
for v in 0 4; do
  WG_LPT_VARIANT=$v timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 $ROOT/bench.py --workload imix --graph --no-cpu-baseline > $O/prof_bench_$v.json 2> $O/prof_$v.log || die prof_$v $?
  python3 $ROOT/tools/prof_window.py trace $(find $O/prof_$v -name "run_kernel_trace.csv" | head -1) $O/prof_bench_$v.json --out $O/window_$v.json > /dev/null || die window_$v $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'lpt_variant': int(sys.argv[2]), **{k: d.get(k) for k in ('window_span_per_step_us', 'kernel_busy_per_step_us', 'planning_busy_per_step_us', 'gap_per_step_us')}}))" $O/window_$v.json $v | tee -a $O/trace.jsonl
done
cd $ROOT
for a in 1 2 3; do
  for g in "" "--graph"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --workload imix $g > $O/tmp.json 2>> $O/bench.err || die "bench $g" $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'graph': d['graph'], 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'verified': d['verified']}))" $O/tmp.json | tee -a $O/ab.jsonl
  done
done
echo "[lptw] done"
