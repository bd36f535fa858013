#!/bin/bash
# Round 6: k_lpt_one's per-key counters on separate 64-B lines (WG_CNT_STRIDE=16, product) against one line
# (ab_libs/s1, WG_CNT_STRIDE=1): parity tests, IMIX bench lines launched and in a graph, and a kernel trace
# of each graph run (the planner's own duration).
set -o pipefail
T=${1:-r06c}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$T
mkdir -p $O
cd $ROOT
die() { echo "[cnt] FAILED: $1 (rc $2)"; exit $2; }
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 600 $PYT tests/test_gpu_configs.py -k "two_lane or imix or random" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; die tests $?; }
tail -1 $O/tests.log
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  WG_LIB_PATH=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --workload imix "$@" > $O/tmp.json 2>> $O/bench.err || die "bench $name" $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'variant': sys.argv[2], 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['roofline']['kernel_ms'], 'verified': d['verified']}))" $O/tmp.json "$name" >> $O/ab.jsonl
  tail -1 $O/ab.jsonl
}
P=$ROOT/wireguard-java_amd/libwgaead.so
S=$ROOT/ab_libs/s1/libwgaead.so
for a in 1 2 3; do
  run stride16 $P
  run stride1 $S
  run stride16_graph $P --graph
  run stride1_graph $S --graph
done
cd /tmp && export TMPDIR=/tmp
for v in stride16:$P stride1:$S; do
  n=${v%%:*}; lib=${v#*:}
  WG_LIB_PATH=$lib timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o run --output-format csv -- python3 $ROOT/bench.py --workload imix --graph --no-cpu-baseline > $O/prof_bench_$n.json 2> $O/prof_$n.log || die prof_$n $?
  python3 $ROOT/tools/prof_window.py trace $(find $O/prof_$n -name "run_kernel_trace.csv" | head -1) $O/prof_bench_$n.json --out $O/window_$n.json > /dev/null || die window_$n $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k: d.get(k) for k in ('window_span_per_step_us', 'kernel_busy_per_step_us', 'planning_busy_per_step_us', 'gap_per_step_us')})" $O/window_$n.json $n
done
echo "[cnt] done"
