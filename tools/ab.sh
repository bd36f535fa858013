#!/bin/bash
# Quick correctness + A/B pass on the GPU box: GPU tests, then C1 / C2 bench lines for the
# product kernel and the round-1 baseline. Usage: bash tools/ab.sh <tag> [tests-args]
set -eo pipefail
T=${1:-ab}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$T
mkdir -p $O
cd $ROOT
echo "[ab] tests"
timeout -k 10 900 python -u -m pytest ${2:-tests} -x -v --timeout 300 --timeout-method thread -m gpu > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
for k in default wave1; do
  for w in c1 c2; do
    echo "[ab] bench $w $k"
    timeout -k 10 300 python bench.py --workload $w --kernel $k --no-cpu-baseline > $O/bench_${w}_$k.json 2>> $O/bench.err
    cat $O/bench_${w}_$k.json
  done
done
echo "[ab] done"
