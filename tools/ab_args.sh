#!/bin/bash
# Alternating A/B of bench.py argument sets on one box: the GPU tests named by AB_TESTS once
# (default: duplex + parity), then C1 and C2 (AB_WORKLOADS) bench lines, AB_REPS (2) rounds over the
# sets, the order rotated every round.
# Usage: bash tools/ab_args.sh <tag> "<args A>" "<args B>" ...  (words NAME=value in a set are
# environment settings for that set, e.g. "WG_SLOT16=0 --variant 1")
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
T=$1; shift
O=$ROOT/gpurun_out/$T
mkdir -p $O
cd $ROOT
if [ "${AB_TESTS:-x}" != none ]; then
  timeout -k 10 400 python -u -m pytest ${AB_TESTS:-tests/test_gpu_duplex.py tests/test_gpu_parity.py} -x -q -m gpu \
    --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
N=$#
for r in $(seq 1 ${AB_REPS:-2}); do
  # rotate the order every rep, so no set always runs first (or after the same set)
  for k in $(seq 0 $((N - 1))); do
    i=$(( (k + r - 1) % N + 1 ))
    a=${!i}
    for w in ${AB_WORKLOADS:-c1 c2}; do
      envs=""; args=""
      for x in $a; do case $x in --*) args="$args $x";; *=*) envs="$envs $x";; *) args="$args $x";; esac; done
      env $envs timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline $AB_BENCH_ARGS $args > $O/v${i}_${w}_$r.json 2>> $O/err.log || { echo "[$a] $w bench failed"; tail -5 $O/err.log; exit 1; }
      python3 -c "import json; d=json.load(open('$O/v${i}_${w}_$r.json')); print('[$a] $w $r', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['verified'])"
    done
  done
done
