#!/bin/bash
# C1/C2 bench (no verification gate, no CPU baseline) for several libwgaead builds; timing studies
# and ablation builds whose output is deliberately wrong. Usage: bash tools/time_libs.sh <tag> lib1.so ...
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
T=$1; shift
O=$ROOT/gpurun_out/$T
mkdir -p $O
cd $ROOT
W=${WORKLOADS:-c1}
for rep in 1 2; do
for lib in "$@"; do
  for w in $W; do
    WG_LIB_PATH=$ROOT/wireguard-java_amd/$lib timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 100 > $O/${lib}_${w}_$rep.json 2>> $O/err.log || true
    python3 -c "import json; d=json.load(open('$O/${lib}_${w}_$rep.json')); print('$lib $w $rep', d['value'], d['roofline']['kernel_ms'], d['roofline']['seal_ms'], d['roofline']['open_ms'], d['verified'])"
  done
done
done
