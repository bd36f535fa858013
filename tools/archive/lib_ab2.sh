#!/bin/bash
# Alternating A/B of libwgaead builds (WG_LIB_PATH): parity subset once per build, then
# C1 and C2 bench lines in A B A B order. Usage: bash tools/lib_ab2.sh <tag> lib1.so lib2.so ...
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
T=$1; shift
O=$ROOT/gpurun_out/$T
mkdir -p $O
cd $ROOT
for lib in "$@"; do
  WG_LIB_PATH=$ROOT/wireguard-java_amd/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_duplex.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/${lib}_tests.log 2>&1 || { echo "$lib tests failed"; tail -30 $O/${lib}_tests.log; exit 1; }
  echo "$lib $(tail -1 $O/${lib}_tests.log)"
done
for r in 1 2; do for lib in "$@"; do for w in ${AB_WORKLOADS:-c1 c2}; do
  WG_LIB_PATH=$ROOT/wireguard-java_amd/$lib timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline $AB_ARGS > $O/${lib}_${w}_$r.json 2>> $O/err.log || { echo "$lib $w bench failed"; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${lib}_${w}_$r.json')); print('$lib $w $r', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['verified'])"
done; done; done
