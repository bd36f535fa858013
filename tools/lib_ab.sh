#!/bin/bash
# Correctness + C1/C2 bench + VALU count for alternative libwgaead builds (WG_LIB_PATH).
# Usage: bash tools/lib_ab.sh <tag> lib1.so [lib2.so ...]   (paths relative to wireguard-java_amd/)
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
T=$1; shift
O=$ROOT/gpurun_out/$T
mkdir -p $O
cd $ROOT
for lib in "$@"; do
  L=$ROOT/wireguard-java_amd/$lib
  echo "[lib] $lib tests"
  WG_LIB_PATH=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_framing.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/${lib}_tests.log 2>&1 || { tail -30 $O/${lib}_tests.log; exit 1; }
  tail -1 $O/${lib}_tests.log
  for w in c1 c2; do
    WG_LIB_PATH=$L timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > $O/${lib}_$w.json 2>> $O/err.log
    python3 -c "import json; d=json.load(open('$O/${lib}_$w.json')); print('$lib $w', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['verified'])"
  done
  mkdir -p $O/pmc_$lib
  cd /tmp && export TMPDIR=/tmp
  WG_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_$lib/p1 -o run --output-format csv -- python3 $ROOT/bench.py --steps 20 --warmup 5 --ramp-ms 100 --no-cpu-baseline > $O/pmc_$lib/p1.log 2>&1
  cd $ROOT
done
echo "[lib] done"
