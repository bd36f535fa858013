#!/bin/bash
# SQ_INSTS_VALU and C1 time for several libwgaead builds (ablation builds included: no
# correctness gate). Usage: bash tools/valu_ab.sh <tag> lib1.so [lib2.so ...]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
T=$1; shift
O=$ROOT/gpurun_out/$T
mkdir -p $O
for lib in "$@"; do
  L=$ROOT/wireguard-java_amd/$lib
  WG_LIB_PATH=$L timeout -k 10 300 python $ROOT/bench.py --no-cpu-baseline --steps 100 > $O/${lib}_c1.json 2>> $O/err.log
  python3 -c "import json; d=json.load(open('$O/${lib}_c1.json')); print('$lib c1', d['value'], d['roofline']['seal_ms'], d['roofline']['open_ms'], d['verified'])"
  mkdir -p $O/pmc_$lib
  (cd /tmp && TMPDIR=/tmp WG_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_$lib/p1 -o run --output-format csv -- python3 $ROOT/bench.py --steps 20 --warmup 5 --ramp-ms 100 --no-cpu-baseline > $O/pmc_$lib/p1.log 2>&1) || echo "pmc $lib failed"
done
echo "[valu] done"
