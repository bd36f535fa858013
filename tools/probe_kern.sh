#!/bin/bash
# GPU probe: per transport-kernel configuration "KERNEL K V" (WG_TRANSPORT_KERNEL,
# WG_LANE_K, WG_LANE_VARIANT / WG_QUAD_VARIANT): full GPU parity, C1 and C3 bench,
# and the 16x-C1 launch time (tools/ablate.py).
# Usage: bash tools/probe_kern.sh <tag> "quad 4 0" "lane 2 5" ...
set -o pipefail
TAG=${1:-kern}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$TAG
mkdir -p $O
cd $ROOT
for cfg in "$@"; do
  set -- $cfg
  export WG_TRANSPORT_KERNEL=$1 WG_LANE_K=$2 WG_LANE_VARIANT=$3 WG_QUAD_VARIANT=$3 WG_WAVE_VARIANT=$3
  id=$1_$2_$3
  echo "[probe] $cfg"
  if [ "${4:-p}" = "p" ]; then
    timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
      > $O/parity_$id.log 2>&1 || { echo "parity FAILED for $cfg"; tail -30 $O/parity_$id.log; exit 1; }
    tail -1 $O/parity_$id.log
    for W in c1 c3; do
      timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 3 --workload $W > $O/bench_${W}_$id.json 2>> $O/bench.err \
        || { echo "bench FAILED for $cfg $W"; exit 1; }
      python3 -c "import json; d=json.load(open('$O/bench_${W}_$id.json')); r=d['roofline']; print('$W $id', d['value'], 'GiB/s seal_ms', r['seal_ms'], 'open_ms', r['open_ms'], 'ok', d['verified'])"
    done
  fi
  N=1048576 ABLATE=transport timeout -k 10 120 python tools/ablate.py 2>&1 | grep -v amdgpu | tr '\n' ' ' || exit 1
  echo
done
echo "[probe] done"
