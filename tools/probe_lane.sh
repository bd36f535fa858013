#!/bin/bash
# GPU probe (run through gpurun from the repo root): k_lane parity (full GPU parity
# suite) and the C1/C3 bench per (K lanes per packet, variant bits), against the default.
# Usage: bash tools/probe_lane.sh <tag> "K V" ...
set -o pipefail
TAG=${1:-lane}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$TAG
mkdir -p $O
cd $ROOT
echo "[probe] default kernel C1"
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/bench_default.json 2>> $O/bench.err \
  || { echo "bench FAILED (default)"; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default.json')); r=d['roofline']; print('C1 default', d['value'], 'GiB/s seal_ms', r['seal_ms'], 'open_ms', r['open_ms'], 'ok', d['verified'])"
for cfg in "$@"; do
  set -- $cfg
  export WG_TRANSPORT_KERNEL=lane WG_LANE_K=$1 WG_LANE_VARIANT=$2
  echo "[probe] parity K=$1 V=$2"
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    > $O/parity_$1_$2.log 2>&1 || { echo "parity FAILED for K=$1 V=$2"; tail -30 $O/parity_$1_$2.log; exit 1; }
  tail -1 $O/parity_$1_$2.log
  for W in c1 c3; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 3 --workload $W > $O/bench_${W}_$1_$2.json 2>> $O/bench.err \
      || { echo "bench FAILED for K=$1 V=$2 $W"; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${W}_$1_$2.json')); r=d['roofline']; print('$W K=$1 V=$2', d['value'], 'GiB/s seal_ms', r['seal_ms'], 'open_ms', r['open_ms'], 'ok', d['verified'])"
  done
done
unset WG_TRANSPORT_KERNEL WG_LANE_K WG_LANE_VARIANT
echo "[probe] done"
