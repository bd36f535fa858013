#!/bin/bash
# GPU probe (run through gpurun from the repo root): instruction-cost microbench,
# transport-kernel parity per variant, C1 bench per (seal variant, open variant,
# waves per workgroup), and per-wave timelines from the diagnostic library.
# Usage: bash tools/probe_variants.sh <tag> "Vs Vo G [p]" ...   (p: also run the parity subset)
set -o pipefail
TAG=${1:-probe}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$TAG
mkdir -p $O
cd $ROOT
echo "[probe] microbench6"
timeout -k 10 120 ./tools/microbench6 > $O/microbench6.txt 2>&1 || { echo "microbench6 failed"; exit 1; }
cat $O/microbench6.txt | tail -6
for cfg in "$@"; do
  set -- $cfg
  export WG_WAVE_VARIANT=$1 WG_WAVE_VARIANT_OPEN=$2 WG_WAVE_WPG=$3
  if [ "$4" = "p" ]; then
  echo "[probe] parity Vs=$1 Vo=$2 G=$3"
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "uniform_lengths or golden or mixed_sizes or unaligned or wire_format or out_of_range or max_packet or full_c1" \
    > $O/parity_$1_$2_$3.log 2>&1 || { echo "parity FAILED for $cfg"; tail -20 $O/parity_$1_$2_$3.log; exit 1; }
  tail -1 $O/parity_$1_$2_$3.log
  fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/bench_$1_$2_$3.json 2>> $O/bench.err \
    || { echo "bench FAILED for $cfg"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/bench_$1_$2_$3.json')); r=d['roofline']; print('C1 Vs=$1 Vo=$2 G=$3', d['value'], 'GiB/s seal_ms', r['seal_ms'], 'open_ms', r['open_ms'], 'frac', r['frac'], 'ok', d['verified'])"
done
unset WG_WAVE_VARIANT WG_WAVE_VARIANT_OPEN WG_WAVE_WPG
echo "[probe] done"
