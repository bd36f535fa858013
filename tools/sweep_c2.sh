#!/bin/bash
# C2 (mixed 64..9000 B, 256 keys) bench per k_wave packets-per-wave setting and per kernel.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out/c2sweep
for P in 4 8 16 32 64; do
  WG_STREAM_PPW_MIXED=$P timeout -k 10 200 python bench.py --workload c2 --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/c2sweep/ppw_$P.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/c2sweep/ppw_$P.json')); print('C2 k_wave ppw=$P', d['value'], d['roofline']['seal_ms'], d['verified'])"
done
for KC in "coop 4 0" "coop 2 0" "lane 4 5" "stream 8 1"; do
  set -- $KC
  WG_TRANSPORT_KERNEL=$1 WG_LANE_K=$2 WG_LANE_VARIANT=$3 timeout -k 10 200 python bench.py --workload c2 --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/c2sweep/$1_$2.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/c2sweep/$1_$2.json')); print('C2 $KC', d['value'], d['roofline']['seal_ms'], d['verified'])"
done
