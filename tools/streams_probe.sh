set -o pipefail
for S in 1 2 4; do
  for KCFG in "wave 1 5" "coop 2 0" "coop 1 0"; do
    set -- $KCFG
    WG_TRANSPORT_KERNEL=$1 WG_LANE_K=$2 WG_LANE_VARIANT=$3 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 5 --streams $S > gpurun_out/streams_$1_$2_$S.json 2>/dev/null || { echo fail; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/streams_$1_$2_$S.json')); print('streams=$S $KCFG', d['value'], d['verified'])"
  done
done
