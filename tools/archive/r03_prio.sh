set -o pipefail
AB_TESTS=none AB_REPS=3 AB_WORKLOADS=c1 AB_BENCH_ARGS="--steps 1000" bash tools/ab_args.sh ab_host "WG_PRIO=0" "WG_PRIO=0 --variant 0"
for f in gpurun_out/ab_host/v*_c1_*.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'])"; done
