set -o pipefail
AB_TESTS=none AB_REPS=3 AB_WORKLOADS=c1 AB_BENCH_ARGS="--steps 1000" bash tools/ab_args.sh ab_prio3 "WG_PRIO=0" "WG_PRIO=1" "WG_PRIO=0 --variant 0"
