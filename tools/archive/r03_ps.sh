set -o pipefail
AB_TESTS=none AB_REPS=2 AB_WORKLOADS=c2 AB_BENCH_ARGS="--steps 300" bash tools/ab_args.sh ab_ps65 "WG_MIXED_PER_SLOT=0" "WG_MIXED_PER_SLOT=4" "WG_MIXED_PER_SLOT=6"
