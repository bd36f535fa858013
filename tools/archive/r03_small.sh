set -o pipefail
AB_TESTS=none AB_REPS=2 AB_WORKLOADS=c2 AB_BENCH_ARGS="--steps 400 --packets 16384" bash tools/ab_args.sh ab_small "WG_MIXED_SPLIT=0" "WG_SLOT16=1" "WG_MIXED_SPLIT=4" "WG_MIXED_SPLIT=1"
AB_TESTS=none AB_REPS=1 AB_WORKLOADS=c2 AB_BENCH_ARGS="--steps 400 --packets 32768" bash tools/ab_args.sh ab_small32 "WG_MIXED_SPLIT=0" "WG_SLOT16=1" "WG_MIXED_SPLIT=4" "WG_MIXED_SPLIT=1"
