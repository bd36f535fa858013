set -o pipefail
AB_TESTS=none AB_REPS=2 AB_WORKLOADS=c2 AB_BENCH_ARGS="--steps 400" bash tools/ab_args.sh ab_c2diag "--packets 65536" "--packets 16384" "--keys 1" "--packets 262144"
AB_TESTS=none AB_REPS=2 AB_WORKLOADS=c1 AB_BENCH_ARGS="--steps 1000" bash tools/ab_args.sh ab_c1diag "--packets 65536" "--keys 256" "--packets 16384" "--packets 262144"
