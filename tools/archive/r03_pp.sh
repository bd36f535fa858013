set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_duplex.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pp_tests.log 2>&1 || { tail -30 gpurun_out/pp_tests.log; exit 1; }
tail -1 gpurun_out/pp_tests.log
AB_TESTS=none AB_REPS=3 AB_WORKLOADS=c1 AB_BENCH_ARGS="--steps 1000" bash tools/ab_args.sh ab_phaseprio "WG_PHASE_PRIO=0" "WG_PHASE_PRIO=1"
