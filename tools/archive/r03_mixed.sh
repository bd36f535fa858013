set -o pipefail
mkdir -p gpurun_out/mixed
WG_MIXED_SPLIT=9 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_duplex.py tests/test_gpu_configs.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/mixed/tests.log 2>&1 || { tail -30 gpurun_out/mixed/tests.log; exit 1; }
tail -1 gpurun_out/mixed/tests.log
AB_TESTS=none AB_REPS=2 AB_WORKLOADS=c2 AB_BENCH_ARGS="--steps 400" bash tools/ab_args.sh ab_mixed "WG_MIXED_SPLIT=0" "WG_MIXED_SPLIT=9" "WG_MIXED_SPLIT=6" "WG_MIXED_SPLIT=12"
