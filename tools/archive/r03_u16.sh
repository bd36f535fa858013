set -o pipefail
WG_UNIFORM16=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_duplex.py tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/u16_tests.log 2>&1 || { tail -30 gpurun_out/u16_tests.log; exit 1; }
tail -1 gpurun_out/u16_tests.log
for n in 8192 16384 32768; do
AB_TESTS=none AB_REPS=2 AB_WORKLOADS=c1 AB_BENCH_ARGS="--steps 500 --packets $n" bash tools/ab_args.sh ab_u16_$n "WG_UNIFORM16=0" "WG_UNIFORM16=1"
done
