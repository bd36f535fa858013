set -o pipefail
mkdir -p gpurun_out/vf
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/vf/tests.log 2>&1 || { tail -30 gpurun_out/vf/tests.log; exit 1; }
tail -1 gpurun_out/vf/tests.log
AB_TESTS=none AB_REPS=2 AB_BENCH_ARGS="--steps 600" bash tools/ab_args.sh ab_vf "WG_LIB_PATH=$PWD/wireguard-java_amd/libwgaead_prev.so" "WG_PRIO=-1"
