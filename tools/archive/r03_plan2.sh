set -o pipefail
mkdir -p gpurun_out/plan2
timeout -k 10 300 python -u -m pytest tests/test_gpu_duplex.py tests/test_gpu_configs.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/plan2/tests.log 2>&1 || { tail -30 gpurun_out/plan2/tests.log; exit 1; }
tail -1 gpurun_out/plan2/tests.log
for n in 65536 98304 131072 262144; do
  timeout -k 10 200 python bench.py --workload c2 --no-cpu-baseline --steps 200 --packets $n > gpurun_out/plan2/c2_$n.json 2>> gpurun_out/plan2/err.log || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/plan2/c2_$n.json')); print('c2 packets $n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['verified'])"
done
AB_TESTS=none AB_REPS=2 AB_WORKLOADS=c2 AB_BENCH_ARGS="--steps 200 --packets 131072" bash tools/ab_args.sh ab_prio131 "WG_PRIO=1" "WG_PRIO=0"
