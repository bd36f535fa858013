set -o pipefail
mkdir -p gpurun_out/plan
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/plan/tests.log 2>&1 || { tail -30 gpurun_out/plan/tests.log; exit 1; }
tail -1 gpurun_out/plan/tests.log
for n in 8192 16384 24576 32768 49152 65536 131072; do
  timeout -k 10 200 python bench.py --workload c2 --no-cpu-baseline --steps 300 --packets $n > gpurun_out/plan/c2_$n.json 2>> gpurun_out/plan/err.log || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/plan/c2_$n.json')); print('c2 packets $n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['verified'])"
done
for n in 8192 16384 32768 65536; do
  timeout -k 10 200 python bench.py --workload c1 --no-cpu-baseline --steps 500 --packets $n > gpurun_out/plan/c1_$n.json 2>> gpurun_out/plan/err.log || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/plan/c1_$n.json')); print('c1 packets $n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['verified'])"
done
