# quick GPU check: parity tests, C1/C2 bench lines (used during development)
set -o pipefail
O=gpurun_out/${1:-q}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -2 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c1.json 2>$O/bench.err && cat $O/bench_c1.json &&
timeout -k 10 300 python bench.py --no-cpu-baseline --workload c2 > $O/bench_c2.json 2>>$O/bench.err && cat $O/bench_c2.json
