set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05v
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
for w in "--workload imix --packets 32768" "--workload imix" "--workload c2" ""; do
  timeout -k 10 300 python bench.py $w --no-cpu-baseline > $O/b.json 2>> $O/bench.err || exit 1
  python3 -c "import json; d=json.load(open('$O/b.json')); print('$w', d['value'], d['verified'], d.get('oracle_sample',{}).get('bit_exact'))" | tee -a $O/bench_lines.txt
done
