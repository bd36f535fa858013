# A/B of the dependent seal -> open step on C1 and C2: WG_F_AFTER_SEAL step vs two serial launches
set -o pipefail
O=gpurun_out/${1:-ab}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_duplex.py tests/test_gpu_rx.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; rc=$?; tail -3 $O/t.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do for m in step serial; do for w in c1 c2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --mode $m --workload $w > $O/${m}_${w}_$r.json || exit 1
  python -c "import json;d=json.load(open('$O/${m}_${w}_$r.json'));print('$m $w', d['value'], d['roofline']['frac'], d['verified'])"
done; done; done
timeout -k 10 100 python tools/bench_rx.py > $O/rx.json && cat $O/rx.json
