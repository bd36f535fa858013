#!/bin/bash
# Round-4 final: whole -m gpu suite, smoke(), the bench lines (c1 twice, c2, c3).
set -o pipefail
out=gpurun_out/${1:-r04end}
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
for w in c1 c2 c3 c1b; do
  wl=${w%b}; extra=""; [ $wl = c3 ] && extra="--steps 5 --warmup 1"
  timeout -k 10 300 python bench.py --workload $wl $extra > $out/$w.json 2>>$out/err || exit 1
  python3 -c "
import json; j=json.loads(open('$out/$w.json').read().strip().splitlines()[-1]); r=j['roofline']
print('$w', j['value'], j['ms_per_step'], r['frac'], r['step']['frac'], r.get('traffic'), j['verified'], j['oracle_sample']['bit_exact'], j['cpu_baseline']['value'])"
done
