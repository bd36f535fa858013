#!/bin/bash
# Kernel trace of tools/bench_rx.py for both replay paths: per-kernel durations and the gaps between
# the kernels of one check (GPU-side launch cost).
set -o pipefail
out=gpurun_out/${1:-r04rp}
mkdir -p $out
for f in 3 5; do
  WG_RX_LAUNCHES=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/f$f -o run --output-format csv -- python3 tools/bench_rx.py > $out/f$f.log 2>&1 || { tail -20 $out/f$f.log; exit 1; }
  grep '^{' $out/f$f.log | tail -1
  python3 - $out/f$f <<'PY'
import csv, glob, sys, collections
tr = glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0]
rows = [r for r in csv.DictReader(open(tr)) if 'k_rp' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
dur = collections.defaultdict(list)
for r in rows:
    dur[r['Kernel_Name'].split('(')[0]].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
for k, v in dur.items():
    v.sort(); print(k, len(v), 'median ns', v[len(v)//2])
# calls: a k_rp_order starts a call; span = first start .. last end of the call
calls, cur = [], []
for r in rows:
    n = r['Kernel_Name']
    if ('k_rp_order' in n or 'k_rp_judge' in n) and cur:
        calls.append(cur); cur = []
    cur.append(r)
if cur: calls.append(cur)
spans = sorted(int(c[-1]['End_Timestamp']) - int(c[0]['Start_Timestamp']) for c in calls)
busy = sorted(sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in c) for c in calls)
print('calls', len(calls), 'median span ns', spans[len(spans)//2], 'median busy ns', busy[len(busy)//2])
PY
done
