#!/bin/bash
# Replay window: parity tests (four- and five-launch paths), then tools/bench_rx.py for both paths, twice, alternating.
set -o pipefail
out=gpurun_out/${1:-r04r}
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rx.py -m gpu > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
for k in 1 2; do
  for f in 3 5; do
    WG_RX_LAUNCHES=$f timeout -k 10 200 python tools/bench_rx.py >> $out/rx.jsonl 2>>$out/err || exit 1
  done
done
python3 - $out/rx.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    j=json.loads(l); print(j['rx_launches'], 'replay', j['replay_us'], 'filter+replay', j['filter+replay_us'], '1024 slots', j['replay_1024_slots_us'], j['replay_1024_slots_status_hist'][:2])
PY
