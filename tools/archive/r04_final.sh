#!/bin/bash
# Round-4 end check: the whole -m gpu suite, smoke(), then the queue harness.
set -o pipefail
out=gpurun_out/${1:-r04fin}
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
tools/r04_queue.sh $1_q
