#!/bin/bash
# Round 6: the step launch that plans its own short-packet order (k_step_mixed_fused, WG_LPT_FUSED) through the
# configuration / step / bench tests, then IMIX and C2 bench lines alternating fused and WG_LPT_FUSED=0.
# Usage: bash tools/r06_fused.sh <tag> [alternations]
set -o pipefail
T=${1:-r06f}
ALT=${2:-3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$T
mkdir -p $O
cd $ROOT
die() { echo "[fused] FAILED: $1 (rc $2)"; exit $2; }
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 600 $PYT tests/test_gpu_configs.py tests/test_gpu_duplex.py tests/test_gpu_bench.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; die tests $?; }
tail -1 $O/tests.log
for a in $(seq 1 $ALT); do
  for w in ${WL:-imix c2}; do
    for f in 1 0; do
      WG_LPT_FUSED=$f timeout -k 10 300 python bench.py --no-cpu-baseline --workload $w > $O/tmp.json 2>> $O/bench.err || die "bench $w $f" $?
      python3 - "$w" "$f" $O/tmp.json >> $O/ab.jsonl <<'PY'
import json, sys
d = json.load(open(sys.argv[3]))
print(json.dumps({"workload": sys.argv[1], "fused": int(sys.argv[2]), "value": d["value"], "ms_per_step": d["ms_per_step"],
                  "kernel_ms": d["roofline"]["kernel_ms"], "step_ms": d["roofline"]["step"]["ms"], "verified": d["verified"]}))
PY
      tail -1 $O/ab.jsonl
    done
  done
done
echo "[fused] done"
