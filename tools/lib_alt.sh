#!/bin/bash
# Alternating A/B of libwgaead builds on one box (WG_LIB_PATH): the C1 and C2 parity tests of each
# build, then R rounds of bench C1 and C2 per build in turn.
# Usage: bash tools/lib_alt.sh <tag> <rounds> lib1.so [lib2.so ...]   (paths relative to the repo root)
set -o pipefail
O=gpurun_out/$1; R=$2; shift 2; mkdir -p $O
for lib in "$@"; do
  WG_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread -m gpu -k "c1 or c2" > $O/tests_$(echo $lib | tr / _).log 2>&1 || { echo "tests $lib"; tail -20 $O/tests_$(echo $lib | tr / _).log; exit 1; }
done
for r in $(seq $R); do
  for lib in "$@"; do
    for w in c1 c2; do
      WG_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 100 --warmup 10 | sed "s|^{|{\"lib\": \"$lib\", |" >> $O/ab.jsonl || { echo "bench rc $?"; exit 1; }
    done
  done
done
python3 - $O <<'PY'
import json, sys
for l in open(sys.argv[1] + "/ab.jsonl"):
    j = json.loads(l)
    print(j["lib"], j["config"]["workload"][:2], j["value"], j["roofline"]["kernel_ms"], j["roofline"]["frac"], j["verified"])
PY
