#!/bin/bash
# Round 6 GPU pass: the whole GPU suite on the product library, the stitched-Horner kernels (WG_STITCH=1) and
# the 5-mad-chain Poly1305 build through the configuration tests, then alternating A/B bench lines.
# Usage: bash tools/ab_r06.sh <tag> [tests|ab|all] [alternations]
set -o pipefail
T=${1:-r06b}
PART=${2:-all}
ALT=${3:-2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$T
mkdir -p $O
cd $ROOT
die() { echo "[ab] FAILED: $1 (rc $2)"; exit $2; }
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
if [ "$PART" != ab ]; then
  echo "[ab] GPU suite (product library), the bench tests first"
  timeout -k 10 900 $PYT tests/test_gpu_bench.py tests > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; die tests $?; }
  tail -1 $O/gpu_tests.log
  echo "[ab] stitched kernels through the configuration and step tests"
  WG_STITCH=1 timeout -k 10 600 $PYT tests/test_gpu_configs.py tests/test_gpu_duplex.py tests/test_gpu_bench.py > $O/st_tests.log 2>&1 || { tail -30 $O/st_tests.log; die st_tests $?; }
  tail -1 $O/st_tests.log
  for v in $(ls ab_libs 2>/dev/null); do
    echo "[ab] $v library through the parity and configuration tests"
    WG_LIB_PATH=$ROOT/ab_libs/$v/libwgaead.so timeout -k 10 600 $PYT tests/test_gpu_parity.py tests/test_gpu_configs.py > $O/${v}_tests.log 2>&1 || { tail -30 $O/${v}_tests.log; die ${v}_tests $?; }
    tail -1 $O/${v}_tests.log
  done
fi
[ "$PART" = tests ] && exit 0
run() {  # name env... -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/tmp.json 2>> $O/bench.err || die "bench $name $*" $?
  python3 - "$name" "$*" $O/tmp.json >> $O/ab.jsonl <<'EOF'
import json, sys
d = json.load(open(sys.argv[3]))
print(json.dumps({"variant": sys.argv[1], "args": sys.argv[2], "value": d["value"], "ms_per_step": d["ms_per_step"],
                  "kernel_ms": d["roofline"]["kernel_ms"], "step_ms": d["roofline"]["step"]["ms"],
                  "frac": d["roofline"]["frac"], "verified": d["verified"], "stagger": d.get("stagger")}))
EOF
  tail -1 $O/ab.jsonl
}
for a in $(seq 1 $ALT); do
  for w in "--workload c1 --streams 1" "--workload c1" "--workload c2" "--workload imix"; do
    run base -- $w
    run st5 WG_STITCH=1 -- $w
    [ "$w" = "--workload imix" ] && run base_lpt2 WG_LPT_ONE=0 -- $w
    for v in $(ls ab_libs 2>/dev/null); do
      run $v WG_LIB_PATH=$ROOT/ab_libs/$v/libwgaead.so WG_STITCH=$([ $v = st6 ] && echo 1 || echo 0) -- $w
    done
  done
  run base20 -- --steps 20 --warmup 5
  run base20_nostagger -- --steps 20 --warmup 5 --stagger 0
done
echo "[ab] done"
