#!/bin/bash
# Round 6: the driver's 20-step command with and without the staggered two-stream schedule, alternating, and
# kernel traces of a staggered 20-step C1 run and of the IMIX step. Usage: bash tools/r06_stagger.sh <tag> [alternations]
set -o pipefail
T=${1:-r06h}
ALT=${2:-6}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$T
mkdir -p $O
cd $ROOT
die() { echo "[stagger] FAILED: $1 (rc $2)"; exit $2; }
line() {
  python3 - "$1" $O/tmp.json >> $O/ab.jsonl <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
print(json.dumps({"variant": sys.argv[1], "value": d["value"], "ms_per_step": d["ms_per_step"],
                  "step_ms": d["roofline"]["step"]["ms"], "kernel_ms": d["roofline"]["kernel_ms"],
                  "verified": d["verified"], "stagger": d.get("stagger")}))
PY
  tail -1 $O/ab.jsonl
}
for a in $(seq 1 $ALT); do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/tmp.json 2>> $O/err.log || die stagger $?
  line stagger20
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --stagger 0 > $O/tmp.json 2>> $O/err.log || die nostagger $?
  line nostagger20
done
for a in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline > $O/tmp.json 2>> $O/err.log || die stagger200 $?
  line stagger200
  timeout -k 10 120 python bench.py --no-cpu-baseline --stagger 0 > $O/tmp.json 2>> $O/err.log || die nostagger200 $?
  line nostagger200
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr20 -o run --output-format csv -- python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/tr20.json 2> $O/tr20.log || die trace20 $?
python3 $ROOT/tools/stream_phase.py $(find $O/tr20 -name "run_kernel_trace.csv" | head -1) $O/tr20.json --out $O/phase_20.json || die phase20 $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trimix -o run --output-format csv -- python3 $ROOT/bench.py --workload imix --no-cpu-baseline > $O/trimix.json 2> $O/trimix.log || die traceimix $?
python3 $ROOT/tools/prof_window.py trace $(find $O/trimix -name "run_kernel_trace.csv" | head -1) $O/trimix.json --out $O/window_imix.json || die windowimix $?
python3 $ROOT/tools/trace_gaps.py $(find $O/trimix -name "run_kernel_trace.csv" | head -1) > $O/imix_gaps.txt || die gaps $?; cat $O/imix_gaps.txt
echo "[stagger] done"
