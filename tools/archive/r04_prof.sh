#!/bin/bash
# Round-4 profiles (run through gpurun from the repo root): rocprofv3 kernel traces of the bench's timed
# window for C1 and C3 with the timed steps replayed from one HIP graph (bench.py --graph: no host enqueue
# between the traced launches), and one PMC pass per counter group for C1 and C3 (FETCH_SIZE,
# WRITE_SIZE, SQ_WAVES + SQ_INSTS_VALU + SQ_WAVE_CYCLES + SQ_BUSY_CYCLES, SQ_WAIT_INST_ANY +
# SQ_ACTIVE_INST_VALU + SQ_INSTS_LDS + GRBM_GUI_ACTIVE), each pass its own run (MI355X guide).
# Usage: bash tools/r04_prof.sh r04 [c1 c3 ...]
set -o pipefail
R=${1:-r04}
shift
WS=${@:-c1 c3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$R
mkdir -p $O/pmc
step() { echo "[prof] $1 $(date +%T)"; }
die() { echo "[prof] FAILED: $1 (rc $2)"; exit $2; }
cd /tmp && export TMPDIR=/tmp
for w in $WS; do
  args="--workload $w --no-cpu-baseline --graph"
  [ $w = c3 ] && args="$args --steps 5 --warmup 1"
  step "kernel trace $w"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- python3 $ROOT/bench.py $args > $O/prof_bench_$w.json 2> $O/prof_$w.log || die prof_$w $?
  python3 $ROOT/tools/prof_window.py trace $(find $O/prof_$w -name "run_kernel_trace.csv" | head -1) $O/prof_bench_$w.json --out $O/window_$w.json > /dev/null || die window_$w $?
  cat $O/window_$w.json | head -30
  i=0
  pargs="--workload $w --no-cpu-baseline --graph --steps 20 --warmup 2"
  [ $w = c3 ] && pargs="--workload $w --no-cpu-baseline --graph --steps 3 --warmup 1"
  for grp in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    step "pmc $w $grp"
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d $O/pmc/${w}_p$i -o run --output-format csv -- python3 $ROOT/bench.py $pargs > $O/pmc/${w}_p$i.json 2> $O/pmc/${w}_p$i.log || die pmc_${w}_$i $?
  done
  pa=""
  for j in 1 2 3 4; do pa="$pa $(find $O/pmc/${w}_p$j -name '*counter_collection.csv' | head -1) $O/pmc/${w}_p$j.json"; done
  python3 $ROOT/tools/prof_window.py pmc $pa --out $O/pmc_$w.json > /dev/null || die pmc_window_$w $?
  head -c 1500 $O/pmc_$w.json
done
step done
