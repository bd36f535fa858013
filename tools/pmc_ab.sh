#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over short C1 bench runs, per transport
# kernel. Usage: bash tools/pmc_ab.sh <tag> "<kernel> ..." [workload]
set -eo pipefail
T=${1:-pmc}
KS=${2:-"default wave1"}
W=${3:-c1}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for k in $KS; do
  mkdir -p $O/$k
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    echo "[pmc] $k $grp"
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $O/$k/p$i -o run --output-format csv -- \
      python3 $ROOT/bench.py --workload $W --kernel $k --steps 20 --warmup 5 --ramp-ms 100 --no-cpu-baseline > $O/$k/p$i.log 2>&1
  done
done
echo "[pmc] done"
