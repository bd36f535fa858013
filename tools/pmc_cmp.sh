#!/bin/bash
# PMC passes over `bench.py --steps 5` for one configuration (env set by the caller).
# Usage: bash tools/pmc_cmp.sh <outdir under gpurun_out> [workload]
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$1
W=${2:-c1}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_INSTS_LDS" "SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d $O/p$i -o run --output-format csv -- python3 $ROOT/bench.py --no-cpu-baseline --steps 5 --warmup 1 --workload $W > $O/p$i.log 2>&1
done
