#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over tools/ablate.py; outputs under gpurun_out/pmc/
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ablate.py > $OUT/p$i.log 2>&1
done
