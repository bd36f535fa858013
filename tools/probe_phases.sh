#!/bin/bash
# Per-wave phase timeline (diagnostic library) and PMC passes for the default
# transport kernel, seal only. Usage: bash tools/probe_phases.sh <tag>
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$1
mkdir -p $O
cd $ROOT
WG_LIB_PATH=$ROOT/wireguard-java_amd/libwgaead_diag.so timeout -k 10 120 python tools/wave_stamps.py > $O/stamps.txt 2>&1 || { cat $O/stamps.txt; exit 1; }
cat $O/stamps.txt
timeout -k 10 900 bash tools/pmc_cmp.sh $1 c1 || exit 1
python3 tools/pmc_table.py $1
