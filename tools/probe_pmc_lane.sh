#!/bin/bash
# PMC passes (tools/pmc_cmp.sh) for k_lane at the given K values, C1, then the table.
# Usage: bash tools/probe_pmc_lane.sh <tag> K...
set -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
for K in "$@"; do
  WG_TRANSPORT_KERNEL=lane WG_LANE_K=$K timeout -k 10 600 bash tools/pmc_cmp.sh ${TAG}_k$K c1 || { echo "pmc failed K=$K"; exit 1; }
  python3 tools/pmc_table.py ${TAG}_k$K
done
