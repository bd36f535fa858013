#!/bin/bash
# k_lane timing ablations (tools/ablate.py, seal/open µs per launch): full, no payload
# memory traffic (V&8), no Poly1305 (V&16), neither; C1-size and 16x batches.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out/ablate_lane
for N in 65536 1048576; do
  for V in 5 13 21 29; do
    echo "N=$N K=2 V=$V"
    N=$N ABLATE=transport WG_TRANSPORT_KERNEL=lane WG_LANE_K=2 WG_LANE_VARIANT=$V timeout -k 10 120 python tools/ablate.py 2>&1 | grep -v amdgpu || exit 1
  done
  echo "N=$N k_wave default"
  N=$N ABLATE=transport timeout -k 10 120 python tools/ablate.py 2>&1 | grep -v amdgpu || exit 1
done
timeout -k 10 120 ./tools/microbench7 || exit 1
