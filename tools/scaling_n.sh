#!/bin/bash
# Transport launch time vs batch size (1420-B packets): separates the fixed per-launch
# cost from the per-packet cost. Usage: bash tools/scaling_n.sh > gpurun_out/scaling_n.txt
for n in 2048 8192 16384 32768 65536 131072 262144 524288 1048576; do
  echo "N=$n"
  N=$n ABLATE=transport timeout -k 10 120 python tools/ablate.py 2>&1 | grep -v amdgpu
done
