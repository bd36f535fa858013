#!/bin/bash
# Host-to-host pipeline (BASELINE configs[4]): stages in turn against pipelined chunks, GPU and CPU
# backends, 8 UDP streams, alternating on one box
set -o pipefail
O=gpurun_out/${1:-r05pipe}; mkdir -p $O
for r in 1 2; do
  for ch in 1 8 16; do
    timeout -k 10 200 ./tools/host_pipeline --backend gpu --packets 65536 --reps 5 --udp-streams 8 --chunks $ch >> $O/gpu.jsonl || { echo "gpu rc $?"; exit 1; }
    timeout -k 10 300 ./tools/host_pipeline --backend cpu --oracle oracle/liboracle.so --threads 16 --packets 65536 --reps 3 --udp-streams 8 --chunks $ch >> $O/cpu.jsonl || { echo "cpu rc $?"; exit 1; }
  done
done
python3 - "$O" <<'PY'
import json, sys
for f in ("gpu", "cpu"):
    for l in open(f"{sys.argv[1]}/{f}.jsonl"):
        j = json.loads(l)
        print(f, j["chunks"], j["seal_gib_s"], j["open_gib_s"], j["end_to_end_gib_s"], j["delivered"], j["dropped"], j["bad_tag"], j["mismatched"])
PY
