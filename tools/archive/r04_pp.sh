#!/bin/bash
# Per-packet server under oversubscription (64 / 128 callers on the box's 16-core share): callers that
# sleep on a futex woken by one waker thread (default) against callers that poll until their result
# lands (WG_PP_SPIN=1e9: the round-3 behaviour without the timed sleeps). Also records the box's CPU
# quota (cgroup cpu.max), which explains the ~70-90 ms tails of spinning callers.
set -o pipefail
O=gpurun_out/${1:-r04pp}
mkdir -p $O
{ echo "nproc $(nproc)"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/cpu.stat 2>/dev/null; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; } > $O/cpu_quota.txt
run() {  # label env...
  local label=$1; shift
  env "$@" timeout -k 10 120 ./tools/batcher_bench $T $((160000 / T)) 1420 | sed "s/^{/{\"policy\": \"$label\", /" >> $O/pp_load.jsonl || exit 1
}
for rep in 1 2; do
  for T in 1 16 64 128; do
    run adaptive WG_PP_SPIN=4096
    run spin_only WG_PP_SPIN=1000000000 WG_PP_SPIN_CALLERS=100000
    run sleep_early WG_PP_SPIN_CALLERS=4
  done
done
cat $O/cpu_quota.txt
python3 - $O/pp_load.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    j = json.loads(l)
    print(j["policy"], j["threads"], j["payload_gib_s"], j["lat_us"])
PY
