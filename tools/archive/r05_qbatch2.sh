set -o pipefail
O=gpurun_out/r05qb2; mkdir -p $O
for r in 1 2 3 4; do
  for cfg in "1 1" "1 2" "2 2"; do
    timeout -k 10 120 ./tools/queue_bench 16 100000 0 8192 $cfg fwd_batch=1 >> $O/mixed.jsonl || { echo "rc $?"; exit 1; }
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r05qb2/mixed.jsonl"):
    j = json.loads(l)
    print(j["forwarders"], j["verifiers"], j["seal_open_gib_s"], j["packets_per_s"], j["bad"], j["cpus_busy"], j["throttled_periods"])
PY
