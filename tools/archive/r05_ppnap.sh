#!/bin/bash
# Per-packet callers beyond the CPUs: the sleeping caller's futex timeout (WG_PP_NAP_US 2000 / 250),
# with the slowest call's stages (stamps=1)
set -o pipefail
O=gpurun_out/${1:-r05ppnap}; mkdir -p $O
for r in 1 2 3; do
  for nap in 2000 250; do
    for t in 64 128; do
      WG_PP_NAP_US=$nap timeout -k 10 120 ./tools/batcher_bench $t $((160000 / t)) 1420 stamps=1 | sed "s/^{/{\"nap_us\": $nap, /" >> $O/ab.jsonl || { echo "rc $?"; exit 1; }
    done
  done
done
python - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for l in open(O + "/ab.jsonl"):
    j = json.loads(l)
    s = j.get("slowest", {})
    print(j["nap_us"], j["threads"], j["payload_gib_s"], j["lat_us"]["p50"], j["lat_us"]["p999"], j["lat_us"]["max"], j["throttled_periods"],
          {k: s.get(k) for k in ("wait_us", "device_service_us", "slept", "involuntary_csw", "claim_us", "publish_us", "copy_out_us")})
PY
