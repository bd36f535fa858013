set -o pipefail
mkdir -p gpurun_out/ppab
for r in 1 2 3; do
  for v in keyfirst mailbox; do
    for t in 16 64; do
      if [ $v = keyfirst ]; then export LD_LIBRARY_PATH=$PWD/wireguard-java_amd/kf; else unset LD_LIBRARY_PATH; fi
      timeout -k 5 60 ./tools/batcher_bench $t $((80000 / t)) 1420 > gpurun_out/ppab/one.json || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/ppab/one.json')); print('$v', $t, $r, d['payload_gib_s'], d['lat_us']['p50'], d['lat_us']['p99'], d['lat_us']['p999'], d['launches'])"
    done
  done
done
