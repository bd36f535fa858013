# per-packet server: waves exit on their own idle time (old, wireguard-java_amd/ppold) vs only when
# no wave has served for idle_us (new; spin1k: callers sleep after 1,024 checks instead of 4,096),
# alternating on one box; callers 16 / 64 / 128
# (wireguard-java_amd/ppold/libwgaead.so: the csrc tree with the variant under test swapped back, built by hand with
# the Makefile's hipcc line; without it both slots load the product library, i.e. a control run)
set -o pipefail
mkdir -p gpurun_out/ppidle
timeout -k 10 300 python -u -m pytest tests/test_batcher.py -x -q -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/ppidle/tests.log 2>&1 || { tail -30 gpurun_out/ppidle/tests.log; exit 1; }
tail -1 gpurun_out/ppidle/tests.log
for r in $(seq 1 ${PP_REPS:-3}); do
  for v in ${PP_SETS:-old new}; do
    for t in 16 64 128; do
      if [ $v = old ]; then export LD_LIBRARY_PATH=$PWD/wireguard-java_amd/ppold; else unset LD_LIBRARY_PATH; fi
      if [ $v = spin1k ]; then export WG_PP_SPIN=1024; else unset WG_PP_SPIN; fi
      timeout -k 5 90 ./tools/batcher_bench $t $((160000 / t)) 1420 > gpurun_out/ppidle/one.json || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/ppidle/one.json')); print('$v', $t, $r, d['payload_gib_s'], d['lat_us']['p50'], d['lat_us']['p99'], d['lat_us']['p999'], d['lat_us']['max'], d['launches'])" | tee -a gpurun_out/ppidle/ab.txt
    done
  done
done
