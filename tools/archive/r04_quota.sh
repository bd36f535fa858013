#!/bin/bash
# Is the ~70-90 ms tail of 64 / 128 per-packet callers CPU-quota throttling? cpu.stat before and after
# one run of each (the box: cpu.max 1600000 100000 = 16 CPUs of quota, affinity over all 256 CPUs).
O=gpurun_out/${1:-r04q}
mkdir -p $O
for T in 64 128; do
  for pol in "WG_PP_SPIN=1000000000 WG_PP_SPIN_CALLERS=100000" "WG_PP_SPIN_CALLERS=32"; do
    echo "== T=$T $pol" >> $O/quota.txt
    grep -E "nr_throttled|throttled_usec|usage_usec" /sys/fs/cgroup/cpu.stat >> $O/quota.txt
    env $pol timeout -k 10 120 ./tools/batcher_bench $T $((160000 / T)) 1420 >> $O/quota.txt || exit 1
    grep -E "nr_throttled|throttled_usec|usage_usec" /sys/fs/cgroup/cpu.stat >> $O/quota.txt
  done
done
cut -c1-300 $O/quota.txt
