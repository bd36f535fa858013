#!/bin/bash
# One measurement round on the GPU box (run through gpurun from the repo root):
#   parity tests, smoke(), bench lines (C1 with cpu_baseline, C2, C3), the
#   rocprofv3 --kernel-trace --stats summary of the C1 bench command, and one PMC
#   pass per counter (FETCH_SIZE, WRITE_SIZE, VALU/wave counters) over the same command.
# Usage: bash tools/gpu_round.sh r01 [quick]
set -eo pipefail
R=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$R
mkdir -p $O $O/pmc
cd $ROOT
echo "[round] tests"; timeout -k 10 600 python -m pytest tests -x -q -m gpu > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
echo "[round] smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
echo "[round] bench c1"; timeout -k 10 400 python bench.py > $O/bench_c1.json 2> $O/bench.err
cat $O/bench_c1.json
echo "[round] bench c2"; timeout -k 10 300 python bench.py --workload c2 > $O/bench_c2.json 2>> $O/bench.err
cat $O/bench_c2.json
if [ "$2" != "quick" ]; then
  echo "[round] bench c3"; timeout -k 10 400 python bench.py --workload c3 --no-cpu-baseline --steps 5 --warmup 1 > $O/bench_c3.json 2>> $O/bench.err
  cat $O/bench_c3.json
fi
echo "[round] host path c4"
timeout -k 10 300 python bench.py --workload c4 --steps 5 --warmup 1 > $O/bench_c4_pinned.json 2>> $O/bench.err
cat $O/bench_c4_pinned.json
WG_HOST_PATH=copy timeout -k 10 300 python bench.py --workload c4 --steps 5 --warmup 1 > $O/bench_c4_pinned_copy.json 2>> $O/bench.err
cat $O/bench_c4_pinned_copy.json
timeout -k 10 300 python bench.py --workload c4 --host-mem pageable --steps 3 --warmup 1 > $O/bench_c4_pageable.json 2>> $O/bench.err
cat $O/bench_c4_pageable.json
echo "[round] host-to-host pipeline (UDP loopback)"
for k in 1 8; do
  timeout -k 10 200 ./tools/host_pipeline --backend gpu --packets 65536 --reps 5 --udp-streams $k --tun >> $O/host_pipeline_gpu.jsonl
done
timeout -k 10 300 ./tools/host_pipeline --backend cpu --oracle oracle/liboracle.so --threads 16 --packets 65536 --reps 3 --udp-streams 8 --tun >> $O/host_pipeline_cpu.jsonl
cat $O/host_pipeline_gpu.jsonl $O/host_pipeline_cpu.jsonl
echo "[round] receive-side checks"; timeout -k 10 120 python tools/bench_rx.py > $O/rx_timing.json; cat $O/rx_timing.json
echo "[round] per-packet batcher"
for t in 1 16 64; do timeout -k 10 120 ./tools/batcher_bench $t $((t == 1 ? 2000 : 160000 / t)) 1420 >> $O/batcher.jsonl; done
timeout -k 10 120 ./tools/batcher_bench 16 10000 0 >> $O/batcher.jsonl
cat $O/batcher.jsonl
cd /tmp && export TMPDIR=/tmp
echo "[round] rocprofv3 stats"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $ROOT/bench.py --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.log
i=0
for grp in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  echo "[round] pmc $grp"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d $O/pmc/p$i -o run --output-format csv -- python3 $ROOT/bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/pmc/p$i.log 2>&1
done
echo "[round] done"
