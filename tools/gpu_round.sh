#!/bin/bash
# One measurement round on the GPU box (run through gpurun from the repo root):
#   parity tests, smoke(), bench lines (C1 step with cpu_baseline, C1 serial, C2, C3, C4 host),
#   the UDP host pipeline, receive-side and per-packet timings, rocprofv3 kernel traces of the
#   C1 and C2 bench commands (tools/prof_window.py keeps the timed region only) and one PMC pass
#   per counter group for C1 and C2 (each pass its own run, as the MI355X guide prescribes).
# Usage: bash tools/gpu_round.sh r03 [bench|prof|all] (bench: everything up to the profiles; prof: the
# rocprofv3 traces and PMC passes; one gpurun call each fits the 600-s call limit)
set -o pipefail
R=${1:-r03}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$R
mkdir -p $O $O/pmc
cd $ROOT
PART=${2:-all}
step() { echo "[round] $1"; }
die() { echo "[round] FAILED: $1 (rc $2)"; exit $2; }
if [ "$PART" != prof ]; then
step "build on the box (every library the tests and the bench load comes from this tree's sources)"
timeout -k 10 400 python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || die build $?
md5sum wireguard-java_amd/libwgaead.so wireguard-java_amd/libwgaead_test.so oracle/liboracle.so > $O/build_md5.txt
git_head=$(cat .git_head 2>/dev/null || echo unknown); echo "head $git_head" >> $O/build_md5.txt
step tests
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || die tests $?
tail -1 $O/gpu_tests.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || die smoke $?
tail -1 $O/smoke.log
step "bench c1: the driver's command (--gpus 1 --steps 20 --warmup 5), three times"
for i in 1 2 3; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c1_driver$i.json 2>> $O/bench.err || die bench_c1_driver $?
done
cat $O/bench_c1_driver1.json
step "bench c1 (step, 200 steps)"
timeout -k 10 400 python bench.py > $O/bench_c1.json 2>> $O/bench.err || die bench_c1 $?
cat $O/bench_c1.json
timeout -k 10 400 python bench.py > $O/bench_c1b.json 2>> $O/bench.err || die bench_c1b $?
step "bench c1 under torchrun (RCCL group of one rank)"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 1 > $O/bench_c1_torchrun1.json 2>> $O/bench.err || die bench_c1_torchrun $?
step "bench c1 (serial)"
timeout -k 10 300 python bench.py --mode serial --no-cpu-baseline > $O/bench_c1_serial.json 2>> $O/bench.err || die bench_c1_serial $?
step "bench c1 (step as two launches)"
timeout -k 10 300 python bench.py --variant 1 --no-cpu-baseline > $O/bench_c1_step2.json 2>> $O/bench.err || die bench_c1_step2 $?
step "bench c2"
timeout -k 10 300 python bench.py --workload c2 > $O/bench_c2.json 2>> $O/bench.err || die bench_c2 $?
cat $O/bench_c2.json
step "bench imix"
timeout -k 10 300 python bench.py --workload imix > $O/bench_imix.json 2>> $O/bench.err || die bench_imix $?
cat $O/bench_imix.json
timeout -k 10 300 python bench.py --workload imix --graph --no-cpu-baseline > $O/bench_imix_graph.json 2>> $O/bench.err || die bench_imix_graph $?
cat $O/bench_imix_graph.json
step "bench c3"
timeout -k 10 400 python bench.py --workload c3 --no-cpu-baseline --steps 5 --warmup 1 > $O/bench_c3.json 2>> $O/bench.err || die bench_c3 $?
cat $O/bench_c3.json
step "host path c4"
timeout -k 10 300 python bench.py --workload c4 --steps 5 --warmup 1 > $O/bench_c4_pinned.json 2>> $O/bench.err || die c4 $?
WG_HOST_PATH=copy timeout -k 10 300 python bench.py --workload c4 --steps 5 --warmup 1 > $O/bench_c4_pinned_copy.json 2>> $O/bench.err || die c4copy $?
timeout -k 10 300 python bench.py --workload c4 --host-mem pageable --steps 3 --warmup 1 > $O/bench_c4_pageable.json 2>> $O/bench.err || die c4pageable $?
cat $O/bench_c4_*.json
step "host-to-host pipeline (UDP loopback)"
for k in 1 8; do
  timeout -k 10 200 ./tools/host_pipeline --backend gpu --packets 65536 --reps 5 --udp-streams $k --tun >> $O/host_pipeline_gpu.jsonl || die pipeline $?
done
timeout -k 10 300 ./tools/host_pipeline --backend cpu --oracle oracle/liboracle.so --threads 16 --packets 65536 --reps 3 --udp-streams 8 --tun >> $O/host_pipeline_cpu.jsonl || die pipeline_cpu $?
# pipelined: seal, UDP and open overlap in 16 chunks
timeout -k 10 200 ./tools/host_pipeline --backend gpu --packets 65536 --reps 5 --udp-streams 8 --chunks 16 >> $O/host_pipeline_gpu.jsonl || die pipeline_pipelined $?
timeout -k 10 300 ./tools/host_pipeline --backend cpu --oracle oracle/liboracle.so --threads 16 --packets 65536 --reps 3 --udp-streams 8 --chunks 16 >> $O/host_pipeline_cpu.jsonl || die pipeline_cpu_pipelined $?
step "receive side"
timeout -k 10 180 python tools/bench_rx.py > $O/rx_timing.json || die rx $?
cat $O/rx_timing.json
fi
[ "$PART" = bench ] && { step done; exit 0; }
cd /tmp && export TMPDIR=/tmp
# c1s: C1 with one stream per step (--streams 1): the launch the line's roofline (kernel_ms, frac, traffic)
# describes; c1: the default two-stream step (the line's value); c2: one stream by default
for w in c1s c1 c2 imix; do
  wl=${w%s}; xs=""; [ $w = c1s ] && xs="--streams 1"; [ $w = imix ] && wl=imix
  step "rocprofv3 kernel trace $w"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- python3 $ROOT/bench.py --workload $wl $xs --no-cpu-baseline > $O/prof_bench_$w.json 2> $O/prof_$w.log || die prof_$w $?
  python3 $ROOT/tools/prof_window.py trace $(find $O/prof_$w -name "run_kernel_trace.csv" | head -1) $O/prof_bench_$w.json --out $O/window_$w.json > /dev/null || die window_$w $?
  [ $w = c1 ] && continue  # counters: the one-stream launches (c1s) and C2
  i=0
  for grp in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    step "pmc $w $grp"
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d $O/pmc/${w}_p$i -o run --output-format csv -- python3 $ROOT/bench.py --workload $wl $xs --no-cpu-baseline --steps 20 --warmup 2 > $O/pmc/${w}_p$i.json 2> $O/pmc/${w}_p$i.log || die pmc_${w}_$i $?
  done
  args=""
  for j in 1 2 3 4; do args="$args $(find $O/pmc/${w}_p$j -name '*counter_collection.csv' | head -1) $O/pmc/${w}_p$j.json"; done
  python3 $ROOT/tools/prof_window.py pmc $args --out $O/pmc_$w.json > /dev/null || die pmc_window_$w $?
done
step done
