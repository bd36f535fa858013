#!/bin/bash
# The IMIX-like mix of SURVEY.md §8d on the GPU box (run through gpurun from the repo root): its parity
# test, bench lines (default plan, and two streams), the timed region's kernel trace and one PMC pass
# per counter group (tools/prof_window.py keeps the timed window; pmc_<R>_imix.json feeds the line's
# roofline.traffic).
# Usage: bash tools/imix_round.sh r05k
set -o pipefail
R=${1:-r05k}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$R
mkdir -p $O/pmc
cd $ROOT
step() { echo "[imix] $1"; }
die() { echo "[imix] FAILED: $1 (rc $2)"; exit $2; }
step test
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -v -m gpu -k imix --timeout 120 --timeout-method thread > $O/imix_test.log 2>&1 || die test $?
tail -1 $O/imix_test.log
step bench
timeout -k 10 300 python bench.py --workload imix > $O/bench_imix.json 2> $O/bench.err || die bench $?
cat $O/bench_imix.json
timeout -k 10 300 python bench.py --workload imix --no-cpu-baseline > $O/bench_imix_b.json 2>> $O/bench.err || die bench_b $?
timeout -k 10 300 python bench.py --workload imix --no-cpu-baseline --streams 2 > $O/bench_imix_streams2.json 2>> $O/bench.err || die bench_s2 $?
cd /tmp && export TMPDIR=/tmp
step "kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_imix -o run --output-format csv -- python3 $ROOT/bench.py --workload imix --no-cpu-baseline > $O/prof_bench_imix.json 2> $O/prof_imix.log || die prof $?
python3 $ROOT/tools/prof_window.py trace $(find $O/prof_imix -name "run_kernel_trace.csv" | head -1) $O/prof_bench_imix.json --out $O/window_imix.json > /dev/null || die window $?
i=0
for grp in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  step "pmc $grp"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d $O/pmc/imix_p$i -o run --output-format csv -- python3 $ROOT/bench.py --workload imix --no-cpu-baseline --steps 20 --warmup 2 > $O/pmc/imix_p$i.json 2> $O/pmc/imix_p$i.log || die pmc_$i $?
done
args=""
for j in 1 2 3 4; do args="$args $(find $O/pmc/imix_p$j -name '*counter_collection.csv' | head -1) $O/pmc/imix_p$j.json"; done
python3 $ROOT/tools/prof_window.py pmc $args --out $O/pmc_imix.json > /dev/null || die pmc_window $?
step done
