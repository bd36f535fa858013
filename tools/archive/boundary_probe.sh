#!/bin/bash
# Where the per-launch time goes at the launch boundary: a kernel trace of serial C1 steps
# (durations, gaps), store / payload-load ablation builds (no correctness: timing only), and
# the multi-stream split. Usage: bash tools/boundary_probe.sh <tag>
set -o pipefail
T=${1:-bprobe}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$T
mkdir -p $O
cd $ROOT
for lib in libwgaead.so libwgaead_abl_NOSTORE.so libwgaead_abl_NODMA.so; do
  WG_LIB_PATH=$ROOT/wireguard-java_amd/$lib timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$lib.json 2>> $O/bench.err
  rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || { echo "bench $lib rc=$rc"; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$lib.json')); r=d['roofline']; print('$lib', d['value'], r['kernel_ms'], r['seal_ms'], r['open_ms'], d['verified'])"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --streams 4 > $O/bench_streams4.json 2>> $O/bench.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench_streams4.json')); print('streams4', d['value'], d['roofline']['kernel_ms'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python3 $ROOT/bench.py --no-cpu-baseline --steps 100 > $O/trace_bench.json 2> $O/trace.log || exit 1
python3 $ROOT/tools/trace_gaps.py $(ls $O/trace/*/run_kernel_trace.csv $O/trace/run_kernel_trace.csv 2>/dev/null | head -1)
echo "[probe] done"
