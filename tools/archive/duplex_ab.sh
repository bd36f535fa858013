#!/bin/bash
# Duplex-launch check on the GPU box: its parity tests, then C1 bench lines for serial steps,
# duplex steps (alternating and split workgroup order), two streams, and a rocprofv3 kernel
# summary of the duplex bench. Usage: bash tools/duplex_ab.sh <tag>
set -eo pipefail
T=${1:-duplex}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$T
mkdir -p $O
cd $ROOT
echo "[dx] tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_duplex.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for run in "serial:--mode serial" "duplex:--mode duplex" "streams2:--streams 2" "duplex_c2:--mode duplex --workload c2" "serial_c2:--mode serial --workload c2"; do
  name=${run%%:*}; a=${run#*:}
  timeout -k 10 300 python bench.py $a --no-cpu-baseline > $O/bench_$name.json 2>> $O/bench.err
  python3 -c "import json; d=json.load(open('$O/bench_$name.json')); print('$name', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['verified'])"
done
WG_LIB_PATH=$ROOT/wireguard-java_amd/libwgaead_split.so timeout -k 10 300 python bench.py --mode duplex --no-cpu-baseline > $O/bench_duplex_split.json 2>> $O/bench.err
python3 -c "import json; d=json.load(open('$O/bench_duplex_split.json')); print('duplex_split', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['verified'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $ROOT/bench.py --mode duplex --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.log
cat $O/prof_bench.json
echo "[dx] done"
