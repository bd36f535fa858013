#!/bin/bash
# The driver's bench command beside the 200-step default, and kernel traces of both, so the two
# streams' phase per step can be read (tools/stream_phase.py). Usage: bash tools/phase_round.sh <tag> [extra bench args]
set -o pipefail
T=${1:-phase}
shift
X="$*"
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$T
mkdir -p $O
cd $ROOT
die() { echo "[phase] FAILED: $1 (rc $2)"; exit $2; }
for i in 1 2; do
  echo "[phase] driver command $i"
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 $X > $O/bench_20_$i.json 2>> $O/bench.err || die bench20 $?
  python3 -c "import json; d=json.load(open('$O/bench_20_$i.json')); print('20-step', d['value'], d['roofline']['kernel_ms'], d['roofline']['step']['ms'], d['verified'])"
  echo "[phase] 200 steps $i"
  timeout -k 10 300 python bench.py --no-cpu-baseline $X > $O/bench_200_$i.json 2>> $O/bench.err || die bench200 $?
  python3 -c "import json; d=json.load(open('$O/bench_200_$i.json')); print('200-step', d['value'], d['roofline']['kernel_ms'], d['roofline']['step']['ms'], d['verified'])"
done
cd /tmp && export TMPDIR=/tmp
for s in 20 200; do
  w=$((s == 20 ? 5 : 20))
  echo "[phase] trace $s steps"
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr$s -o run --output-format csv -- python3 $ROOT/bench.py --steps $s --warmup $w --no-cpu-baseline $X > $O/tr$s.json 2> $O/tr$s.log || die trace$s $?
  python3 $ROOT/tools/stream_phase.py $(find $O/tr$s -name "run_kernel_trace.csv" | head -1) $O/tr$s.json --out $O/phase_$s.json || die phase$s $?
done
echo "[phase] done"
