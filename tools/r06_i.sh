#!/bin/bash
# Round 6: the bench / configuration tests after the k_lpt_one and spin-sync changes, IMIX one-launch vs two-launch
# planning, the 20-step line with and without spin-sync, the SQ counter list and a VALU-busy PMC pass on C1.
set -o pipefail
T=${1:-r06i}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$T
mkdir -p $O $O/pmc
cd $ROOT
die() { echo "[r06i] FAILED: $1 (rc $2)"; exit $2; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bench.py tests/test_gpu_configs.py tests/test_gpu_duplex.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; die tests $?; }
tail -1 $O/tests.log
line() {
  python3 - "$1" $O/tmp.json >> $O/ab.jsonl <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
print(json.dumps({"variant": sys.argv[1], "value": d["value"], "ms_per_step": d["ms_per_step"],
                  "step_ms": d["roofline"]["step"]["ms"], "kernel_ms": d["roofline"]["kernel_ms"],
                  "verified": d["verified"], "spin_sync": d.get("spin_sync")}))
PY
  tail -1 $O/ab.jsonl
}
for a in 1 2 3; do
  timeout -k 10 120 python bench.py --workload imix --no-cpu-baseline > $O/tmp.json 2>> $O/err.log || die imix $?; line imix_one
  WG_LPT_ONE=0 timeout -k 10 120 python bench.py --workload imix --no-cpu-baseline > $O/tmp.json 2>> $O/err.log || die imix2 $?; line imix_two
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/tmp.json 2>> $O/err.log || die spin $?; line c1_20_spin
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --spin-sync 0 > $O/tmp.json 2>> $O/err.log || die nospin $?; line c1_20_nospin
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > $O/list_avail.txt 2>&1 || echo "list-avail rc $?"
grep -E "^\s*SQ_|SQ_[A-Z_]+" $O/list_avail.txt | head -5
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $O/pmc/c1s_p$i -o run --output-format csv -- python3 $ROOT/bench.py --streams 1 --no-cpu-baseline --steps 20 --warmup 2 > $O/pmc/c1s_p$i.json 2> $O/pmc/c1s_p$i.log || echo "pmc pass $i rc $?"
done
echo "[r06i] done"
