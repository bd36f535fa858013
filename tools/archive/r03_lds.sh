set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/lds; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM -d $O/p1 -o run --output-format csv -- python3 $ROOT/bench.py --no-cpu-baseline --steps 20 --warmup 2 > $O/p1.json 2> $O/p1.log || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAVES -d $O/p2 -o run --output-format csv -- python3 $ROOT/bench.py --no-cpu-baseline --steps 20 --warmup 2 > $O/p2.json 2> $O/p2.log || exit 1
cd $ROOT
python3 tools/prof_window.py pmc $(find $O/p1 -name '*counter_collection.csv' | head -1) $O/p1.json $(find $O/p2 -name '*counter_collection.csv' | head -1) $O/p2.json --out $O/pmc_lds.json > /dev/null && python3 -c "
import json; d=json.load(open('$O/pmc_lds.json'))['k_step']['counters_mean']; print({k: round(v) for k,v in d.items()})"
