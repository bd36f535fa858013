set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05o
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  WG_SLOT4=$v timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/p$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload imix --no-cpu-baseline --steps 20 --warmup 2 > $O/p$v.json 2> $O/p$v.log || exit 1
done
