#!/bin/bash
# Kernel trace of the default C1 bench command (two streams) and its timed window.
set -o pipefail
out=gpurun_out/${1:-r04p2s}
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --workload c1 > $out/bench.json 2> $out/prof.log || { tail -20 $out/prof.log; exit 1; }
python3 tools/prof_window.py trace $out/prof/run_kernel_trace.csv $out/bench.json --out $out/window.json && cat $out/window.json
