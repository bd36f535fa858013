# end-of-session check on the final tree: GPU tests, smoke, then the per-packet order control
# (the kept library in both A/B slots, tools/r03_ppidle.sh)
set -o pipefail
mkdir -p gpurun_out/final2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final2/gpu_tests.log 2>&1 || { tail -30 gpurun_out/final2/gpu_tests.log; exit 1; }
tail -1 gpurun_out/final2/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
AB_CONTROL=1 PP_REPS=2 bash tools/r03_ppidle.sh
