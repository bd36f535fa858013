set -o pipefail
mkdir -p gpurun_out/r06f
timeout -k 5 60 ./tools/stitch_check > gpurun_out/r06f/stitch_check.txt 2>&1; echo "stitch_check rc $?"; cat gpurun_out/r06f/stitch_check.txt
WG_STITCH=1 timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_duplex.py tests/test_gpu_configs.py -k "step or c1 or c3 or imix" > gpurun_out/r06f/st.log 2>&1; echo "st tests rc $?"; grep -E "passed|failed|FAILED" gpurun_out/r06f/st.log | tail -30
