set -o pipefail
O=gpurun_out/s16; mkdir -p $O
WG_LIB_PATH=$PWD/wireguard-java_amd/lib_base.so timeout -k 10 120 python -u -m pytest tests/test_batcher.py -q -s -k new_context --timeout 100 --timeout-method thread > $O/old_lib.log 2>&1; echo "old lib rc $?"; grep -E "passed|failed|batch seal" $O/old_lib.log
timeout -k 10 600 python -u -m pytest tests -x -q -s -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log; grep "batch seal while" $O/gpu_tests.log
for r in 1 2; do for v in 0 1; do
  WG_SLOT16=$v timeout -k 10 200 python bench.py --workload c2 --no-cpu-baseline > $O/c2_s${v}_$r.json 2>>$O/err.log || exit 1
  python -c "import json;d=json.load(open('$O/c2_s${v}_$r.json'));print('slot16=$v', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['verified'])"
done; done
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/c1.json 2>>$O/err.log && python -c "import json;d=json.load(open('$O/c1.json'));print('c1', d['value'], d['roofline']['frac'], d['verified'])"
