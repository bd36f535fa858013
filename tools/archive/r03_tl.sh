set -o pipefail
mkdir -p gpurun_out/tl
timeout -k 10 120 python tools/phase_stamps.py --mode seal --keys 1 > gpurun_out/tl/seal.json 2> gpurun_out/tl/err.log || { tail -3 gpurun_out/tl/err.log; exit 1; }
timeout -k 10 120 python tools/phase_stamps.py --mode step --keys 1 > gpurun_out/tl/step.json 2>> gpurun_out/tl/err.log || exit 1
python3 -c "
import json
for m in ('seal','step'):
  d=json.load(open('gpurun_out/tl/%s.json'%m)); print(m, d['kernel_span_us'], d['wave_life_us_mean'], d['wave_end_us'], d['tail_idle_frac'], d['live_waves_over_time'])
"
AB_TESTS=none bash tools/ab_args.sh ab_prio "--variant 0" "WG_PRIO=0 --variant 0" "WG_PRIO=1 --variant 0"
