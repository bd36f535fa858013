"""Sweep launch tunables of libwgaead on the GPU box; one bench.py subprocess per point."""
import itertools
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
grid = json.loads(sys.argv[1]) if len(sys.argv) > 1 else {"WG_TILE_PASSES": ["1", "2", "3"], "WG_POLY_WAVES": ["1", "2", "4"]}
workload = sys.argv[2] if len(sys.argv) > 2 else "c1"
keys = list(grid)
for vals in itertools.product(*[grid[k] for k in keys]):
    env = dict(os.environ)
    env.update(dict(zip(keys, vals)))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--steps", "20",
                        "--workload", workload], env=env, capture_output=True, text=True, timeout=300)
    try:
        d = json.loads(r.stdout.strip().splitlines()[-1])
        print(dict(zip(keys, vals)), "value", d["value"], "seal_ms", d["roofline"]["seal_ms"], "open_ms",
              d["roofline"]["open_ms"], "frac", d["roofline"]["frac"], "ok", d["verified"], flush=True)
    except Exception:
        print(dict(zip(keys, vals)), "FAILED", r.returncode, r.stderr[-500:], flush=True)
        sys.exit(1)
