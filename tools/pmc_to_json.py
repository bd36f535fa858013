"""Turn a round's rocprofv3 output (gpurun_out/<round>/) into committed summaries:
profiles/<round>_kernel_stats.csv (the --stats table) and profiles/pmc_<round>.json
(per-launch HBM bytes for the seal and open kernels).

HBM bytes follow MI355X_MICROARCH.md's rocprofv3 section: FETCH_SIZE and WRITE_SIZE
are in KB, each collected in its own pass; on gfx950 FETCH_SIZE reports half the
bytes of a wide coalesced streaming read, so it is doubled; WRITE_SIZE is exact for
16-B-per-lane streaming stores.
Usage: python tools/pmc_to_json.py r01
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rnd = sys.argv[1]
src = os.path.join(ROOT, "gpurun_out", rnd)
prof = os.path.join(ROOT, "profiles")
os.makedirs(prof, exist_ok=True)

stats = glob.glob(os.path.join(src, "prof", "**", "*kernel_stats.csv"), recursive=True)
if stats:
    shutil.copy(stats[0], os.path.join(prof, f"{rnd}_kernel_stats.csv"))


def kind(name):
    if not any(k in name for k in ("k_transport", "k_wave", "k_stream", "k_tile", "k_lean", "k_pipe")):
        return None
    # template arg 0 = MODE: 0 seal, 1 open
    inner = name.split("<", 1)[1] if "<" in name else ""
    return "seal" if inner.startswith("0") else "open" if inner.startswith("1") else None


vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(src, "pmc", "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        k = kind(r["Kernel_Name"])
        if k:
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            vals[k]["_name"] = r["Kernel_Name"].split("(")[0]
            vals[k]["_vgpr"] = int(r["VGPR_Count"])

out = {"round": rnd, "source": "rocprofv3 --kernel-trace --pmc <one counter group per pass> -- python3 bench.py "
                                "--no-cpu-baseline --steps 5 --warmup 1 (C1: 65536 x 1420 B)",
       "correction": "FETCH_SIZE x 2 (gfx950 half-count of 16 B/lane streaming reads) + WRITE_SIZE; both KB x 1024"}
for k, cs in vals.items():
    m = {c: sum(v) / len(v) for c, v in cs.items() if not c.startswith("_")}
    d = {"kernel": cs["_name"], "vgpr": cs["_vgpr"], "launches": len(cs.get("FETCH_SIZE", [])), "counters_mean": m}
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        d["read_bytes"] = m["FETCH_SIZE"] * 1024 * 2
        d["write_bytes"] = m["WRITE_SIZE"] * 1024
        d["hbm_bytes_per_launch"] = d["read_bytes"] + d["write_bytes"]
        out[f"{k}_hbm_bytes_per_launch"] = round(d["hbm_bytes_per_launch"])
    out[k] = d
json.dump(out, open(os.path.join(prof, f"pmc_{rnd}.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
