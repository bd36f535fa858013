"""Per-kernel mean of every PMC counter under gpurun_out/<dir>/p*/ (tools/pmc_cmp.sh output),
plus derived figures: mean resident waves and cycles per VALU instruction per SIMD."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "k_transport" not in k and "k_wave" not in k and "k_tile" not in k:
                continue
            k = f.split("/")[-3] + ":" + k.split("(")[0].replace("void ", "")
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] == "SQ_WAVES":
                dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for k, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        print(d, k, "dur_us %.1f" % (sum(dur[k]) / len(dur[k]) / 1e3 if dur[k] else 0))
        for c, v in sorted(m.items()):
            print(f"    {c:24s} {v:.4g}")
        if "GRBM_GUI_ACTIVE" in m and "SQ_WAVE_CYCLES" in m:
            cyc = m["GRBM_GUI_ACTIVE"] / 8
            print(f"    kernel cycles/XCD {cyc:.4g}  mean resident waves {4 * m['SQ_WAVE_CYCLES'] / cyc:.0f}"
                  f"  cyc per VALU per SIMD {cyc * 1024 / m['SQ_INSTS_VALU']:.2f}")
