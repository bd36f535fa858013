"""Per-kernel durations and the idle gaps between consecutive launches of the transport
kernels in a rocprofv3 --kernel-trace CSV. Usage: python tools/trace_gaps.py run_kernel_trace.csv [name-substring]"""
import csv
import statistics as st
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
key = sys.argv[2] if len(sys.argv) > 2 else "wgt::k_"
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows if key in r["Kernel_Name"])
# the timed region of bench.py: the longest run of back-to-back launches (gaps < 50 us)
runs, cur = [], [ks[0]]
for a, b in zip(ks, ks[1:]):
    if b[0] - a[1] < 50_000:
        cur.append(b)
    else:
        runs.append(cur)
        cur = [b]
runs.append(cur)
run = max(runs, key=len)
by = {}
for s, e, n in run:
    by.setdefault(n.split("(")[0], []).append((e - s) / 1e3)
for n, d in by.items():
    print(f"{n}: launches {len(d)} mean {st.mean(d):.2f} us median {st.median(d):.2f} us")
gaps = [(b[0] - a[1]) / 1e3 for a, b in zip(run, run[1:])]
span = (run[-1][1] - run[0][0]) / 1e3
print(f"run of {len(run)} launches over {span:.1f} us: gap mean {st.mean(gaps):.2f} us median {st.median(gaps):.2f} us, "
      f"busy {100 * sum(e - s for s, e, _ in run) / 1e3 / span:.1f}%")
