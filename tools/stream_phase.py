"""Per-step phase of the K streams of a bench.py step, from a rocprofv3 --kernel-trace CSV.

bench.py --streams 2 cuts each step's batch into two runs, one k_step launch per run and stream.
Whether the second stream's launch fills the first one's tail depends on how far apart the two
launches start. This tool takes the timed window's transport-kernel dispatches (the same window
as tools/prof_window.py), groups them by stream and prints, per step, each stream's start and end
relative to the window start, the offset between the streams' starts and the step's span.

Usage: python tools/stream_phase.py <kernel_trace.csv> <bench.json> [--out profiles/x.json]
"""
import argparse
import csv
import json
import os
import statistics as st
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_window import bench_line, window  # noqa: E402

KEY = "wgt::k_"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench")
    ap.add_argument("--out")
    a = ap.parse_args()
    b = bench_line(a.bench)
    skip, count, per = window(b)
    rows = [r for r in csv.DictReader(open(a.trace)) if KEY in r["Kernel_Name"] and "k_lpt" not in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Correlation_Id"]))  # issue order
    win = rows[skip:skip + count]
    if len(win) != count:
        raise SystemExit(f"window needs {count} dispatches after {skip}, trace has {len(rows)}")
    t0 = min(int(r["Start_Timestamp"]) for r in win)
    steps = []
    for s in range(min(b["steps"], len(win) // per)):
        d = win[s * per:(s + 1) * per]
        st_ = [(int(r["Start_Timestamp"]) - t0) / 1e3 for r in d]
        en_ = [(int(r["End_Timestamp"]) - t0) / 1e3 for r in d]
        steps.append({"step": s, "queues": [r["Queue_Id"] for r in d], "start_us": st_, "end_us": en_,
                      "dur_us": [e - x for x, e in zip(st_, en_)],
                      "start_offset_us": (max(st_) - min(st_)) if per > 1 else 0.0})
    # per stream (queue): its launches back to back, first start and last end
    by_q = {}
    for r in win:
        by_q.setdefault(r["Queue_Id"], []).append(((int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3))
    streams = {q: {"launches": len(v), "first_start_us": round(min(x for x, _ in v), 2),
                   "last_end_us": round(max(e for _, e in v), 2)} for q, v in by_q.items()}
    span = (max(int(r["End_Timestamp"]) for r in win) - t0) / 1e3
    offs = [x["start_offset_us"] for x in steps]
    durs = [d for x in steps for d in x["dur_us"]]
    res = {"bench_value": b["value"], "steps": b["steps"], "launches_per_step": per,
           "window_span_us": round(span, 2), "us_per_step": round(span / b["steps"], 3),
           "launch_dur_mean_us": round(st.mean(durs), 2),
           "start_offset_first5_us": [round(o, 2) for o in offs[:5]],
           "start_offset_last5_us": [round(o, 2) for o in offs[-5:]],
           "start_offset_mean_us": round(st.mean(offs), 2), "streams": streams,
           "per_step": steps}
    print(json.dumps({k: v for k, v in res.items() if k != "per_step"}, indent=1))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
