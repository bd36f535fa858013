"""Kernel statistics over bench.py's TIMED REGION only, from a rocprofv3 --kernel-trace CSV.

rocprofv3 --stats averages every dispatch of a kernel, including the clock-ramp and warmup steps
that bench.py runs before its timed region and the seal-only / open-only trains after it, so its
averages do not describe the launches the bench line's `ms_per_step` and `roofline.frac` come
from (Weak #1). bench.py's JSON line carries ramp_steps / warmup / steps and the
kernel launches per step; this tool takes the transport kernel's dispatches in issue order,
skips (ramp_steps + warmup) x launches, keeps the next steps x launches and reports their
durations, the window's span and the roofline fraction recomputed from them.

PMC passes (--pmc): the same window over a counter_collection.csv gives per-dispatch counter
means for the timed launches.
Usage:
  python tools/prof_window.py trace <kernel_trace.csv> <bench.json> [--out profiles/x.json]
  python tools/prof_window.py pmc <counter_collection.csv> <bench.json> [<csv> <json> ...] [--out ...]
"""
import argparse
import collections
import csv
import json
import re
import sys

KERNELS = r"k_step|k_transport|k_duplex|k_wave|k_tile"


def bench_line(path):
    for line in open(path):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    raise SystemExit(f"no bench JSON line in {path}")


def window(b):
    # a K-stream step (bench.py --streams K > 1) cuts the batch into K runs, one launch each
    st = b["roofline"].get("step") or {}
    per = st["launches"] if st.get("streams", 1) > 1 else b["roofline"].get("launches_per_step", 1)
    if b.get("launches_before_window") is not None and b.get("window_launches") is not None:
        # bench.py counts its transport launches (a staggered two-stream schedule has one more per run)
        return b["launches_before_window"], b["window_launches"], per
    skip = (b["ramp_steps"] + b["warmup"] + b.get("graph_warm_steps", 0)) * per
    return skip, b["steps"] * per, per


def kind(name):
    m = re.search(KERNELS, name)
    if not m:
        return None
    k = m.group(0)
    if k in ("k_transport", "k_wave", "k_tile"):
        inner = name.split("<", 1)[1] if "<" in name else ""
        k += "<seal>" if inner.startswith("0") else "<open>" if inner.startswith("1") else ""
    return k


def trace(args):
    b = bench_line(args.bench)
    skip, take, per = window(b)
    rows = [r for r in csv.DictReader(open(args.csv)) if kind(r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the step kernel(s): the name(s) used by the timed region (the last launches before the trains)
    names = [kind(r["Kernel_Name"]) for r in rows]
    want = b["roofline"]["kernel_names"]
    sel = [r for r, k in zip(rows, names) if k in want]
    win = sel[skip:skip + take]
    if len(win) != take:
        raise SystemExit(f"window wants {take} dispatches after {skip}, trace has {len(sel)}")
    per_kernel = collections.defaultdict(list)
    for r in win:
        per_kernel[kind(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    span_us = (int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])) * 1e-3
    busy_us = sum(sum(v) for v in per_kernel.values())
    out = {
        "source": f"rocprofv3 --kernel-trace of the bench command; dispatches {skip}..{skip + take - 1} of {sorted(want)} "
                  f"(ramp {b['ramp_steps']} + warmup {b['warmup']} + graph warm {b.get('graph_warm_steps', 0)} steps "
                  f"skipped, {b['steps']} timed steps x {per}{', one graph replay' if b.get('graph') else ''})",
        "bench_ms_per_step": b["ms_per_step"],
        "bench_frac": b["roofline"]["frac"],
        "window_span_us": round(span_us, 2),
        "window_span_per_step_us": round(span_us / b["steps"], 3),
        "kernel_busy_per_step_us": round(busy_us / b["steps"], 3),
        "kernels": {k: {"dispatches": len(v), "avg_us": round(sum(v) / len(v), 3), "min_us": round(min(v), 3),
                        "max_us": round(max(v), 3), "median_us": round(sorted(v)[len(v) // 2], 3)}
                    for k, v in sorted(per_kernel.items())},
    }
    # the step's other launches inside the window (the mixed plans' k_lpt_* planning): the device time a
    # step needs besides the transport kernel, so that the gaps left are the host's
    t0, t1 = int(win[0]["Start_Timestamp"]), int(win[-1]["End_Timestamp"])
    plan_us = sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
                  for r in csv.DictReader(open(args.csv)) if re.search(r"k_lpt_", r["Kernel_Name"])
                  and t0 <= int(r["Start_Timestamp"]) and int(r["End_Timestamp"]) <= t1)
    if plan_us:
        out["planning_busy_per_step_us"] = round(plan_us / b["steps"], 3)
        out["gap_per_step_us"] = round((span_us - busy_us - plan_us) / b["steps"], 3)
    st = b["roofline"].get("step") or {}
    multi = st.get("streams", 1) > 1
    # per step: a K-stream step's K launches together move one batch (the one-stream kernel's bytes)
    alg = b["roofline"]["alg_bytes_per_launch"] * (b["roofline"].get("launches_per_step", 1) if multi else per)
    if multi:  # compare with the K-stream step's own fraction, not the one-stream kernel's
        out["bench_frac"] = st["frac"]
        out["streams"] = st["streams"]
    # the bench's frac is bytes per step over the device time of a step (HIP events around the
    # whole timed region): the profile's counterpart is the window's span per step (launches of
    # one step may overlap on two streams, so their summed durations can exceed it)
    out["frac_from_profile"] = round(alg / (span_us / b["steps"] * 1e-6) / 8.0e12, 4)
    out["frac_vs_bench"] = round(out["frac_from_profile"] / out["bench_frac"], 4)
    out["span_le_bench_ms_per_step"] = span_us / b["steps"] * 1e-3 <= b["ms_per_step"]
    # the same fraction from the kernels' own durations: under rocprofv3 the host can take longer to
    # enqueue a step than the GPU takes to run it (the profiler intercepts every dispatch), and
    # then the span holds idle gaps that the unprofiled bench does not have
    out["frac_from_kernel_time"] = round(alg / (busy_us / b["steps"] * 1e-6) / 8.0e12, 4)
    # K streams overlap their launches: the summed durations exceed the span, so only the span says
    # whether the host kept the device fed
    out["host_bound_under_profiler"] = span_us > 1.05 * (busy_us + plan_us) if not multi else \
        span_us / b["steps"] * 1e-3 > 1.05 * b["ms_per_step"]
    return out


def pmc(args):
    # alternating <counter_collection.csv> <bench json of that pass>: every pass has its own ramp
    pairs = list(zip(args.csv[0::2], args.csv[1::2]))
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for f, bf in pairs:
        b = bench_line(bf)
        skip, take, per = window(b)
        want = b["roofline"]["kernel_names"]
        rows = [r for r in csv.DictReader(open(f)) if kind(r["Kernel_Name"]) in want]
        by_counter = collections.defaultdict(list)
        for r in rows:
            by_counter[r["Counter_Name"]].append(r)
        for c, rs in by_counter.items():
            rs.sort(key=lambda r: int(r["Start_Timestamp"]))
            for r in rs[skip:skip + take]:
                k = kind(r["Kernel_Name"])
                vals[k][c].append(float(r["Counter_Value"]))
                meta[k] = {"vgpr": int(r["VGPR_Count"]), "sgpr": int(r["SGPR_Count"]), "grid": int(r["Grid_Size"]),
                           "workgroup": int(r["Workgroup_Size"]), "lds": int(r["LDS_Block_Size"])}
    out = {"source": "rocprofv3 --kernel-trace --pmc (one counter group per pass), each pass's timed-window "
                     "dispatches only (ramp + warmup skipped)",
           "workload": b["config"]["workload"], "step": b["config"]["step"],
           "correction": "HBM bytes = FETCH_SIZE x 1024 x 2 (gfx950 counts half of 16-B/lane streaming reads) + "
                         "WRITE_SIZE x 1024 (MI355X_MICROARCH.md, HBM)"}
    for k, cs in vals.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = dict(meta[k], counters_mean=m, dispatches=max(len(v) for v in cs.values()))
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            d["read_bytes"] = round(m["FETCH_SIZE"] * 1024 * 2)
            d["write_bytes"] = round(m["WRITE_SIZE"] * 1024)
            d["hbm_bytes_per_launch"] = d["read_bytes"] + d["write_bytes"]
            d["alg_bytes_per_launch"] = b["roofline"]["alg_bytes_per_launch"]
            d["traffic_over_alg"] = round(d["hbm_bytes_per_launch"] / d["alg_bytes_per_launch"], 4)
        if "SQ_WAVES" in m and "SQ_INSTS_VALU" in m:
            d["valu_per_wave"] = round(m["SQ_INSTS_VALU"] / m["SQ_WAVES"], 1)
        out[k] = d
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["trace", "pmc"])
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--bench", required=False)
    ap.add_argument("--out")
    a = ap.parse_args()
    if a.what == "trace":
        if not a.bench:
            a.csv, a.bench = a.csv[:1], a.csv[1]
        a.csv = a.csv[0]
        out = trace(a)
    else:
        out = pmc(a)
    s = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    sys.exit(main())
