"""Per-kernel breakdown of ONE cfg3 decode step (dev tool, CPU) from a rocprofv3 kernel trace of
tools/decode_prof.py (800 graph-replayed steps, B = 32) and, optionally, the FETCH_SIZE /
WRITE_SIZE passes of tools/decode_traffic.py (the same kernels launched eagerly).

The step's launch sequence repeats every P dispatches; P is found from the trace (the
smallest period over which the kernel names repeat for the whole loop).  For each position
in the step: kernel, average duration over all steps, over the first and the last 100 steps
(the self-attention's keys grow with t), and PMC HBM bytes per launch.

    python tools/summarize_decode_step.py <tag> <dir with kt/ [dtr/fetch dtr/write]>
"""
from __future__ import annotations

import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(n: str) -> str:
    return n.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:70]


def find(src, suffix):
    return next((os.path.join(d, f) for d, _, fs in os.walk(src) for f in fs if f.endswith(suffix)), None)


def loop_span(names, steps):
    """(start, period) of the longest run of `steps` identical windows."""
    n = len(names)
    for p in range(20, 200):
        for s0 in range(0, n - p * steps + 1):
            if all(names[s0 + i] == names[s0 + i + p] for i in range(p * (steps - 1))):
                return s0, p
    raise SystemExit("no periodic decode loop found")


def pmc(path, counter):
    if not path:
        return None
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0) or 0))
    return [(short(r["Kernel_Name"]), float(r["Counter_Value"])) for r in rows]


def main(tag, src, steps=800):
    tr = find(os.path.join(src, "kt"), "kernel_trace.csv")
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                for r in csv.DictReader(open(tr)))
    names = [e[2] for e in ev]
    s0, P = loop_span(names, steps)
    wall = (ev[s0 + P * steps - 1][1] - ev[s0][0]) / 1e3 / steps
    rows = []
    for i in range(P):
        d = [(ev[s0 + t * P + i][1] - ev[s0 + t * P + i][0]) / 1e3 for t in range(steps)]
        rows.append({"pos": i, "kernel": names[s0 + i], "avg_us": sum(d) / steps,
                     "first100_us": sum(d[:100]) / 100, "last100_us": sum(d[-100:]) / 100})
    # PMC bytes per position: the eager run's dispatches of the loop, same order
    fe, wr = pmc(find(os.path.join(src, "dtr", "fetch"), "counter_collection.csv"), "FETCH_SIZE"), \
        pmc(find(os.path.join(src, "dtr", "write"), "counter_collection.csv"), "WRITE_SIZE")
    if fe and wr:
        fn, wn = [n for n, _ in fe], [n for n, _ in wr]
        f0, _ = loop_span(fn, steps)
        w0, _ = loop_span(wn, steps)
        for r in rows:
            i = r["pos"]
            fb = sum(fe[f0 + t * P + i][1] for t in range(steps)) / steps * 2 * 1024   # gfx950: x2, KiB
            wb = sum(wr[w0 + t * P + i][1] for t in range(steps)) / steps * 1024
            r["hbm_bytes"] = fb + wb
    busy = sum(r["avg_us"] for r in rows)
    lines = [f"# One cfg3 decode step, per kernel — {tag}", "",
             "B = 32, 128 phonemes, 800 forced frames, bf16, libtt2's captured step graph replayed 800 times "
             "(tools/decode_prof.py under `rocprofv3 --kernel-trace --stats`); bytes from FETCH_SIZE x2 + WRITE_SIZE "
             "passes over the same kernels launched eagerly (tools/decode_traffic.py).", "",
             f"{P} kernels per step; {wall:.1f} us per step wall, {busy:.1f} us of kernel time "
             f"({wall - busy:.1f} us of launch gaps, {(wall - busy) / P:.2f} us per boundary).", "",
             "| # | kernel | avg us | first 100 steps | last 100 steps | HBM KB |", "|---|---|---|---|---|---|"]
    for r in rows:
        hb = f"{r['hbm_bytes'] / 1024:.0f}" if "hbm_bytes" in r else "-"
        lines.append(f"| {r['pos']} | `{r['kernel']}` | {r['avg_us']:.2f} | {r['first100_us']:.2f} | "
                     f"{r['last100_us']:.2f} | {hb} |")
    agg = {}
    for r in rows:
        a = agg.setdefault(r["kernel"], [0, 0.0])
        a[0] += 1
        a[1] += r["avg_us"]
    lines += ["", "| kernel | per step | us per step |", "|---|---|---|"]
    for k, (c, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"| `{k}` | {c} | {us:.1f} |")
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    open(os.path.join(ROOT, "profiles", f"{tag}_decode_step.md"), "w").write("\n".join(lines) + "\n")
    json.dump({"period": P, "wall_us_per_step": wall, "kernel_us_per_step": busy, "rows": rows},
              open(os.path.join(ROOT, "profiles", f"{tag}_decode_step.json"), "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
