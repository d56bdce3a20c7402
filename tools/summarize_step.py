"""Per-step kernel table of the TIMED graph-replayed training steps only (dev tool, CPU).

Input: a `rocprofv3 --kernel-trace --stats --output-format csv` run of
`bench.py --profile-run --steps K --warmup W` (tools/prof_step.sh).  That run executes, in
order on one stream: W eager warm-up steps, 2 untimed graph replays, K timed graph replays,
1 eager probe step and 5 graph-node probe replays (the roofline leg).  Every step runs `adam_kernel` exactly once, so the
adam dispatches delimit the steps: the timed region is every dispatch that starts after the
(W + 2)-th adam dispatch ends and ends no later than the (W + 2 + K)-th one.

Writes profiles/<tag>_step_kernels.md (+ .json): per kernel, launches per step, average
duration and share of the step, over the timed replays only, and the dominant kernel's
per-launch average beside bench.py's live figure.

    python tools/summarize_step.py <tag> [gpurun_out/<dir>]
"""
from __future__ import annotations

import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# one dispatch per step in every schedule (the pipelined optimizer splits Adam over two launches
# in the next step's forward): the loss kernel's dispatches delimit the steps
DELIM = "_ZN12_GLOBAL__N_111loss_kernel"


def short(name: str) -> str:
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:80]


def main(tag: str, src: str | None = None):
    src = src or os.path.join(ROOT, "gpurun_out", tag)
    kt = os.path.join(src, "kt") if os.path.isdir(os.path.join(src, "kt")) else src   # not dk/ (decode)
    trace = next((os.path.join(d, f) for d, _, fs in os.walk(kt) for f in fs if f.endswith("kernel_trace.csv")), None)
    if trace is None:
        raise SystemExit(f"no *kernel_trace.csv under {src}")
    bench = json.loads([ln for ln in open(os.path.join(src, "bench_step.json")) if ln.startswith("{")][-1])
    K, W = bench["steps"], bench["warmup"]
    rows = list(csv.DictReader(open(trace)))
    ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    adam = [e for e in ev if short(e[2]).startswith(DELIM)]
    # W eager + 2 untimed replays + K timed, then the probe steps (eager, graph-node replays)
    assert len(adam) >= W + 2 + K + 1, f"{len(adam)} {DELIM} dispatches, expected >= {W + 2 + K + 1}"
    t0, t1 = adam[W + 1][1], adam[W + 1 + K][1]
    timed = [e for e in ev if e[0] >= t0 and e[1] <= t1]
    wall_ms = (t1 - t0) / 1e6 / K
    agg: dict[str, list] = {}
    for s, e, n in timed:
        d = agg.setdefault(short(n), [0, 0.0])
        d[0] += 1
        d[1] += (e - s) / 1e3
    busy = sum(v[1] for v in agg.values()) / K
    dom = (bench.get("roofline") or {}).get("kernel", "gemm7_kernel<true, true>")
    lines = [f"# Timed training steps under rocprofv3 — {tag}", "",
             f"`rocprofv3 --kernel-trace --stats -- python3 bench.py --profile-run --steps {K} --warmup {W}` "
             f"(tools/prof_step.sh); summary by tools/summarize_step.py over the {K} timed graph replays only "
             "(the loss-kernel dispatches delimit steps; eager warm-up, untimed replays and the probe step excluded).", "",
             f"bench under the profiler: {bench['ms_per_step']} ms/step.  Timed window: {wall_ms:.3f} ms/step "
             f"wall, {busy / 1e3:.3f} ms/step of kernel time, {len(timed) / K:.0f} kernels/step.", "",
             "| kernel | launches/step | avg us | ms/step | % of kernel time |", "|---|---|---|---|---|"]
    table = []
    for n, (c, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        table.append({"kernel": n, "launches_per_step": c / K, "avg_us": us / c, "ms_per_step": us / K / 1e3,
                      "pct": 100 * us / K / busy})
        lines.append(f"| `{n}` | {c / K:g} | {us / c:.2f} | {us / K / 1e3:.3f} | {100 * us / K / busy:.1f} |")
    d = next((t for t in table if t["kernel"] == dom), None)
    rl = bench.get("roofline") or {}
    out = {"tag": tag, "steps": K, "warmup": W, "wall_ms_per_step": wall_ms, "kernel_ms_per_step": busy / 1e3,
           "kernels": table, "dominant": dom}
    if d:
        agree = d["avg_us"] / rl["avg_launch_us"] - 1 if rl.get("avg_launch_us") else None
        out["dominant_avg_us"] = d["avg_us"]
        out["bench_avg_launch_us"] = rl.get("avg_launch_us")
        out["bench_vs_profile"] = agree
        lines += ["", f"Dominant kernel `{dom}`: {d['launches_per_step']:g} launches/step, rocprof average "
                      f"{d['avg_us']:.2f} us over the timed replays; bench.py's live figure in the same run "
                      f"{rl.get('avg_launch_us')} us (differs by {100 * agree:+.1f} %)." if agree is not None else ""]
    dst = os.path.join(ROOT, "profiles")
    open(os.path.join(dst, f"{tag}_step_kernels.md"), "w").write("\n".join(lines) + "\n")
    json.dump(out, open(os.path.join(dst, f"{tag}_step_kernels.json"), "w"), indent=1)
    print("\n".join(lines[:40]))


if __name__ == "__main__":
    main(*sys.argv[1:])
