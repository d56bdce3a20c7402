"""Where the timed training step's wall time goes between kernels (dev tool, CPU).

Input: the same rocprofv3 kernel trace as tools/summarize_step.py (`tools/prof_step.sh <tag>`:
`bench.py --profile-run` under `--kernel-trace`).  Over the K timed graph replays only (the adam
dispatches delimit steps), every dispatch is ordered by start time and the idle time in front of
it is max(0, start - latest end so far): the time no kernel of the step was running.  Each gap is
charged to its seam, the (previous kernel -> next kernel) pair of short names.

Writes profiles/<tag>_step_gaps.md (+ .json): the gap-size histogram, the worst seams by total
gap per step, and kernel time / window.

    python tools/step_gaps.py <tag> [gpurun_out/<dir>]
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
sys.path.insert(0, os.path.join(ROOT, "tools"))
from summarize_step import short  # noqa: E402


def gaps(ev: list[tuple[int, int, str]]):
    """ev: (start_ns, end_ns, name) of one window, sorted by start.  Returns [(gap_ns, prev, next)]
    for every dispatch after the first, and the union of busy time."""
    out, busy = [], 0
    hi = ev[0][1]
    prev = ev[0][2]
    busy = ev[0][1] - ev[0][0]
    for s, e, n in ev[1:]:
        g = max(0, s - hi)
        out.append((g, prev, n))
        busy += max(0, e - max(s, hi))
        if e > hi:
            hi, prev = e, n
    return out, busy


def main(tag: str, src: str | None = None):
    src = src or os.path.join(ROOT, "gpurun_out", tag)
    kt = os.path.join(src, "kt") if os.path.isdir(os.path.join(src, "kt")) else src   # not dk/ (decode)
    trace = next((os.path.join(d, f) for d, _, fs in os.walk(kt) for f in fs if f.endswith("kernel_trace.csv")), None)
    if trace is None:
        raise SystemExit(f"no *kernel_trace.csv under {src}")
    bench = json.loads([ln for ln in open(os.path.join(src, "bench_step.json")) if ln.startswith("{")][-1])
    K, W = bench["steps"], bench["warmup"]
    rows = list(csv.DictReader(open(trace)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    adam = [e for e in ev if e[2].startswith(DELIM)]
    assert len(adam) >= W + 2 + K + 1, f"{len(adam)} {DELIM} dispatches, expected >= {W + 2 + K + 1}"
    seams: dict[tuple[str, str], list] = {}
    hist = [0] * 8   # < 1, 1-2, 2-3, 3-4, 4-6, 6-10, 10-20, >= 20 us
    edges = [1, 2, 3, 4, 6, 10, 20]
    wall = busy_tot = gap_tot = 0
    n_disp = 0
    for k in range(K):
        t0, t1 = adam[W + 1 + k][1], adam[W + 2 + k][1]
        win = [e for e in ev if e[0] >= t0 and e[1] <= t1]
        n_disp += len(win)
        g, busy = gaps(win)
        wall += t1 - t0
        busy_tot += busy
        # the idle time between the previous step's loss and this window's first dispatch
        lead = win[0][0] - t0
        g.insert(0, (lead, "loss_kernel(prev step)", win[0][2]))
        for ns, a, b in g:
            gap_tot += ns
            us = ns / 1e3
            hist[sum(us >= x for x in edges)] += 1
            d = seams.setdefault((a, b), [0, 0])
            d[0] += 1
            d[1] += ns
    wall_ms, busy_ms, gap_ms = wall / K / 1e6, busy_tot / K / 1e6, gap_tot / K / 1e6
    labels = ["< 1", "1-2", "2-3", "3-4", "4-6", "6-10", "10-20", ">= 20"]
    top = sorted(seams.items(), key=lambda kv: -kv[1][1])[:30]
    lines = [f"# Gaps between kernels of the timed training step — {tag}", "",
             f"Source: the rocprofv3 kernel trace of `bench.py --profile-run --steps {K} --warmup {W}` "
             "(tools/prof_step.sh), the timed graph replays only; tools/step_gaps.py.", "",
             f"Per step: window {wall_ms:.3f} ms, kernels running {busy_ms:.3f} ms "
             f"(kernel time / window = {busy_ms / wall_ms:.3f}), idle {gap_ms:.3f} ms over "
             f"{n_disp / K:.0f} dispatches ({1e3 * gap_ms / max(1, n_disp / K):.2f} us per seam).", "",
             "Gap sizes (count per step):", "",
             "| gap (us) | " + " | ".join(labels) + " |", "|---" * (len(labels) + 1) + "|",
             "| seams | " + " | ".join(f"{h / K:g}" for h in hist) + " |", "",
             "Worst seams by idle time per step:", "",
             "| previous kernel | next kernel | per step | avg gap us | us per step |", "|---|---|---|---|---|"]
    for (a, b), (c, ns) in top:
        lines.append(f"| `{a}` | `{b}` | {c / K:g} | {ns / c / 1e3:.2f} | {ns / K / 1e3:.1f} |")
    out = {"tag": tag, "steps": K, "wall_ms_per_step": wall_ms, "busy_ms_per_step": busy_ms,
           "idle_ms_per_step": gap_ms, "busy_over_window": busy_ms / wall_ms, "dispatches_per_step": n_disp / K,
           "hist_us_edges": edges, "hist_per_step": [h / K for h in hist],
           "seams": [{"prev": a, "next": b, "per_step": c / K, "avg_us": ns / c / 1e3, "us_per_step": ns / K / 1e3}
                     for (a, b), (c, ns) in sorted(seams.items(), key=lambda kv: -kv[1][1])]}
    dst = os.path.join(ROOT, "profiles")
    open(os.path.join(dst, f"{tag}_step_gaps.md"), "w").write("\n".join(lines) + "\n")
    json.dump(out, open(os.path.join(dst, f"{tag}_step_gaps.json"), "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main(*sys.argv[1:])
