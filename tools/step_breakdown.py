"""Per-step kernel breakdown of one graph-replayed train step from a rocprofv3
kernel trace of bench.py (dev tool).

    python tools/step_breakdown.py gpurun_out/.../run_kernel_trace.csv [step_index]

Steps are delimited by the Adam kernel (one launch per step); the default picks
the median-length step among the timed replays.
"""
import csv
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    m = re.search(r"_ZN12_GLOBAL__N_1\d+(\w+?)I", name)
    if m:
        return m.group(1)
    m = re.match(r"(?:void )?([\w:]+(?:<[^()]*>)?)", name)
    return m.group(1) if m else name[:40]


def main(path, pick=None):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    steps = []
    for k in range(len(idx) - 1):
        seg = rows[idx[k] + 1: idx[k + 1] + 1]
        span = int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
        steps.append((k, span, busy, seg))
    # graph replays have (almost) no gaps: pick the median-busy of those
    tight = [s for s in steps if s[1] < 1.05 * s[2]] or steps
    tight.sort(key=lambda s: s[2])
    k, span, busy, seg = tight[len(tight) // 2] if pick is None else steps[int(pick)]
    print(f"step {k}: {len(seg)} launches, span {span / 1e3:.1f} us, kernel-busy {busy / 1e3:.1f} us")
    agg = defaultdict(lambda: [0, 0.0])
    for r in seg:
        key = (short(r["Kernel_Name"]), r.get("Grid_Size_X", ""), r.get("Grid_Size_Y", ""))
        agg[key][0] += 1
        agg[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    fam = defaultdict(lambda: [0, 0.0])
    for (n, _, _), (c, t) in agg.items():
        fam[n][0] += c
        fam[n][1] += t
    print("\n-- by kernel --")
    for n, (c, t) in sorted(fam.items(), key=lambda x: -x[1][1]):
        print(f"{n:48s} {c:4d} {t:9.1f} us {100 * t * 1e3 / busy:5.1f}%")
    print("\n-- by kernel and grid (top 40) --")
    for (n, gx, gy), (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:40]:
        print(f"{n:40s} grid {gx:>8s}x{gy:<4s} {c:4d} {t:9.1f} us  avg {t / c:7.1f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
