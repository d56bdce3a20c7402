"""Turn a `tools/gpu_pass.sh <tag> prof` run (gpurun_out/<tag>/kt, bench_kt.json; called on the GPU
box by tools/summarize_pass.sh) into committed summaries under profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats table (as produced)
  profiles/<tag>_kernel_stats.md    top kernels, per-step times, vs bench.py's live figure
  profiles/<tag>_traffic.json       PMC HBM bytes per launch of the dominant kernel
                                    (FETCH_SIZE x 2 per the gfx950 correction + WRITE_SIZE, KiB -> B)

    python tools/summarize_prof.py r01
"""
from __future__ import annotations

import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOMINANT = "gemm2_kernel<true, true>"   # fallback; the bench run's roofline names the live one


def per_kernel_counter(path, counter):
    out = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            d = out.setdefault(r["Kernel_Name"], [0, 0.0])
            d[0] += 1
            d[1] += float(r["Counter_Value"])
    return out


def main(tag: str):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    if not os.path.isdir(src):  # tools/gpu_pass.sh layout (prof_<tag>: the round-1 layout)
        src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "kt", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    bench = json.loads(open(os.path.join(src, "bench_kt.json")).read().strip().splitlines()[-1])
    global DOMINANT
    DOMINANT = (bench.get("roofline") or {}).get("kernel", DOMINANT).split(" (")[0]
    steps_total = bench["steps"] + bench["warmup"] + 2 + 1 + 1  # timed + eager warm-up + graph warm + capture-free roofline step (+1 graph record)
    total_ns = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = [f"# rocprofv3 kernel stats — {tag}", "",
             f"Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py --steps {bench['steps']} "
             f"--warmup {bench['warmup']} --profile-run` (tools/gpu_pass.sh prof).", "",
             f"bench under the profiler: {bench['ms_per_step']} ms/step, {bench['value']} frames/s.", "",
             f"Total kernel time {total_ns / 1e6:.1f} ms over ~{steps_total} executed steps.", "",
             "| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
        name = r["Name"].replace("(anonymous namespace)::", "").split("(")[0][:90]
        lines.append(f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
                     f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")
    dom = [r for r in rows if DOMINANT in r["Name"]]
    rl = bench.get("roofline") or {}
    if dom:
        avg_us = float(dom[0]["AverageNs"]) / 1e3
        lines += ["", f"Dominant kernel `{DOMINANT}`: rocprof average {avg_us:.2f} us/launch over "
                      f"{dom[0]['Calls']} launches; bench.py's live HIP-event figure in the same run: "
                      f"{rl.get('avg_launch_us')} us/launch ({rl.get('achieved')} TFLOP/s)."]
    traffic = {}
    fpath = os.path.join(src, "pmc_fetch", "run_counter_collection.csv")
    wpath = os.path.join(src, "pmc_write", "run_counter_collection.csv")
    if os.path.exists(fpath) and os.path.exists(wpath):
        fe = per_kernel_counter(fpath, "FETCH_SIZE")
        wr = per_kernel_counter(wpath, "WRITE_SIZE")
        for name, (n, v) in fe.items():
            if DOMINANT in name:
                wn, wv = next(((a, b) for k, (a, b) in wr.items() if DOMINANT in k), (1, 0.0))
                fetch = 2.0 * v / n * 1024.0
                write = wv / wn * 1024.0
                traffic = {"kernel": DOMINANT, "dispatches": n, "fetch_bytes_per_launch": fetch,
                           "write_bytes_per_launch": write, "hbm_bytes_per_launch": fetch + write,
                           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; FETCH_SIZE x2 "
                                     "(gfx950 counts 128-B requests as 64 B), KiB -> bytes"}
        # per launch shape (grid size) of the dominant kernel: which launches re-read
        by_grid = {}
        for path, cname, col in ((fpath, "FETCH_SIZE", 0), (wpath, "WRITE_SIZE", 1)):
            with open(path) as f:
                for r in csv.DictReader(f):
                    if r["Counter_Name"] == cname and DOMINANT in r["Kernel_Name"]:
                        d = by_grid.setdefault(int(float(r.get("Grid_Size", 0))), [0, 0.0, 0, 0.0])
                        d[2 * col] += 1
                        d[2 * col + 1] += float(r["Counter_Value"]) * 1024.0 * (2.0 if col == 0 else 1.0)
        if traffic:
            # every kernel's PMC bytes per dispatch, the 12 with the most fetched bytes
            top = sorted(fe.items(), key=lambda kv: -kv[1][1])[:12]
            traffic["top_kernels"] = {
                name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:80]: {"dispatches": n, "fetch_bytes": round(2.0 * v / n * 1024.0),
                                          "write_bytes": round(wr.get(name, (1, 0.0))[1] / max(wr.get(name, (1, 0.0))[0], 1)
                                                               * 1024.0)}
                for name, (n, v) in top}
            traffic["by_grid_size"] = {str(g): {"fetch_bytes": round(v[1] / max(v[0], 1)),
                                                "write_bytes": round(v[3] / max(v[2], 1)),
                                                "dispatches": v[0]} for g, v in sorted(by_grid.items())}
        lines += ["", "PMC HBM traffic of the dominant kernel (separate --pmc passes): "
                      f"{json.dumps(traffic)}"]
    open(os.path.join(dst, f"{tag}_kernel_stats.md"), "w").write("\n".join(lines) + "\n")
    if traffic:
        json.dump(traffic, open(os.path.join(dst, f"{tag}_traffic.json"), "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
