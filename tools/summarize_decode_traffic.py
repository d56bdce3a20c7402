"""HBM traffic of one decode run (cfg3, or cfg5 with --longform) from the two PMC passes of
tools/decode_traffic.py (dev tool).  Sums FETCH_SIZE x 2 (gfx950 counts 128-B requests as 64 B) + WRITE_SIZE
(KiB -> bytes) over every dispatch from the encoder's embedding lookup to the end of the
run, and separately over the decode steps alone (first to last attn_decode dispatch).
Writes profiles/<tag>_decode_traffic.json, or profiles/<tag>_longform_traffic.json when
<src>/decode_run.json (written by the traffic run's --out=<src>) says the run was cfg5.

    python tools/summarize_decode_traffic.py gpurun_out/dtr r04
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEC_BYTES = 2.019e11   # SURVEY 8(d) cfg3 algorithmic bytes per run
DEC_T = 800


def per_dispatch(path, counter):
    rows = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            d = int(r["Dispatch_Id"])
            name, v = rows.get(d, (r["Kernel_Name"], 0.0))
            rows[d] = (name, v + float(r["Counter_Value"]))
    return rows


def main(src, tag):
    fe = per_dispatch(os.path.join(src, "fetch"), "FETCH_SIZE")
    wr = per_dispatch(os.path.join(src, "write"), "WRITE_SIZE")

    def window(rows):
        ids = sorted(rows)
        start = max(i for i in ids if "embed_fwd_kernel" in rows[i][0])
        dec = [i for i in ids if "attn_decode_kernel" in rows[i][0]]
        run = [i for i in ids if i >= start]
        steps = [i for i in ids if dec[0] <= i <= dec[-1]]
        return run, steps

    fr, fs = window(fe)
    wrr, ws = window(wr)
    fetch_run = 2.0 * 1024 * sum(fe[i][1] for i in fr)
    write_run = 1024 * sum(wr[i][1] for i in wrr)
    fetch_steps = 2.0 * 1024 * sum(fe[i][1] for i in fs)
    write_steps = 1024 * sum(wr[i][1] for i in ws)
    run_info = os.path.join(src, "decode_run.json")
    info = json.load(open(run_info)) if os.path.exists(run_info) else {"kind": "decode", "steps": DEC_T,
                                                                       "algorithmic_bytes_per_run": DEC_BYTES}
    lf = info["kind"] == "longform"
    steps, algo = info["steps"], info["algorithmic_bytes_per_run"]
    out = {
        "workload": ("cfg5 long-form run: B=64 fp16 decode steps until every injected stop + post-net"
                     if lf else "cfg3 decode run: encoder + 800 forced decode steps + post-net")
                    + " (tools/decode_traffic.py, steps launched eagerly: the graph's kernels)",
        "steps": steps, "dispatches_run": len(fr), "dispatches_steps": len(fs),
        "dispatches_per_step": len(fs) / steps,
        "hbm_bytes_per_run": fetch_run + write_run, "fetch_bytes_per_run": fetch_run, "write_bytes_per_run": write_run,
        "hbm_bytes_per_step": (fetch_steps + write_steps) / steps,
        "algorithmic_bytes_per_run": algo,
        "traffic_over_algorithmic": (fetch_run + write_run) / algo,
        "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; FETCH_SIZE x2 (gfx950), KiB -> bytes; "
                  "Infinity-Cache hits are counted by these counters (MI355X_MICROARCH.md)",
    }
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    name = f"{tag}_longform_traffic.json" if lf else f"{tag}_decode_traffic.json"
    json.dump(out, open(os.path.join(ROOT, "profiles", name), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "r02")
