"""Per-queue timeline of one timed training step from a rocprofv3 kernel trace (dev tool, CPU):
which hardware queue each kernel ran on and when, from a given offset into the step, so the
overlapped backward's side-stream work can be read against the encoder chain.

    python tools/stream_timeline.py gpurun_out/<dir> [from_ms] [count]
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_step import short  # noqa: E402


def main(src, from_ms=0.0, count=80):
    trace = next(os.path.join(d, f) for d, _, fs in os.walk(src) for f in fs if f.endswith("kernel_trace.csv"))
    bench = json.loads([ln for ln in open(os.path.join(src, "bench_step.json")) if ln.startswith("{")][-1])
    K, W = bench["steps"], bench["warmup"]
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"])
                for r in csv.DictReader(open(trace)))
    adam = [e for e in ev if e[2].startswith("adam")]
    t0, t1 = adam[W + 1][1], adam[W + 2][1]
    win = [e for e in ev if t0 <= e[0] and e[1] <= t1]
    busy = defaultdict(float)
    for e in win:
        busy[e[3]] += (e[1] - e[0]) / 1e6
    print("step %.3f ms; busy per queue (ms): %s" % ((t1 - t0) / 1e6, {q: round(v, 3) for q, v in busy.items()}))
    for e in [e for e in win if (e[0] - t0) / 1e6 >= from_ms][:count]:
        print("%8.3f %7.2f q%s %s" % ((e[0] - t0) / 1e3, (e[1] - e[0]) / 1e3, e[3], e[2][:56]))


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 0.0, int(sys.argv[3]) if len(sys.argv) > 3 else 80)
