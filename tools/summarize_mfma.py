"""MFMA-busy evidence from a rocprofv3 PMC pass (dev tool, CPU):

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/prof_mfma -o run \
        --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-decode --no-cpu-baseline --no-ragged
    python tools/summarize_mfma.py gpurun_out/prof_mfma/run_counter_collection.csv profiles/r01g_mfma_busy.json

Per kernel: mean SQ_VALU_MFMA_BUSY_CYCLES per launch (summed over the chip's SIMDs), the
launch duration under the profiler, and busy / (1024 SIMDs x duration x 2.4 GHz): the
fraction of the chip's matrix-pipe cycles that were busy.  For the v7 GEMM the busy cycles
per launch divided by the algorithmic MFMA count (2MNK / 16384 per v_mfma_f32_16x16x32_bf16)
give the cycles per MFMA: 16 means the kernel issues no MFMA work beyond the algorithmic."""
import csv
import json
import sys
from collections import defaultdict

SIMDS, CLOCK = 1024, 2.4e9


def main(src, dst):
    per = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(src)):
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        per[r["Kernel_Name"]][r["Counter_Name"]].append((float(r["Counter_Value"]), dur))
    out = {}
    for k, v in per.items():
        b = v.get("SQ_VALU_MFMA_BUSY_CYCLES")
        if not b:
            continue
        n = len(b)
        busy = sum(x[0] for x in b) / n
        dur = sum(x[1] for x in b) / n
        if busy <= 0:
            continue
        out[k] = {"launches": n, "mfma_busy_cycles_per_launch": busy, "duration_us_under_profiler": dur * 1e6,
                  "busy_fraction": busy / (SIMDS * dur * CLOCK)}
    top = dict(sorted(out.items(), key=lambda kv: -kv[1]["mfma_busy_cycles_per_launch"] * kv[1]["launches"])[:12])
    json.dump({"source": src, "simds": SIMDS, "clock_hz": CLOCK, "kernels": top}, open(dst, "w"), indent=1)
    for k, v in top.items():
        print(f"{k[:60]:60s} {v['launches']:5d} busy/launch {v['mfma_busy_cycles_per_launch']:.3e} "
              f"{v['duration_us_under_profiler']:6.1f} us  busy {v['busy_fraction']:.3f}")


if __name__ == "__main__":
    main(*sys.argv[1:3])
