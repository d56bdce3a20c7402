"""Work-group timeline of one GEMM launch (dev tool, GPU): per-work-group {start, end} from the
launch probe's span record, for a shape under given variants (replayed warm, then the last
launch's records): work groups, span, median / max duration, starts by round.

    python tools/gemm_wgt.py m n k [variant ...] [--epi brd]
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
import torch  # noqa: E402

from tt2 import ops  # noqa: E402
from tt2._lib import ACT_RELU, lib  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    epi = sys.argv[sys.argv.index("--epi") + 1] if "--epi" in sys.argv else ""
    if epi in args:
        args.remove(epi)
    m, n, k = (int(x) for x in args[:3])
    variants = [int(x) for x in args[3:]] or [13]
    A = torch.randn(m, k, device="cuda").bfloat16()
    B = (torch.randn(n, k, device="cuda") / k ** 0.5).bfloat16()
    C_ = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
    seed = torch.tensor([7], dtype=torch.int32, device="cuda")
    kw = {}
    if "b" in epi:
        kw["bias"] = torch.randn(n, device="cuda")
    if "r" in epi:
        kw["act"] = ACT_RELU
    if "d" in epi:
        kw["drop"] = ops.Drop(seed, 5, 0.1)
    L = lib()
    buf = (C.c_uint64 * 16384)()
    for v in variants:
        for _ in range(5):
            ops.gemm(A, B, C_, m, n, k, k, k, n, variant=v, **kw)
        torch.cuda.synchronize()
        ops.PROBE = probe = ops.LaunchProbe()
        try:
            ops.gemm(A, B, C_, m, n, k, k, k, n, variant=v, **kw)
            torch.cuda.synchronize()
            slot = probe.rec[0][2]
            cnt = L.tt2_probe_span_records(slot, buf, 8192)
        finally:
            ops.PROBE = None
        us = lambda t: t / 100.0   # noqa: E731   (100 MHz wall clock -> us)
        st = [buf[2 * i] for i in range(cnt)]
        en = [buf[2 * i + 1] for i in range(cnt)]
        t0 = min(st)
        du = sorted(e - s for s, e in zip(st, en))
        starts = sorted(us(s - t0) for s in st)
        print(f"v{v} {m}x{n}x{k} {epi}: {cnt} WGs, span {us(max(en) - t0):.1f} us, WG median {us(du[cnt // 2]):.1f} "
              f"max {us(du[-1]):.1f} min {us(du[0]):.1f}")
        hist = {}
        for s in starts:
            hist[int(s // 2) * 2] = hist.get(int(s // 2) * 2, 0) + 1
        print("   starts (2-us bins):", " ".join(f"{b}:{c}" for b, c in sorted(hist.items())))
        probe.close()


if __name__ == "__main__":
    main()
