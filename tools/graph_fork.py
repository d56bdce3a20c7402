"""Do hipGraph branches run concurrently? (dev tool, GPU)

Captures K under-filled GEMM launches (2048x512x512: 32 workgroups) on a side stream
alongside K launches of a second independent GEMM chain on the capture stream (fork /
join through events), and compares the replay time with the two chains captured
serially on one stream."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
import torch  # noqa: E402

from tt2 import ops  # noqa: E402


def main():
    K = 20
    dev = "cuda"
    A = [torch.randn(2048, 512, device=dev).bfloat16() for _ in range(2)]
    W = [torch.randn(512, 512, device=dev).bfloat16() for _ in range(2)]
    C = [torch.empty(2048, 512, device=dev).bfloat16() for _ in range(2)]
    big_a = torch.randn(12800, 512, device=dev).bfloat16()
    big_w = torch.randn(2048, 512, device=dev).bfloat16()
    big_c = torch.empty(12800, 2048, device=dev).bfloat16()

    def chain(i):
        for _ in range(K):
            ops.gemm(A[i], W[i], C[i], 2048, 512, 512, 512, 512, 512)

    def bigchain():
        for _ in range(K // 4):
            ops.gemm(big_a, big_w, big_c, 12800, 2048, 512, 512, 512, 2048)

    for _ in range(2):
        chain(0); chain(1); bigchain()
    torch.cuda.synchronize()

    def capture(fork, second):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        side = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            g.capture_begin(capture_error_mode="thread_local")
            if fork:
                ev = torch.cuda.Event()
                ev.record(s)
                side.wait_event(ev)
                with torch.cuda.stream(side):
                    chain(0)
                second()
                ev2 = torch.cuda.Event()
                ev2.record(side)
                s.wait_event(ev2)
            else:
                chain(0)
                second()
            g.capture_end()
        torch.cuda.current_stream().wait_stream(s)
        return g

    def timeit(g):
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            g.replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / 10 * 1e6

    for name, second in (("small||small", lambda: chain(1)), ("small||big", bigchain)):
        ser = timeit(capture(False, second))
        par = timeit(capture(True, second))
        print(f"{name}: serial {ser:.1f} us, forked {par:.1f} us", flush=True)


if __name__ == "__main__":
    main()
