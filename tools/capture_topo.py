"""Minimal stream-capture topologies (dev tool, GPU): which fork/join pattern makes
hipStreamEndCapture segfault (round 5: SyncBatchNorm exchanges issued from the encoder's side
stream, tools/capture_probe.py).  One topology per process; tiny elementwise kernels only.

    python tools/capture_topo.py <topo>

O = capture origin, S = side stream, C = comm stream; "X<-Y" = X waits on Y's last work.
  simple    O: k; S<-O; S: k; O<-S
  nested2o  O: k; S<-O; S: k; C<-S; C: k; O<-C; O<-S           (C forked from S, joined into O)
  nested2s  O: k; S<-O; S: k; C<-S; C: k; S<-C; S: k; O<-S     (C forked from S, joined into S)
  refork    nested2s, then C<-O; C: k; O<-C                      (C forked again, from O)
  reforks   nested2s, then S<-O; S: k; C<-S; C: k; O<-C; O<-S  (C forked again, from S)
Prints the join status of S and C before the end and "TOPO OK <topo>" after a replay."""
import faulthandler
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))

import torch  # noqa: E402

from tt2.capture import StepCapture, joined_status  # noqa: E402


def main():
    faulthandler.enable()
    topo = sys.argv[1]
    x = torch.zeros(1 << 20, device="cuda")
    O, S, C = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    O.wait_stream(torch.cuda.current_stream())
    torch.cuda.synchronize()

    def k(s, v):
        with torch.cuda.stream(s):
            x.add_(v)

    def nested2s():
        k(O, 1)
        S.wait_stream(O)
        k(S, 2)
        C.wait_stream(S)
        k(C, 3)
        S.wait_stream(C)
        k(S, 4)
        O.wait_stream(S)

    g = torch.cuda.CUDAGraph()
    with StepCapture(g, O, lambda: {"S": S, "C": C}):
        if topo == "simple":
            k(O, 1)
            S.wait_stream(O)
            k(S, 2)
            O.wait_stream(S)
        elif topo == "nested2o":
            k(O, 1)
            S.wait_stream(O)
            k(S, 2)
            C.wait_stream(S)
            k(C, 3)
            O.wait_stream(C)
            O.wait_stream(S)
        elif topo == "nested2s":
            nested2s()
        elif topo == "refork":
            nested2s()
            C.wait_stream(O)
            k(C, 5)
            O.wait_stream(C)
        elif topo == "reforks":
            nested2s()
            S.wait_stream(O)
            k(S, 5)
            C.wait_stream(S)
            k(C, 6)
            O.wait_stream(C)
            O.wait_stream(S)
        else:
            raise SystemExit(f"unknown topology {topo}")
        print("status", joined_status(O, {"S": S, "C": C}), flush=True)
    g.replay()
    torch.cuda.synchronize()
    print("TOPO OK", topo, x[0].item(), flush=True)


if __name__ == "__main__":
    main()
