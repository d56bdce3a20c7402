"""Build libtt2.so (gfx950) in-tree: csrc/*.hip + csrc/*.cpp -> tt2/libtt2.so.

Plain hipcc, one object per source compiled in parallel, incremental on
source/header mtimes.  Usage: python transformer-tacotron2_amd/build_lib.py [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
BUILD = os.path.join(PKG, "build")
OUT = os.path.join(PKG, "tt2", "libtt2.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I" + INCLUDE, "-I" + CSRC,
         "-Wno-unused-result"]
# Per-file extras.  Attention keeps MFMA accumulators in arch VGPRs: its softmax reads
# and rescales them every tile, and the default AGPR placement adds a copy per use.
EXTRA = {"attention.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]}


def _headers_mtime() -> float:
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs += [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE) if f.endswith(".h")]
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _compile(src: str, obj: str) -> tuple[str, int, str]:
    cmd = [HIPCC] + FLAGS + EXTRA.get(os.path.basename(src), []) + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    return src, r.returncode, r.stdout + r.stderr


def build(jobs: int = 8, verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))
    hmt = _headers_mtime()
    todo, objs = [], []
    for f in srcs:
        src = os.path.join(CSRC, f)
        obj = os.path.join(BUILD, f + ".o")
        objs.append(obj)
        if not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), hmt):
            todo.append((src, obj))
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for src, rc, log in ex.map(lambda so: _compile(*so), todo):
            if rc != 0:
                raise RuntimeError(f"hipcc failed on {src}:\n{log}")
            if verbose:
                print(f"compiled {os.path.basename(src)}", flush=True)
    if todo or not os.path.exists(OUT) or os.path.getmtime(OUT) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n" + r.stdout + r.stderr)
        if verbose:
            print("linked", OUT, flush=True)
    return OUT


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 4))
    a = ap.parse_args()
    print(build(a.j, verbose=True))
    sys.exit(0)
