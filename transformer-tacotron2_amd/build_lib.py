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


# --asan: the host side of every source under AddressSanitizer (device code unchanged; GPU
# sanitizers are not available) into build_asan/libtt2_asan.so, for CPU tests of the host
# logic (size queries, plans, validation) with the runtime preloaded (tests/test_asan_host.py)
ASAN_FLAGS = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer"]
ASAN_BUILD = os.path.join(PKG, "build_asan")
ASAN_OUT = os.path.join(ASAN_BUILD, "libtt2_asan.so")


def _compile(src: str, obj: str, asan: bool = False) -> tuple[str, int, str]:
    cmd = [HIPCC] + FLAGS + (ASAN_FLAGS if asan else []) + EXTRA.get(os.path.basename(src), []) + ["-c", src,
                                                                                                  "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    return src, r.returncode, r.stdout + r.stderr


def build(jobs: int = 8, verbose: bool = False, asan: bool = False) -> str:
    build_dir, out = (ASAN_BUILD, ASAN_OUT) if asan else (BUILD, OUT)
    os.makedirs(build_dir, exist_ok=True)
    srcs = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))
    hmt = _headers_mtime()
    todo, objs = [], []
    for f in srcs:
        src = os.path.join(CSRC, f)
        obj = os.path.join(build_dir, f + ".o")
        objs.append(obj)
        if not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), hmt):
            todo.append((src, obj))
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for src, rc, log in ex.map(lambda so: _compile(*so, asan=asan), todo):
            if rc != 0:
                raise RuntimeError(f"hipcc failed on {src}:\n{log}")
            if verbose:
                print(f"compiled {os.path.basename(src)}", flush=True)
    if todo or not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs
        if asan:
            cmd += ["-fsanitize=address", "-shared-libsan"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n" + r.stdout + r.stderr)
        if verbose:
            print("linked", out, flush=True)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--asan", action="store_true", help="host-side AddressSanitizer build (build_asan/)")
    a = ap.parse_args()
    print(build(a.j, verbose=True, asan=a.asan))
    sys.exit(0)
