"""The C ABI's host-side logic under AddressSanitizer (SURVEY §5 aux: host ASan debug
build), on CPU: build_lib.py --asan instruments the host code of every source (device code
unchanged; GPU sanitizers are not available on this pool), and the host-only C-ABI tests
(tests/test_capi.py: symbol exports, struct layouts, block size queries, plans and
validation errors) run against it with the ASan runtime preloaded."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))


def test_capi_under_asan():
    import build_lib
    rt = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    if not rt:
        pytest.skip("no ASan runtime in this image")
    lib = build_lib.build(jobs=min(8, os.cpu_count() or 4), asan=True)
    env = dict(os.environ, LD_PRELOAD=rt[-1], ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", TT2_LIB=lib)
    check = ("import sys; sys.path.insert(0, 'transformer-tacotron2_amd'); from tt2 import _lib; "
             "_lib.load(); print(open('/proc/self/maps').read().count('libtt2_asan.so') > 0)")
    r = subprocess.run([sys.executable, "-c", check], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and r.stdout.strip() == "True", r.stderr[-2000:]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_capi.py")], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "AddressSanitizer" not in r.stderr
