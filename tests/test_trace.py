"""roctx ranges (SURVEY §5 tracing aux): the switch and the library binding, on CPU."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(env_val):
    code = ("import sys; sys.path.insert(0, 'transformer-tacotron2_amd'); from tt2 import trace; "
            "f = trace.ranged('t')(lambda a: a + 1); "
            "r = trace.Range('r'); r.__enter__(); r.__exit__(None, None, None); "
            "print(f(1), hasattr(f, '__wrapped__'), trace._roctx is not None)")
    env = dict(os.environ, TT2_ROCTX=env_val)
    return subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=120)


def test_roctx_off_is_identity():
    r = _run("0")
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["2", "False", "False"]


def test_roctx_on_pushes_ranges():
    r = _run("1")
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["2", "True", "True"]
