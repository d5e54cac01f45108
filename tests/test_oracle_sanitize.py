"""The C oracle under AddressSanitizer + UndefinedBehaviorSanitizer (host code only; VERDICT r3
item 3): oracle/Makefile builds oracle/asan/liblgx_oracle.so with -fsanitize=address,undefined
(-fno-sanitize-recover: any UB aborts), and the oracle's own CPU tests - the golden replays of the
reference's outputs (env logic, Go1 dVel, SEA), the SEA step and the physics known-answer tests -
run against it in a child process with the ASan runtime preloaded (the python interpreter itself is
not instrumented; leak checking is off for the interpreter's arenas)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN_SO = os.path.join(ROOT, "oracle", "asan", "liblgx_oracle.so")


def _runtime():
    try:
        p = subprocess.check_output(["gcc", "-print-file-name=libasan.so"], text=True).strip()
    except (OSError, subprocess.CalledProcessError):
        return None
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.timeout(600)
def test_oracle_tests_pass_under_asan_ubsan():
    rt = _runtime()
    if rt is None:
        pytest.skip("no gcc ASan runtime on this host")
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan/liblgx_oracle.so"])
    env = dict(os.environ, LD_PRELOAD=rt, LGX_ORACLE_SO=ASAN_SO, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", PYTHONDONTWRITEBYTECODE="1")
    # the sanitized build is the one the child process maps
    probe = ("import sys; sys.path.insert(0, 'tests'); import oracle_backend as o; o.load_oracle(); "
             "maps = open('/proc/self/maps').read(); assert o.ORACLE_SO.endswith('asan/liblgx_oracle.so'); "
             "assert 'asan/liblgx_oracle.so' in maps and 'libasan' in maps; print('sanitized oracle mapped')")
    r = subprocess.run([sys.executable, "-c", probe], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "sanitized oracle mapped" in r.stdout, r.stderr[-2000:]
    tests = [os.path.join("tests", t) for t in ("test_golden.py", "test_sea.py", "test_oracle_physics.py")]
    r = subprocess.run([sys.executable, "-m", "pytest", *tests, "-x", "-q", "-p", "no:cacheprovider"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=540)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert " passed" in r.stdout and "error" not in r.stderr.lower(), r.stderr[-2000:]
