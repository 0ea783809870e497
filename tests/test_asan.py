"""Host AddressSanitizer run of the C ABI: scripts/asan_check.sh rebuilds
libpetdiff.so with ASan on its host code and the MH C checker with clang ASan, then runs
tests/test_abi.py and tests/test_cpu_mh.py against those builds (LD_PRELOAD of the clang ASan
runtime, halt_on_error).  CPU only; about a minute for the first (uncached) build."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c_abi_and_mh_checker_under_asan():
    r = subprocess.run(['bash', os.path.join(ROOT, 'scripts', 'asan_check.sh')], capture_output=True, text=True,
                       timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert 'ERROR: AddressSanitizer' not in out
    assert ' passed' in out
