"""ASan + UBSan run of the library's host code: `make -C aimet_amd/csrc sanitize` builds
every source with the host side under -fsanitize=address,undefined (device code unchanged) and links
tests/cpp/sanitize_host.cpp; here it drives the encoding math and the host TF-E / percentile / MSE /
entropy searches (tfe_core.hpp, mse_core.hpp, entropy_kl.hpp) over randomized and degenerate
statistics. The quantizer life cycle on a device (create_many / device-memory cache / host entropy
thread pool / destroy) is the `gpu` argument of the same binary (run on the MI355X box; log in
profiles/r02/sanitize_gpu.log)."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "build", "san", "sanitize_host")


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="needs hipcc")
def test_host_code_clean_under_asan_ubsan():
    subprocess.run(["make", "-s", "-j", str(min(8, os.cpu_count() or 2)), "-C",
                    os.path.join(REPO, "aimet_amd", "csrc"), "sanitize"], check=True, capture_output=True,
                   timeout=900)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([BIN], env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr, p.stderr[-4000:]
    assert "sanitize_host: clean" in p.stdout
