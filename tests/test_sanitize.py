"""ASan + UBSan run of the library's host code: `make -C aimet_amd/csrc sanitize` builds
every source with the host side under -fsanitize=address,undefined (device code unchanged) and links
tests/cpp/sanitize_host.cpp; here it drives the encoding math and the host TF-E / percentile / MSE /
entropy searches (tfe_core.hpp, mse_core.hpp, entropy_kl.hpp) over randomized and degenerate
statistics. The quantizer life cycle on a device (create_many / device-memory cache / host entropy
thread pool / destroy) is the `gpu` argument of the same binary: its plain build, linked against
the product library (tests/cpp/bin/sanitize_host_plain, built by __graft_entry__.build()), runs
under -m gpu on the legacy null stream and on a created stream -- the driver that faulted while
device scratch came from the stream-ordered pool (profiles/r02/sanitize_gpu.log)."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "build", "san", "sanitize_host")
PLAIN = os.path.join(REPO, "tests", "cpp", "bin", "sanitize_host_plain")


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


@pytest.mark.gpu
@pytest.mark.parametrize("stream", [[], ["stream"]], ids=["null_stream", "created_stream"])
def test_device_lifecycle_scratch_reuse_on_gpu(stream):
    """create_many -> batched statistics (job tables uploaded into reused scratch) -> batched
    TF-E / MSE / entropy searches -> destroy, 60 rounds (`long`), on the legacy null stream and on a
    created stream; any fault, error status or unclean exit fails."""
    from conftest import gpu_available
    if not gpu_available():
        pytest.skip("needs an MI355X")
    assert os.path.exists(PLAIN), "build the driver first: make -C aimet_amd/csrc plain_driver"
    p = subprocess.run([PLAIN, "gpu", "long"] + stream, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "sanitize_host: clean" in p.stdout
