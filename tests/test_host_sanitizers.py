"""The engine's host code under AddressSanitizer + UndefinedBehaviorSanitizer (the reference's CI runs
its own tests with ASan + UBSan, /root/reference/.github/workflows/ci.yml:24-25).

`make -C hsig-picotls_amd asan` compiles the host units with -fsanitize=address,undefined (device code objects unchanged)
into asan/host_check (tests/host_check/host_check.cpp), which drives, without a GPU, every host path that reads caller
or wire bytes: 100 000 random and damaged TLS record streams through ptls_hip_tls13_parse (each in an exactly-sized heap
buffer, so a one-byte over-read is a report), the record framing, the launch planner on random descriptor sets, the
byte partition, and the C ABI's argument checks and no-device paths.  A sanitizer report aborts the driver.  (The Python
CPU suite loads the product library through ctypes into an uninstrumented interpreter, so the sanitized build is
exercised by this native driver instead.)"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "hsig-picotls_amd", "asan", "host_check")


@pytest.mark.skipif(shutil.which("g++") is None or not os.path.exists("/opt/rocm/include/hip"), reason="g++ / HIP headers missing")
def test_host_code_is_clean_under_asan_ubsan():
    r = subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "hsig-picotls_amd"), "asan"], capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([BIN, "1"], capture_output=True, text=True, timeout=900, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "host_check: ok (0 failed checks)" in out, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]


@pytest.mark.gpu
def test_host_pipelines_clean_under_asan_ubsan_on_device():
    """the same driver on the GPU box (argument "device"): 80 random pipeline layouts per key size -- both transports,
    64 KiB and 1 MiB slices, records in and out of output order, 1-64-byte gaps, exactly-sized heap buffers for the copy
    transport -- sealed and opened back, every record compared with the CPU oracle and every byte between records checked
    unchanged, with pipeline.cpp's slicing and gap planning instrumented (the kernels are the product's).  Built here by
    __graft_entry__.build() (make tests-builds); the GPU box runs the shipped binary."""
    if not os.path.exists(BIN):
        pytest.skip("asan/host_check not built (make -C hsig-picotls_amd asan)")
    env = dict(os.environ, ASAN_OPTIONS="protect_shadow_gap=0:detect_leaks=0:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([BIN, "device", "40"], capture_output=True, text=True, timeout=600, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "host_check: ok (0 failed checks)" in out and "device paths run" in out, out[-4000:]
