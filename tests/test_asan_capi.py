"""Host-side AddressSanitizer run of the C-ABI validation layer (tools/asan_capi.py), CPU.

Runs when the ASan build exists (`make -C tensorflow2-machine-vision_amd asan`, ~2 min, not
part of the default build); the committed log of the last run is profiles/r03_asan_capi.log."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tensorflow2-machine-vision_amd", "lib", "libedet_asan.so")


@pytest.mark.skipif(not os.path.exists(LIB), reason="ASan build absent (make -C tensorflow2-machine-vision_amd asan)")
def test_capi_validation_under_asan():
    rt = subprocess.run(["/opt/rocm/bin/hipcc", "-print-file-name=libclang_rt.asan-x86_64.so"],
                        capture_output=True, text=True).stdout.strip()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", LD_PRELOAD=rt, EDET_LIB=LIB,
               HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "asan_capi.py")], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "asan_capi: OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
    assert "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
