"""The C-ABI from C (tools/capi/capi_smoke.c): what a non-Python host (cgo / JNI / plain C) binding sees.

CPU: build the program against the in-tree library and check the error contract (bad dimensions, NULL
engine: -1 + wm_last_error, never an abort).  GPU: the prebuilt plain and host-sanitized (ASan + UBSan on the
library's host C++ and the program; `make -C tools/capi asan`) binaries run a whole tiny-dims engine through
the C-ABI — every weight enumerated and uploaded, log-mel, encode, cross-KV, greedy and beam generate,
forward, align."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CAPI = os.path.join(ROOT, "tools", "capi")
LIB = os.path.join(ROOT, "vlog_amd", "libwhisper_mi355.so")


@pytest.mark.skipif(not os.path.isfile(LIB) or not shutil.which("make"), reason="library not built")
def test_c_error_contract_builds_and_runs():
    subprocess.run(["make", "-C", CAPI, "-s"], check=True, capture_output=True, timeout=300)
    exe = os.path.join(CAPI, "out", "capi", "capi_smoke")
    env = dict(os.environ, HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", ""))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "capi_smoke:" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["capi/capi_smoke", "asan/capi_smoke_asan"])
def test_c_smoke_on_gpu(variant):
    exe = os.path.join(CAPI, "out", *variant.split("/"))
    if not os.path.isfile(exe):
        pytest.skip(f"{exe} not built (make -C tools/capi all asan)")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "capi_smoke: ok" in r.stdout, r.stdout
