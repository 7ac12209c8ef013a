"""§5.2 race / memory-error detection for the host C++ runtime: the data
library (threaded loader, TFRecord codec, synthetic generator) is built with
ASan+UBSan and with TSan and driven by csrc/data/tests/selftest.cpp. Host
code only (GPU sanitizers and XNACK are not available on the MI355X pool)."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SRCS = sorted(str(p) for p in (ROOT / "csrc" / "data").glob("*.cpp"))
DRIVER = str(ROOT / "csrc" / "data" / "tests" / "selftest.cpp")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_data_library_under_sanitizer(san, tmp_path):
    exe = tmp_path / "selftest"
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-pthread", f"-fsanitize={san}",
           "-fno-omit-frame-pointer", *SRCS, DRIVER, "-o", str(exe), "-lz"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    env = {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1",
           "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1",
           "TSAN_OPTIONS": "halt_on_error=1", "PATH": "/usr/bin:/bin"}
    r = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, timeout=600,
                       env=env)
    assert r.returncode == 0 and "selftest ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
