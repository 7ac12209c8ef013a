"""The native library registers every op schema at load time; a bad schema
aborts the process. Loading it here (CPU, no GPU needed) catches that before
a GPU run does."""
import subprocess
import sys
from pathlib import Path

import pytest

LIB = Path(__file__).resolve().parents[1] / "tdfo_amd" / "lib" / "libtdfo_hip.so"


@pytest.mark.skipif(not LIB.exists(), reason="native library not built")
def test_native_library_registers_ops():
    code = ("import torch; torch.ops.load_library(%r); "
            "import tdfo_amd.ops as o; n = o._native(); "
            "assert hasattr(n, 'dense_optimizer') and hasattr(n, 'attention_fwd'); print('ok')"
            % str(LIB))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]
