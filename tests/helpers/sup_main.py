"""torchrun worker for tests/test_supervise.py: supervise helpers/sup_child.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tdfo_amd.utils.supervise import supervise  # noqa: E402

child = [sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)), "sup_child.py"),
         sys.argv[1]]
sys.exit(supervise(child, attempts=[{}, {"TDFO_COMM": "torch"}], fallback_argv=[["--fb"]],
                   timeout_s=120))
