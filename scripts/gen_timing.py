"""Time the C++ synthetic Criteo generator per batch at several thread counts."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tdfo_amd.data.synthetic import HostSyntheticCriteo  # noqa: E402
from tdfo_amd.models.dlrm import CRITEO_1TB_ROWS  # noqa: E402

for th in (1, 8, 12, 16):
    g = HostSyntheticCriteo(CRITEO_1TB_ROWS, 8192, seed=1, threads=th, nbuf=3)
    g.batch(0)
    t = time.perf_counter()
    for i in range(20):
        g.batch(i)
    print(th, "threads:", round((time.perf_counter() - t) / 20 * 1e3, 3), "ms/batch", flush=True)
