"""Child of tests/helpers/sup_main.py: rendezvous (per-attempt store
prefix), one gloo all-reduce, then the exit code the scenario prescribes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from tdfo_amd.parallel import dist as tdist  # noqa: E402

scenario = sys.argv[1]
attempt = int(os.environ["TDFO_ATTEMPT"])
info = tdist.init_distributed("cpu", "gloo", timeout_s=60)
t = torch.ones(1)
torch.distributed.all_reduce(t)
assert t.item() == info.world_size
codes = {"ok": [[0, 0], [9, 9]], "watchdog": [[0, 3], [0, 0]], "diverged": [[4, 4], [0, 0]],
         "crash": [[-11 & 0xFF, 0], [0, 0]], "both": [[3, 3], [5, 5]]}[scenario]
rc = codes[attempt][info.rank]
print(f"child rank={info.rank} attempt={attempt} comm={os.environ.get('TDFO_COMM')} "
      f"fb={'--fb' in sys.argv} rc={rc}", flush=True)
tdist.reset()
sys.exit(rc)
