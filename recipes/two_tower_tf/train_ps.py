"""Parameter-server TwoTower training (reference: tensorflow2/train_ps.py).

The gRPC parameter servers are replaced by sharded embedding tables in HBM
(row-wise by default, all-to-all over xGMI); cluster.json is read only to
report the requested topology. Writes ./ckpt (per-epoch sharded checkpoints),
./backup (resume point, restored automatically, removed on success) and
./log/metrics.jsonl.
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train_ps.py
"""
from pathlib import Path

import _path  # noqa: F401
from _bootstrap import config
from tdfo_amd.utils.guarded import supervised
from tdfo_amd.config import read_cluster
from tdfo_amd.train.two_tower import run


def main():
    cl = read_cluster(Path(__file__).resolve().parent / "cluster.json")
    print(f"===== cluster.json: {cl['num_workers']} workers, {cl['num_ps']} ps "
          "-> sharded embeddings over the launched ranks =====")
    run(config(__file__), mode="ps", flavor="keras")


if __name__ == "__main__":
    supervised(main)
