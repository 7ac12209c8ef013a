"""Bert4Rec training (reference: torchrec/train.py).
  python train.py                                  # one rank
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train.py
model_parallel=true shards the item table over ranks (DMP); false replicates it (DDP)."""
import _path  # noqa: F401
from _bootstrap import config
from tdfo_amd.utils.guarded import supervised
from tdfo_amd.train.bert4rec import run

if __name__ == "__main__":
    supervised(lambda: run(config(__file__)))
