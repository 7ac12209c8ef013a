"""Data-parallel TwoTower training (reference: jax-flax/train_dp.py).
One process per GPU over RCCL:
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train_dp.py
(plain `python train_dp.py` runs one rank)."""
import _path  # noqa: F401
from _bootstrap import config
from tdfo_amd.utils.guarded import supervised
from tdfo_amd.train.two_tower import run

if __name__ == "__main__":
    supervised(lambda: run(config(__file__), mode="dp", flavor="flax"))
