"""Data-parallel TwoTower training, Keras flavor (reference: tensorflow2/train_dp.py,
MirroredStrategy -> one process per GPU over RCCL)."""
import _path  # noqa: F401
from _bootstrap import config
from tdfo_amd.utils.guarded import supervised
from tdfo_amd.train.two_tower import run

if __name__ == "__main__":
    supervised(lambda: run(config(__file__), mode="dp", flavor="keras"))
