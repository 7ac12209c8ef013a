"""Data-parallel DLRM (BASELINE config 3): one process per GPU, dense gradients
all-reduced over RCCL; tables up to 256 MB replicated on every rank (their
dense fp32 gradient all-reduced, or ids + pooled gradients all-gathered), the
larger ones owner-partitioned row-wise (sparse/planner.py "data_parallel"):
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train_dp.py"""
import _path  # noqa: F401
from _bootstrap import config
from tdfo_amd.utils.guarded import supervised
from tdfo_amd.train.dlrm import run

if __name__ == "__main__":
    supervised(lambda: run(config(__file__), mode="dp"))
