"""Sharded-embedding DLRM / DCN-v2 (BASELINE configs 4-5; the reference's
parameter-server entry point collapsed into in-node table/row-wise sharding):
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train_ps.py \
      (TDFO_CONFIG=config_1tb.toml or config_dcnv2.toml)"""
import _path  # noqa: F401
from _bootstrap import config
from tdfo_amd.utils.guarded import supervised
from tdfo_amd.train.dlrm import run

if __name__ == "__main__":
    supervised(lambda: run(config(__file__), mode="ps"))
