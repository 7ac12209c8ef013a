"""Bert4Rec ETL (reference: torchrec/preprocessing.py) ->
data_dir/parquet_bert4rec/{train,eval}_part_{1,2}.parquet + size_map_bert4rec.json."""
import _path  # noqa: F401
from _bootstrap import config
from tdfo_amd.data.bert4rec_etl import run_etl

if __name__ == "__main__":
    cfg = config(__file__)
    print(run_etl(cfg.data_dir, cfg.max_len, cfg.sliding_step, cfg.mask_prob, cfg.seed))
