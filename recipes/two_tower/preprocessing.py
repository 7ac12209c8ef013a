"""Goodreads ETL -> data_dir/parquet/{train,eval}_part_{1..8}.parquet + size_map.json
(reference: jax-flax/preprocessing.py). `python preprocessing.py`"""
import _path  # noqa: F401
from _bootstrap import config
from tdfo_amd.data.goodreads import run_etl

if __name__ == "__main__":
    cfg = config(__file__)
    run_etl(cfg.data_dir, fmt="parquet")
