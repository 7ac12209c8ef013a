"""Goodreads ETL, TF flavor (reference: tensorflow2/preprocessing.py + data.py):
GZIP TFRecord parts (or parquet, per `write_format`) + size_map.json +
{train,eval}_data_size.json."""
import _path  # noqa: F401
from _bootstrap import config
from tdfo_amd.data.goodreads import run_etl

if __name__ == "__main__":
    cfg = config(__file__)
    run_etl(cfg.data_dir, fmt=cfg.write_format)
