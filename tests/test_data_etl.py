"""Goodreads ETL transforms, TFRecord codec, C++ host loader,
HBM-resident columnar batches and the typed config."""
import gzip
import json
import struct
from pathlib import Path

import numpy as np
import pytest
import torch

from tdfo_amd.config import from_dict, read_configs
from tdfo_amd.data import goodreads as G
from tdfo_amd.data import native as N
from tdfo_amd.data.columnar import DeviceColumns

REPO = Path(__file__).resolve().parents[1]


def test_decade_buckets_keep_reference_boundaries():
    got = G.year_to_decade(["1900", "1909", "1910", "1911", "1999", "2000", "2001", "2020",
                            "2021", "2030", "2031", "1899", "", "n/a"])
    assert list(got) == ["1900s", "1900s", "1900s", "1910s", "1990s", "1990s", "2000s", "2010s",
                         "2020s", "2020s", "unknown", "unknown", "unknown", "unknown"]


def test_continuous_transform_fills_median_and_minmax():
    vals = ["10", "", "20", "5000", "30"]
    out = G.transform_continuous(vals)
    # stats over {10, 20, 30}: min 10, max 30, median 20 fills "" and 5000
    np.testing.assert_allclose(out, [0.0, 0.5, 0.5, 0.5, 1.0])


def test_sparse_mapping_sorted_with_unknown():
    m = G.sparse_mapping(["eng", "", "spa", "eng", None])
    assert m == {"eng": 0, "spa": 1, "unknown": 2}
    np.testing.assert_array_equal(G.transform_categorical(["spa", "", "eng"], m, np.int16), [1, 2, 0])


def test_split_mask_80_20_by_sorted_book():
    user = np.array([0] * 10 + [1] * 6 + [2] * 3)
    book = np.array([9, 8, 7, 6, 5, 4, 3, 2, 1, 0, 30, 10, 20, 60, 50, 40, 7, 5, 6])
    m = G.split_mask(user, book)
    assert m[:10].sum() == 8 and set(book[:10][m[:10]]) == set(range(8))
    assert m[10:16].tolist() == [True, True, True, False, True, True]   # ceil(4.8) = 5
    assert m[16:].all()                                                  # ceil(2.4) = 3


def test_etl_end_to_end(tmp_path):
    d = tmp_path / "gr"
    G.make_synthetic_raw(d, 120, 200, seed=1, mean_inter=30)
    sm, n_tr, n_ev = G.run_etl(d, verbose=False)
    assert json.loads((d / "size_map.json").read_text()) == sm
    assert set(sm) == {"user", "item", "language", "is_ebook", "format", "publisher",
                       "pub_decade"}
    parts = sorted((d / "parquet").glob("train_part_*.parquet"))
    assert len(parts) == G.FILE_NUM
    cols = G.read_parquet_columns(str(d / "parquet" / "train_part_*.parquet"))
    assert list(cols) == G.FINAL_COLUMNS
    for k, dt in G.COLUMN_DTYPES.items():
        assert cols[k].dtype == dt, k
    ev = G.read_parquet_columns(str(d / "parquet" / "eval_part_*.parquet"))
    assert len(cols["user_id"]) == n_tr and len(ev["user_id"]) == n_ev
    # every user's eval books sort after its train books; no overlap
    for u in np.unique(ev["user_id"])[:20]:
        assert cols["item_id"][cols["user_id"] == u].max() < ev["item_id"][ev["user_id"] == u].min()
    assert 0.74 < n_tr / (n_tr + n_ev) < 0.86
    assert cols["avg_rating"].min() >= 0 and cols["avg_rating"].max() <= 1
    for k in ("language", "format", "publisher", "pub_decade", "is_ebook"):
        assert cols[k].max() < sm[k]
    # TF flavor: tfrecord parts + size sidecar, is_read/is_reviewed dropped
    G.run_etl(d, fmt="tfrecord", verbose=False)
    tf = G.read_tfrecord_columns(str(d / "tfrecord" / "train_part_*.tfrecord"))
    assert set(tf) == set(G.TFRECORD_COLUMNS)
    assert G.data_size(str(d / "tfrecord" / "train_part_*.tfrecord"), "tfrecord") == n_tr
    np.testing.assert_array_equal(np.sort(tf["user_id"]), np.sort(cols["user_id"]))


def test_legacy_sort_quirk_detaches_labels(tmp_path):
    d = tmp_path / "gr"
    G.make_synthetic_raw(d, 60, 100, seed=2, mean_inter=25)
    fixed = G.read_interactions(d)
    legacy = G.read_interactions(d, legacy_sort=True)
    # same multiset of (user, book) pairs, but labels follow different books
    a = sorted(zip(fixed["user_id"].tolist(), fixed["book_id"].tolist()))
    b = sorted(zip(legacy["user_id"].tolist(), legacy["book_id"].tolist()))
    assert a == b
    fa = {(u, bk): lb for u, bk, lb in zip(fixed["user_id"], fixed["book_id"], fixed["label"])}
    mism = sum(fa[(u, bk)] != lb for u, bk, lb in
               zip(legacy["user_id"], legacy["book_id"], legacy["label"]))
    assert mism > 0


def test_crc32c_and_tfrecord_framing(tmp_path):
    assert N.crc32c(b"123456789") == 0xE3069283
    p = tmp_path / "x.tfrecord"
    cols = {"a": np.array([1, -2, 3]), "f": np.array([0.5, 1.5, -2.0], dtype=np.float32)}
    N.tfrecord_write(str(p), cols)
    raw = gzip.open(p).read()
    ln = struct.unpack("<Q", raw[:8])[0]
    assert 0 < ln < len(raw)
    lc = struct.unpack("<I", raw[8:12])[0]
    crc = N.crc32c(raw[:8])
    assert lc == ((((crc >> 15) | (crc << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF
    back = N.tfrecord_read(str(p), {"a": "int64", "f": "float32"})
    np.testing.assert_array_equal(back["a"], cols["a"])
    np.testing.assert_array_equal(back["f"], cols["f"])
    # corruption is detected
    bad = bytearray(raw)
    bad[20] ^= 0xFF
    q = tmp_path / "bad.tfrecord"
    with gzip.open(q, "wb") as f:
        f.write(bytes(bad))
    with pytest.raises(IOError):
        N.tfrecord_read(str(q), {"a": "int64", "f": "float32"})


def test_host_loader_epochs_and_ranks():
    n = 257
    cols = {"a": np.arange(n, dtype=np.int64), "b": np.arange(n, dtype=np.int16)}
    L = N.HostLoader(cols, 16, shuffle=True, seed=5, num_workers=3, prefetch=3)
    orders = []
    for ep in range(2):
        L.set_epoch(ep)
        got = torch.cat([b["a"].clone() for b in L])
        assert sorted(got.tolist()) == list(range(n))
        orders.append(got)
    assert not torch.equal(orders[0], orders[1])
    L.set_epoch(0)
    assert torch.equal(torch.cat([b["a"].clone() for b in L]), orders[0])   # deterministic
    parts = []
    for r in range(3):
        Lr = N.HostLoader(cols, 16, shuffle=True, seed=5, drop_last=True, rank=r, world_size=3)
        parts.append(torch.cat([b["a"].clone() for b in Lr]))
        assert len(Lr) == n // 48
    u = torch.cat(parts)
    assert len(u) == (n // 48) * 48 and len(set(u.tolist())) == len(u)
    L.close()


def test_device_columns_rank_split_matches_loader_contract():
    cols = {"a": np.arange(100, dtype=np.int64)}
    dc = DeviceColumns(cols, "cpu")
    parts = [torch.cat([b["a"] for b in dc.batches(8, shuffle=True, seed=1, epoch=2, rank=r,
                                                    world_size=3)]) for r in range(3)]
    u = torch.cat(parts)
    assert sorted(u.tolist()) == list(range(100))
    assert dc.num_batches(8, 3, drop_last=True) == 4


def test_config_accepts_reference_tomls_and_rejects_typos(tmp_path):
    for rel in ("recipes/two_tower/config.toml", "recipes/two_tower_tf/config.toml"):
        cfg = read_configs(REPO / rel)
        assert cfg.embed_dim == 16 and cfg.per_device_train_batch_size == 2048
    cfg = read_configs(REPO / "recipes/two_tower_tf/config.toml")
    assert cfg.write_format == "tfrecord" and cfg.jit_xla is True
    with pytest.raises(TypeError):
        from_dict({"learning_rte": 1.0})
    with pytest.raises(ValueError):
        from_dict({"write_format": "csv"})
    with pytest.raises(ValueError):
        from_dict({"max_len": 5, "sliding_step": 10})
    p = tmp_path / "c.toml"
    p.write_text('data_dir = "d"\n')
    (tmp_path / "d").mkdir()
    (tmp_path / "d" / "size_map.json").write_text('{"user": 3}')
    cfg = read_configs(p, ["n_epochs=3", "sharding.strategy=row_wise"])
    assert cfg.size_map == {"user": 3} and cfg.n_epochs == 3
    assert cfg.sharding.strategy == "row_wise"
