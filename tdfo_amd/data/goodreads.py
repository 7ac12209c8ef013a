"""Goodreads TwoTower ETL (reference jax-flax/preprocessing.py, its TF twin
tensorflow2/preprocessing.py + data.py) on pyarrow/numpy — Polars is not
available, and the per-user group work is done with vectorised sort/bincount
instead of Python group-apply.

Steps (file:line of jax-flax/preprocessing.py):
  * interactions: keep users with 10..250 rows (:51-52); label = rating >= 4
    (:56-60); book ids sorted per user (:66).
  * books: language / is_ebook / format / publisher / decade -> sorted-unique
    integer ids with "" -> "unknown" (:131-144); avg_rating / num_pages:
    drop ""/>2000 for the stats, fill with the median, min-max scale
    (:110-128); publication year -> 13 decade buckets + "unknown" (:74-107).
  * per user 80/20 split by sorted book id (:212-220, quirk Q12);
  * 8 parquet parts per split, train parts shuffled with seed 42 (:240-270);
    size_map.json (:273-275). TF variant: GZIP TFRecord parts without
    is_read / is_reviewed (quirk Q15) + {split}_data_size.json sidecars.

Deliberate choices:
  * Quirk "per-user sort": the reference sorts only the ``book_id`` column
    inside ``over("user_id")`` (:66), detaching labels from their books. We
    sort whole rows (labels stay with their book); ``legacy_sort=True``
    reproduces the reference behaviour.
  * Decade quirk: polars ``is_between`` is closed on both ends, so a year that
    is a multiple of 10 falls in the *previous* decade ("1910" -> "1900s").
    Preserved for parity.
"""
from __future__ import annotations

import json
import math
import time
from pathlib import Path
from typing import Dict, Tuple

import numpy as np
import pyarrow as pa
import pyarrow.csv as pacsv
import pyarrow.parquet as pq

SPLIT_RATIO = 0.8
FILE_NUM = 8
MIN_INTER, MAX_INTER = 10, 250
FINAL_COLUMNS = ["user_id", "item_id", "language", "is_ebook", "format", "publisher",
                 "pub_decade", "avg_rating", "num_pages", "is_read", "is_reviewed", "label"]
COLUMN_DTYPES = {"user_id": np.int32, "item_id": np.int32, "language": np.int16,
                 "is_ebook": np.int8, "format": np.int16, "publisher": np.int32,
                 "pub_decade": np.int8, "avg_rating": np.float32, "num_pages": np.float32,
                 "is_read": np.int8, "is_reviewed": np.int8, "label": np.int8}
TFRECORD_COLUMNS = [c for c in FINAL_COLUMNS if c not in ("is_read", "is_reviewed")]
CATEGORY_COLS = [("language", "language_code"), ("is_ebook", "is_ebook"), ("format", "format"),
                 ("publisher", "publisher"), ("pub_decade", None)]


# ------------------------------------------------------------ interactions
def read_interactions(data_dir: Path, legacy_sort: bool = False) -> Dict[str, np.ndarray]:
    tbl = pacsv.read_csv(
        Path(data_dir) / "goodreads_interactions.csv",
        convert_options=pacsv.ConvertOptions(column_types={
            "user_id": pa.int32(), "book_id": pa.int32(), "is_read": pa.int8(),
            "rating": pa.int8(), "is_reviewed": pa.int8()}))
    user = tbl["user_id"].to_numpy()
    cnt = np.bincount(user)
    keep = (cnt[user] >= MIN_INTER) & (cnt[user] <= MAX_INTER)
    cols = {k: tbl[k].to_numpy()[keep] for k in ("user_id", "book_id", "is_read", "is_reviewed",
                                                 "rating")}
    label = (cols.pop("rating") >= 4).astype(np.int8)
    cols["label"] = label
    user = cols["user_id"]
    if legacy_sort:
        # reference: only book_id is sorted within each user's rows, the other
        # columns keep their original row order (jax-flax/preprocessing.py:66)
        order_rows = np.argsort(user, kind="stable")
        by_user_book = np.lexsort((cols["book_id"], user))
        out = {k: v[order_rows] for k, v in cols.items()}
        out["book_id"] = cols["book_id"][by_user_book]
        # restore the original row positions
        inv = np.empty_like(order_rows)
        inv[order_rows] = np.arange(len(order_rows))
        return {k: v[inv] for k, v in out.items()}
    order = np.lexsort((cols["book_id"], user))     # rows sorted by (user, book)
    return {k: v[order] for k, v in cols.items()}


def split_mask(user: np.ndarray, book: np.ndarray) -> np.ndarray:
    """True for train rows: per user, the first ceil(0.8 n) books in sorted
    book-id order (jax-flax/preprocessing.py:212-220)."""
    order = np.lexsort((book, user))
    u_sorted = user[order]
    n = np.bincount(user)
    starts = np.zeros(len(n) + 1, dtype=np.int64)
    np.cumsum(n, out=starts[1:])
    rank = np.arange(len(order)) - starts[u_sorted]
    train_n = np.ceil(n * SPLIT_RATIO - 1e-9).astype(np.int64)
    mask = np.empty(len(order), dtype=bool)
    mask[order] = rank < train_n[u_sorted]
    return mask


# ------------------------------------------------------------ book features
def year_to_decade(years) -> np.ndarray:
    """Publication-year strings -> decade labels (reference when-chain order:
    both-ends-closed ranges, so "1910" -> "1900s")."""
    out = np.full(len(years), "unknown", dtype=object)
    for i, y in enumerate(years):
        s = (y or "").strip()
        if not s.isdigit():
            continue
        v = int(s)
        if 1900 <= v <= 2030:
            out[i] = f"{1900 + max(0, v - 1901) // 10 * 10}s"
    return out


def transform_continuous(values) -> np.ndarray:
    vals = np.array([v if v is not None else "" for v in values], dtype=object)
    nonempty = vals != ""
    num = np.zeros(len(vals), dtype=np.float64)
    num[nonempty] = vals[nonempty].astype(np.float64)
    ok = nonempty & (num <= 2000)
    good = num[ok].astype(np.float32)
    mn, mx = float(good.min()), float(good.max())
    med = round(float(np.median(good)), 4)
    num[~nonempty] = med
    num[num > 2000] = med
    return ((num.astype(np.float32) - mn) / (mx - mn)).astype(np.float32)


def sparse_mapping(values) -> Dict[str, int]:
    vals = ["unknown" if (v is None or v == "") else str(v) for v in values]
    return {v: i for i, v in enumerate(sorted(set(vals)))}


def transform_categorical(values, mapping: Dict[str, int], dtype) -> np.ndarray:
    return np.array([mapping["unknown" if (v is None or v == "") else str(v)] for v in values],
                    dtype=dtype)


def _read_id_map(path: Path) -> Tuple[np.ndarray, np.ndarray]:
    tbl = pacsv.read_csv(path)
    a = tbl.column(0).to_numpy()
    b = np.array([str(x) for x in tbl.column(1).to_pylist()], dtype=object)
    return a.astype(np.int64), b


def _read_books(path: Path) -> Dict[str, list]:
    keys = ["book_id", "language_code", "is_ebook", "average_rating", "format", "publisher",
            "num_pages", "publication_year"]
    cols = {k: [] for k in keys}
    with open(path) as f:
        for line in f:
            if not line.strip():
                continue
            r = json.loads(line)
            for k in keys:
                v = r.get(k, "")
                cols[k].append("" if v is None else str(v))
    return cols


def book_features(data_dir: Path) -> Tuple[Dict[str, np.ndarray], Dict[str, int]]:
    """Per csv book id (row i = book id i) feature arrays + size_map."""
    data_dir = Path(data_dir)
    size_map: Dict[str, int] = {}
    user_ids, _ = _read_id_map(data_dir / "user_id_map.csv")
    size_map["user"] = int(len(user_ids))
    book_ids, book_orig = _read_id_map(data_dir / "book_id_map.csv")
    size_map["item"] = int(len(book_ids))
    books = _read_books(data_dir / "goodreads_books.json")
    books["pub_decade"] = list(year_to_decade(books["publication_year"]))
    feats = {}
    dtypes = {"language": np.int16, "is_ebook": np.int8, "format": np.int16,
              "publisher": np.int32, "pub_decade": np.int8}
    for col, src in CATEGORY_COLS:
        vals = books[src or col]
        mp = sparse_mapping(vals)
        feats[col] = transform_categorical(vals, mp, dtypes[col])
        size_map[col] = len(mp)
    feats["avg_rating"] = transform_continuous(books["average_rating"])
    feats["num_pages"] = transform_continuous(books["num_pages"])
    # left join book_id_map -> books on the original id
    pos = {b: i for i, b in enumerate(books["book_id"])}
    idx = np.array([pos.get(b, -1) for b in book_orig], dtype=np.int64)
    if (idx < 0).any():
        raise ValueError(f"{int((idx < 0).sum())} mapped books have no features "
                         "(reference asserts no nulls: jax-flax/preprocessing.py:208)")
    n_items = int(book_ids.max()) + 1
    out = {}
    for k, v in feats.items():
        arr = np.zeros(n_items, dtype=v.dtype)
        arr[book_ids] = v[idx]
        out[k] = arr
    return out, size_map


# ------------------------------------------------------------ writers
def _rows_for_split(inter: Dict[str, np.ndarray], feats: Dict[str, np.ndarray]):
    book = inter["book_id"]
    cols = {"user_id": inter["user_id"], "item_id": book}
    for k in ("language", "is_ebook", "format", "publisher", "pub_decade", "avg_rating",
              "num_pages"):
        cols[k] = feats[k][book]
    cols["is_read"] = inter["is_read"]
    cols["is_reviewed"] = inter["is_reviewed"]
    cols["label"] = inter["label"]
    return {k: np.asarray(cols[k]).astype(COLUMN_DTYPES[k]) for k in FINAL_COLUMNS}


def _parts(n_total: int, mask: np.ndarray):
    """Part i holds the split's rows whose original position falls in the
    i-th of FILE_NUM equal slices of the interaction table."""
    unit = math.ceil(n_total / FILE_NUM)
    for i, off in enumerate(range(0, n_total, unit), start=1):
        sl = np.zeros(n_total, dtype=bool)
        sl[off: off + unit] = True
        yield i, np.nonzero(sl & mask)[0]


def write_split(data_dir: Path, inter, feats, mask, prefix: str, fmt: str = "parquet",
                verbose: bool = True) -> int:
    write_dir = Path(data_dir) / fmt
    write_dir.mkdir(parents=True, exist_ok=True)
    n_total = len(inter["user_id"])
    total = 0
    for i, rows in _parts(n_total, mask):
        t0 = time.perf_counter()
        if prefix == "train":
            rows = rows[np.random.default_rng(42).permutation(len(rows))]
        part = _rows_for_split({k: v[rows] for k, v in inter.items()}, feats)
        total += len(rows)
        if fmt == "parquet":
            pq.write_table(pa.table(part), write_dir / f"{prefix}_part_{i}.parquet")
        else:
            from .native import tfrecord_write
            tfrecord_write(write_dir / f"{prefix}_part_{i}.tfrecord",
                           {k: part[k] for k in TFRECORD_COLUMNS})
        if verbose:
            print(f"{prefix} part_{i} finished in {(time.perf_counter() - t0):.2f}s")
    if fmt == "tfrecord":
        (write_dir / f"{prefix}_data_size.json").write_text(json.dumps({"data_size": total}))
    return total


def run_etl(data_dir, fmt: str = "parquet", legacy_sort: bool = False, verbose: bool = True):
    data_dir = Path(data_dir)
    feats, size_map = book_features(data_dir)
    (data_dir / "size_map.json").write_text(json.dumps(size_map, indent=4))
    inter = read_interactions(data_dir, legacy_sort=legacy_sort)
    if verbose:
        print(f"data size: {len(inter['user_id']):,}")
    mask = split_mask(inter["user_id"], inter["book_id"])
    n_tr = write_split(data_dir, inter, feats, mask, "train", fmt, verbose)
    n_ev = write_split(data_dir, inter, feats, ~mask, "eval", fmt, verbose)
    if verbose:
        print(f"train data size: {n_tr:,}, eval data size: {n_ev:,}")
    return size_map, n_tr, n_ev


# ------------------------------------------------------------ synthetic raw
def make_synthetic_raw(data_dir, n_users: int = 300, n_books: int = 500, seed: int = 0,
                       mean_inter: int = 40):
    """Write Goodreads-format raw files (goodreads_interactions.csv,
    user_id_map.csv, book_id_map.csv, goodreads_books.json) with learnable
    structure: users and books have latent tastes; rating >= 4 iff aligned."""
    rng = np.random.default_rng(seed)
    d = Path(data_dir)
    d.mkdir(parents=True, exist_ok=True)
    ut = rng.normal(size=(n_users, 4))
    bt = rng.normal(size=(n_books, 4))
    rows = []
    for u in range(n_users):
        k = int(np.clip(rng.poisson(mean_inter), 3, 300))
        bs = rng.choice(n_books, size=min(k, n_books), replace=False)
        score = bt[bs] @ ut[u] + rng.normal(scale=0.5, size=len(bs))
        rating = np.clip(np.round(3 + score), 0, 5).astype(int)
        for b, r in zip(bs, rating):
            rows.append((u, int(b), int(rng.random() < 0.7), int(r), int(rng.random() < 0.2)))
    with open(d / "goodreads_interactions.csv", "w") as f:
        f.write("user_id,book_id,is_read,rating,is_reviewed\n")
        for r in rows:
            f.write(",".join(map(str, r)) + "\n")
    with open(d / "user_id_map.csv", "w") as f:
        f.write("user_id_csv,user_id\n")
        for u in range(n_users):
            f.write(f"{u},u{u:08x}\n")
    with open(d / "book_id_map.csv", "w") as f:
        f.write("book_id_csv,book_id\n")
        for b in range(n_books):
            f.write(f"{b},{1000 + b * 7}\n")
    langs = ["eng", "en-US", "spa", "fre", "ger", ""]
    fmts = ["Paperback", "Hardcover", "ebook", "Kindle Edition", ""]
    with open(d / "goodreads_books.json", "w") as f:
        for b in rng.permutation(n_books):
            year = "" if rng.random() < 0.1 else str(int(rng.integers(1890, 2025)))
            pages = "" if rng.random() < 0.1 else str(int(rng.integers(20, 1500)))
            if rng.random() < 0.02:
                pages = "5000"                     # outlier (> 2000) -> median
            rec = {"book_id": str(1000 + int(b) * 7),
                   "language_code": langs[int(rng.integers(len(langs)))],
                   "is_ebook": "true" if rng.random() < 0.3 else "false",
                   "average_rating": f"{rng.uniform(2.5, 4.8):.2f}",
                   "format": fmts[int(rng.integers(len(fmts)))],
                   "publisher": "" if rng.random() < 0.1 else f"pub{int(rng.integers(30))}",
                   "num_pages": pages, "publication_year": year}
            f.write(json.dumps(rec) + "\n")
    return len(rows)


# ------------------------------------------------------------ readers
def read_parquet_columns(pattern: str) -> Dict[str, np.ndarray]:
    """Concatenate every part matching a glob (sorted by name)."""
    p = Path(pattern)
    files = sorted(p.parent.glob(p.name), key=lambda x: (len(x.name), x.name))
    if not files:
        raise FileNotFoundError(pattern)
    tables = [pq.read_table(f) for f in files]
    tbl = pa.concat_tables(tables)
    return {c: tbl[c].to_numpy() for c in tbl.column_names}


def read_tfrecord_columns(pattern: str) -> Dict[str, np.ndarray]:
    from .native import tfrecord_read
    p = Path(pattern)
    files = sorted(p.parent.glob(p.name), key=lambda x: (len(x.name), x.name))
    if not files:
        raise FileNotFoundError(pattern)
    schema = {c: ("float32" if COLUMN_DTYPES[c] == np.float32 else "int64")
              for c in TFRECORD_COLUMNS}
    parts = [tfrecord_read(str(f), schema) for f in files]
    return {c: np.concatenate([q[c] for q in parts]).astype(COLUMN_DTYPES[c])
            for c in TFRECORD_COLUMNS}


def data_size(pattern: str, fmt: str = "parquet") -> int:
    """Row count (tensorflow2/utils.py:41-48: sidecar json for tfrecord)."""
    p = Path(pattern)
    if fmt == "tfrecord":
        prefix = p.name.split("_part")[0]
        side = p.parent / f"{prefix}_data_size.json"
        if side.exists():
            return int(json.loads(side.read_text())["data_size"])
        from .native import tfrecord_count
        return sum(tfrecord_count(str(f)) for f in p.parent.glob(p.name))
    return sum(pq.ParquetFile(f).metadata.num_rows for f in p.parent.glob(p.name))
