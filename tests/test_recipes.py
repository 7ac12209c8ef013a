"""Reference-compatible entry points run end to end on CPU:
preprocessing.py -> train.py for TwoTower (Flax and Keras flavors, parquet and
tfrecord), Bert4Rec, and DLRM-tiny (BASELINE config 1)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]


def _run(script, args, cwd, env_extra=None, timeout=600):
    env = dict(os.environ)
    env.update(env_extra or {})
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, str(REPO / script), *args], cwd=cwd, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


@pytest.fixture(scope="module")
def raw(tmp_path_factory):
    from tdfo_amd.data.goodreads import make_synthetic_raw
    d = tmp_path_factory.mktemp("goodreads")
    make_synthetic_raw(d, 160, 300, seed=5, mean_inter=40)
    return d


def test_two_tower_flax_recipe(raw, tmp_path):
    _run("recipes/two_tower/preprocessing.py", [f"data_dir={raw}"], tmp_path)
    out = _run("recipes/two_tower/train.py",
               [f"data_dir={raw}", "n_epochs=2", "per_device_train_batch_size=256",
                "per_device_eval_batch_size=256"], tmp_path)
    assert "===== train size:" in out and "Epoch 2 eval loss:" in out
    assert (tmp_path / "model_params.pt").exists()
    from tdfo_amd.utils.checkpoint import load_flax_params
    p = load_flax_params(str(tmp_path / "model_params.pt"))
    assert p["item_fc1"]["kernel"].shape == (98, 16)


def test_two_tower_keras_tfrecord_recipes(raw, tmp_path):
    _run("recipes/two_tower_tf/preprocessing.py", [f"data_dir={raw}"], tmp_path)
    assert (raw / "tfrecord" / "train_data_size.json").exists()
    out = _run("recipes/two_tower_tf/train.py",
               [f"data_dir={raw}", "n_epochs=1", "per_device_train_batch_size=256"], tmp_path)
    assert "train auc:" in out and "eval auc:" in out
    out = _run("recipes/two_tower_tf/train_ps.py",
               [f"data_dir={raw}", "n_epochs=2", "per_device_train_batch_size=256"], tmp_path)
    assert "cluster.json: 4 workers, 2 ps" in out
    assert (tmp_path / "ckpt" / "epoch_2" / "manifest.json").exists()
    assert (tmp_path / "log" / "metrics.jsonl").exists()
    assert not list((tmp_path / "backup").glob("*"))         # removed after success


def test_bert4rec_recipe(raw, tmp_path):
    _run("recipes/bert4rec/preprocessing.py", [f"data_dir={raw}"], tmp_path)
    sm = json.loads((raw / "size_map_bert4rec.json").read_text())
    assert set(sm) == {"n_users", "n_items"}
    out = _run("recipes/bert4rec/train.py", [f"data_dir={raw}", "n_epochs=1"], tmp_path)
    assert "Epoch 0, metrics" in out and "Epoch 1, average loss" in out


def test_dlrm_tiny_cpu_recipe(tmp_path):
    out = _run("recipes/dlrm/train.py", ["synthetic.num_batches=40", "log_every=20",
                                         "eval_every=40", f"metrics_file={tmp_path}/m.jsonl"],
               tmp_path)
    assert "step 40 train loss" in out and "eval auc" in out
    recs = [json.loads(x) for x in (tmp_path / "m.jsonl").read_text().splitlines()]
    assert recs[-1]["step"] == 40 and recs[-1]["eval_auc"] > 0.5
