"""Multi-rank guards of the contract entrypoints (utils/guarded.py): the
recipes' torchrun launches get the collective pre-flight (a mismatch takes
every rank onto c10d + staged) and the per-rank supervisor (a killed rank
makes every rank rerun once on the fallback path, resuming from the latest
checkpoint). CPU, gloo, torchrun, world size 2.

Reference: GRPC_FAIL_FAST + BackupAndRestore (tensorflow2/train_ps.py:39,
148-157), c10d DDP as the known-good path (torchrec/train.py:197-198)."""
import os
import re
import socket
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
TINY = ["per_device_train_batch_size=32", "synthetic.rows=tiny", "log_every=5", "eval_every=0",
        "max_steps=10", "bottom_mlp=32,16", "top_mlp=32,1"]


def _torchrun(script, args, env_extra, timeout=300):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    for k in ("TDFO_COMM", "TDFO_RESUME", "TDFO_STREAM_GRAPHS", "TDFO_PREFLIGHT_INJECT",
              "TDFO_FAULT_AT_STEP", "TDFO_FAULT_RANK", "TDFO_FAULT_ATTEMPT", "TDFO_SUPERVISE"):
        env.pop(k, None)
    env.update(env_extra)
    env["CUDA_VISIBLE_DEVICES"] = ""
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=2", "--master-addr", "127.0.0.1",
                        f"--master-port={port}", str(REPO / script), *args],
                       capture_output=True, text=True, timeout=timeout, env=env,
                       cwd=str(REPO / Path(script).parent))
    return p.returncode, p.stdout + p.stderr


def test_dlrm_recipe_preflight_mismatch_takes_c10d():
    rc, out = _torchrun("recipes/dlrm/train_ps.py", TINY, {"TDFO_PREFLIGHT_INJECT": "1"})
    assert rc == 0, out
    assert '"comm_path": "c10d-staged"' in out, out
    assert "collectives: c10d, stream graphs: False, preflight: FAILED" in out, out
    assert "replicated state consistent across ranks: True" in out, out
    assert "attempt failed" not in out, out        # handled in-process, no second attempt


def test_dlrm_recipe_killed_rank_resumes_from_checkpoint(tmp_path):
    ck = tmp_path / "ck"
    rc, out = _torchrun("recipes/dlrm/train_ps.py",
                        TINY + [f"ckpt_dir={ck}", "ckpt_every=4"],
                        {"TDFO_FAULT_AT_STEP": "7", "TDFO_FAULT_RANK": "1",
                         "TDFO_FAULT_ATTEMPT": "0"})
    assert rc == 0, out
    assert '"supervisor": "attempt failed"' in out, out
    # the second attempt: c10d, staged, resumed at the last checkpoint
    assert "attempt 1, collectives: c10d, stream graphs: False" in out, out
    m = re.search(r"resumed from (\S+) at step (\d+)", out)
    assert m and int(m.group(2)) == 4 and m.group(1).endswith("step_4"), out
    assert "replicated state consistent across ranks: True" in out, out
    assert (ck / "step_10" / "manifest.json").exists()


def test_recipes_route_through_supervisor():
    """Every multi-rank contract entrypoint is wrapped (static check)."""
    for script in ("recipes/dlrm/train_dp.py", "recipes/dlrm/train_ps.py",
                   "recipes/bert4rec/train.py", "recipes/two_tower/train_dp.py",
                   "recipes/two_tower_tf/train_dp.py", "recipes/two_tower_tf/train_ps.py"):
        src = (REPO / script).read_text()
        assert "supervised(" in src, script


@pytest.mark.parametrize("one_gpu,env,expect", [
    (True, None, ("0", "tdfo default (one GPU)")),
    (False, None, ("1", "runtime default")),
    (True, "1", ("1", "environment")),
])
def test_one_gpu_runtime_mode(monkeypatch, one_gpu, env, expect):
    from tdfo_amd.utils.guarded import PACKET_CAPTURE, one_gpu_runtime_mode
    if env is None:
        monkeypatch.delenv(PACKET_CAPTURE, raising=False)
    else:
        monkeypatch.setenv(PACKET_CAPTURE, env)
    r = one_gpu_runtime_mode(one_gpu)
    assert (r["value"], r["source"]) == expect
    if one_gpu and env is None:
        assert os.environ[PACKET_CAPTURE] == "0"
