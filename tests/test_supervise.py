"""bench.py's per-rank supervisor (utils/supervise.py): a failed first
attempt on any rank (watchdog exit 3, replica mismatch exit 4, a crash)
reruns every rank once on the fallback path; CPU, torchrun, gloo."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _run(scenario):
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.pop("TDFO_COMM", None)
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=2", "--master-addr", "127.0.0.1",
                        f"--master-port={port}", os.path.join(HERE, "helpers", "sup_main.py"),
                        scenario], capture_output=True, text=True, timeout=240, env=env)
    return p.returncode, p.stdout + p.stderr


def test_all_ok_runs_once():
    rc, out = _run("ok")
    assert rc == 0, out
    assert "attempt=1" not in out
    assert out.count("attempt=0") == 2


@pytest.mark.parametrize("scenario", ["watchdog", "diverged", "crash"])
def test_failed_attempt_falls_back_on_every_rank(scenario):
    rc, out = _run(scenario)
    assert rc == 0, out
    for r in range(2):
        assert f"child rank={r} attempt=1 comm=torch fb=True rc=0" in out, out
    assert '"supervisor": "attempt failed"' in out


def test_both_attempts_fail_reports_failure():
    rc, out = _run("both")
    assert rc != 0, out
