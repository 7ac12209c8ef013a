"""bench.py picks the HIP graph launch mode before any GPU call: graph nodes
dispatched at launch (DEBUG_CLR_GRAPH_PACKET_CAPTURE=0) only for one process
on one GPU, not for rank processes or emulated ranks (host issue cost), and
an explicit setting always wins (profiles/r05/notes.md "HIP graph launch
mode")."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _mode(args, env_extra=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "WORLD_SIZE")}
    env.update(env_extra or {})
    code = ("import sys, os; sys.argv = ['bench.py'] + sys.argv[1:]; "
            "import runpy; g = runpy.run_path('bench.py', run_name='not_main'); "
            "print(os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE', 'unset'))")
    r = subprocess.run([sys.executable, "-c", code] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout.strip().splitlines()[-1]


@pytest.mark.parametrize("args,env,want", [
    ([], None, "0"),
    (["--gpus", "1", "--steps", "5"], None, "0"),
    (["--gpus", "8"], None, "unset"),
    (["--emulate-world", "8", "--emulate-rank", "1"], None, "unset"),
    ([], {"WORLD_SIZE": "2"}, "unset"),
    ([], {"DEBUG_CLR_GRAPH_PACKET_CAPTURE": "1"}, "1"),
])
def test_bench_launch_mode(args, env, want):
    assert _mode(args, env) == want
