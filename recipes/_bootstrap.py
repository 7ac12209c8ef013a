"""Make the in-tree ``tdfo_amd`` package importable from recipe scripts and
parse the optional ``key=value`` overrides (the reference scripts take no
CLI arguments: all configuration comes from ``config.toml`` next to them)."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def config(script_file: str):
    from tdfo_amd.config import read_configs

    here = Path(script_file).resolve().parent
    cfg_path = os.environ.get("TDFO_CONFIG", str(here / "config.toml"))
    return read_configs(cfg_path, sys.argv[1:])
