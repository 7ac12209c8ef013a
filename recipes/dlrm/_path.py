import sys
from pathlib import Path

_here = Path(__file__).resolve()
sys.path.insert(0, str(_here.parents[1]))   # recipes/ (for _bootstrap)
sys.path.insert(0, str(_here.parents[2]))   # repo root (for tdfo_amd)
