"""Single-device TwoTower training (reference: jax-flax/train.py).
`python train.py` -> prints per-epoch train/eval loss, writes ./model_params.pt
(Flax msgpack layout)."""
import _path  # noqa: F401
from _bootstrap import config
from tdfo_amd.train.two_tower import run

if __name__ == "__main__":
    run(config(__file__), mode="single", flavor="flax")
