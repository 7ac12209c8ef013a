"""Single-device TwoTower training, Keras flavor (reference: tensorflow2/train.py):
lecun_normal dense init, `train loss / train auc` log lines."""
import _path  # noqa: F401
from _bootstrap import config
from tdfo_amd.train.two_tower import run

if __name__ == "__main__":
    run(config(__file__), mode="single", flavor="keras")
