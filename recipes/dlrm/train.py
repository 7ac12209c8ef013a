"""Single-process DLRM training: DLRM-tiny on CPU (BASELINE config 1) or one MI355X
(config 2: `python train.py synthetic.rows=kaggle embed_dim=128 ...`)."""
import _path  # noqa: F401
from tdfo_amd.utils.guarded import one_gpu_runtime_mode

one_gpu_runtime_mode(True)     # before any GPU call: the bench's one-GPU runtime mode
from _bootstrap import config  # noqa: E402
from tdfo_amd.train.dlrm import run  # noqa: E402

if __name__ == "__main__":
    run(config(__file__), mode="single")
