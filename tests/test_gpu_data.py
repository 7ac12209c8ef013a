"""Host data plane on the GPU: the C++ synthetic generator behind the pinned,
copy-stream prefetcher delivers exactly the batches the generator defines,
and the DLRM trainer steps on them."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_prefetcher_delivers_generator_batches_in_order():
    from tdfo_amd.data.prefetch import host_prefetcher
    from tdfo_amd.data.synthetic import HostSyntheticCriteo

    rows, L = [1000, 50, 70000], [1, 3, 2]
    pf = host_prefetcher(rows, 512, "cuda", pooling=L, seed=4, rank=1, start=3)
    ref = HostSyntheticCriteo(rows, 512, pooling=L, seed=4, rank=1, nbuf=1)
    for k in range(3, 12):
        (d, i, y), slot = pf.next()
        # consumer work on the current stream after the copy-stream H2D
        got = (d.clone(), i.clone(), y.clone())
        pf.release(slot)
        e = ref.batch(k)
        torch.cuda.synchronize()
        for a, b in zip(got, e):
            assert torch.equal(a.cpu(), b), k
    pf.close()


def test_dlrm_host_data_trains():
    from tdfo_amd.config import from_dict
    from tdfo_amd.train.dlrm import run

    cfg = from_dict({"model": "dlrm", "embed_dim": 64, "per_device_train_batch_size": 1024,
                     "bottom_mlp": [128, 64], "top_mlp": [128, 1], "table_rows": [5000, 300, 20000],
                     "log_every": 10, "max_steps": 30,
                     "synthetic": {"enabled": True, "host_data": True}})
    out = run(cfg, mode="single", device="cuda")
    h = out["history"]
    assert len(h) == 3 and all(r["train_loss"] == r["train_loss"] for r in h)
    assert h[-1]["train_loss"] < h[0]["train_loss"] + 0.05


@pytest.mark.parametrize("dist", ["uniform", "zipf"])
def test_device_generator_matches_host_generator(dist):
    """The one-launch HIP generator (csrc/kernels/synthetic.hip) is the twin
    of the C++ host generator: same ids and dense features for a batch index
    (the counter-based hash chain; float ln with FMA contraction off), labels
    equal up to draws within ~1e-16 of their probability."""
    from tdfo_amd.data.synthetic import DeviceSyntheticStream, HostSyntheticCriteo

    rows, L = [1000, 50, 70000, 40_000_000], [1, 3, 2, 4]
    ds = DeviceSyntheticStream(rows, 777, "cuda", pooling=L, seed=4, rank=1, dist=dist, start=5)
    ref = HostSyntheticCriteo(rows, 777, pooling=L, seed=4, rank=1, nbuf=1, dist=dist)
    for k in range(5, 9):
        (d, i, y), slot = ds.next()
        got = (d.cpu(), i.cpu(), y.cpu())
        ds.release(slot)
        ed, ei, ey = ref.batch(k)
        if dist == "uniform":
            assert torch.equal(got[1], ei), k
        else:    # double pow: equal up to an ulp at a rounding boundary
            assert (got[1] != ei).float().mean() < 1e-3, k
        assert torch.equal(got[0], ed), k
        assert (got[2] != ey).float().mean() < 2e-3, k
        assert 0 <= int(got[1].min()) and int(got[1].max()) < max(rows)
