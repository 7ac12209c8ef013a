"""In-step synthetic batches (data.synthetic.InStepSynthetic; csrc/kernels/
synthetic.hip synth_ids / synth_dense): the ids, bf16 dense features and
labels the step draws from its device step counter equal the side-stream
generator's batch of the same index bit for bit, and a trainer whose per-stream
graphs generate their own batches trains exactly like one fed the same
batches through load_batch."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)
ROWS = [1000, 20, 5000, 3]


@pytest.mark.parametrize("dist,pooling", [("uniform", None), ("zipf", [2, 1, 3, 1])])
def test_in_step_batches_equal_device_stream(dist, pooling):
    from tdfo_amd import ops
    from tdfo_amd.data.synthetic import DeviceSyntheticStream, InStepSynthetic

    B, nd = 300, 13
    ref = DeviceSyntheticStream(ROWS, B, DEV, pooling=pooling, seed=5, dist=dist, start=7)
    ins = InStepSynthetic(ROWS, B, DEV, pooling=pooling, seed=5, dist=dist, start=7)
    counter = torch.tensor([3.0], device=DEV)
    ins.bind(counter)
    x0 = torch.zeros(B, 64, dtype=torch.bfloat16, device=DEV)
    x0[:, nd] = 1.0
    ids = torch.empty(ref.nnz, dtype=torch.int64, device=DEV)
    label = torch.empty(B, device=DEV)
    for k in range(3):
        (d, i, y), slot = ref.next()
        ins.gen_ids(ids)
        ins.gen_dense(x0, label)
        torch.cuda.synchronize()
        assert torch.equal(ids, i), k
        assert torch.equal(label, y), k
        # the same bf16 conversion batch_load applies
        xr = torch.zeros_like(x0)
        xr[:, nd] = 1.0
        ops.batch_load(d, xr, i[:0], i[:0], y, torch.empty_like(y))
        assert torch.equal(x0, xr), k
        ref.release(slot)
        counter += 1.0


def test_trainer_in_step_matches_loaded_batches():
    from tdfo_amd.data.synthetic import DeviceSyntheticStream, InStepSynthetic
    from tdfo_amd.models.dlrm import DLRMConfig, DLRMTrainer
    from tdfo_amd.train.loop import StepLoop

    cfg = DLRMConfig(embedding_dim=128, table_rows=ROWS, bottom=[128], top=[256, 1], ids_stream=False)
    B = 512
    a = DLRMTrainer(cfg, B, DEV)
    b = DLRMTrainer(cfg, B, DEV)
    la = StepLoop(a, DeviceSyntheticStream(ROWS, B, DEV, seed=2))
    lb = StepLoop(b, InStepSynthetic(ROWS, B, DEV, seed=2))
    for lp in (la, lb):
        lp.run(2)
        lp.tr.capture_graph(warmup=0)
        assert lp.tr.graph == "streams"
        lp.run(6)
    torch.cuda.synchronize()
    for t in (a, b):
        t.sync_streams()
    torch.cuda.synchronize()
    assert torch.equal(a.fp.p, b.fp.p)
    assert torch.equal(a.emb.tw_store.weight, b.emb.tw_store.weight)
    assert a.pop_loss() == b.pop_loss()


@pytest.mark.parametrize("interaction", ["dot", "dcn"])
def test_producer_stream_ids_copy_matches_embedding_stream_copy(interaction, monkeypatch):
    """StepLoop hands the device generator's stream to the trainer, which then
    copies each batch's ids there (behind the previous step's sort) instead of
    on the embedding stream: same training, bit for bit."""
    from tdfo_amd.data.synthetic import DeviceSyntheticStream
    from tdfo_amd.models.dlrm import DLRMConfig, DLRMTrainer
    from tdfo_amd.train.loop import StepLoop

    kw = dict(embedding_dim=128, table_rows=ROWS, bottom=[128], top=[256, 1], ids_stream=False)
    if interaction == "dcn":
        kw.update(interaction="dcn", dcn_layers=2, dcn_rank=64, pooling=[2, 1, 3, 1])
    cfg = DLRMConfig(**kw)
    B = 512
    from tdfo_amd.data.synthetic import SyntheticCriteo
    gen = SyntheticCriteo(ROWS, B, pooling=cfg.pooling_factors(), device=DEV, seed=9)
    foreign = [gen.next() for _ in range(2)]
    torch.cuda.synchronize()
    out = []
    for flag in ("1", "0"):
        monkeypatch.setenv("TDFO_SRC_COPY", flag)
        t = DLRMTrainer(cfg, B, DEV)
        src = DeviceSyntheticStream(ROWS, B, DEV, seed=3, pooling=cfg.pooling_factors())
        lp = StepLoop(t, src)
        assert (t._src_copy_stream is not None) == (flag == "1")
        lp.run(2)
        t.capture_graph(warmup=0)
        assert t.graph == "streams"
        lp.run(6)
        # then batches of another producer through load_batch (the embedding
        # stream path, behind the MLP stream)
        for b in foreign:
            t.load_batch(*b, on_device=True)
            t.step()
        t.sync_streams()
        torch.cuda.synchronize()
        out.append((t.fp.p.clone(), t.emb.tw_store.weight.clone(), t.pop_loss()))
    assert torch.equal(out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])
    assert out[0][2] == out[1][2]
