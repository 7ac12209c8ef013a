"""Fused three-layer bottom-MLP forward (csrc/kernels/mlp_fused.hip,
ops.mlp3_fwd) against the three-GEMM path and an fp32 torch reference, and a
trainer using it against one that does not."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _layers(B, gen):
    bf = torch.bfloat16
    x = torch.zeros(B, 64, device=DEV, dtype=bf)
    x[:, :13] = torch.randn(B, 13, generator=gen, device=DEV).to(bf)
    x[:, 13] = 1.0                                     # bias column of layer 0
    Ws = [(torch.randn(512, 64, generator=gen, device=DEV) * 0.2).to(bf),
          (torch.randn(256, 576, generator=gen, device=DEV) * 0.05).to(bf),
          (torch.randn(128, 320, generator=gen, device=DEV) * 0.08).to(bf)]
    P1 = torch.randn(256, 576, generator=gen, device=DEV) * 0.1
    P2 = torch.randn(128, 320, generator=gen, device=DEV) * 0.1
    biases = [None, P1[:, 512], P2[:, 256]]
    return x, Ws, biases, [64, 576, 320]


@pytest.mark.parametrize("B", [32, 8192])
def test_mlp3_matches_gemms_and_reference(B):
    from tdfo_amd import ops

    gen = torch.Generator(device=DEV).manual_seed(3)
    x, Ws, biases, strides = _layers(B, gen)
    bf = torch.bfloat16
    outs = [torch.full((B, 576), 7.0, device=DEV, dtype=bf)[:, :512],
            torch.full((B, 320), 7.0, device=DEV, dtype=bf)[:, :256],
            torch.empty(B, 128, device=DEV, dtype=bf)]
    ops.mlp3_fwd(x, Ws, biases, strides, outs, [64, 512, 256, 128])
    # three GEMMs (the unfused path)
    ref = [torch.empty(B, 512, device=DEV, dtype=bf), torch.empty(B, 256, device=DEV, dtype=bf),
           torch.empty(B, 128, device=DEV, dtype=bf)]
    K = [64, 512, 256]
    inp = x
    for l in range(3):
        ops.gemm(inp[:, :K[l]], False, Ws[l][:, :K[l]], False, biases[l], True, None, ref[l],
                 None, 1)
        inp = ref[l]
    torch.cuda.synchronize()
    for l in range(3):
        torch.testing.assert_close(outs[l].float(), ref[l].float(), rtol=1e-2, atol=1e-2)
    # fp32 reference of the same chain (bf16 rounding between layers)
    h = x.float()
    for l in range(3):
        y = h[:, :K[l]] @ Ws[l][:, :K[l]].float().t()
        if biases[l] is not None:
            y = y + biases[l]
        h = torch.relu(y).to(bf).float()
        torch.testing.assert_close(outs[l].float(), h, rtol=2e-2, atol=2e-2)
    # the padding past each layer's width is untouched
    assert torch.all(outs[0].as_strided((B, 64), (576, 1), 512) == 7.0)


def test_trainer_fused_bottom_matches_unfused():
    import dataclasses

    from tdfo_amd.data.synthetic import SyntheticCriteo
    from tdfo_amd.models.dlrm import DLRMConfig, DLRMTrainer

    rows = [1000, 20, 5000, 3]
    cfg = DLRMConfig(embedding_dim=128, table_rows=rows, bottom=[512, 256, 128], top=[256, 1])
    B = 256
    a = DLRMTrainer(cfg, B, DEV)
    b = DLRMTrainer(dataclasses.replace(cfg, fused_bottom=True), B, DEV)
    assert b._bottom_fused_ok() and not a._bottom_fused_ok()
    data = SyntheticCriteo(rows, B, device=DEV, seed=2)
    batches = [data.next() for _ in range(4)]
    for t in (a, b):
        for d in batches:
            t.load_batch(*d)
            t.step()
    torch.cuda.synchronize()
    torch.testing.assert_close(a.fp.p, b.fp.p, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(a.emb.tw_store.weight, b.emb.tw_store.weight, rtol=1e-3,
                               atol=1e-4)
