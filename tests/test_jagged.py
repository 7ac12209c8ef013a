"""KeyedJaggedTensor, jagged<->dense ops and the local embedding collections
 against plain torch."""
import pytest
import torch

from tdfo_amd import ops
from tdfo_amd.sparse.jagged import (EmbeddingBagCollection, EmbeddingCollection, JaggedToDense,
                                    KeyedJaggedTensor)
from tdfo_amd.sparse.tables import EmbOptimConfig, TableConfig


def test_kjt_basics_and_padded_dense():
    kjt = KeyedJaggedTensor.from_lengths_sync(["a", "b"], torch.arange(1, 10),
                                              [2, 0, 3, 1, 2, 1])
    assert kjt.stride() == 3 and kjt.keys() == ["a", "b"]
    a = kjt["a"]
    assert a.values.tolist() == [1, 2, 3, 4, 5] and a.offsets.tolist() == [0, 2, 2, 5]
    d = kjt["b"].to_padded_dense(2, padding_value=0)
    assert d.tolist() == [[6, 0], [7, 8], [9, 0]]
    d = kjt["a"].to_padded_dense(2)                 # truncation at T
    assert d.tolist() == [[1, 2], [0, 0], [3, 4]]


def test_jagged_to_dense_grad():
    torch.manual_seed(0)
    off = torch.tensor([0, 3, 3, 7, 8])
    v = torch.randn(8, 4, requires_grad=True)
    out = JaggedToDense.apply(v, off, 3, -1.0)
    assert out.shape == (4, 3, 4)
    assert torch.equal(out[1], torch.full((3, 4), -1.0))
    assert torch.equal(out[2], v[3:6].detach())
    g = torch.randn(4, 3, 4)
    (out * g).sum().backward()
    exp = torch.zeros(8, 4)
    exp[0:3] = g[0]
    exp[3:6] = g[2]          # 4th element of bag 2 truncated -> 0
    exp[7] = g[3, 0]
    torch.testing.assert_close(v.grad, exp)


@pytest.mark.parametrize("D", [4, 6])
def test_ops_reference_roundtrip(D):
    off = torch.tensor([0, 2, 5])
    vals = torch.randn(5, D)
    out = torch.empty(2, 4, D)
    ops.jagged_to_dense(vals, off, 4, 0.0, out)
    back = torch.empty(5, D)
    ops.dense_to_jagged(out, off, back)
    torch.testing.assert_close(back, vals)


def _tables():
    return [TableConfig("t0", 50, 8, ["f0"]), TableConfig("t1", 30, 8, ["f1", "f2"])]


def test_embedding_bag_collection_forward_backward():
    torch.manual_seed(1)
    ebc = EmbeddingBagCollection(_tables(), EmbOptimConfig("sgd", lr=0.5), "cpu", seed=3)
    W0 = ebc.store.weight.clone()
    lengths = torch.tensor([2, 1, 0, 3, 1, 2, 2, 0, 1])       # keys f0,f1,f2 x B=3
    vals = torch.randint(0, 30, (int(lengths.sum()),))
    kjt = KeyedJaggedTensor(["f0", "f1", "f2"], vals, lengths)
    out = ebc(kjt)
    off = kjt.offsets()
    ro = {"f0": 0, "f1": 50, "f2": 50}
    for i, k in enumerate(["f0", "f1", "f2"]):
        for b in range(3):
            lo, hi = int(off[i * 3 + b]), int(off[i * 3 + b + 1])
            exp = W0[vals[lo:hi] + ro[k]].sum(0) if hi > lo else torch.zeros(8)
            torch.testing.assert_close(out[k][b], exp)
    g = {k: torch.randn(3, 8) for k in out}
    sum((out[k] * g[k]).sum() for k in out).backward()
    exp = W0.clone()
    for i, k in enumerate(["f0", "f1", "f2"]):
        for b in range(3):
            lo, hi = int(off[i * 3 + b]), int(off[i * 3 + b + 1])
            for j in range(lo, hi):
                exp[vals[j] + ro[k]] -= 0.5 * g[k][b]
    torch.testing.assert_close(ebc.store.weight, exp, rtol=1e-5, atol=1e-5)


def test_embedding_collection_sequences():
    ec = EmbeddingCollection([TableConfig("item", 40, 4, ["item"])], EmbOptimConfig("sgd", lr=1.0),
                             "cpu", seed=2)
    W0 = ec.store.weight.clone()
    kjt = KeyedJaggedTensor(["item"], torch.tensor([3, 4, 5, 3, 9]), torch.tensor([3, 2]))
    res = ec(kjt)["item"]
    torch.testing.assert_close(res.values, W0[[3, 4, 5, 3, 9]])
    dense = res.to_padded_dense(3)
    assert dense.shape == (2, 3, 4) and torch.equal(dense[1, 2], torch.zeros(4))
    dense.sum().backward()
    exp = W0.clone()
    for i in [3, 4, 5, 3, 9]:
        exp[i] -= 1.0
    torch.testing.assert_close(ec.store.weight, exp)
