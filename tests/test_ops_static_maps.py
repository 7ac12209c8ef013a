"""CPU references of the static data-movement ops the multi-rank step uses
(ops.SegmentMap, ops.PieceCopy, ops.slab_reduce): the GPU kernels are checked
against the same definitions in tests/test_gpu_mailbox.py."""
import torch

from tdfo_amd import ops


def test_segment_map_cpu_is_a_gather_of_runs():
    src = torch.arange(100, dtype=torch.int64) * 7
    pieces = [(40, 0, 5), (0, 5, 3), (90, 8, 10)]
    m = ops.SegmentMap(pieces, "cpu")
    out = torch.full((18,), -1, dtype=torch.int64)
    m.apply(src, out)
    ref = torch.cat([src[a:a + n] for a, _, n in pieces])
    assert torch.equal(out, ref)
    assert m.src_n == 100 and m.dst_n == 18 and m.n == 18
    # the pieces of an index that is a union of runs
    idx = torch.tensor([5, 6, 7, 20, 21, 3])
    m2 = ops.SegmentMap.from_index(idx, "cpu")
    out2 = torch.empty(6, dtype=torch.int64)
    m2.apply(src, out2)
    assert torch.equal(out2, src[idx])


def test_piece_copy_cpu_and_reverse():
    B, w = 5, 8
    buf = torch.arange(400, dtype=torch.float32).bfloat16()
    pieces = [(0, 16, 200, 24), (8, 16, 208, 24)]
    pc = ops.PieceCopy(pieces, B, w, "cpu")
    ref = buf.clone()
    for a, la, c, lc in pieces:
        for b in range(B):
            ref[c + b * lc: c + b * lc + w] = ref[a + b * la: a + b * la + w]
    pc.apply(buf)
    assert torch.equal(buf, ref)
    # reverse moves the pieces back (sources overwritten from the copies)
    buf[0:16 * B] = 0
    pc.reverse().apply(buf)
    for a, la, c, lc in pieces:
        for b in range(B):
            assert torch.equal(buf[a + b * la: a + b * la + w], ref[c + b * lc: c + b * lc + w])
    assert pc.extent == max(208 + 4 * 24, 8 + 4 * 16) + w


def test_slab_reduce_cpu():
    segs = []
    for S, n in [(3, 8), (1, 4), (5, 12)]:
        sl = torch.randn(S * n)
        out = torch.empty(n)
        segs.append((sl, S, out))
    ops.slab_reduce(segs)
    for sl, S, out in segs:
        assert torch.allclose(out, sl.view(S, -1).sum(0))

