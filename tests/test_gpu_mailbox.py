"""Host mailbox (parallel/mailbox.py, ``host_publish_kernel``), the batched
split-K slab reduce (``slab_reduce_kernel``) and the static id permute
(``seg_copy_kernel``, ops.SegmentMap) and column-wise piece copy (ops.PieceCopy) on the GPU, against their definitions:
eager and hipGraph-replayed publishes land with the expected sequence numbers
and values; the one-launch reduce of several slab sets equals the fp32 torch
sum of each; the segment copy equals torch.index_select with the same index."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_mailbox_eager_and_replayed():
    from tdfo_amd.parallel.mailbox import HostMailbox
    from tdfo_amd.utils.capture import graph_capture

    dev = torch.device("cuda", 0)
    mb = HostMailbox(2, dev)
    v = torch.tensor([7], dtype=torch.int32, device=dev)
    mb.publish(v)
    assert mb.read() == 7
    v.fill_(-3)
    mb.publish(v, slot=1)
    assert mb.read(1) == -3 and mb.read(0) == 7
    # captured: a kernel writes v, then the publish; each replay is one launch
    x = torch.zeros(1, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with graph_capture(g, stream=s):
        x.add_(5)
        mb.publish(x)
    for k in range(1, 6):
        g.replay()
        mb.note_launch()
        assert mb.read() == 5 * k
    assert mb.wait_s >= 0.0


def test_mailbox_read_survives_a_long_kernel():
    """A read issued while the producing stream is still busy waits for the
    value instead of returning the previous one."""
    from tdfo_amd import ops
    from tdfo_amd.parallel.mailbox import HostMailbox

    dev = torch.device("cuda", 0)
    mb = HostMailbox(1, dev)
    v = torch.tensor([1], dtype=torch.int32, device=dev)
    mb.publish(v)
    assert mb.read() == 1
    ops.spin_us(20000.0)                   # 20 ms of device time ahead of the publish
    v2 = torch.tensor([2], dtype=torch.int32, device=dev)
    mb.publish(v2)
    assert mb.read() == 2


@pytest.mark.parametrize("shapes", [[(4, 1024 * 1088)], [(2, 256 * 576), (8, 128 * 320), (1, 64)],
                                    [(3, 4096)] * 17])
def test_slab_reduce_matches_torch(shapes):
    from tdfo_amd import ops

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    segs, refs = [], []
    for S, n in shapes:
        sl = torch.randn(S * n, generator=g, device=dev)
        out = torch.full((n,), float("nan"), device=dev)
        segs.append((sl, S, out))
        refs.append(sl.view(S, n).sum(0))
    ops.slab_reduce(segs)
    torch.cuda.synchronize()
    for (sl, S, out), ref in zip(segs, refs):
        torch.testing.assert_close(out, ref, rtol=1e-6, atol=1e-5)


def test_segment_map_matches_index_select():
    from tdfo_amd import ops

    dev = torch.device("cuda", 0)
    src = torch.randint(0, 1 << 40, (30000,), dtype=torch.int64, device=dev)
    # runs of assorted lengths (one longer than a chunk), out of order
    pieces = [(20000, 0, 9000), (100, 9000, 3), (5000, 9003, 4096), (0, 13099, 1)]
    m = ops.SegmentMap(pieces, dev)
    idx = torch.cat([torch.arange(a, a + n) for a, _, n in pieces]).to(dev)
    out = torch.full((13100,), -1, dtype=torch.int64, device=dev)
    m.apply(src, out)
    torch.testing.assert_close(out, torch.index_select(src, 0, idx), rtol=0, atol=0)
    assert m.nchunks == 3 + 1 + 1 + 1


def test_piece_copy_matches_strided_copies():
    from tdfo_amd import ops

    dev = torch.device("cuda", 0)
    B, w = 37, 24
    buf = torch.randn(20000, device=dev).bfloat16()
    pieces = [(0, 64, 8000, 48), (40, 64, 8024, 48), (3000, 32, 12000, 24)]
    ref = buf.cpu().clone()
    ops.PieceCopy(pieces, B, w, "cpu").apply(ref)
    pc = ops.PieceCopy(pieces, B, w, dev)
    pc.apply(buf)
    torch.testing.assert_close(buf.cpu(), ref, rtol=0, atol=0)
    back = ref.clone()
    pc.reverse().reverse().apply(buf)             # idempotent re-apply
    torch.testing.assert_close(buf.cpu(), back, rtol=0, atol=0)
