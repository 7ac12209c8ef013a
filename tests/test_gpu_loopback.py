"""Loopback collectives on the GPU (parallel/comm.py LoopbackComm): the
native piece copies (seg_copy over an int64 view) and the slab-reduce read of
the reduce-scatter give the same data as the CPU definitions in
tests/test_comm.py, for 8-byte, 4-byte and 2-byte element types."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("dtype", [torch.int64, torch.int32, torch.bfloat16, torch.float32])
def test_loopback_device_copies_match_cpu(dtype):
    from tdfo_amd.parallel.comm import LoopbackComm

    W, r = 8, 3
    n = 4096 + 64                                     # > one seg_copy chunk in int64 units
    inp = (torch.arange(W * n) % 977).to(dtype)
    for eq in (True, False):
        osp = [n] * W if eq else [n + 8 * k for k in range(W)]
        isp = [n] * W
        outs = []
        for dev in ("cpu", DEV):
            c = LoopbackComm(W, r, dev if dev != "cpu" else None)
            out = torch.full((sum(osp),), -1, dtype=dtype, device=dev)
            c.all_to_all(out, inp.to(dev), osp, isp)
            outs.append(out.cpu())
        if not eq and dtype.is_floating_point:
            continue                                  # values: a plain prefix copy on both
        assert torch.equal(outs[0], outs[1]), (dtype, eq)
    x = inp[:n]
    for dev in ("cpu", DEV):
        c = LoopbackComm(W, r, dev if dev != "cpu" else None)
        g = torch.zeros(W * n, dtype=dtype, device=dev)
        c.all_gather(g, x.to(dev))
        assert torch.equal(g.cpu(), x.repeat(W)), dtype
        rs = torch.zeros(n, dtype=dtype, device=dev)
        c.reduce_scatter(rs, inp.to(dev))
        assert torch.equal(rs.cpu(), inp[r * n:(r + 1) * n]), dtype
    torch.cuda.synchronize()


def test_loopback_async_work_orders_the_caller():
    """An async loopback exchange on its own stream is waited through the
    returned work, so the caller's next kernel sees the copied data."""
    from tdfo_amd.parallel.comm import LoopbackComm

    W, n = 4, 1 << 16
    c = LoopbackComm(W, 1, DEV)
    inp = torch.arange(W * n, device=DEV, dtype=torch.int64)
    out = torch.empty_like(inp)
    w = c.all_to_all(out, inp, [n] * W, [n] * W, async_op=True)
    w.wait()
    s = out.view(W, n).sum(1)
    assert torch.equal(s.cpu(), inp[n:2 * n].sum().cpu().repeat(W))
