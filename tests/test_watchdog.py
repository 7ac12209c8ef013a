"""Hang guard (utils/watchdog.py) and the cross-rank replica check
(parallel/replicas.py) on CPU / gloo: a rank that stops stepping ends every
rank of the job with exit code 3 and a diagnostic; replicated state is
bit-identical after pipelined multi-rank training, and one perturbed replica
is reported by every rank."""
import os
import time

import pytest
import torch
import torch.multiprocessing as mp

from tests.dist_harness import _free_port, run_distributed

ROWS = [50, 7, 300, 1000, 3]


def test_watchdog_unit_checks():
    from tdfo_amd.utils.watchdog import StepWatchdog

    wd = StepWatchdog("cpu", timeout_s=5.0, exit_code=-1, poll_s=60.0)
    try:
        assert wd.check() is None
        with wd.active():
            wd.beat(step=1)
            assert wd.check() is None and wd.completed == 1
            t = time.monotonic()
            assert wd.check(now=t + 1.0) is None
            why = wd.check(now=t + 10.0)
            assert why is not None and why.startswith("host")
        assert wd.check(now=time.monotonic() + 10.0) is None       # left the step loop
        # a heartbeat that does not land (the device view lags behind)
        wd._landed = lambda: 0
        wd.beat(step=7)
        why = wd.check(now=time.monotonic() + 10.0)
        assert why is not None and "step 7" in why and why.startswith("device")
        wd._fire(why)                                   # exit_code < 0: records only
        assert wd.fired["rank"] == 0 and wd.fired["steps_issued"] == 2
    finally:
        wd.close()


def _trainer(rank, world, pipeline=True):
    from tdfo_amd.models.dlrm import DLRMConfig, DLRMTrainer
    from tdfo_amd.parallel.dist import get_info

    cfg = DLRMConfig(embedding_dim=16, table_rows=ROWS, bottom=[32, 16], top=[32, 16, 1],
                     sharding="auto", pooling=[1, 2, 1, 1, 1], pipeline=pipeline,
                     dense_lr=1e-2, emb_lr=0.05)
    return DLRMTrainer(cfg, 8, "cpu", group=get_info().group, rank=rank, world_size=world), cfg


def _hang_worker(rank, world, port, hang_rank):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), TDFO_WATCHDOG_S="")
    torch.set_num_threads(1)
    from tdfo_amd.parallel.dist import init_distributed
    from tdfo_amd.train.loop import StepLoop, make_source
    from tdfo_amd.utils.watchdog import StepWatchdog

    init_distributed("cpu", "gloo", timeout_s=120)
    tr, cfg = _trainer(rank, world)
    wd = StepWatchdog("cpu", timeout_s=3.0, rank=rank, describe=tr.progress, poll_s=0.2)
    src = make_source(cfg.table_rows, 8, "cpu", cfg.pooling_factors(), 1, rank, kind="cpu")
    loop = StepLoop(tr, src, watchdog=wd, beat_every=1)
    loop.run(3)
    if rank == hang_rank:
        real = tr.step

        def stuck():
            time.sleep(60)            # a rank that stops making progress
            real()
        tr.step = stuck
    loop.run(3)                       # every rank: stuck here -> watchdog exit 3
    os._exit(0)


def test_watchdog_ends_a_hung_job(capfd):
    """Rank 1 stops inside a step; rank 0 then blocks in the next exchange.
    Both watchdogs fire within seconds (long before gloo's 120 s timeout)."""
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_hang_worker, args=(r, 2, port, 1)) for r in range(2)]
    t0 = time.time()
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=90)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    assert not alive, "a rank outlived its watchdog"
    assert [p.exitcode for p in procs] == [3, 3]
    assert time.time() - t0 < 80
    err = capfd.readouterr().err
    assert err.count('"watchdog": "hang"') == 2 and '"why": "host' in err


def _replica_worker(rank, world, inject):
    from tdfo_amd.data.synthetic import SyntheticCriteo
    from tdfo_amd.parallel.dist import get_info
    from tdfo_amd.parallel.replicas import check_replicas

    tr, cfg = _trainer(rank, world)
    data = SyntheticCriteo(ROWS, 8, pooling=cfg.pooling, device="cpu", seed=3 + rank)
    tr.prime(*data.next())
    for _ in range(4):
        tr.set_next_batch(*data.next())
        tr.step()
    tr.pop_loss()
    state = tr.replicated_state()
    assert any(k.startswith("emb.dp.") for k in state)     # replicated tables included
    ok0, _ = check_replicas(state, get_info().group)
    if inject == rank:
        state["dense.p"].view(-1)[3] += 1e-6
    ok1, per = check_replicas(state, get_info().group)
    return ok0, ok1, per


def test_replicas_agree_and_divergence_is_caught():
    res = run_distributed(_replica_worker, 2, 1)
    for ok0, ok1, per in res:
        assert ok0 is True
        assert ok1 is False and per["dense.p"] is False
        assert all(v for k, v in per.items() if k != "dense.p")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.int64])
def test_fingerprint_is_exact(dtype):
    from tdfo_amd.parallel import replicas

    x = (torch.randn(5000) * 10).to(dtype)
    y = x.clone()
    assert torch.equal(replicas.fingerprint([x]), replicas.fingerprint([y]))
    bits = {torch.float32: torch.int32, torch.bfloat16: torch.int16, torch.int64: torch.int64}
    y.view(bits[dtype])[4321] += 1                     # one ulp / one unit apart
    assert not torch.equal(replicas.fingerprint([x]), replicas.fingerprint([y]))
    # a swap of two elements changes the position-weighted half
    z = x.clone()
    z[[10, 20]] = z[[20, 10]]
    if not torch.equal(x[10], x[20]):
        f0, f1 = replicas.fingerprint([x]), replicas.fingerprint([z])
        assert f0[0] == f1[0] and f0[1] != f1[1]
