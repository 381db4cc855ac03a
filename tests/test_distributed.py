"""Multi-rank search on CPU: world_size 2 over gloo (the GPU path uses nccl=RCCL).

Each rank searches its shard of the candidate range with the host-emulator
device double; the all-reduced MIN must equal a single-process search."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from mythril_amd.distributed import shard_range


def test_shard_range_partitions_exactly():
    for count in (1, 7, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            parts = [shard_range(100, count, r, world) for r in range(world)]
            assert parts[0][0] == 100
            for (b0, c0), (b1, _) in zip(parts, parts[1:]):
                assert b0 + c0 == b1
            assert sum(c for _, c in parts) == count


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mythril_amd.distributed import sharded_search
    from mythril_amd.engine import WitnessEngine, prepare
    from mythril_amd.ir import Ctx
    from tests.fakedev import FakeDevice
    c = Ctx()
    x, y = c.var("x", 256), c.var("y", 64)
    queries = [prepare([c.app("bvult", x, c.const(1 << 250, 256)), c.app("bvugt", y, c.const(1 << 62, 64))], c,
                       use_pools=False),
               prepare([c.app("=", y, c.const(12345, 64))], c, use_pools=False)]
    eng = WitnessEngine(dev=FakeDevice(chunk=512), seed=7)
    found, _ = sharded_search(eng, queries, count=4096, begin=0, flags=0)
    q.put((rank, found))
    dist.destroy_process_group()


def test_world_size_2_gloo_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res[0] == res[1]
    from mythril_amd.engine import WitnessEngine, prepare
    from mythril_amd.ir import Ctx
    from tests.fakedev import FakeDevice
    c = Ctx()
    x, y = c.var("x", 256), c.var("y", 64)
    queries = [prepare([c.app("bvult", x, c.const(1 << 250, 256)), c.app("bvugt", y, c.const(1 << 62, 64))], c,
                       use_pools=False),
               prepare([c.app("=", y, c.const(12345, 64))], c, use_pools=False)]
    eng = WitnessEngine(dev=FakeDevice(chunk=512), seed=7)
    single, _ = eng.dev.search([eng.dev.load(qq.program) for qq in queries], 7, 0, 4096, 0)
    assert res[0] == single
    assert res[0][0] is not None and res[0][1] is None


def test_u64_indices_survive_the_int64_all_reduce():
    """indices >= 2^63 (pool digits reach bit 63) and 2^63-1 must not
    overflow torch.int64 or read as "no witness"; MIN order is the u64 order."""
    from mythril_amd.distributed import _from_i64, _to_i64
    vals = [0, 1, (1 << 63) - 1, 1 << 63, (1 << 64) - 2, None]
    enc = [_to_i64(v) for v in vals]
    assert all(-(1 << 63) <= e < (1 << 63) for e in enc)
    assert enc == sorted(enc)
    assert [_from_i64(e) for e in enc] == vals
    with pytest.raises(ValueError):
        _to_i64(1 << 64)
