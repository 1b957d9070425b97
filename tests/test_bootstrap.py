"""Multi-process rendezvous on CPU: world_size-2 `gloo` group distributes the ncclUniqueId (as
bench.py does for --gpus N) and the library's TCP bootstrap allgathers over it."""
import os
import socket

import pytest
import torch.multiprocessing as mp

import msccl_amd as M


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    obj = [M.get_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    out = M.bootstrap_allgather(obj[0], rank, world, bytes([rank + 1]) * 16)
    # second round on a fresh root proves independence of ids
    obj2 = [M.get_unique_id() if rank == 1 else None]
    dist.broadcast_object_list(obj2, src=1)
    out2 = M.bootstrap_allgather(obj2[0], rank, world, rank.to_bytes(4, "little"))
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, out, out2))


@pytest.mark.parametrize("world", [2, 3])
def test_bootstrap_allgather_multiprocess(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r, out, out2 = q.get(timeout=120)
        res[r] = (out, out2)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = b"".join(bytes([r + 1]) * 16 for r in range(world))
    want2 = b"".join(r.to_bytes(4, "little") for r in range(world))
    for r in range(world):
        assert res[r] == (want, want2)


def _root_addr(uid):
    # BootstrapId: magic u64, addr u32 (network order), port u16 (network order), pad, nonce
    # (msccl_amd/csrc/bootstrap.h)
    return socket.inet_ntoa(uid[8:12]), int.from_bytes(uid[12:14], "big")


def _stray_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    stray = None
    if rank == 0:
        uid = M.get_unique_id()
        # a client that connects and never says Hello must not stall the root's accept loop
        stray = socket.create_connection(_root_addr(uid))
    obj = [uid if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    out = M.bootstrap_allgather(obj[0], rank, world, bytes([rank + 7]) * 8)
    dist.barrier()
    dist.destroy_process_group()
    if stray is not None:
        stray.close()
    q.put((rank, out))


def test_bootstrap_survives_silent_client():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_stray_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = b"".join(bytes([r + 7]) * 8 for r in range(world))
    assert res == {0: want, 1: want}


def test_unique_id_shape():
    uid = M.get_unique_id()
    assert len(uid) == 128 and uid != M.get_unique_id()
