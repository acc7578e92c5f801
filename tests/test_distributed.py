"""World-size-2 test of the frame-sharded result gather on the gloo backend
(CPU tensors): the gathered rows equal the concatenation of the per-rank rows,
bit for bit (no reduction anywhere)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_outputs(rank, F=3, D=16, R=28):
    rng = np.random.default_rng(100 + rank)
    counts = rng.integers(0, D + 1, F).astype(np.int32)
    dets = np.zeros((F, D, 5), np.float32)
    cls = np.zeros((F, D), np.int32)
    masks = []
    for f in range(F):
        dets[f, :counts[f]] = rng.uniform(0, 100, (counts[f], 5))
        cls[f, :counts[f]] = rng.integers(1, 81, counts[f])
        masks.append(rng.uniform(0, 1, (counts[f], R, R)).astype(np.float32))
    return dets, cls, counts, np.concatenate(masks) if masks else np.zeros((0, R, R), np.float32)


def _worker(rank, world, port, outq):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vosdetectron_amd.runner import ResultGatherer, shard_frames
    dets, cls, counts, masks = _rank_outputs(rank)
    g = ResultGatherer(3, 16, 28, world, "cpu")
    out = g.gather(torch.from_numpy(dets), torch.from_numpy(cls), torch.from_numpy(counts),
                   torch.from_numpy(masks), counts.tolist())
    # double-buffered async path: two gathers in flight order, second slot
    p1 = g.gather_async(torch.from_numpy(dets), torch.from_numpy(cls), torch.from_numpy(counts),
                        torch.from_numpy(masks), counts.tolist())
    r1 = {k: v.clone() for k, v in p1.wait().items()}
    p2 = g.gather_async(torch.from_numpy(dets) + 1, torch.from_numpy(cls),
                        torch.from_numpy(counts), torch.from_numpy(masks), counts.tolist())
    r2 = p2.wait()
    same = all(torch.equal(r1[k], out[k]) for k in out)
    shifted = torch.equal(r2["dets"], out["dets"] + 1) and torch.equal(r2["masks"], out["masks"])
    if rank == 0:
        outq.put({k: v.numpy().copy() for k, v in out.items()})
        outq.put(shard_frames(10, world, 1))
        outq.put((same, shifted))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_world2_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    shard = q.get(timeout=60)
    same, shifted = q.get(timeout=60)
    assert same and shifted
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    exp = [_rank_outputs(r) for r in range(world)]
    assert np.array_equal(got["dets"], np.concatenate([e[0] for e in exp]))
    assert np.array_equal(got["classes"], np.concatenate([e[1] for e in exp]))
    assert np.array_equal(got["counts"], np.concatenate([e[2] for e in exp]))
    for r, (d, c, n, m) in enumerate(exp):
        o = 0
        for f in range(3):
            k = n[f]
            assert np.array_equal(got["masks"][r * 3 + f, :k], m[o:o + k])
            assert not got["masks"][r * 3 + f, k:].any()
            o += k
    assert shard == [5, 6, 7, 8, 9]
