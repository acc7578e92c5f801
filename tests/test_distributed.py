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
    """Per-rank engine outputs; the masks are frame-major like the engine's."""
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
    from vosdetectron_amd.runner import ResultGatherer, frame_masks, shard_frames
    dets, cls, counts, masks = _rank_outputs(rank)
    g = ResultGatherer(3, 16, 28, world, "cpu", mask_rows=48)
    out = g.gather(torch.from_numpy(dets), torch.from_numpy(cls), torch.from_numpy(counts),
                   torch.from_numpy(masks))
    out = {k: v.clone() for k, v in out.items()}
    per_frame = [frame_masks(out, 3, i).numpy().copy() for i in range(world * 3)]
    # double-buffered async path: two gathers in flight order, second slot
    p1 = g.gather_async(torch.from_numpy(dets), torch.from_numpy(cls), torch.from_numpy(counts),
                        torch.from_numpy(masks))
    r1 = p1.wait(clone=True)
    p2 = g.gather_async(torch.from_numpy(dets) + 1, torch.from_numpy(cls),
                        torch.from_numpy(counts), torch.from_numpy(masks))
    r2 = p2.wait()
    same = all(torch.equal(r1[k], out[k]) for k in out)
    shifted = torch.equal(r2["dets"], out["dets"] + 1) and torch.equal(r2["masks"], out["masks"])
    # a view of a reused slot raises instead of showing a later step's rows
    for _ in range(2):  # the gather after next reuses p2's slot
        g.gather_async(torch.from_numpy(dets), torch.from_numpy(cls), torch.from_numpy(counts),
                       torch.from_numpy(masks)).wait(views=False)
    try:
        p2.wait()
        stale_raises = False
    except RuntimeError:
        stale_raises = True
    # more masks than the packet's mask rows: nothing is truncated -- finish()
    # ships the rows past mask_rows in a second gather, on every rank alike
    small = ResultGatherer(3, 16, 28, world, "cpu", mask_rows=20)
    fin = small.gather_async(torch.from_numpy(dets), torch.from_numpy(cls),
                             torch.from_numpy(counts), torch.from_numpy(masks)).finish()
    over_frames = [frame_masks(fin, 3, i).numpy().copy() for i in range(world * 3)]
    overflow_raises = all(np.array_equal(a, b) for a, b in zip(over_frames, per_frame)) \
        and "masks_extra" in fin
    # only rank 1 overflows (29 and 32 rows vs 30): rank 0 sends zero padding
    one = ResultGatherer(3, 16, 28, world, "cpu", mask_rows=30)
    fin1 = one.gather_async(torch.from_numpy(dets), torch.from_numpy(cls),
                            torch.from_numpy(counts), torch.from_numpy(masks)).finish()
    overflow_raises &= fin1["masks_extra"].shape[1] == 2 and all(
        np.array_equal(frame_masks(fin1, 3, i).numpy(), per_frame[i]) for i in range(world * 3))
    if rank == 0:
        got = {k: v.numpy().copy() for k, v in out.items()}
        got["per_frame"] = per_frame
        outq.put(got)
        outq.put(shard_frames(10, world, 1))
        outq.put((same, shifted, stale_raises, overflow_raises))
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
    same, shifted, stale_raises, overflow_raises = q.get(timeout=60)
    assert same and shifted and stale_raises and overflow_raises
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
            assert np.array_equal(got["per_frame"][r * 3 + f], m[o:o + k])
            assert got["mask_offsets"][r, f] == o
            o += k
    assert shard == [5, 6, 7, 8, 9]


def test_bench_launch_world2_dry_run():
    """`bench.py --gpus 2` without a launcher spawns 2 ranks (torch.distributed.run)
    and the bench line reports n_gpus from the live world; --dry-run runs the
    packed all-gather on gloo and checks every gathered row."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--steps", "3", "--dry-run"], capture_output=True, text=True,
                       timeout=300, env=env, cwd=root)
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["dry_run"] and line["gather_ok"]
    # the N>1 diagnostics: per-rank step time and gather share
    rk = line["rank_ms_per_step"]
    assert len(rk["per_rank"]) == 2 and rk["min"] <= rk["max"]
    assert line["gather"]["gather_ms"] > 0 and line["gather"]["share_of_step"] > 0
    assert "dp2" in line["config"]["parallelism"]
    # a launcher world that disagrees with --gpus is refused
    env2 = dict(env, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p2 = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                         "--dry-run"], capture_output=True, text=True, timeout=120, env=env2,
                        cwd=root)
    assert p2.returncode != 0 and "formed a world of 1" in p2.stderr


def test_gather_overflow_single_process():
    """Without a process group the gatherer's send slot is the result; rows past
    mask_rows come back through finish() (no collective), and frame_masks raises
    when a caller skips finish()."""
    from vosdetectron_amd.runner import ResultGatherer, frame_masks
    dets, cls, counts, masks = _rank_outputs(1)  # counts [5, 16, 11]
    g = ResultGatherer(3, 16, 28, 1, "cpu", mask_rows=10)
    t = [torch.from_numpy(a) for a in (dets, cls, counts, masks)]
    v = g.gather_async(*t).wait(clone=True)
    with pytest.raises(RuntimeError):
        frame_masks(v, 3, 1)
    fin = g.gather_async(*t).finish()
    o = 0
    for f in range(3):
        assert np.array_equal(frame_masks(fin, 3, f).numpy(), masks[o:o + counts[f]])
        o += counts[f]
    # the engine path: the packet had only mask_rows rows, complete() added the rest
    fin2 = g.gather_async(t[0], t[1], t[2], t[3][:10]).finish(masks_full=t[3])
    assert torch.equal(fin2["masks_extra"][0], t[3][10:])
