"""bench.py's timed loop run as timed, on the GPU (VERDICT r4 "do this" item 1).

The driver's N-GPU run uses exactly this concurrency on every rank, so it is
tested here in the same shape at N = 1:
  * the DEFAULT_FRAMES-frame step captured once per upload slot and replayed as
    a hipGraph (bench.StepLoop.capture -> bench.capture_graphs);
  * FrameUploader's side-stream H2D of the next batch issued during each step
    (four distinct pinned host batches, the bench's seeds);
  * a one-rank RCCL ("nccl") group: each step's packed all_gather is left in
    flight on RCCL's stream while the next step's graph replays, and the
    previous step's host read (complete) runs while it computes;
  * bench.timed_region with the per-rank watchdog armed.
Every step's GATHERED results (dets, classes, counts, class-selected masks) must
equal an eager, synchronous pipe.run of the same host batch bit for bit.
Reference: lib/core/test_engine.py:168-213 (per-GPU shards, collated results)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def rccl_world1():
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=DEV)
    try:
        yield
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_bench_timed_loop_with_rccl_gather_matches_eager(rccl_world1):
    import bench
    from vosdetectron_amd import config as vcfg
    from vosdetectron_amd import ops
    from vosdetectron_amd.runner import FrameUploader, ResultGatherer, StepWatchdog
    from vosdetectron_amd.weights import build_model

    cfg = vcfg.get("e2e_mask_rcnn_R-50-FPN_1x")
    F = bench.DEFAULT_FRAMES
    model, _ = build_model(cfg, seed=0, device=DEV, channels_last=True)
    pipe, fh, fw = bench.make_pipeline(cfg, model, F, "nhwc", DEV)
    n_host = 4
    host = [bench.synthetic_frames(F, 1 + i * F, fh, fw) for i in range(n_host)]
    uploader = FrameUploader(host, DEV)
    gatherer = ResultGatherer(F, pipe.det_cap, cfg.MRCNN.RESOLUTION, 1, DEV,
                              mask_rows=pipe.mask_rows(F))
    assert gatherer.collective
    gathered = {}

    def on_gathered(t, pending):
        gathered[t] = pending.wait(clone=True)

    loop = bench.StepLoop(pipe, uploader, gatherer, on_gathered=on_gathered)
    warm = 2
    for i in range(warm):
        loop.step(prefetch=i < warm - 1)
    loop.drain()
    torch.cuda.synchronize()
    assert loop.capture() == "captured"
    gathered.clear()
    steps = 6
    trips = []
    wd = StepWatchdog(on_trip=lambda *a: trips.append(a))
    try:
        dt, last = bench.timed_region(loop, steps, torch.cuda.synchronize, None, wd)
    finally:
        wd.stop()
    assert not trips, trips
    assert sorted(gathered) == list(range(steps))
    # which GEMM plans keep state in a workspace (the shared-workspace hazard of
    # two concurrently replayed steps): reported, not asserted
    ws_plans = [p for p in ops.gemm_plan_list() if p[6] > 0]
    print("gemm plans with a workspace:", ws_plans)
    R = cfg.MRCNN.RESOLUTION
    for b in range(n_host):
        ref = pipe.run(torch.from_numpy(host[b]).to(DEV), sync=True)
        torch.cuda.synchronize()
        counts = ref["counts_host"]
        M = sum(counts)
        assert M > 0
        for t in range(b, steps, n_host):  # step t uploaded host batch t % 4
            v = gathered[t]
            assert v["counts"].cpu().tolist() == counts, (t, b)
            assert torch.equal(v["dets"], ref["dets"]), (t, b)
            assert torch.equal(v["classes"], ref["classes"]), (t, b)
            m = v["masks"][0, :M]
            assert m.shape == (M, R, R)
            assert torch.equal(m, ref["masks"]), (t, b, float((m - ref["masks"]).abs().max()))
    assert last["counts_host"] == pipe.run(
        torch.from_numpy(host[(steps - 1) % n_host]).to(DEV), sync=True)["counts_host"]


def test_gemm_workspace_private_per_stream_and_capture():
    """ops.gemm_workspace: one workspace per (device, stream) eagerly, and a fresh
    one from the graph's own pool while a stream is capturing -- two captured
    steps never share a GEMM workspace."""
    from vosdetectron_amd import ops
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(s1):
        a = ops.gemm_workspace(DEV)
        a2 = ops.gemm_workspace(DEV)
    with torch.cuda.stream(s2):
        b = ops.gemm_workspace(DEV)
    assert a.data_ptr() == a2.data_ptr() and a.data_ptr() != b.data_ptr()
    ptrs, graphs = [], []
    x = torch.randn(256, 256, device=DEV)
    w = torch.randn(64, 256, device=DEV)
    bias = torch.zeros(64, device=DEV)
    for _ in range(2):
        g = torch.cuda.CUDAGraph()
        graphs.append(g)  # both graphs (and their pools) stay alive
        cs = torch.cuda.Stream()
        with torch.cuda.graph(g, stream=cs):
            ws = ops.gemm_workspace(DEV)
            ptrs.append(ws.data_ptr())
            y = ops.gemm_bias_act(x, w, bias, relu=False)
        g.replay()
        torch.cuda.synchronize()
        if y is not None:
            assert torch.allclose(y, x @ w.t(), rtol=1e-4, atol=1e-4)
    assert ptrs[0] != ptrs[1] and a.data_ptr() not in ptrs and b.data_ptr() not in ptrs
