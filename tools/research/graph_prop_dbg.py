"""Round 5 debug: vd_generate_proposals (radix select) under hipGraph capture.
(1) the op alone at the 32-frame R-50-FPN level shapes, captured and replayed with
new scores; (2) the test_graph_replay fixture flow, replaying the capture batch
and a new one."""
import sys
import os
import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from vosdetectron_amd import ops  # noqa: E402

DEV = torch.device("cuda")


def op_alone():
    g = torch.Generator(device="cuda").manual_seed(0)
    F, A = 32, 3
    shapes = [(200, 336), (100, 168), (50, 84), (25, 42), (13, 21)]
    scales = [1 / 4., 1 / 8., 1 / 16., 1 / 32., 1 / 64.]
    cls = [torch.rand(F, A, h, w, device=DEV, generator=g) for h, w in shapes]
    box = [torch.randn(F, 4 * A, h, w, device=DEV, generator=g) * .1 for h, w in shapes]
    anc = [torch.rand(h * w * A, 4, device=DEV, generator=g, dtype=torch.float64) * 500
           for h, w in shapes]
    for a in anc:
        a[:, 2:] += a[:, :2] + 16
    info = torch.tensor([[800., 1344., 1.]] * F, device=DEV)
    eager = ops.generate_proposals(cls, box, anc, scales, info, 1000, 1000, 0.7, 0.)
    print("eager counts min", int(eager[2].min()), flush=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.generate_proposals(cls, box, anc, scales, info, 1000, 1000, 0.7, 0.)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        out = ops.generate_proposals(cls, box, anc, scales, info, 1000, 1000, 0.7, 0.)
    for it in range(3):
        gr.replay()
        torch.cuda.synchronize()
        same = all(torch.equal(a, b) for a, b in zip(out, eager))
        print("replay", it, "counts min", int(out[2].min()), "same as eager", same, flush=True)
    for c in cls:
        c.uniform_(generator=g)
    eager2 = ops.generate_proposals(cls, box, anc, scales, info, 1000, 1000, 0.7, 0.)
    gr.replay()
    torch.cuda.synchronize()
    print("new scores: counts min", int(out[2].min()), "same as eager",
          all(torch.equal(a, b) for a, b in zip(out, eager2)), flush=True)


def fixture_flow():
    import bench
    from vosdetectron_amd import config as vcfg
    from vosdetectron_amd.engine import FramePipeline
    from vosdetectron_amd.weights import build_model
    cfg = vcfg.get("e2e_mask_rcnn_R-50-FPN_1x")
    model, sd = build_model(cfg, seed=0, device=DEV, channels_last=True)
    B = bench.DEFAULT_FRAMES
    pipe = FramePipeline(model, cfg, batch=B, channels_last=True, device=DEV)
    host = [bench.synthetic_frames(B, 1 + i * B, 800, 1333) for i in range(3)]
    slots = [torch.from_numpy(host[0]).to(DEV), torch.from_numpy(host[1]).to(DEV)]
    for x in slots:
        pipe.complete(pipe.run(x, sync=False))
    torch.cuda.synchronize()
    graphs, note = {}, [None]
    bench.capture_graphs(pipe, slots, graphs, note)
    print("capture:", note[0], flush=True)
    for si, hb in ((0, 0), (0, 2), (1, 1), (1, 2)):
        slot = slots[si]
        slot.copy_(torch.from_numpy(host[hb]).to(DEV))
        g, gout = graphs[slot.data_ptr()]
        g.replay()
        torch.cuda.synchronize()
        c = gout["counts"].cpu().tolist() if "counts" in gout else None
        print("slot", si, "batch", hb, "counts[:4]", c[:4] if c else None, flush=True)


if __name__ == "__main__":
    op_alone()
    fixture_flow()
