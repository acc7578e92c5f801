"""Two captured steps replayed concurrently on two streams (the round-4 stall,
DESIGN §6), after the GEMM-workspace fix: both graphs captured as
bench.capture_graphs does (own capture stream and pool each), then

  sequential: replay A, replay B on one stream, K times;
  concurrent: replay A on stream sA and B on stream sB, K times (each stream
              waits for its own previous replay only);

prints the frames/s of both and checks every concurrent output against the
eager step bit for bit.  Run under a short `timeout -k 10`.

  python tools/research/concurrent_replay.py [--frames 32] [--reps 6]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--reps", type=int, default=6)
    args = ap.parse_args()
    import bench
    from vosdetectron_amd import config as vcfg
    from vosdetectron_amd import ops
    from vosdetectron_amd.weights import build_model
    dev = torch.device("cuda", 0)
    cfg = vcfg.get("e2e_mask_rcnn_R-50-FPN_1x")
    F = args.frames
    model, _ = build_model(cfg, seed=0, device=dev, channels_last=True)
    pipe, fh, fw = bench.make_pipeline(cfg, model, F, "nhwc", dev)
    host = [bench.synthetic_frames(F, 1 + i * F, fh, fw) for i in range(2)]
    slots = [torch.from_numpy(h).to(dev) for h in host]
    for x in slots:
        pipe.complete(pipe.run(x, sync=False))
    torch.cuda.synchronize()
    graphs, note = {}, [None]
    bench.capture_graphs(pipe, slots, graphs, note)
    assert note[0] == "captured", note[0]
    print("plans with a workspace:", [p for p in ops.gemm_plan_list() if p[6] > 0],
          flush=True)
    (ga, oa), (gb, ob) = graphs[slots[0].data_ptr()], graphs[slots[1].data_ptr()]
    refs = [pipe.run(x, sync=True) for x in slots]
    refs = [{k: refs[i][k].clone() for k in ("dets", "counts", "masks")} for i in range(2)]
    torch.cuda.synchronize()

    def seq():
        for _ in range(args.reps):
            ga.replay()
            gb.replay()
        torch.cuda.synchronize()

    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()

    def conc():
        cur = torch.cuda.current_stream()
        sa.wait_stream(cur)
        sb.wait_stream(cur)
        for _ in range(args.reps):
            with torch.cuda.stream(sa):
                ga.replay()
            with torch.cuda.stream(sb):
                gb.replay()
        cur.wait_stream(sa)
        cur.wait_stream(sb)
        torch.cuda.synchronize()

    res = {}
    for name, fn in (("sequential", seq), ("concurrent", conc), ("sequential2", seq),
                     ("concurrent2", conc)):
        t0 = time.perf_counter()
        fn()
        dt = time.perf_counter() - t0
        res[name] = round(2 * F * args.reps / dt, 2)
        print(name, res[name], "frames/s", flush=True)
    ok = True
    for i, o in enumerate((oa, ob)):
        M = sum(int(c) for c in o["counts"].cpu().tolist())
        ok &= torch.equal(o["dets"], refs[i]["dets"]) and torch.equal(o["counts"], refs[i]["counts"])
        ok &= torch.equal(o["masks"][:M], refs[i]["masks"][:M])
    res["bit_identical_to_eager"] = bool(ok)
    print(json.dumps(res), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
