import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle import oracle as orc
from vosdetectron_amd import ops
dev = "cuda"
N = int(sys.argv[1]) if len(sys.argv) > 1 else 32
shapes = {2: (200, 336), 3: (100, 168), 4: (50, 84), 5: (25, 42), 6: (13, 21)}
rng = np.random.default_rng(0)
probs = [torch.from_numpy(rng.uniform(0, 1, (N, 3, H, W)).astype(np.float32)).to(dev) for H, W in shapes.values()]
deltas = [torch.from_numpy(rng.normal(0, .5, (N, 12, H, W)).astype(np.float32)).to(dev) for H, W in shapes.values()]
an = [torch.from_numpy(orc.fpn_level_anchors(l)).to(dev) for l in shapes]
info = torch.tensor([[800, 1344, 1.0]] * N, device=dev)
def run(thr, lv=None):
    idx = range(5) if lv is None else [lv]
    return ops.generate_proposals([probs[i] for i in idx], [deltas[i] for i in idx], [an[i] for i in idx],
                                  [1. / 2 ** (i + 2) for i in idx], info, 1000, 1000, thr, 0)
for presel, mlds in (("1", "1"), ("0", "1"), ("1", "0")):  # profiles/r05: lds 1 slower
  os.environ["VOSDET_RPN_PRESEL"] = presel
  os.environ["VOSDET_RPN_MASK_LDS"] = mlds
  print("VOSDET_RPN_PRESEL=%s VOSDET_RPN_MASK_LDS=%s, %d images" % (presel, mlds, N), flush=True)
  for name, thr, lv in [("all nms", 0.7, None), ("all no-nms", 0.0, None), ("P2 nms", 0.7, 0), ("P2 no-nms", 0.0, 0), ("P3 nms", 0.7, 1)]:
    for _ in range(3): run(thr, lv)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(20): run(thr, lv)
    e1.record(); e1.synchronize()
    print(name, round(e0.elapsed_time(e1) / 20 * 1e3, 1), "us", flush=True)
