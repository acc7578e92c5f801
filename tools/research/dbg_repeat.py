"""Run-to-run determinism of a small (3-frame) step on a batch-B pipeline: which
intermediate differs between two identical runs."""
import sys

import torch

sys.path.insert(0, '.')
import bench  # noqa: E402
from vosdetectron_amd import config as vcfg  # noqa: E402
from vosdetectron_amd.engine import FramePipeline  # noqa: E402
from vosdetectron_amd.weights import build_model  # noqa: E402

DEV = torch.device('cuda')
B, NF = int(sys.argv[1]), int(sys.argv[2])
cfg = vcfg.get("e2e_mask_rcnn_R-50-FPN_1x")
model, sd = build_model(cfg, seed=0, device=DEV, channels_last=True)
pipe = FramePipeline(model, cfg, batch=B, channels_last=True, device=DEV)
frames = torch.from_numpy(bench.synthetic_frames(B, 1, 800, 1333)[:NF]).to(DEV)


def snap(r):
    out = {}
    for k, v in r.items():
        if isinstance(v, torch.Tensor):
            out[k] = v.clone()
        elif isinstance(v, (list, tuple)) and v and isinstance(v[0], torch.Tensor):
            for i, t in enumerate(v):
                out["%s[%d]" % (k, i)] = t.clone()
    return out


runs = []
for it in range(3):
    r = pipe.run(frames, sync=True, keep_intermediates=True)
    torch.cuda.synchronize()
    runs.append(snap(r))
for it in (1, 2):
    for k in runs[0]:
        a, b = runs[0][k], runs[it][k]
        if a.shape != b.shape:
            print(it, k, "shape", tuple(a.shape), tuple(b.shape))
        elif not torch.equal(a, b):
            print(it, k, "diff", tuple(a.shape), float((a.float() - b.float()).abs().max()), flush=True)
print("keys", list(runs[0].keys()))
