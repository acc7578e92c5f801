"""Where variants 11 / 13 (pipelined sweep) differ from variant 10 on the schedule test's
frames: mismatch counts by (P, row ph, bin pw, lane, component) and a few RoIs."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bench import fpn_levels_np, synthetic_rois  # noqa: E402
from vosdetectron_amd import ops  # noqa: E402

DEV = "cuda"
C, F = 256, 3
g = torch.Generator(device=DEV).manual_seed(7)
sizes = [(200, 336), (100, 168), (50, 84), (25, 42)]
pyr = [torch.randn((F, h, w, C), generator=g, device=DEV) for h, w in sizes]
rois = np.concatenate([synthetic_rois(f, 500, batch_idx=f) for f in range(F)])
lv = fpn_levels_np(rois) - 2
rt, lt = torch.from_numpy(rois).to(DEV), torch.from_numpy(lv).to(DEV)
scales = [1. / 4, 1. / 8, 1. / 16, 1. / 32]
for P, v in ((7, "11"), (7, "13"), (14, "11"), (14, "13")):
    print("variant", v)
    os.environ["VOSDET_ROIALIGN_VARIANT"] = "10"
    a = ops.roi_align_fpn(pyr, scales, rt, lt, P, 2, out_layout="nhwc").cpu().numpy()
    os.environ["VOSDET_ROIALIGN_VARIANT"] = v
    b = ops.roi_align_fpn(pyr, scales, rt, lt, P, 2, out_layout="nhwc").cpu().numpy()
    bad = a != b
    print("P", P, "mismatch", bad.sum(), "of", bad.size, flush=True)
    if bad.sum():
        r, ph, pw, c = np.nonzero(bad)
        print(" rois", np.unique(r)[:20], len(np.unique(r)))
        print(" ph", np.bincount(ph, minlength=P))
        print(" pw", np.bincount(pw, minlength=P))
        print(" lane", np.bincount(c // 4, minlength=64))
        print(" comp", np.bincount(c % 4, minlength=4))
        i = np.unique(r)[0]
        print(" roi", i, rois[i], "level", lv[i])
        for q in range(P):
            row = np.nonzero(bad[i, q].any(axis=1))[0]
            if len(row):
                print("  ph", q, "bad pw", row, "lanes", np.unique(np.nonzero(bad[i, q])[1] // 4)[:10])
