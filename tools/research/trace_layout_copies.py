"""Research: report every layout conversion (a copy) ops._like / _fmt / torch
.contiguous() makes inside one VOS engine step at the benched batch, with a short stack,
to find the step's large direct copies."""
import traceback

import torch

import bench
from vosdetectron_amd import config as vcfg, ops
from vosdetectron_amd.weights import build_model

orig_like = ops._like


def like(x, layout, name):
    y = orig_like(x, layout, name)
    if y is not x:
        print("ops._like copy", name, tuple(x.shape), x.numel() * 4 / 1e6, "MB")
        print("".join(traceback.format_stack(limit=5)[:-1]))
    return y


ops._like = like
orig_contig = torch.Tensor.contiguous


def contig(self, *a, **k):
    y = orig_contig(self, *a, **k)
    if y.data_ptr() != self.data_ptr() and self.numel() * 4 > 64e6:
        print("contiguous copy", tuple(self.shape), self.numel() * 4 / 1e6, "MB", k)
        print("".join(traceback.format_stack(limit=5)[:-1]))
    return y


torch.Tensor.contiguous = contig
cfg = vcfg.get("vos_R-101-FPN_3x_gn_dynamic_davis")
dev = torch.device("cuda")
model, sd = build_model(cfg, seed=0, device=dev, channels_last=True)
F_ = bench.default_frames(cfg)
pipe = bench.make_pipeline(cfg, model, F_, "nhwc", dev)[0]
fr = torch.from_numpy(bench.synthetic_frames(F_, 1, 480, 854)).to(dev)
for i in range(2):
    print("=== step", i, flush=True)
    pipe.run(fr)
    torch.cuda.synchronize()

# the copies themselves: aten::copy_ calls of > 64 MB in one step, with Python stacks
from torch.profiler import ProfilerActivity, profile

with profile(activities=[ProfilerActivity.CPU], record_shapes=True, with_stack=True) as prof:
    pipe.run(fr)
    torch.cuda.synchronize()
for ev in prof.events():
    if ev.name in ("aten::copy_", "aten::clone", "aten::contiguous", "aten::reshape",
                   "aten::_reshape_alias", "aten::cat", "aten::to", "aten::_to_copy"):
        shp = ev.input_shapes[0] if ev.input_shapes else []
        n = 1
        for d in shp:
            n *= d
        if n * 4 > 64e6:
            print(ev.name, shp, "\n   ", "\n    ".join(ev.stack[:6]))
