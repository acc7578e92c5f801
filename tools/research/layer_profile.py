#!/usr/bin/env python3
"""Per-op (by input shape) device time of one steady-state FramePipeline step
(torch.profiler), to see which convolutions dominate the MFMA side.
usage: tools/layer_profile.py [config] [batch]"""
import os
import sys

import numpy as np
import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vosdetectron_amd import config as vcfg  # noqa: E402
from vosdetectron_amd.engine import FramePipeline  # noqa: E402
from vosdetectron_amd.weights import build_model  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "e2e_mask_rcnn_R-50-FPN_1x"
    F = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    dev = torch.device("cuda")
    torch.backends.cudnn.benchmark = True
    cfg = vcfg.get(name)
    model, _ = build_model(cfg, device=dev, channels_last=True)
    pipe = FramePipeline(model, cfg, batch=F, channels_last=True, device=dev)
    fr = torch.from_numpy(np.random.RandomState(1).randint(0, 256, (F, 800, 1333, 3),
                                                           np.uint8)).to(dev)
    for _ in range(3):
        pipe.run(fr)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                 record_shapes=True) as prof:
        pipe.run(fr)
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(
        sort_by="device_time_total", row_limit=40, max_name_column_width=40,
        max_shapes_column_width=90))


if __name__ == "__main__":
    main()
