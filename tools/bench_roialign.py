#!/usr/bin/env python3
"""RoIAlign (FPN, NHWC) roofline microbenchmark: the §8(d) synthetic workload,
8 distinct frames per launch.  Prints one JSON line (bench.py's roofline object).
VOSDET_ROIALIGN_VARIANT selects the kernel variant (see roi_align.hip)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import measure_roialign_roofline  # noqa: E402

if __name__ == "__main__":
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    order = os.environ.get("ORDER", "1") == "1"
    frames = int(os.environ.get("FRAMES", "8"))
    r = measure_roialign_roofline(torch.device("cuda"), frames=frames, R=R, P=P, use_order=order,
                                  out_layout=os.environ.get("RA_OUT_LAYOUT", "nhwc"),
                                  deal=int(os.environ["XCD_DEAL"]) if "XCD_DEAL" in os.environ
                                  else None,
                                  window=int(os.environ["XCD_WINDOW"]) if "XCD_WINDOW" in os.environ
                                  else None)
    r["variant"] = os.environ.get("VOSDET_ROIALIGN_VARIANT", "default")
    r["xcd_order"] = order
    print(json.dumps(r), flush=True)
