#!/usr/bin/env python3
"""Benchmark: frames/s of e2e_mask_rcnn_R-50-FPN_1x inference on synthetic
800x1333 frames (BASELINE.json configs[1]), plus the RoIAlign HBM roofline and
the reference CPU path timed on the host.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch F]

One process per GPU (torchrun for N>1, RCCL).  A step = every rank uploads its own
F u8 frames from pinned host memory (side stream, inside the timed region) and runs
the full per-frame hot path on them, then one all_gather of the packed detections +
masks collects every rank's results (weak scaling: per-GPU work is fixed).  Rank 0
prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import platform
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def synthetic_frames(n, seed0, h=800, w=1333):
    return np.stack([np.random.RandomState(seed0 + i).randint(0, 256, (h, w, 3), np.uint8)
                     for i in range(n)])


def synthetic_rois(seed, R=1000, img_w=1333, img_h=800, batch_idx=0):
    """SURVEY.md §8(d) synthetic proposals."""
    rng = np.random.default_rng(seed)
    s = np.exp(rng.uniform(np.log(16), np.log(512), R))
    a = np.exp(rng.uniform(np.log(0.5), np.log(2), R))
    w, h = s / np.sqrt(a), s * np.sqrt(a)
    cx, cy = rng.uniform(0, img_w, R), rng.uniform(0, img_h, R)
    x1 = np.clip(cx - w / 2, 0, img_w - 1)
    y1 = np.clip(cy - h / 2, 0, img_h - 1)
    x2 = np.clip(cx + w / 2, 0, img_w - 1)
    y2 = np.clip(cy + h / 2, 0, img_h - 1)
    return np.stack([np.full(R, batch_idx), x1, y1, x2, y2], 1).astype(np.float32)


def fpn_levels_np(rois):
    w = rois[:, 3] - rois[:, 1] + 1
    h = rois[:, 4] - rois[:, 2] + 1
    s = np.sqrt(np.maximum(w * h, 0))
    return np.clip(np.floor(4 + np.log2(s / 224 + 1e-6)), 2, 5).astype(np.int32)


def roi_align_algorithmic_bytes(rois, lvls, sizes, C, P):
    """4*C*|union of per-RoI footprints| per level + outputs + rois."""
    touched = 0
    for li, (H, W) in enumerate(sizes):
        m = np.zeros((H, W), bool)
        sel = rois[lvls == li]
        sc = 1.0 / 2 ** (li + 2)
        for r in sel:
            x1, y1, x2, y2 = r[1] * sc, r[2] * sc, r[3] * sc, r[4] * sc
            ya, xa = int(math.floor(y1)), int(math.floor(x1))
            yb = int(math.floor(max(y2, y1 + 1))) + 1
            xb = int(math.floor(max(x2, x1 + 1))) + 1
            m[max(ya, 0):min(yb + 1, H), max(xa, 0):min(xb + 1, W)] = True
        touched += int(m.sum())
    return 4 * C * touched + 4 * len(rois) * C * P * P + 20 * len(rois)


def xcd_order(rois, lvls, n_xcd=8):
    """Scheduling permutation for the RoIAlign launch: RoIs sorted by (frame, level,
    y-band, x) and dealt so that XCD k (blocks b with b % 8 == k) walks the k-th
    contiguous slice of that order -- spatial neighbours share an L2."""
    band = np.floor((rois[:, 2] + rois[:, 4]) * 0.5 / 2.0 ** (lvls + 2) / 8).astype(np.int64)
    cx = (rois[:, 1] + rois[:, 3]) * 0.5
    srt = np.lexsort((cx, band, lvls, rois[:, 0]))
    n = len(srt)
    per = -(-n // n_xcd)
    order = np.empty(n, np.int32)
    b = np.arange(n)
    slot = (b % n_xcd) * per + b // n_xcd
    # blocks whose slot runs past n (last partial slice) take the leftovers in order
    ok = slot < n
    order[ok] = srt[slot[ok]]
    rest = np.setdiff1d(np.arange(n), order[ok], assume_unique=False)
    order[~ok] = srt[np.isin(srt, rest)]
    return order


ROIALIGN_KERNEL = {"3": "vd::roi_align_fpn_nhwc_kernel<7,2,2> (reference order)",
                   "8": "vd::roi_align_fpn_nhwc_sep_kernel<2,true> (separable, nt stores)",
                   "10": "vd::roi_align_fpn_nhwc_sep_buf_kernel<2,true,true> (separable, buffer loads, "
                         "nt stores)",
                   "30": "vd::ratile::tile_kernel (tile-binned, LDS-DMA windows, reference "
                         "arithmetic) + bin_count / tile_scan / bin_scatter / direct"}


# rocprofv3 --pmc passes of this exact launch (tools/prof_roialign.sh, separate
# passes per counter group; FETCH_SIZE doubled per the MI355X guide): L2<->fabric
# bytes per launch, committed under profiles/ and reported as "traffic".
ROIALIGN_PMC = {"8": "r02_roialign_pmc/separable_v8_xcd.json",
                # re-measured at the end of round 6 (1,530,243,616 B; round 3: 1,531,124,880)
                "10": "r06/roialign_pmc/separable_buf_v10_xcd.json"}


def measure_roialign_roofline(dev, frames=8, R=1000, C=256, P=7, sr=2, iters=None,
                              use_order=True, out_layout="nhwc", deal=None, window=None):
    """RoIAlign (FPN NHWC, one launch over 4 levels x `frames` images) timed with HIP
    events on the launch stream; >= 8 distinct frames so the working set (>700 MB)
    exceeds the 256 MB Infinity Cache."""
    from vosdetectron_amd import ops
    iters = iters or int(os.environ.get("RA_ITERS", "50"))
    sizes = [(200, 336), (100, 168), (50, 84), (25, 42)]
    scales = [1. / 4, 1. / 8, 1. / 16, 1. / 32]
    g = torch.Generator(device=dev).manual_seed(1)
    pyr = [torch.randn((frames, h, w, C), generator=g, device=dev) for h, w in sizes]
    rois, lvls, nbytes = [], [], 0
    for f in range(frames):
        r = synthetic_rois(f, R, batch_idx=f)
        lv = fpn_levels_np(r) - 2
        nbytes += roi_align_algorithmic_bytes(r, lv, sizes, C, P)
        rois.append(r)
        lvls.append(lv)
    rois_np, lv_np = np.concatenate(rois), np.concatenate(lvls)
    rois_t = torch.from_numpy(rois_np).to(dev)
    lv_t = torch.from_numpy(lv_np).to(dev)
    variant = os.environ.get("VOSDET_ROIALIGN_VARIANT", "10")
    order = ops.xcd_roi_order(rois_t, lv_t, n_xcd=deal, window=window) if use_order else None
    shape = (frames * R, P, P, C) if out_layout == "nhwc" else (frames * R, C, P, P)
    out = torch.empty(shape, device=dev)
    s = torch.cuda.current_stream()
    for _ in range(3):
        ops.roi_align_fpn(pyr, scales, rois_t, lv_t, P, sr, out=out, roi_order=order,
                          out_layout=out_layout)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        ops.roi_align_fpn(pyr, scales, rois_t, lv_t, P, sr, out=out, roi_order=order,
                          out_layout=out_layout)
    e1.record(s)
    e1.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / iters
    achieved = nbytes / t / 1e9
    traffic, tsrc = None, None
    pmc = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles",
                       ROIALIGN_PMC.get(variant, "-"))
    if use_order and out_layout == "nhwc" and (frames, R, C, P, sr) == (8, 1000, 256, 7, 2) \
            and os.path.exists(pmc):
        traffic = int(json.load(open(pmc))["traffic_bytes"])
        tsrc = os.path.relpath(pmc, os.path.dirname(os.path.abspath(__file__)))
    extra = {}
    if traffic:
        # the bytes the launch really moves through the fabric (PMC) per second:
        # beside the algorithmic rate, what the memory system delivers to it
        extra = {"traffic_over_algorithmic": round(traffic / nbytes, 3),
                 "traffic_GBs": round(traffic / t / 1e9, 1),
                 "traffic_frac": round(traffic / t / 1e9 / HBM_PEAK_GBS, 4)}
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "traffic_source": tsrc, **extra,
            "kernel": ROIALIGN_KERNEL.get(variant,
                                          "vd::roi_align_fpn_nhwc_kernel")
                      + (" (XCD-ordered)" if use_order else "") + ", out " + out_layout,
            "launch": "%d frames x %d RoIs, C=%d, P=%d, sr=%d" % (frames, R, C, P, sr),
            "algorithmic_bytes_per_launch": int(nbytes), "avg_launch_us": round(t * 1e6, 2)}


def cpu_roialign_1thread(C=256, P=7, sr=2, seed=0):
    """The reference's RoIAlign semantics on the host, single thread (oracle/roi_ops.c,
    the per-level roi_feature_transform loop): one frame of the roofline launch's
    synthetic RoIs (1000, P=7) -- SURVEY.md 8(d) asks for this number beside the
    multi-thread e2e baseline."""
    from oracle import oracle as orc
    sizes = [(200, 336), (100, 168), (50, 84), (25, 42)]
    rng = np.random.default_rng(seed + 1)
    feats = [rng.standard_normal((1, C, h, w), dtype=np.float32) for h, w in sizes]
    rois = synthetic_rois(seed, 1000)
    lv = fpn_levels_np(rois)
    d = {}
    order = []
    for k in range(2, 6):
        idx = np.where(lv == k)[0]
        d["rois_fpn%d" % k] = rois[idx]
        order.append(idx)
    d["rois_idx_restore_int32"] = np.argsort(np.concatenate(order), kind="stable").astype(np.int32)
    nbytes = roi_align_algorithmic_bytes(rois, lv - 2, sizes, C, P)
    t0 = time.perf_counter()
    orc.roi_feature_transform(feats[::-1], d, "rois", P, [1. / 32, 1. / 16, 1. / 8, 1. / 4], sr)
    dt = time.perf_counter() - t0
    return {"ms_per_frame": round(dt * 1e3, 1), "GBs_algorithmic": round(nbytes / dt / 1e9, 3),
            "threads": 1, "sample": "1 frame, 1000 synthetic RoIs (seed 0), C=256, P=7, sr=2"}


def cpu_nms_1thread(n=1000, thresh=0.7, reps=20):
    """The reference's NMS semantics on the host, one thread (oracle: cython_nms.nms
    restated in C, pinned to the executed .pyx by tests/golden/nms.npz) on the
    same N = 1000 set measure_nms times on the GPU."""
    from oracle import oracle as orc
    d = nms_bench_dets(n)
    orc.nms(d, thresh)
    t0 = time.perf_counter()
    for _ in range(reps):
        keep = orc.nms(d, thresh)
    dt = (time.perf_counter() - t0) / reps
    return {"latency_us": round(dt * 1e6, 1), "kept": int(len(keep)), "threads": 1,
            "sample": "N=%d, thresh %.1f, %d calls" % (n, thresh, reps)}


def cpu_share():
    """(threads, how) for the CPU baseline: the host CPUs this process may use --
    its affinity set, capped by a cgroup quota and by OMP_NUM_THREADS when the
    launcher sets one (the GPU box exports 16 while nproc shows the whole
    machine, and threads beyond the share only time-slice)."""
    n_aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    caps = {"affinity": n_aff}
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            caps["cgroup_quota"] = max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        caps["OMP_NUM_THREADS"] = int(omp)
    threads = min(caps.values())
    return threads, caps


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def ref_cpu_pipeline(sd, n_frames, cfg):
    """(pipeline, frames, description): the reference's CPU im_detect_all for the
    config (oracle/pipeline.py, oracle/vos_pipeline.py) and its synthetic frames."""
    from oracle.pipeline import RefCPUPipeline
    if cfg.get("VOS", False):
        from oracle.vos_pipeline import RefCPUVOSPipeline
        ref = RefCPUVOSPipeline(sd, dynamic=cfg.CONVGRU.DYNAMIC_MODEL,
                                num_classes=cfg.MODEL.NUM_CLASSES, max_size=cfg.TEST.MAX_SIZE)
        fr = synthetic_frames(n_frames + 1, 1000, 480, 854)
        what = "DAVIS-shaped 480x854 frames of one sequence, Generalized_VOS_RCNN"
    elif not cfg.FPN.FPN_ON:
        from oracle.pipeline import RefCPUPipelineC4
        from vosdetectron_amd.c4 import _conv4_counts
        ref = RefCPUPipelineC4(sd, block_counts=_conv4_counts(cfg.MODEL.CONV_BODY),
                               groups=cfg.RESNETS.NUM_GROUPS,
                               post_nms=cfg.TEST.RPN_POST_NMS_TOP_N)
        fr = synthetic_frames(n_frames + 1, 1000)
        what = "800x1333 frames, C4 (res5 head on every proposal)"
    else:
        from vosdetectron_amd.modeling import _stage_counts
        ref = RefCPUPipeline(sd, block_counts=_stage_counts(cfg.MODEL.CONV_BODY),
                             groups=cfg.RESNETS.NUM_GROUPS)
        fr = synthetic_frames(n_frames + 1, 1000)
        what = "800x1333 frames"
    return ref, fr, what


def frame_flops(sd, cfg, frames=16):
    """Algorithmic FLOPs of one frame (torch.utils.flop_counter,
    2 per MAC, convs + linears incl. the mask head at that frame's detections),
    counted on the reference's CPU path -- independent of how the GPU path
    fuses or lays out the contractions.  Returns (flops, detections, direct-form
    FLOPs the `frames`-frame engine runs as Winograd F(2x2), as F(4x4))."""
    from torch.utils.flop_counter import FlopCounterMode
    ref, fr, _ = ref_cpu_pipeline(sd, 0, cfg)
    with FlopCounterMode(display=False) as fc, _WinoFlops(frames) as wf:
        res = ref(fr[0])
    return (int(fc.get_total_flops()), int(len(res[1])), wf.flops, wf.flops4, wf.split3,
            wf.grouped_adj)


class _WinoFlops(torch.overrides.TorchFunctionMode):
    """Direct-form FLOPs of the frame's 3x3 convolutions the engine runs as
    Winograd F(2x2,3x3) (`flops`) and F(4x4,3x3) (`flops4`): the engine's own
    routing rule (modeling.conv3x3_route, incl. the mosaic choice and the
    block-occupancy gates) applied to the `frames`-frame batch of each conv the
    reference path runs.  Their MFMA work is 1/2.25 (16 positions per 2x2 tile) and
    1/4 (36 per 4x4 tile) of the direct form's.  Only stride-1 / pad-1 / ungrouped
    3x3s with a frame-level batch qualify (the mask head's RoI maps: N = frames x
    dets)."""

    def __init__(self, frames=16):
        super().__init__()
        self.flops, self.flops4, self.split3, self.frames = 0, 0, 0, frames
        # grouped 3x3s on the F(4x4) kernel's block-diagonal form: executed MFMA work
        # minus what the flop counter counts for them (16 / (C / groups) x its count)
        self.grouped_adj = 0

    def __torch_function__(self, func, types, args=(), kwargs=None):
        from vosdetectron_amd import ops
        kwargs = kwargs or {}
        out = func(*args, **kwargs)
        # GEMM-shaped contractions the engine runs on the split-bf16 kernel
        # (ops.gemm_bias_act's rule: K >= SPLIT3_MIN_K, N a multiple of 64; the box
        # head's cls_score / bbox_pred run fused, N padded to 448)
        if ops.split3_enabled():
            if func in (torch.nn.functional.linear,):
                x, w = args[0], args[1]
                if w.shape[1] >= ops.SPLIT3_MIN_K and w.shape[1] % 16 == 0:
                    self.split3 += 2 * x.numel() // x.shape[-1] * w.shape[0] * w.shape[1]
            elif func in (torch.nn.functional.conv2d, torch.conv2d):
                w = args[1]
                if tuple(w.shape[2:]) == (1, 1) and w.shape[1] >= ops.SPLIT3_MIN_K and \
                        w.shape[1] % 16 == 0 and w.shape[0] % 64 == 0:
                    self.split3 += 2 * out.numel() * w.shape[1]
                elif (tuple(w.shape) == (64, 3, 7, 7)
                      and os.environ.get("VOSDET_STEM", "split") == "split"):
                    self.split3 += 2 * out.numel() * 147  # the split-bf16 stem
            elif func in (torch.nn.functional.conv_transpose2d, torch.conv_transpose2d):
                x, w = args[0], args[1]  # w: Cin x Cout x kh x kw
                n = w.shape[1] * w.shape[2] * w.shape[3]
                if w.shape[0] >= ops.SPLIT3_MIN_K and n % 64 == 0:
                    self.split3 += 2 * x.numel() * n
        if func in (torch.nn.functional.conv2d, torch.conv2d):
            from vosdetectron_amd.modeling import conv3x3_route
            x, w = args[0], args[1]
            rest = list(args[3:]) + [None] * 4
            stride = kwargs.get("stride", rest[0] if rest[0] is not None else 1)
            padding = kwargs.get("padding", rest[1] if rest[1] is not None else 0)
            groups = kwargs.get("groups", rest[3] if rest[3] is not None else 1)
            st = tuple(stride) if isinstance(stride, (tuple, list)) else (stride, stride)
            pd = tuple(padding) if isinstance(padding, (tuple, list)) else (padding, padding)
            Cout, Cin = w.shape[0], w.shape[1]
            N, H, W = out.shape[0], out.shape[2], out.shape[3]
            if tuple(w.shape[2:]) == (3, 3) and st == (1, 1) and pd == (1, 1) and groups > 1:
                from vosdetectron_amd.modeling import conv3x3_grouped_route
                if conv3x3_grouped_route(N * self.frames, Cin * groups, Cout, H, W,
                                         groups) is not None:
                    fc_ = 2 * N * H * W * Cout * Cin * 9  # Cin = C / groups here
                    self.grouped_adj += fc_ * 16 // Cin - fc_
            dil = kwargs.get("dilation", rest[2] if rest[2] is not None else 1)
            dl = tuple(dil) if isinstance(dil, (tuple, list)) else (dil, dil)
            if (tuple(w.shape[2:]) == (3, 3) and st == (1, 1) and pd == (2, 2) and dl == (2, 2)
                    and groups == 1 and H % 2 == 0 and W % 2 == 0):
                # dilation 2: the plain conv of 4 polyphase sub-maps (modeling._conv3x3_mfma)
                algo = conv3x3_route(4 * N * self.frames, Cin, Cout, H // 2, W // 2)[0]
                if algo == "wino":
                    self.flops += 2 * N * H * W * Cout * Cin * 9
                elif algo == "wino4":
                    self.flops4 += 2 * N * H * W * Cout * Cin * 9
            if tuple(w.shape[2:]) == (3, 3) and st == (1, 1) and pd == (1, 1) and groups == 1:
                # one reference frame's conv -> the engine's batch of `frames` frames
                algo = conv3x3_route(N * self.frames, Cin, Cout, H, W)[0]
                if algo == "wino":
                    self.flops += 2 * N * H * W * Cout * Cin * 9
                elif algo == "wino4":
                    self.flops4 += 2 * N * H * W * Cout * Cin * 9
        return out


def measure_hbm_copy(dev, nbytes=2 << 30, iters=20):
    """Device-to-device copy bandwidth (read + write bytes / time), SURVEY.md 8(d)'s
    'measured stream-copy bandwidth' beside the 8 TB/s spec peak."""
    n = nbytes // 4
    src = torch.empty(n, device=dev).uniform_()
    dst = torch.empty_like(src)
    for _ in range(3):
        dst.copy_(src)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        dst.copy_(src)
    e1.record(s)
    e1.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / iters
    del src, dst
    return {"GBs": round(2 * n * 4 / t / 1e9, 1), "frac_of_spec": round(2 * n * 4 / t / 1e9 /
                                                                         HBM_PEAK_GBS, 4),
            "bytes_per_copy": 2 * n * 4, "how": "torch copy_ of a 2 GiB fp32 buffer, HIP events"}


MFMA_FP32_PEAK_TFS = 157.3  # MI355X dense fp32 matrix peak


def measure_dominant_conv(dev, F, H, W, C=256, iters=None):
    """The step's dominant kernel by time: the P2 3x3 256 -> 256 convolution (FPN
    posthoc and RPN conv) on the kernel the engine routes it to
    (modeling.conv3x3_route: Winograd F(4x4,3x3) at the benched 64 frames, F(2x2)
    below its workgroup gate), timed alone at the benched shape with HIP events on
    its stream.  Algorithmic FLOPs are the direct convolution's 2*9*C*Cout per
    output pixel (what the reference computes; Winograd takes the rate past the
    peak), executed FLOPs the MFMA positions actually run: 16 per 2x2 tile (4/9 of
    the direct form) or 36 per 4x4 tile (1/4)."""
    from vosdetectron_amd import modeling, ops
    iters = iters or int(os.environ.get("CONV_ITERS", "10"))
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn((F, C, H, W), generator=g, device=dev).contiguous(
        memory_format=torch.channels_last)
    w = torch.randn((C, C, 3, 3), generator=g, device=dev) / (9 * C) ** .5
    b = torch.randn((C,), generator=g, device=dev)
    algo, mos = modeling.conv3x3_route(F, C, C, H, W)
    if algo == "wino4":
        u = ops.conv3x3_wino4_weight(w)
        run = lambda out=None: ops.conv3x3_wino4_bias_act(  # noqa: E731
            x, u, b, out=out, mosaic=mos or False)
        name = "vd::conv3x3_wino4_kernel (Winograd F(4x4,3x3), v_mfma_f32_16x16x4_f32)"
        share, positions = 1 / 4, "36 positions per 4x4 tile, 1/4"
    else:
        u = ops.conv3x3_wino_weight(w)
        run = lambda out=None: ops.conv3x3_wino_bias_act(x, u, b, out=out,  # noqa: E731
                                                         mosaic=mos or False)
        name = "vd::conv3x3_wino2_kernel (Winograd F(2x2,3x3), v_mfma_f32_16x16x4_f32)"
        share, positions = 4 / 9, "16 positions per 2x2 tile, 4/9"
    y = run()
    if y is None:
        return None
    for _ in range(2):
        run(y)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        run(y)
    e1.record(s)
    e1.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / iters
    alg = 2.0 * F * H * W * C * C * 9
    exe = alg * share
    del x, y, u
    return {"kernel": name, "route": algo + ("_" + mos if isinstance(mos, str) else ""),
            "bound": "mfma", "shape": [F, C, H, W, C], "avg_launch_us": round(t * 1e6, 1),
            "unit": "TFLOP/s", "peak": MFMA_FP32_PEAK_TFS,
            "achieved": round(exe / t / 1e12, 1),
            "frac": round(exe / t / 1e12 / MFMA_FP32_PEAK_TFS, 4),
            "direct_conv_equivalent_TFs": round(alg / t / 1e12, 1),
            "how": "HIP events over %d launches; achieved / frac = the MFMA work Winograd "
                   "executes (%s of the direct FLOPs); direct_conv_equivalent_TFs = "
                   "direct-conv FLOPs / time, a rate that exceeds the peak by design, "
                   "not a fraction" % (iters, positions)}


MFMA_BF16_PEAK_TFS = 2516.6  # dense bf16 matrix peak: 256 CUs x 4 SIMDs x 1024 flop/clk x 2.4 GHz


def measure_split_gemm(dev, M=32000, N=1024, K=12544, iters=10):
    """The largest split-bf16 GEMM of the step, fc6 of the box head (F x 1000 RoIs
    x 12,544 -> 1,024, ReLU), timed alone with HIP events on its stream: fp32 work per
    second, and the bf16 matrix-core work it executes (six bf16 products per fp32 MAC)
    as a fraction of the dense bf16 peak."""
    from vosdetectron_amd import ops
    if not ops.split3_enabled():
        return None
    g = torch.Generator(device=dev).manual_seed(5)
    a = torch.randn((M, K), generator=g, device=dev).relu_()
    w = torch.randn((N, K), generator=g, device=dev) / K ** .5
    b = torch.zeros((N,), device=dev)
    wp = ops.gemm_split3_weight(w)
    out = torch.empty((M, N), device=dev)
    for _ in range(2):
        ops.gemm_split3_bias_act(a, wp, b, out=out)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        ops.gemm_split3_bias_act(a, wp, b, out=out)
    e1.record(s)
    e1.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / iters
    flops = 2.0 * M * N * K
    del a, w, wp, out
    return {"kernel": "vd::gemm_split3_kernel (three-piece bf16 split, six "
                      "v_mfma_f32_32x32x16_bf16 products per fp32 MAC)",
            "shape": [M, N, K], "avg_launch_us": round(t * 1e6, 1),
            "fp32_work_TFs": round(flops / t / 1e12, 1),
            "fp32_matrix_peak_TFs": MFMA_FP32_PEAK_TFS,
            "bf16_executed_TFs": round(6 * flops / t / 1e12, 1),
            "bf16_peak_TFs": MFMA_BF16_PEAK_TFS,
            "frac": round(6 * flops / t / 1e12 / MFMA_BF16_PEAK_TFS, 4),
            "how": "HIP events over %d launches; frac = executed bf16 MFMA work / the dense "
                   "bf16 peak (fp32_work_TFs exceeds the fp32 matrix peak by design)" % iters}


def step_roofline(flops_frame, dets_cpu, frames, ms_per_step, engine_launch, frame_hw, blob_hw,
                  wino_flops_frame=0, wino4_flops_frame=0, split3_flops_frame=0,
                  grouped_adj_frame=0):
    """the FPS as a fraction of the roofline = sum of per-stage
    bound times / measured step time.  MFMA-bound stages: the FLOPs the engine's
    MFMAs execute for one frame at the fp32 matrix peak -- the reference's
    algorithmic FLOPs (torch.utils.flop_counter on its CPU path) with the
    convolutions the engine runs as Winograd F(2x2,3x3) / F(4x4,3x3) priced at the
    1/2.25 / 1/4 of their direct form that Winograd multiplies; HBM-bound stages: the box
    RoIAlign's algorithmic bytes (the engine's own launch) and frame prep (u8 read
    + fp32 blob write) at 8 TB/s; latency-bound stages (proposals, NMS) carry no
    bound.  `frac` is that executed-work fraction (<= 1 by construction).  Pricing
    every conv in its direct form instead gives a rate, not a fraction (Winograd
    takes it past 1): reported as `direct_conv_equivalent`, never as a frac.  The
    1x1 convs / fc layers the engine runs on the split-bf16 GEMM (round 6) execute
    six bf16 products per fp32 MAC on the bf16 matrix cores: priced at 6 x their
    FLOPs at the dense bf16 peak (0.38 of their time at the fp32 peak)."""
    exec_flops = (flops_frame - wino_flops_frame * (1 - 1 / 2.25)
                  - wino4_flops_frame * (1 - 1 / 4.0) + grouped_adj_frame)
    exec_ms = ((exec_flops - split3_flops_frame) / (MFMA_FP32_PEAK_TFS * 1e12)
               + 6 * split3_flops_frame / (MFMA_BF16_PEAK_TFS * 1e12)) * frames * 1e3
    direct_ms = flops_frame * frames / (MFMA_FP32_PEAK_TFS * 1e12) * 1e3
    h, w = frame_hw
    blob_bytes = frames * (h * w * 3 + 3 * 4 * blob_hw[0] * blob_hw[1])
    ra_bytes = engine_launch["algorithmic_bytes_per_launch"] if engine_launch else 0
    hbm_ms = (blob_bytes + ra_bytes) / (HBM_PEAK_GBS * 1e9) * 1e3
    bound = exec_ms + hbm_ms
    return {"bound_ms_per_step": round(bound, 3), "mfma_bound_ms": round(exec_ms, 3),
            "hbm_bound_ms": round(hbm_ms, 3), "frac": round(bound / ms_per_step, 4),
            "executed_gflop_per_frame": round(exec_flops / 1e9, 2),
            "winograd_direct_gflop_per_frame": round(wino_flops_frame / 1e9, 2),
            "winograd4_direct_gflop_per_frame": round(wino4_flops_frame / 1e9, 2),
            "split_bf16_gemm_gflop_per_frame": round(split3_flops_frame / 1e9, 2),
            "mfma_util_step": round(exec_ms / ms_per_step, 4),
            "direct_conv_equivalent": {
                "gflop_per_frame": round(flops_frame / 1e9, 2),
                "TFs": round(flops_frame * frames / (ms_per_step * 1e-3) / 1e12, 1),
                "ms_at_peak": round(direct_ms, 3),
                "note": "reference FLOPs (every conv direct) / step time: a rate, not a "
                        "roofline fraction"},
            "dets_in_counted_frame": dets_cpu,
            "peaks": {"fp32_matrix_TFs": MFMA_FP32_PEAK_TFS, "bf16_matrix_TFs": MFMA_BF16_PEAK_TFS,
                      "hbm_GBs": HBM_PEAK_GBS},
            "flops_source": "torch.utils.flop_counter over one frame of the reference CPU path "
                            "(oracle/pipeline.py), 2 flop per MAC; Winograd convs by the "
                            "engine's routing rule (modeling.conv3x3_route)"}


def cpu_baseline(cfg_name, sd, n_frames=16, threads=None, cfg=None, min_seconds=10.0):
    """The reference's CPU path (oracle/pipeline.py, oracle/vos_pipeline.py) on a
    bounded sample: frames are run until ``min_seconds`` of CPU work (at least 2 frames,
    at most ``n_frames``), so the sample is ~10-30 s whatever the host."""
    share, caps = cpu_share()
    threads = threads or share
    torch.set_num_threads(threads)
    ref, fr, what = ref_cpu_pipeline(sd, n_frames, cfg)
    ref(fr[0])  # warm-up
    t0 = time.perf_counter()
    done = 0
    while done < n_frames and (done < 2 or time.perf_counter() - t0 < min_seconds):
        ref(fr[done + 1])
        done += 1
    dt = time.perf_counter() - t0
    n_frames = done
    ra = None if (cfg is not None and (cfg.get("VOS", False) or not cfg.FPN.FPN_ON)) \
        else cpu_roialign_1thread()
    return {"value": round(n_frames / dt, 4), "unit": "frames/s", "cores": threads,
            "kind": "port", "roialign_1thread": ra, "nms_1thread": cpu_nms_1thread(),
            "cpu_model": cpu_model(),
            "nproc": os.cpu_count(), "cpu_share": caps,
            "sample": "%d synthetic %s, im_detect_all path (torch-CPU convs on %d threads, "
                      "oracle C RoIAlign/NMS, numpy proposals; segm_results excluded as in "
                      "the GPU line), %.1f s" % (n_frames, what, threads, dt)}


def measure_pipeline_roialign(pipe, frames_dev, reps=20):
    """Roofline of the engine's OWN box RoIAlign launch: the real proposals and
    pyramid of one batch (keep_intermediates), algorithmic bytes from those
    RoIs (§8d formula), time = HIP events around `reps` launches on the stream
    the engine launches on."""
    from vosdetectron_amd import ops
    cfg = pipe.cfg
    out = pipe.run(frames_dev, keep_intermediates=True)
    pyr = out["pyramid"]
    F = frames_dev.shape[0]
    rois_all, lv_all, nbytes = [], [], 0
    counts = out["roi_counts"].cpu().tolist()
    sizes = [tuple(p.shape[1:3]) for p in pyr]
    C = pyr[0].shape[3]
    P = cfg.FAST_RCNN.ROI_XFORM_RESOLUTION
    for f in range(F):
        r = out["rois"][f, :counts[f]].cpu().numpy()
        lv = fpn_levels_np(r) - 2
        nbytes += roi_align_algorithmic_bytes(r, lv, sizes, C, P)
        rois_all.append(r)
        lv_all.append(lv)
    rois_t = torch.from_numpy(np.concatenate(rois_all)).to(frames_dev.device)
    lv_t = torch.from_numpy(np.concatenate(lv_all).astype(np.int32)).to(frames_dev.device)
    order = ops.xcd_roi_order(rois_t, lv_t)
    res = torch.empty((rois_t.shape[0], P, P, C), device=frames_dev.device)
    sr = cfg.FAST_RCNN.ROI_XFORM_SAMPLING_RATIO
    for _ in range(3):
        ops.roi_align_fpn(pyr, pipe.roi_scales, rois_t, lv_t, P, sr, roi_order=order, out=res,
                          out_layout="nhwc")
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        ops.roi_align_fpn(pyr, pipe.roi_scales, rois_t, lv_t, P, sr, roi_order=order, out=res,
                          out_layout="nhwc")
    e1.record(s)
    e1.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / reps
    return {"bound": "hbm", "achieved": round(nbytes / t / 1e9, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(nbytes / t / 1e9 / HBM_PEAK_GBS, 4),
            "launch": "engine box RoIAlign, %d frames x %d real proposals, C=%d, P=%d, sr=%d"
                      % (F, rois_t.shape[0] // max(F, 1), C, P, sr),
            "algorithmic_bytes_per_launch": int(nbytes), "avg_launch_us": round(t * 1e6, 2)}


def _event_time(fn, reps, warm=3):
    """Average seconds of fn() over `reps` calls, HIP events on the current stream
    (the stream the ops launch on)."""
    for _ in range(warm):
        fn()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / 1e3 / reps


def nms_bench_dets(n=1000, seed=3):
    """SURVEY 8(d) synthetic proposals (1333 x 800 frame) with uniform scores: the
    BASELINE.md NMS row's N = 1000 input."""
    r = synthetic_rois(seed, n)
    sc = np.random.default_rng(seed + 1).random(n).astype(np.float32)
    return np.concatenate([r[:, 1:5], sc[:, None]], 1).astype(np.float32)


def measure_nms(dev, n=1000, thresh=0.7, reps=200):
    """BASELINE.md 3 'NMS latency N=1000, thr 0.7': vd_nms (cython_nms semantics,
    bit-exact vs the executed reference: tests/golden/nms.npz) on one set of N
    boxes, HIP events over `reps` launches with preallocated workspace -- the
    device latency of one call, no host read.  SURVEY 8(d): latency bound; the
    greedy algorithm's work is N^2/2 IoU evaluations."""
    from vosdetectron_amd import _lib
    d = torch.from_numpy(nms_bench_dets(n)).to(dev)
    keep = torch.empty((n,), dtype=torch.int64, device=dev)
    num = torch.zeros((1,), dtype=torch.int32, device=dev)
    L = _lib.lib()
    ws = torch.empty((max(int(L.vd_nms_workspace_size(n)), 256),), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    th = float(np.float32(thresh))

    def run():
        _lib.check(L.vd_nms(d.data_ptr(), n, 5, th, keep.data_ptr(), num.data_ptr(),
                            ws.data_ptr(), ws.numel(), stream), "vd_nms")
    t = _event_time(run, reps)
    kept = int(num.item())
    evals = n * (n - 1) // 2
    return {"kernel": "vd_nms: nms_prep_kernel + nms_mask_kernel + nms_resolve_kernel",
            "bound": "latency", "n": n, "thresh": thresh, "kept": kept,
            "latency_us": round(t * 1e6, 2), "iou_evals": evals,
            "iou_evals_per_s": round(evals / t, 1),
            "input": "SURVEY 8(d) synthetic RoIs (seed 3), uniform scores (seed 4)",
            "how": "HIP events over %d launches, preallocated workspace" % reps,
            "rocprof": "profiles/r06/head_d/trace/post_launches.txt: nms_prep 14.5 + nms_mask "
                       "8.1 + nms_resolve 30.6 us per launch (rocprofv3 --kernel-trace, 203 calls)"}


def measure_step_post(pipe, frames_dev, reps=20):
    """The step's proposal and detection kernels on the engine's own tensors
    (keep_intermediates): vd_generate_proposals over P2-P6 x F frames (anchors,
    decode, clip, filter, top-k, NMS 0.7) priced against SURVEY 8(d)'s HBM bytes
    -- 20 B per anchor read (4 B score + 16 B deltas) + 24 B per written proposal
    -- and vd_box_detections (decode, 80-class NMS 0.5, top-100) as a latency."""
    from vosdetectron_amd import ops
    cfg = pipe.cfg
    tst = cfg.TEST
    out = pipe.run(frames_dev, keep_intermediates=True)
    probs, deltas = out["rpn_probs"], out["rpn_deltas"]
    F = frames_dev.shape[0]
    bufs = [torch.zeros((F, len(probs), tst.RPN_POST_NMS_TOP_N, 5), device=frames_dev.device),
            torch.zeros((F, len(probs), tst.RPN_POST_NMS_TOP_N), device=frames_dev.device),
            torch.zeros((F, len(probs)), dtype=torch.int32, device=frames_dev.device)]

    def prop():
        ops.generate_proposals(probs, deltas, pipe.anchors, pipe.rpn_scales, pipe.im_info[:F],
                               tst.RPN_PRE_NMS_TOP_N, tst.RPN_POST_NMS_TOP_N, tst.RPN_NMS_THRESH,
                               tst.RPN_MIN_SIZE, out=bufs)
    t_p = _event_time(prop, reps)
    anchors = sum(int(p.shape[1]) * int(p.shape[2]) * int(p.shape[3]) for p in probs)  # per frame
    nbytes = F * (20 * anchors + 24 * len(probs) * tst.RPN_POST_NMS_TOP_N)
    K = out["cls_prob"].shape[1]
    post = out["rois"].shape[1]
    dbufs = [torch.zeros((F, pipe.det_cap, 5), device=frames_dev.device),
             torch.zeros((F, pipe.det_cap), dtype=torch.int32, device=frames_dev.device),
             torch.zeros((F,), dtype=torch.int32, device=frames_dev.device)]

    def dets():
        ops.box_detections(out["rois"], out["cls_prob"].view(F, post, K),
                           out["bbox_pred"].view(F, post, -1), out["roi_counts"],
                           pipe.im_scale_t[:F], pipe.im_hw[:F], tst.SCORE_THRESH, tst.NMS,
                           tst.DETECTIONS_PER_IM, cfg.MODEL.BBOX_REG_WEIGHTS, pipe.det_cap,
                           out=dbufs)
    t_d = _event_time(dets, reps)
    return {"proposals": {
                "kernel": "vd_generate_proposals: rpn_proposals_kernel + rpn_nms_mask_kernel + "
                          "rpn_nms_finish_kernel (P2-P6, all frames, one launch each)",
                "bound": "hbm", "achieved": round(nbytes / t_p / 1e9, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(nbytes / t_p / 1e9 / HBM_PEAK_GBS, 4),
                "algorithmic_bytes": int(nbytes), "avg_us": round(t_p * 1e6, 1),
                "anchors_per_frame": anchors, "frames": F,
                "note": "20 B read per anchor (score + 4 deltas) + 24 B per written proposal "
                        "(SURVEY 8d); the select / NMS phases are latency-bound, so the "
                        "byte rate is far below the roofline"},
            "class_nms": {
                "kernel": "vd_box_detections: decode + class_nms_kernel (80 classes x F) + "
                          "det_limit_kernel", "bound": "latency",
                "avg_us": round(t_d * 1e6, 1), "frames": F, "rois_per_frame": post,
                "us_per_frame": round(t_d * 1e6 / F, 2)},
            "how": "HIP events over %d launches on the engine's own step tensors" % reps,
            "rocprof": "profiles/r06/head_i/trace/post_launches.txt (64 frames): rpn_proposals "
                       "85.5 (+ 6 rpn_sel_hist, rpn_sel_compact) + rpn_nms_mask 244.0 + "
                       "rpn_nms_finish 64.7 us; class_nms 818.7 + det_limit 41.6 us per launch "
                       "(rocprofv3 --kernel-trace, 36 calls)"}


def measure_segm(pipe, out, frames=16):
    """segm_results (fused device paste + RLE, device rleToString, host string
    slicing and class grouping) per frame over one step's frames -- outside the
    FPS by SURVEY §8d's definition, reported beside it."""
    from vosdetectron_amd.engine import frame_segms
    sub = dict(out)
    k = min(frames, len(out["counts_host"]))
    sub["counts_host"] = out["counts_host"][:k]
    frame_segms(pipe, sub)  # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    frame_segms(pipe, sub)
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / k * 1e3, 3)


def capture_graphs(pipe, slots, graphs, note):
    """Capture one hipGraph of the whole step per frame slot (sync=False: no host
    read inside).  Each graph is captured on a stream of its own and into a
    memory pool of its own, so nothing a launch keeps state in is shared between
    the two graphs: torch's BLAS workspaces are per (handle, stream), and
    ops.gemm_workspace allocates from the capturing graph's pool (a
    shared GEMM workspace is what stalled two concurrently replayed steps in
    round 4).  Eager execution stays in place if capture fails."""
    try:
        for x in slots[:2]:
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                pipe.run(x, sync=False)  # warm on the capture stream
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                gout = pipe.run(x, sync=False)
            torch.cuda.synchronize()
            graphs[x.data_ptr()] = (g, gout)
        note[0] = "captured"
    except Exception as e:  # noqa: BLE001 -- report and run eagerly
        graphs.clear()
        note[0] = "capture failed: %s" % (str(e).splitlines()[0][:200],)
        print("bench: hipGraph %s; running eagerly" % note[0], file=sys.stderr, flush=True)
        torch.cuda.synchronize()


class StepLoop:
    """The step bench.py times, shared by main() and by the GPU test
    that runs it as timed (tests/test_timed_loop_gpu.py).  One step: take the
    next u8 batch (FrameUploader: its H2D was issued on a side stream during the
    previous step; the next batch's copy is issued now), replay the step's
    captured hipGraph for that upload slot (or run the pipeline eagerly), then
    the previous step's one host read (pipe.complete) while this step runs, then
    -- when a process group exists -- wait for the previous step's all_gather
    (stream-ordered) and issue this step's, left in flight on RCCL's stream while
    the next step computes.  At most one gather is in flight.

    on_gathered(step, pending): called with each step's PendingGather just before
    the loop waits on it (a test collects wait(clone=True) there)."""

    def __init__(self, pipe, uploader, gatherer, vos=False, seq_len=50, resident=None,
                 on_gathered=None):
        self.pipe, self.uploader, self.gatherer = pipe, uploader, gatherer
        self.vos, self.seq_len, self.resident = vos, seq_len, resident
        self.on_gathered = on_gathered
        self.asynchronous = getattr(pipe, "ASYNC", False)
        self.graphs = {}  # upload slot data_ptr -> (CUDAGraph, static outputs)
        self.graph_note = None
        self.t = 0
        self.pending = None  # (step, PendingGather)
        self.prev_out = None
        self.last_out = None

    def frames(self, t, prefetch):
        if self.resident is not None:
            return self.resident[t % len(self.resident)]
        return self.uploader.get(t, prefetch)

    def drain(self):
        """The previous step's gather has landed (stream-ordered)."""
        if self.pending is not None:
            t, p = self.pending
            self.pending = None
            if self.on_gathered is not None:
                self.on_gathered(t, p)
            p.wait(views=False)

    def step(self, prefetch=True):
        t = self.t
        self.t += 1
        pipe = self.pipe
        if self.vos and t % self.seq_len == 0:
            pipe.reset()
        frames = self.frames(t, prefetch)
        key = frames.data_ptr()
        if key in self.graphs:  # replay the captured step (one launch, no host work)
            g, gout = self.graphs[key]
            g.replay()
            out = dict(gout)
        else:
            out = pipe.run(frames, sync=not self.asynchronous)
        if self.resident is None:
            self.uploader.release(t)
        if self.asynchronous:
            # the previous step's one host read (counts, capacity, rare overflow
            # masks) while this step runs on the GPU
            if self.prev_out is not None:
                pipe.complete(self.prev_out)
            self.prev_out = out
        if self.gatherer is not None and self.gatherer.collective:
            # ONE packed all_gather per step over RCCL (runner.py)
            self.drain()
            self.pending = (t, self.gatherer.gather_async(out["dets"], out["classes"],
                                                          out["counts"], out["masks"]))
        self.last_out = out
        return out

    def capture(self):
        """Capture the step once per upload slot (after warm-up) and restart the
        upload cycle at slot 0."""
        slots = self.resident if self.resident is not None else self.uploader.dev
        note = [None]
        capture_graphs(self.pipe, slots, self.graphs, note)
        self.graph_note = note[0]
        self.t = 0
        return self.graph_note

    def finish(self):
        """The last step's gather and host read: its completed outputs."""
        self.drain()
        if self.asynchronous and self.prev_out is not None:
            self.pipe.complete(self.prev_out)
            return self.prev_out
        return self.last_out


def timed_region(loop, steps, sync, barrier=None, watchdog=None, clock=time.perf_counter):
    """bench.py's timed region: barrier + device sync, `steps` loop steps, then
    -- still inside -- the last step's gather and complete() (loop.finish: the
    counts read and any overflow mask batch), device sync + barrier.  Returns
    (seconds, the last step's completed outputs)."""
    if barrier is not None:
        barrier()
    sync()
    t0 = clock()
    for i in range(steps):
        if watchdog:
            watchdog.start_step(i)
        loop.step(prefetch=i < steps - 1)
        if watchdog:
            watchdog.end_step()
    if watchdog:
        watchdog.start_step(steps)
    out = loop.finish()
    sync()
    if watchdog:
        watchdog.end_step()
    if barrier is not None:
        barrier()
    sync()
    return clock() - t0, out


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n):
    """`python bench.py --gpus N` without a launcher: start N ranks through
    torch.distributed.run (one process per GPU, like the reference's per-GPU
    subprocesses, lib/utils/subprocess.py:41-115) and return its exit code.  Runs
    before anything touches the GPU; the ranks are children, not an exec."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(n), "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.call(cmd, env=env)


def dry_run(args, world, rank):
    """--dry-run: the N-rank plumbing on CPU (gloo): forms the world, runs K steps
    of the packed result all-gather on synthetic per-rank results, checks every
    gathered row, and prints the bench line shape with n_gpus from the live world."""
    import torch.distributed as dist
    from vosdetectron_amd.runner import ResultGatherer, frame_masks
    F, D, R = args.batch or 3, 16, 28
    g = ResultGatherer(F, D, R, world, "cpu", mask_rows=F * D)

    def results(r, t):
        rng = np.random.default_rng(1000 * t + r)
        counts = rng.integers(0, D + 1, F).astype(np.int32)
        dets = rng.uniform(0, 100, (F, D, 5)).astype(np.float32)
        cls = rng.integers(1, 81, (F, D)).astype(np.int32)
        masks = rng.uniform(0, 1, (int(counts.sum()), R, R)).astype(np.float32)
        return dets, cls, counts, masks

    t0 = time.perf_counter()
    ok = True
    for t in range(args.steps):
        d, c, n, m = results(rank, t)
        v = g.gather(torch.from_numpy(d), torch.from_numpy(c), torch.from_numpy(n),
                     torch.from_numpy(m))
        for r in range(world):
            d2, c2, n2, m2 = results(r, t)
            ok &= bool(np.array_equal(v["dets"][r * F:(r + 1) * F].numpy(), d2))
            ok &= bool(np.array_equal(v["counts"][r * F:(r + 1) * F].numpy(), n2))
            o = 0
            for f in range(F):
                ok &= bool(np.array_equal(frame_masks(v, F, r * F + f).numpy(),
                                          m2[o:o + n2[f]]))
                o += n2[f]
    dt = time.perf_counter() - t0
    # the N>1 line's diagnostics, as main() reports them: every rank's own step
    # time (value uses the slowest) and the gather's share of the step
    t = torch.tensor([dt], dtype=torch.float64)
    allt = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(allt, t)
    per = [float(x.item()) / args.steps * 1e3 for x in allt]
    tmax = max(float(x.item()) for x in allt)
    okt = torch.tensor([int(ok)])
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    tg0 = time.perf_counter()
    for _ in range(args.steps):
        g.gather_async(*[torch.from_numpy(a) for a in results(rank, 0)]).wait(views=False)
    tg = torch.tensor([time.perf_counter() - tg0], dtype=torch.float64)
    dist.all_reduce(tg, op=dist.ReduceOp.MAX)
    g_ms = float(tg.item()) / args.steps * 1e3
    if rank == 0:
        print(json.dumps({"metric": "dry-run (gloo, CPU): frame-sharded result all_gather",
                          "value": round(world * F * args.steps / tmax, 3),
                          "unit": "frames/s", "n_gpus": world, "steps": args.steps,
                          "warmup": 0, "dry_run": True, "gather_ok": bool(okt.item()),
                          "bytes_per_rank": g.bytes_per_rank,
                          "config": {"parallelism": "frame-sharded dp%d + one all_gather per "
                                                    "step (gloo rehearsal)" % world},
                          "rank_ms_per_step": {"min": round(min(per), 3),
                                               "max": round(max(per), 3),
                                               "spread": round(max(per) / min(per) - 1, 4),
                                               "per_rank": [round(v, 3) for v in per]},
                          "gather": {"gather_ms": round(g_ms, 3),
                                     "share_of_step": round(g_ms / (tmax / args.steps * 1e3), 4),
                                     "bytes_per_rank": g.bytes_per_rank}}), flush=True)
    dist.destroy_process_group()
    return 0 if okt.item() else 1


# Frames per GPU per step for the FPN engines (the metric's config): 32 measured
# 3.0 % more frames/s than 16 on one box (344.0 -> 354.3, profiles/r04/batch32/) --
# the step's latency-bound tail (proposal select, class NMS) and the small
# kernels are amortised over twice the frames; per-step latency doubles (~90 ms).
# The VOS and C4 engines stay at 16.  --batch overrides.  Round 6: 64 frames, +2.2 %
# over 32 on one box (456.7-457.6 -> 466.6-468.0 frames/s, 48: 462.1-462.6,
# profiles/r06/batch64/): the tail and the small P5 / P6 / res5 kernels amortised
# again, per-step latency ~137 ms.
DEFAULT_FRAMES = 64


def default_frames(cfg) -> int:
    return DEFAULT_FRAMES if cfg.FPN.FPN_ON and not cfg.get("VOS", False) else 16


def make_pipeline(cfg, model, F, layout, dev):
    """The engine the bench times for a config, and its frame size: the VOS loop
    (configs[3]: DAVIS-shaped 480p sequences; batch row b = sequence b of this
    rank, SURVEY.md §8e, a step = the next frame of every sequence), the C4
    single-scale family (configs[0]) or the FPN engine, at 800 x 1333."""
    from vosdetectron_amd.engine import FramePipeline
    nhwc = layout == "nhwc"
    if cfg.get("VOS", False):
        from vosdetectron_amd.engine import VOSPipeline
        return VOSPipeline(model, cfg, frame_hw=(480, 854), batch=F, channels_last=nhwc,
                           device=dev), 480, 854
    if not cfg.FPN.FPN_ON:
        from vosdetectron_amd.c4 import C4FramePipeline
        return C4FramePipeline(model, cfg, batch=F, channels_last=nhwc, device=dev), 800, 1333
    return FramePipeline(model, cfg, batch=F, channels_last=nhwc, device=dev), 800, 1333


def step_calls(pipe, vos):
    """The pipeline calls the timed step makes (bench.main's step()), as
    (callable, args, kwargs): a test binds them against the engines' signatures
    on CPU (a drift in a VOS / C4 signature otherwise costs a GPU run)."""
    asynchronous = getattr(pipe, "ASYNC", False)
    frames = object()
    calls = [(pipe.run, (frames,), {"sync": not asynchronous}), (pipe.run, (frames,), {}),
             (pipe.run, (frames,), {"keep_intermediates": True}),
             (pipe.enable_timers, (), {}), (pipe.enable_timers, (False,), {}),
             (pipe.timer_summary, (), {})]
    if vos:
        calls.append((pipe.reset, (), {}))
    if asynchronous:
        calls += [(pipe.complete, ({},), {}), (pipe.mask_rows, (1,), {})]
    return calls


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of one node; default: the launcher's WORLD_SIZE or 1. "
                         "Without a launcher, N > 1 spawns N ranks via torch.distributed.run")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None,
                    help="frames per GPU per step (default: DEFAULT_FRAMES = 64 for the FPN "
                         "engines, 16 for VOS / C4)")
    ap.add_argument("--config", default="e2e_mask_rcnn_R-50-FPN_1x")
    ap.add_argument("--layout", default="nhwc", choices=["nchw", "nhwc"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=16,
                    help="max frames in the CPU-baseline sample (run until 10 s, >= 2 frames)")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-timers", dest="timers", action="store_false",
                    help="skip the per-stage breakdown: by default, after the timed steps, "
                         "min(--steps, 3) more steps run with HIP-event stage timers and "
                         "stages_ms is reported (not part of the timed region)")
    ap.add_argument("--resident", action="store_true",
                    help="frames uploaded once before timing (round-1 definition); default: "
                         "every step uploads its u8 frames from pinned host memory inside the "
                         "timed region (SURVEY §8d)")
    ap.add_argument("--seq-len", type=int, default=50,
                    help="VOS configs: frames per synthetic sequence (hidden states reset)")
    ap.add_argument("--no-graph", dest="graph", action="store_false",
                    help="launch every step eagerly instead of replaying a captured hipGraph")
    ap.add_argument("--rccl-gather", action="store_true",
                    help="issue the per-step all-gather even at world 1 (forms a 1-rank "
                         "RCCL group), so the collective is inside the timed step")
    ap.add_argument("--no-watchdog", dest="watchdog", action="store_false",
                    help="no per-rank step watchdog (default: a timed step running longer than "
                         "10x the median step prints its index and exits the rank with status 3)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU/gloo rehearsal of the N-rank launch and gather (no GPU)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal on a one-GPU box: every rank uses device 0 and the "
                         "collectives run on gloo (RCCL refuses duplicate devices); the N-rank "
                         "launch, timing and packed gather end to end, not a measurement")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "0"))
    if world == 0:  # no launcher
        if args.gpus and args.gpus > 1:
            return spawn_ranks(args.gpus)
        world = 1
    if args.gpus is not None and args.gpus != world:
        raise SystemExit("bench: --gpus %d but the launcher formed a world of %d ranks"
                         % (args.gpus, world))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29512")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        return dry_run(args, dist.get_world_size(), rank)
    if args.share_gpu:
        local = 0
    if world > 1 or args.rccl_gather:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1:  # a one-rank RCCL group (--rccl-gather): no launcher env
            os.environ.setdefault("MASTER_PORT", str(free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        torch.cuda.set_device(local)
        if args.share_gpu:  # RCCL refuses two ranks on one device: gloo carries the rehearsal
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        world = dist.get_world_size()  # n_gpus from the live world
    dev = torch.device("cuda", local)
    torch.backends.cudnn.benchmark = True

    from vosdetectron_amd import config as vcfg
    from vosdetectron_amd.runner import FrameUploader, ResultGatherer
    from vosdetectron_amd.weights import build_model

    cfg = vcfg.get(args.config)
    vos = bool(cfg.get("VOS", False))
    model, sd = build_model(cfg, seed=0, device=dev, channels_last=args.layout == "nhwc")
    F = args.batch or default_frames(cfg)
    n_host = 4  # distinct pinned host batches cycled through
    pipe, fh, fw = make_pipeline(cfg, model, F, args.layout, dev)
    host = [synthetic_frames(F, 1 + rank * F * n_host + i * F + (7919 if vos else 0), fh, fw)
            for i in range(n_host)]
    uploader = FrameUploader(host, dev)
    if args.resident:
        resident = [torch.from_numpy(h).to(dev) for h in host]
    else:
        resident = None
    any_frames = resident[0] if args.resident else uploader.dev[0]  # post-run measurements

    # FPN engines queue a step without any host read (sync=False): the mask
    # batch has pipe.mask_rows(F) rows and the gather ships exactly those
    asynchronous = getattr(pipe, "ASYNC", False)
    mask_rows = (pipe.mask_rows(F) if asynchronous
                 else F * max(100, int(cfg.TEST.DETECTIONS_PER_IM)) + 64)
    gatherer = ResultGatherer(F, pipe.det_cap, cfg.MRCNN.RESOLUTION, world, dev,
                              mask_rows=mask_rows)
    use_graph = args.graph and getattr(pipe, "ASYNC", False) and not vos
    loop = StepLoop(pipe, uploader, gatherer, vos=vos, seq_len=args.seq_len,
                    resident=resident if args.resident else None)

    # MIOpen's first-shape search (cudnn.benchmark) keeps the first warm-up step
    # silent for a minute or more: a heartbeat on stderr shows the run is alive.
    import threading
    warm_done = threading.Event()

    def heartbeat():
        t_hb = time.perf_counter()
        while not warm_done.wait(30.0):
            print("bench: warm-up in progress (%.0f s)" % (time.perf_counter() - t_hb),
                  file=sys.stderr, flush=True)

    if rank == 0:
        threading.Thread(target=heartbeat, daemon=True).start()
    for i in range(args.warmup):
        loop.step(prefetch=i < args.warmup - 1)
        if rank == 0:
            print("bench: warm-up step %d/%d issued" % (i + 1, args.warmup),
                  file=sys.stderr, flush=True)
    loop.drain()
    torch.cuda.synchronize()
    if use_graph:
        loop.capture()  # restarts the upload cycle at slot 0 for the timed region
    warm_done.set()
    from vosdetectron_amd.runner import StepWatchdog
    watchdog = StepWatchdog(rank=rank) if args.watchdog else None
    dt, out = timed_region(loop, args.steps, torch.cuda.synchronize,
                           dist.barrier if world > 1 else None, watchdog)
    if watchdog:
        watchdog.stop()
    rank_ms = None
    if world > 1:  # every rank's own step time; the line's value uses the slowest
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        allt = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allt, t)
        per = [float(x.item()) / args.steps * 1e3 for x in allt]
        rank_ms = {"min": round(min(per), 3), "max": round(max(per), 3),
                   "spread": round(max(per) / min(per) - 1, 4), "per_rank": [round(v, 3) for v in per]}
        dt = max(float(x.item()) for x in allt)
    gather_share = None
    if gatherer.collective and not args.share_gpu:
        # the packed all_gather ALONE (no compute to hide behind), K times: an upper
        # bound on its share of the step, where it overlaps the next step's compute
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        tg0 = time.perf_counter()
        for i in range(args.steps):
            gatherer.gather_async(out["dets"], out["classes"], out["counts"],
                                  out["masks"]).wait(views=False)
        torch.cuda.synchronize()
        tg = torch.tensor([time.perf_counter() - tg0], device=dev, dtype=torch.float64)
        if world > 1:
            dist.all_reduce(tg, op=dist.ReduceOp.MAX)
        g_ms = float(tg.item()) / args.steps * 1e3
        gather_share = {"gather_ms": round(g_ms, 3),
                        "share_of_step": round(g_ms / (dt / args.steps * 1e3), 4),
                        "bytes_per_rank": gatherer.bytes_per_rank,
                        "bus_GBs": round(gatherer.bytes_per_rank * (world - 1) / (g_ms * 1e-3)
                                         / 1e9, 2) if world > 1 else None,
                        "how": "the step's packed all_gather alone, %d times after the timed "
                               "region (in the step it overlaps the next step's compute)"
                               % args.steps}
    dets_per_frame = float(np.mean(out["counts_host"]))

    stages = None
    extra = {}
    if args.timers and rank == 0:  # local steps only: no collective on one rank
        pipe.enable_timers()
        for i in range(min(args.steps, 3)):
            pipe.run(any_frames)
        stages = {k: round(v * 1e3, 3) for k, v in pipe.timer_summary().items()}
        pipe.enable_timers(False)
        if not vos and cfg.FPN.FPN_ON:
            segm_ms = measure_segm(pipe, out)
            extra["segm_results_ms_per_frame"] = segm_ms
            # the reference's whole im_detect_all incl. segm_results (RLE strings
            # on the host), serialised after the timed step: one GPU's rate
            step_ms_frame = dt / args.steps * 1e3 / F
            extra["frames_per_s_incl_segm_per_gpu"] = round(1e3 / (step_ms_frame + segm_ms), 2)

    roof = None
    if not args.no_roofline and rank == 0:
        roof = measure_roialign_roofline(dev)
        if "X-101" in args.config:
            # SURVEY 8(d) config 5 stress: R = 1000 RoIs at P = 14 (282.1 MB per frame)
            roof["stress_launch"] = measure_roialign_roofline(dev, P=14)
        if not vos and cfg.FPN.FPN_ON:
            roof["engine_launch"] = measure_pipeline_roialign(pipe, any_frames)
            extra["nms"] = measure_nms(dev)
            extra.update(measure_step_post(pipe, any_frames))
    if not args.no_roofline and rank == 0 and world == 1:  # N=1 line only (no ranks waiting)
        extra["hbm_copy"] = measure_hbm_copy(dev)
        if not vos and cfg.FPN.FPN_ON:
            extra["dominant_kernel"] = measure_dominant_conv(
                dev, F, getattr(pipe, "Hp", fh) // 4, getattr(pipe, "Wp", fw) // 4)
            extra["split_gemm"] = measure_split_gemm(dev, M=F * 1000)
        nthr = torch.get_num_threads()
        torch.set_num_threads(cpu_share()[0])
        flops, dets_cpu, wino_flops, wino4_flops, split3_flops, grouped_adj = \
            frame_flops(sd, cfg, F)
        torch.set_num_threads(nthr)
        extra["step_roofline"] = step_roofline(
            flops, dets_cpu, F, dt / args.steps * 1e3, roof.get("engine_launch") if roof else None,
            (fh, fw),
            (getattr(pipe, "Hp", fh), getattr(pipe, "Wp", fw)),
            wino_flops, wino4_flops, split3_flops, grouped_adj)
    cpu = None
    if not args.no_cpu_baseline and rank == 0 and world == 1:
        cpu = cpu_baseline(args.config, sd, args.cpu_frames, cfg=cfg)

    if rank == 0:
        fps = world * F * args.steps / dt
        h2d = "resident in HBM before timing" if args.resident else (
            "u8 frames uploaded every step inside the timed region (pinned host, side "
            "stream, %.1f MB/step/GPU)" % (uploader.nbytes / 1e6))
        line = {
            "metric": "frames/sec @1333x800 e2e_mask_rcnn_R-50-FPN, 1/2/4/8 MI355X; "
                      "RoIAlign HBM GB/s",
            "value": round(fps, 3), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "arith": "fp32 tensors end to end; the 1x1 convs / fc layers with K >= %d and "
                     "the stem's conv1 run on "
                     "the bf16 matrix cores with each fp32 operand split into three bf16 "
                     "pieces (six products, fp32 accumulate: error vs fp64 at or below the "
                     "fp32 GEMM's, tests/test_gemm_split3_gpu.py)%s" % (
                         __import__("vosdetectron_amd.ops", fromlist=["ops"]).SPLIT3_MIN_K,
                         "" if __import__("vosdetectron_amd.ops", fromlist=["ops"])
                         .split3_enabled() else " -- OFF in this run (VOSDET_GEMM_SPLIT3=0)"),
            "data": "synthetic (u8 800x1333 frames, RandomState seeds; deterministic "
                    "N(0,1/fan_in) weights)",
            "config": {"workload": (
                "%s inference, %d DAVIS-shaped 480x854 synthetic sequences per GPU (one frame "
                "of each per step, ConvGRU hidden states carried, reset every %d frames), full "
                "vos im_detect_all path" % (args.config, F, args.seq_len)) if vos else (
                "%s inference, %d synthetic %dx%d frames per GPU per step: blob, body, RPN, "
                "proposals, box head, class NMS, mask head -> class-selected masks "
                "(segm_results paste/RLE excluded, SURVEY 8d)" % (args.config, F, fh, fw)),
                       "frames_per_gpu_step": F, "global_batch": world * F,
                       "parallelism": ("frame-sharded dp%d + one RCCL all_gather per step"
                                       % world) if gatherer.collective else
                       "single GPU, frame-sharded dp1: no collective at N=1 (nothing to "
                       "gather; --rccl-gather issues it anyway)",
                       "layout": args.layout, "dets_per_frame": dets_per_frame, "h2d": h2d,
                       "gather_bytes_per_rank": gatherer.bytes_per_rank
                       if gatherer.collective else 0,
                       "launch": "hipGraph replay per step" if loop.graphs else
                       ("eager (%s)" % loop.graph_note if loop.graph_note else "eager")},
            "roofline": roof, "cpu_baseline": cpu,
        }
        if rank_ms:
            line["rank_ms_per_step"] = rank_ms
        if gather_share:
            line["gather"] = gather_share
        if args.share_gpu:
            line["rehearsal"] = "--share-gpu: %d ranks on one device, not a measurement" % world
        if stages:
            line["stages_ms"] = stages
        line.update(extra)
        print(json.dumps(line), flush=True)
    if world > 1 or args.rccl_gather:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
