#!/usr/bin/env python3
"""L2 model of the RoIAlign product kernel's schedule (research aid, CPU only).

One XCD = one LRU cache of 4 MiB at 1 KiB-pixel granularity (a pixel's 256
fp32 channels are always fetched together).  The XCD runs K RoIs at a time
(K = resident workgroups: 4 per CU x 32 CUs at 8 waves/SIMD), each RoI's P
output rows in parallel (one wave per row), each row sweeping its distinct
columns left to right (roi_align.hip sep_row_sweep).  Accesses are interleaved
one column step per resident row per tick; a finished RoI's slot takes the next
RoI of the XCD's slice.  Prints misses / accesses for a schedule so orderings
and residency limits can be compared before spending GPU time."""
import os
import sys
from collections import OrderedDict

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bench import synthetic_rois, fpn_levels_np  # noqa: E402

SIZES = [(200, 336), (100, 168), (50, 84), (25, 42)]


def row_columns(r, li, P=7, SR=2):
    sc = 1.0 / 2 ** (li + 2)
    H, W = SIZES[li]
    sw, sh, ew, eh = (np.float32(r[1]) * sc, np.float32(r[2]) * sc,
                      np.float32(r[3]) * sc, np.float32(r[4]) * sc)
    rw, rh = max(ew - sw, 1.), max(eh - sh, 1.)
    bh, bw = rh / P, rw / P
    cols = []
    for pw in range(P):
        for ix in range(SR):
            x = sw + pw * bw + (ix + .5) * bw / SR
            if x < -1 or x > W:
                continue
            x = max(x, 0)
            xl = int(x)
            xh = xl if xl >= W - 1 else xl + 1
            xl = min(xl, W - 1)
            for c in (xl, xh):
                if not cols or cols[-1] != c:
                    if c not in cols[-2:]:
                        cols.append(c)
    rows = []
    for ph in range(P):
        taps = set()
        for iy in range(SR):
            y = sh + ph * bh + (iy + .5) * bh / SR
            if y < -1 or y > H:
                continue
            y = max(y, 0)
            yl = int(y)
            yh = yl if yl >= H - 1 else yl + 1
            taps.add(min(yl, H - 1))
            taps.add(yh)
        rows.append(sorted(taps))
    return [[[(li, y, x) for y in taps] for x in cols] for taps in rows]


def simulate(seq, K, cap=4096):
    """seq: list of per-RoI [row][step] -> list of pixel keys."""
    lru = OrderedDict()
    hits = miss = 0
    slots = []
    nxt = 0

    def fill():
        nonlocal nxt
        while len(slots) < K and nxt < len(seq):
            slots.append([seq[nxt], [0] * len(seq[nxt])])
            nxt += 1
    fill()
    while slots:
        done = []
        for si, (roi, pos) in enumerate(slots):
            live = False
            for ri, row in enumerate(roi):
                if pos[ri] < len(row):
                    live = True
                    for key in row[pos[ri]]:
                        if key in lru:
                            hits += 1
                            lru.move_to_end(key)
                        else:
                            miss += 1
                            lru[key] = 1
                            if len(lru) > cap:
                                lru.popitem(last=False)
                    pos[ri] += 1
            if not live:
                done.append(si)
        for si in reversed(done):
            slots.pop(si)
        fill()
    return hits, miss


def morton(y, x):
    k = 0
    for b in range(10):
        k |= ((x >> b) & 1) << (2 * b) | ((y >> b) & 1) << (2 * b + 1)
    return k


def hilbert(y, x, n=512):
    d, s = 0, n // 2
    while s > 0:
        rx = 1 if (x & s) else 0
        ry = 1 if (y & s) else 0
        d += s * s * ((3 * rx) ^ ry)
        if ry == 0:
            if rx == 1:
                x, y = s - 1 - x, s - 1 - y
            x, y = y, x
        s //= 2
    return d


def order_keys(rois, lv, curve, band=8):
    keys = []
    for r, li in zip(rois, lv):
        sc = 1.0 / 2 ** (li + 2)
        cy = int((r[2] + r[4]) * .5 * sc)
        cx = int((r[1] + r[3]) * .5 * sc)
        if curve == "band":
            k = (cy // band) * 65536 + cx
        elif curve == "morton":
            k = morton(cy, cx)
        elif curve == "hilbert":
            k = hilbert(cy, cx)
        else:
            k = 0
        keys.append((li, k))
    return keys


if __name__ == "__main__":
    rois = synthetic_rois(0, 1000)
    lv = fpn_levels_np(rois) - 2
    acc = [row_columns(r, l) for r, l in zip(rois, lv)]
    total = sum(len(s) for a in acc for row in a for s in row)
    print("accesses/RoI-set", total)
    for curve in sys.argv[1].split(","):
        keys = order_keys(rois, lv, curve)
        idx = sorted(range(len(rois)), key=lambda i: keys[i]) if curve != "none" else list(range(len(rois)))
        seq = [acc[i] for i in idx]
        for K in [int(k) for k in sys.argv[2].split(",")]:
            h, m = simulate(seq, K)
            print("%-8s K=%4d  miss %7d  (%.3f of accesses, %.2f MB)" % (curve, K, m, m / (h + m),
                                                                         m / 1024))
