#!/usr/bin/env python3
"""Tie semantics study: execute the REFERENCE's own
GenerateProposalsOp (lib/modeling/generate_proposals.py:104-168: argpartition +
argsort(-s) top-k, NMS, keep[:post]) and collect()
(collect_and_distribute_fpn_rpn_proposals.py:91-106: argsort(-scores)) on
tie-bearing scores (quantised to 1/8, 1/64, 1/1024), compare with the package's
stable reading (oracle/oracle.py, which the HIP kernels match bit for bit), and
record what numpy's unstable sorts do on this host.

Writes tests/golden/proposals_ties.npz (inputs + reference outputs) and
tests/golden/proposals_ties.json (summary).  Container-only: imports the
reference through tools/gen_goldens.py's runtime shims (NMS = the reference's own
cython_nms.pyx, built by tools/ref_cython_nms.py, as for the other fixtures).

Usage: python tools/tie_study.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)


def main():
    import gen_goldens as gg
    gg.install_shims()
    import torch
    from core.config import cfg
    from modeling.generate_anchors import generate_anchors
    from modeling.generate_proposals import GenerateProposalsOp
    import modeling.collect_and_distribute_fpn_rpn_proposals as cdp
    from oracle import oracle as orc

    cfg.TEST.RPN_PRE_NMS_TOP_N, cfg.TEST.RPN_POST_NMS_TOP_N = 1000, 1000
    cfg.TEST.RPN_NMS_THRESH, cfg.TEST.RPN_MIN_SIZE = 0.7, 0
    cfg.FPN.RPN_COLLECT_SCALE = 1
    cfg.FPN.RPN_MIN_LEVEL, cfg.FPN.RPN_MAX_LEVEL = 2, 6
    im_info = np.array([[800, 1344, 1.0]], np.float32)
    rng = np.random.default_rng(20241018)
    shapes = {2: (100, 168), 4: (25, 42), 6: (7, 11)}
    fx, summary = {"im_info": im_info}, {"cases": []}
    for q in (8, 64, 1024):
        rl, pl, ol, opl = [], [], [], []
        for lvl, (H, W) in shapes.items():
            an = generate_anchors(stride=2. ** lvl, sizes=(32 * 2. ** (lvl - 2),),
                                  aspect_ratios=(0.5, 1, 2))
            probs = (np.round(rng.uniform(0, 1, (1, 3, H, W)) * q) / q).astype(np.float32)
            deltas = rng.normal(0, 0.3, (1, 12, H, W)).astype(np.float32)
            op = GenerateProposalsOp(an, 1. / 2 ** lvl)
            op.eval()
            r, p = op(torch.from_numpy(probs), torch.from_numpy(deltas), torch.from_numpy(im_info))
            r2, p2 = orc.generate_proposals(an, 1. / 2 ** lvl, probs, deltas, im_info)
            tag = "q%d_fpn%d" % (q, lvl)
            if lvl != 2:  # fixtures stay small: the P2-sized inputs are summarised only
                fx[tag + "_probs"], fx[tag + "_deltas"] = probs, deltas
                fx[tag + "_ref_rois"], fx[tag + "_ref_probs"] = r, p
            n_tied = int(len(probs.ravel()) - len(np.unique(probs)))
            same_set = bool(r.shape == r2.shape and np.array_equal(
                r[np.lexsort(r.T[::-1])], r2[np.lexsort(r2.T[::-1])]))
            summary["cases"].append({
                "case": tag, "anchors": int(probs.size), "tied_scores": n_tied,
                "ref_rows": int(len(r)), "stable_rows": int(len(r2)),
                "ref_equals_stable": bool(r.shape == r2.shape and np.array_equal(r, r2)),
                "same_rows_as_a_set": same_set})
            rl.append(r)
            pl.append(p)
            ol.append(r2)
            opl.append(p2)
    # collect(): argsort(-scores) over concatenated levels with ties
    scores = (np.round(rng.uniform(0, 1, 3000) * 16) / 16).astype(np.float32)
    rois = np.hstack([np.zeros((3000, 1)), rng.uniform(0, 500, (3000, 4))]).astype(np.float32)
    inputs = [rois[i * 600:(i + 1) * 600] for i in range(5)] + \
             [scores[i * 600:(i + 1) * 600, None] for i in range(5)]
    ref_col = cdp.collect(inputs, False)
    stable_col = orc.collect(inputs[:5], inputs[5:], 1000)
    fx["collect_rois"], fx["collect_scores"], fx["collect_ref"] = rois, scores, ref_col
    score_of = {rois[i].tobytes(): scores[i] for i in range(len(rois))}
    sel_ref = np.sort([score_of[x.tobytes()] for x in ref_col])
    sel_stable = np.sort([score_of[x.tobytes()] for x in stable_col])
    summary["collect"] = {"rows": 3000, "distinct_scores": int(len(np.unique(scores))),
                          "ref_equals_stable": bool(np.array_equal(ref_col, stable_col)),
                          "same_selected_score_multiset": bool(np.array_equal(sel_ref,
                                                                              sel_stable))}
    # numpy's own tie order on this host
    t = np.full(1000, 0.5, np.float32)
    a = np.argsort(-t)
    summary["numpy"] = {
        "version": np.__version__,
        "argsort_1000_equal_keys_is_stable": bool(np.array_equal(a, np.arange(1000))),
        "argsort_1000_equal_keys_head": [int(v) for v in a[:12]],
        "argsort_16_equal_keys_is_stable": bool(np.array_equal(np.argsort(-t[:16]),
                                                               np.arange(16))),
        "simd_found": np.__config__.CONFIG.get("SIMD Extensions", {}).get("found")
        if hasattr(np.__config__, "CONFIG") else None}
    out = os.path.join(REPO, "tests", "golden")
    np.savez(os.path.join(out, "proposals_ties.npz"), **fx)
    json.dump(summary, open(os.path.join(out, "proposals_ties.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
