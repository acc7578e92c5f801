"""Per-kernel averages of tools/prop_time.py's calls from a rocprofv3 kernel trace:
5 configurations x 23 calls, (VOSDET_RPN_PRESEL, VOSDET_RPN_MASK_LDS) = (1, 1), (0, 1),
(1, 0) (first 3 calls = warm-up)."""
import collections
import csv
import sys

KEYS = ['rpn_sel_hist', 'rpn_sel_compact', 'rpn_proposals_kernel', 'rpn_nms_mask_lds',
        'rpn_nms_mask_kernel', 'rpn_nms_finish', 'fillBuffer', 'FillFunctor<float>',
        'FillFunctor<int>']
NAMES = ["all nms", "all no-nms", "P2 nms", "P2 no-nms", "P3 nms"]


def short(n):
    for k in KEYS:
        if k in n:
            return k
    return n[:40]


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
seq = [(short(r['Kernel_Name']), int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in rows]
calls, cur = [], []
for s in seq:  # a call starts with the zero fill of its rois (FillFunctor<float>)
    if s[0] == 'FillFunctor<float>' and cur and cur[-1][0] != 'FillFunctor<float>':
        calls.append(cur)
        cur = []
    cur.append(s)
calls.append(cur)
for b in range(len(calls) // 23):
    blk = calls[b * 23 + 3:(b + 1) * 23]
    agg, span = collections.defaultdict(float), 0.
    for c in blk:
        for k, s0, e0 in c:
            agg[k] += (e0 - s0) / 1e3 / len(blk)
        ks = [x for x in c if x[0].startswith('rpn')]
        span += (ks[-1][2] - ks[0][1]) / 1e3 / len(blk)
    print("%s %-10s span %6.1f us  " % (["sel1 lds1", "sel0 lds1", "sel1 lds0"][b // 5],
                                         NAMES[b % 5], span)
          + "  ".join("%s %.1f" % (k, v) for k, v in agg.items()))
