"""segm_results on the device (lib/core/test.py:801-855).

cv2 and pycocotools are absent, so the oracle restates cv2.resize INTER_LINEAR
(OpenCV's scalar float path) and pycocotools' rleEncode/rleToString: parity
unpinned against the executed libraries; the known answers below follow their
published algorithms.  GPU: vd_paste_masks and vd_mask_rle bit-exact against
the oracle restatement, and the RLE strings equal."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc


def test_cv2_resize_linear_known_answers():
    # half-pixel centres, border replicate on x via clamped taps
    np.testing.assert_array_equal(orc.cv2_resize_linear(np.array([[0., 1.]]), 4, 1),
                                  np.array([[0, .25, .75, 1]], np.float32))
    src = np.random.default_rng(0).standard_normal((16, 16)).astype(np.float32)
    np.testing.assert_array_equal(orc.cv2_resize_linear(src, 16, 16), src)  # identity
    # 2x downscale samples the midpoint of each pair
    d = orc.cv2_resize_linear(src, 8, 8)
    e = (src[0::2] * .5 + src[1::2] * .5)
    e = e[:, 0::2] * .5 + e[:, 1::2] * .5
    np.testing.assert_allclose(d, e, atol=1e-6)


def test_rle_known_answers():
    rle_to_string = orc.rle_to_string
    assert orc.rle_encode(np.zeros((2, 2), np.uint8))[0]["counts"] == "4"
    assert orc.rle_encode(np.ones((2, 2), np.uint8))[0]["counts"] == "04"
    r, c = orc.rle_encode(np.array([[0, 1, 1], [0, 1, 0]], np.uint8))  # Fortran order 0,0,1,1,1,0
    assert list(c) == [2, 3, 1] and r["counts"] == "231"
    rng = np.random.default_rng(1)
    for _ in range(300):
        a = (rng.uniform(size=(rng.integers(1, 60), rng.integers(1, 60))) > rng.uniform())
        r, c = orc.rle_encode(a.astype(np.uint8))
        assert c.sum() == a.size
        # independent column-walk restatement of rleEncode's change positions
        f = a.astype(np.uint8).flatten(order="F")
        pos = [i for i in range(f.size) if f[i] != (f[i - 1] if i else 0)]
        assert list(np.diff([0] + pos + [f.size])) == list(c)


def test_leb_encoding_values():
    rle_to_string = orc.rle_to_string
    # single counts: 0..15 -> one char '0'+x; 16 needs a continuation
    assert rle_to_string([5]) == chr(48 + 5)
    assert rle_to_string([16]) == chr(48 + (16 | 0x20)) + chr(48 + 0)
    # negative deltas (i > 2): 3 - 10 = -7 -> one char with the sign bit set
    assert rle_to_string([1, 2, 10, 4, 3])[-1] == chr(48 + ((-7) & 0x1f))


def _cases(rng, n, im_h, im_w, R):
    """Detections as segm_results receives them: clipped to the image
    (clip_tiled_boxes), so only the (R+2)/R expansion reaches past the border
    (the reference's slicing would fail on a box wholly outside the frame)."""
    masks = rng.uniform(0, 1, (n, R, R)).astype(np.float32)
    masks[: n // 4] = (masks[: n // 4] > 0.5).astype(np.float32) * 0.9 + 0.05
    xy = rng.uniform(-60, max(im_w, im_h), (n, 2))
    wh = np.exp(rng.uniform(np.log(1), np.log(900), (n, 2)))
    boxes = np.hstack([xy, xy + wh, rng.uniform(0, 1, (n, 1))]).astype(np.float32)
    boxes[0, :4] = [0, 0, im_w - 1, im_h - 1]  # full frame
    boxes[1, :4] = [10.2, 10.7, 10.2, 10.7]  # degenerate
    boxes[2, :4] = [im_w - 5.5, im_h - 3.2, im_w - 1, im_h - 1]  # corner sliver
    boxes[:, 0:4:2] = np.clip(boxes[:, 0:4:2], 0, im_w - 1)
    boxes[:, 1:4:2] = np.clip(boxes[:, 1:4:2], 0, im_h - 1)
    return masks, boxes


@pytest.mark.gpu
@pytest.mark.parametrize("R,im_h,im_w", [(28, 800, 1333), (14, 480, 854), (28, 37, 53)])
def test_paste_masks_and_rle_vs_oracle(R, im_h, im_w):
    from vosdetectron_amd import ops, segm
    rng = np.random.default_rng(R + im_h)
    masks, boxes = _cases(rng, 48, im_h, im_w, R)
    ref = orc.paste_masks(masks, boxes, im_h, im_w)
    planes = ops.paste_masks(torch.from_numpy(masks).cuda(), torch.from_numpy(boxes).cuda(),
                             im_h, im_w)
    got = planes.cpu().numpy()
    for i in range(len(masks)):
        assert np.array_equal(got[i], ref[i]), i
    rles = segm.encode_planes(planes)
    for i in range(len(masks)):
        r, _ = orc.rle_encode(ref[i])
        assert rles[i] == r, i
    # capacity retry path: a checkerboard needs H*W runs
    cb = ((np.arange(im_h)[:, None] + np.arange(im_w)[None]) % 2).astype(np.uint8)[None]
    cnt, n = ops.mask_rle_counts(torch.from_numpy(cb).cuda(), cap=16)
    assert int(n[0]) == len(orc.rle_encode(cb[0])[1]) > 16
    assert np.array_equal(cnt[0, :int(n[0])].cpu().numpy(), orc.rle_encode(cb[0])[1])


@pytest.mark.gpu
def test_engine_frame_segms():
    """The pipeline's class-selected masks through device segm_results equal the
    oracle's segm_results loop on the same masks and boxes."""
    from vosdetectron_amd import config as vcfg
    from vosdetectron_amd.engine import FramePipeline, frame_segms
    from vosdetectron_amd.weights import build_model
    cfg = vcfg.get("e2e_mask_rcnn_R-50-FPN_1x")
    model, _ = build_model(cfg, device="cuda", channels_last=True)
    frame = np.random.RandomState(5).randint(0, 256, (800, 1333, 3), np.uint8)
    pipe = FramePipeline(model, cfg, batch=1, device="cuda", channels_last=True)
    out = pipe.run(torch.from_numpy(frame[None]).cuda())
    segms = frame_segms(pipe, out)[0]
    k = out["counts_host"][0]
    assert k > 0 and sum(len(s) for s in segms) == k
    dets = out["dets"][0, :k].cpu().numpy()
    cls = out["classes"][0, :k].cpu().numpy()
    ref = orc.paste_masks(out["masks"][:k].cpu().numpy(), dets, 800, 1333)
    seen = {}
    for i in range(k):
        j = int(cls[i])
        r, _ = orc.rle_encode(ref[i])
        assert segms[j][seen.get(j, 0)] == r, i
        seen[j] = seen.get(j, 0) + 1


def _edge_boxes(im_h, im_w):
    """Boxes whose pasted masks hit every branch of the fused column walk: full
    height (a column's last pixel meets the next column's first), full height at
    the last column (the plane's end), first column, a 15 x 15 expanded box
    (R = 28: OpenCV's INTER_AREA 2x path), a 1-pixel box."""
    return np.array([[0, 0, im_w - 1, im_h - 1, 1], [5.5, 0, 40.2, im_h - 1, 1],
                     [im_w - 30.5, 0, im_w - 1, im_h - 1, 1], [0, 3.3, 9.1, 20.7, 1],
                     [100.2, 10.2, 113.2, 23.2, 1], [7, 7, 7, 7, 1],
                     [im_w - 12.4, im_h - 9.6, im_w - 1, im_h - 1, 1]], np.float32)


@pytest.mark.gpu
@pytest.mark.parametrize("R,im_h,im_w", [(28, 800, 1333), (14, 480, 854), (28, 37, 53),
                                         (28, 24, 9000)])
def test_segm_rle_fused_vs_oracle(R, im_h, im_w):
    """vd_segm_rle (paste + RLE without planes) and vd_rle_strings equal the
    oracle's segm_results loop (paste, rleEncode, rleToString) bit for bit; a
    frame wider than the fused kernel's 8192-column table (9000) takes the
    planes path (paste_masks + mask_rle) with the same results."""
    from vosdetectron_amd import ops, segm
    rng = np.random.default_rng(3 * R + im_w)
    masks, boxes = _cases(rng, 40, im_h, im_w, R)
    eb = np.clip(_edge_boxes(im_h, im_w), 0, None)
    eb[:, 0:4:2] = np.minimum(eb[:, 0:4:2], im_w - 1)
    eb[:, 1:4:2] = np.minimum(eb[:, 1:4:2], im_h - 1)
    em = rng.uniform(0, 1, (len(eb), R, R)).astype(np.float32)
    em[0] = 0.9  # all ones in a full-frame box: counts [0, H*W]
    em[1] = 0.9  # all ones, full height, several columns
    em[2, :, -3:] = 0.9  # ones up to the plane's last pixel
    masks = np.concatenate([masks, em])
    boxes = np.concatenate([boxes, eb])
    ref = orc.paste_masks(masks, boxes, im_h, im_w)
    mt, bt = torch.from_numpy(masks).cuda(), torch.from_numpy(boxes).cuda()
    for cap in (None, 3):  # default capacity, and the retry path
        cnt, n = ops.segm_rle_counts(mt, bt, im_h, im_w, cap=cap)
        cnt, n = cnt.cpu().numpy(), n.cpu().numpy()
        for i in range(len(masks)):
            _, c = orc.rle_encode(ref[i])
            assert np.array_equal(cnt[i, :n[i]], c), i
    rles = segm.encode_masks(mt, bt, im_h, im_w)
    for i in range(len(masks)):
        assert rles[i] == orc.rle_encode(ref[i])[0], i


@pytest.mark.gpu
def test_rle_strings_kernel():
    """vd_rle_strings vs the oracle's rleToString on run lengths with large
    values (multi-char), negative deltas, one count, and no counts."""
    from vosdetectron_amd import ops
    rng = np.random.default_rng(11)
    rows = [rng.integers(0, 2 ** rng.integers(1, 31), rng.integers(1, 700)) for _ in range(60)]
    rows += [np.array([1066400]), np.array([0, 1066400]), np.array([5, 1, 2 ** 31 - 1, 3, 0]),
             np.array([], np.int64)]
    cap = max(len(r) for r in rows)
    counts = np.zeros((len(rows), cap), np.int32)
    for i, r in enumerate(rows):
        counts[i, :len(r)] = r
    n = np.array([len(r) for r in rows], np.int32)
    got = ops.rle_strings(torch.from_numpy(counts).cuda(), torch.from_numpy(n).cuda())
    for i, r in enumerate(rows):
        assert got[i] == orc.rle_to_string(r), i
