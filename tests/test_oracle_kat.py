"""Known-answer checks of the oracle's C restatements (oracle/roi_ops.c), which
cannot be executed against the reference CUDA code in this image: analytic
properties of the reference algorithms pin them instead."""
import numpy as np

from oracle import oracle as orc


def ramp(B, C, H, W, a=0.5, b=0.25, c=1.0):
    y, x = np.meshgrid(np.arange(H, dtype=np.float64), np.arange(W, dtype=np.float64),
                       indexing="ij")
    base = (a * y + b * x + c).astype(np.float32)
    f = np.empty((B, C, H, W), np.float32)
    for bi in range(B):
        for ci in range(C):
            f[bi, ci] = base * (ci + 1) + bi
    return f


def test_roi_align_affine_exactness():
    """Bilinear interpolation is exact on affine features, so an interior RoI's
    bin value is the affine function at the bin's mean sample position
    (roi_align_kernel.cu:104-117)."""
    B, C, H, W = 2, 3, 20, 24
    f = ramp(B, C, H, W)
    rois = np.array([[0, 8., 8., 40., 36.], [1, 12., 4., 44., 36.]], np.float32)
    P, sr, scale = 4, 2, 0.5
    out = orc.roi_align(f, rois, P, P, scale, sr)
    for n, r in enumerate(rois):
        b = int(r[0])
        x0, y0, x1, y1 = r[1:] * scale
        bw, bh = (x1 - x0) / P, (y1 - y0) / P
        for ph in range(P):
            for pw in range(P):
                cy = y0 + (ph + 0.5) * bh
                cx = x0 + (pw + 0.5) * bw
                for ci in range(C):
                    exp = (0.5 * cy + 0.25 * cx + 1.0) * (ci + 1) + b
                    assert abs(out[n, ci, ph, pw] - exp) < 1e-4


def test_roi_align_out_of_bounds_and_malformed():
    f = ramp(1, 1, 10, 10)
    # entirely outside (x > W, y > H) -> 0 (roi_align_kernel.cu:19-22)
    rois = np.array([[0, 100., 100., 120., 120.]], np.float32)
    assert np.all(orc.roi_align(f, rois, 2, 2, 1.0, 2) == 0)
    # malformed (x2 < x1) -> forced 1x1 (:85-86), stays finite
    rois = np.array([[0, 5., 5., 2., 2.]], np.float32)
    o = orc.roi_align(f, rois, 2, 2, 1.0, 2)
    assert np.isfinite(o).all()
    # sampling_ratio 0 -> adaptive grid ceil(roi/P) (:94-98): same as sr=ceil for exact fits
    rois = np.array([[0, 0., 0., 8., 8.]], np.float32)
    assert np.array_equal(orc.roi_align(f, rois, 2, 2, 1.0, 0), orc.roi_align(f, rois, 2, 2, 1.0, 4))


def test_nms_known_answers():
    # identical boxes: survey-observed reference order keeps the higher index
    d = np.array([[0, 0, 10, 10, 0.9], [0, 0, 10, 10, 0.9]], np.float32)
    assert orc.nms(d, 0.5).tolist() == [1]
    d = np.array([[0, 0, 10, 10, 0.9], [0, 0, 10, 10, 0.8], [20, 20, 30, 30, 0.7]], np.float32)
    assert orc.nms(d, 0.5).tolist() == [0, 2]
    # IoU exactly at threshold suppresses (>=, cython_nms.pyx:84): two 10x10 boxes
    # (+1 convention -> 11x11=121) overlapping in 11x? region
    a = [0, 0, 10, 10]
    b = [0, 0, 10, 10 + 11]  # area 11*22 = 242, inter 121 -> IoU = 121/242 = 0.5
    d = np.array([a + [0.9], b + [0.8]], np.float32)
    assert orc.nms(d, 0.5).tolist() == [0]
    assert orc.nms(d, 0.5000001).tolist() == [0, 1]
    assert orc.nms(np.zeros((0, 5), np.float32), 0.5).tolist() == []
    # output is ascending index order, not score order (cython_nms.pyx:87)
    d = np.array([[50, 50, 60, 60, 0.1], [0, 0, 10, 10, 0.9]], np.float32)
    assert orc.nms(d, 0.3).tolist() == [0, 1]


def test_roi_pool_and_crop_basics():
    f = ramp(1, 2, 8, 8)
    rois = np.array([[0, 0, 0, 7, 7]], np.float32)
    out, arg = orc.roi_pool(f, rois, 2, 2, 1.0)
    # max of an increasing ramp is the bottom-right of each bin
    assert out[0, 0, 1, 1] == f[0, 0, 7, 7]
    assert arg[0, 1, 1, 1] == 64 + 7 * 8 + 7
    # identity grid at the pixel centres reproduces the input
    G = 8
    lin = np.linspace(-1, 1, G, dtype=np.float32)
    gy, gx = np.meshgrid(lin, lin, indexing="ij")
    grid = np.stack([gy, gx], -1)[None].astype(np.float32)
    crop = orc.roi_crop(f, grid)
    assert np.allclose(crop[0], f[0], atol=1e-5)


def test_resize_known_answers():
    """The oracle's restatement of cv2.resize INTER_LINEAR (prep_im_for_blob,
    lib/utils/blob.py:117-139) on known answers -- cv2 is not importable here, so
    these pin the restatement, not an executed cv2: a 2x upscale of [a, b] is
    OpenCV's well-known [a, .75a+.25b, .25a+.75b, b] in each direction; scale 1 is
    the identity; dsize = round(size * fx) (half to even); both scales exactly 2
    take INTER_AREA's fast path (2 x 2 means)."""
    src = np.array([[0., 4.]], np.float32)[:, :, None]
    assert np.array_equal(orc.cv2_resize_fx(src, 2.0)[0, :, 0], [0, 1, 3, 4])
    assert np.array_equal(orc.cv2_resize_fx(src.transpose(1, 0, 2), 2.0)[:, 0, 0], [0, 1, 3, 4])
    x = np.random.default_rng(0).standard_normal((9, 11, 3)).astype(np.float32)
    assert np.array_equal(orc.cv2_resize_fx(x, 1.0), x)
    assert orc.cv2_resize_fx(np.zeros((353, 500, 3), np.float32), 800 / 353).shape == (800, 1133, 3)
    assert orc.cv2_resize_fx(np.zeros((5, 7, 1), np.float32), 0.5).shape == (2, 4, 1)  # 2.5->2, 3.5->4
    y = np.arange(8 * 6, dtype=np.float32).reshape(8, 6)
    down = orc.cv2_resize_fx(y[:, :, None], 0.5)[:, :, 0]
    assert np.array_equal(down, (y[0::2, 0::2] + y[0::2, 1::2] + y[1::2, 0::2] + y[1::2, 1::2]) / 4)
    m = np.random.default_rng(1).uniform(0, 1, (30, 30)).astype(np.float32)
    area = orc.cv2_resize_linear(m, 15, 15)
    assert np.array_equal(area, (((m[0::2, 0::2] + m[0::2, 1::2]) + m[1::2, 0::2]) + m[1::2, 1::2])
                          * np.float32(0.25))
    blob, scale, info = orc.get_image_blob(np.zeros((353, 500, 3), np.uint8))
    assert blob.shape == (1, 3, 800, 1152) and info[0, 0] == 800 and abs(scale - 800 / 353) < 1e-15
