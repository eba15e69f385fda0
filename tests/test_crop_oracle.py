"""CPU checks of the crop-pipeline restatement (oracle/crop_ref.py) and the host box helpers of
zebrapose_amd/crop.py against the reference's semantics (bop_dataset_pytorch.py:36-72, 124-194,
333-347; class_id_encoder_decoder.py:6-15, 43-63).  OpenCV itself is absent: the resize arithmetic
is parity-unpinned, checked here for its defining properties (copy at equal size, 2x2 box at an
exact 2x downscale, within 1 LSB of exact bilinear elsewhere, nearest-neighbour index rule)."""
import numpy as np

from oracle import crop_ref as C


def _img(seed=0, H=120, W=160):
    return np.random.default_rng(seed).integers(0, 256, (H, W, 3), dtype=np.uint8)


def test_square_roi_matches_reference_slicing():
    img = _img()
    # tall box partially left of / above the image: roi column j <-> image column x1 + j
    roi = C.square_roi(img, np.array([-7, -5, 20, 31]))
    assert roi.shape == (31, 31, 3)
    c = -7 + 20 / 2
    x1, x2 = int(c - 31 / 2), int(c + 31 / 2)  # int() truncation: x2 - x1 = 30 < 31 here
    for j in range(31):
        col = x1 + j
        if 0 <= col < min(img.shape[1], x2):
            assert np.array_equal(roi[5:, j], img[:26, col])
        else:
            assert not roi[:, j].any()
    assert not roi[:5].any()


def test_resize_linear_properties():
    img = _img(1, 300, 300)
    roi = C.square_roi(img, np.array([0, 0, 256, 256]))
    assert np.array_equal(C.cv_resize_linear_u8(roi, 256), roi)
    roi = C.square_roi(img, np.array([10, 20, 200, 200]))  # not a multiple: bilinear
    out = C.cv_resize_linear_u8(roi, 256).astype(float)
    n, sc = roi.shape[0], roi.shape[0] / 256
    f = np.clip((np.arange(256) + 0.5) * sc - 0.5, 0, n - 1)
    s0 = np.floor(f).astype(int)
    s1 = np.minimum(s0 + 1, n - 1)
    a = f - s0
    r = roi.astype(float)
    h = r[:, s0] * (1 - a)[None, :, None] + r[:, s1] * a[None, :, None]
    v = h[s0] * (1 - a)[:, None, None] + h[s1] * a[:, None, None]
    assert np.abs(out - v).max() < 1.0
    big = np.random.default_rng(2).integers(0, 256, (512, 512, 3), dtype=np.uint8)
    o2 = C.cv_resize_linear_u8(big, 256).astype(int)
    b = big.astype(int)
    assert np.array_equal(o2, (b[0::2, 0::2] + b[0::2, 1::2] + b[1::2, 0::2] + b[1::2, 1::2] + 2) >> 2)


def test_nearest_and_codes():
    img = _img(3)
    roi = C.square_roi(img, np.array([5, 5, 90, 90]))
    nn = C.cv_resize_nearest(roi, 128)
    idx = np.minimum(np.floor(np.arange(128) * (90 / 128)).astype(int), 89)
    assert np.array_equal(nn, roi[idx][:, idx])
    code, m, e = C.crop_gt(img, img[:, :, 0], img[:, :, 2], np.array([5, 5, 90, 90]))
    g = nn.astype(np.int64)
    cid = (g[:, :, 0] << 16) | (g[:, :, 1] << 8) | g[:, :, 2]
    for i in range(16):
        assert np.array_equal(code[i], (cid >> (15 - i)) & 1)
    assert m.dtype == np.float32 and np.array_equal(m, (nn[:, :, 0] / 255.).astype(np.float32))


def test_dummy_crop_and_normalisation():
    img = _img(4)
    assert not C.crop_image(img, np.array([0, 0, 0, 0])).any()
    x = C.crop_image(img, np.array([0, 0, 256, 256]) // 2)  # 128 px box -> upscale
    assert x.shape == (3, 256, 256) and x.dtype == np.float32
    roi = C.cv_resize_linear_u8(C.square_roi(img, np.array([0, 0, 128, 128])), 256)
    ref = ((roi.astype(np.float32) / np.float32(255) - C.MEAN) / C.STD).transpose(2, 0, 1)
    assert np.array_equal(x, ref)


def test_host_box_helpers():
    from zebrapose_amd.crop import CropPipeline, get_final_Bbox, padding_Bbox
    assert list(padding_Bbox(np.array([100, 50, 40, 60]), 1.5)) == [90, 35, 60, 90]
    assert list(get_final_Bbox(np.array([90, 35, 60, 90]), "crop_square_resize", 640, 480)) == [75, 35, 90, 90]
    assert list(get_final_Bbox(np.array([-5, 35, 60, 900]), "crop_resize", 640, 480)) == [0, 35, 55, 445]
    pad, fin = CropPipeline().boxes([[100, 50, 40, 60], [-1, -1, -1, -1]], 640, 480)
    assert pad.tolist() == [[90, 35, 60, 90], [0, 0, 0, 0]] and fin.tolist()[0] == [75, 35, 90, 90]
