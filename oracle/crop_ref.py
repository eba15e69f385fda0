"""CPU restatement of the reference's crop pipeline -- TEST INFRASTRUCTURE ONLY (the product never
imports this module).

Reference (bop_dataset_pytorch.py):
  padding_Bbox           :124-139   (host box arithmetic, mirrored in zebrapose_amd/crop.py)
  crop_square_resize     :36-72     square-ify, int() truncation, zero-padded s x s ROI, cv2.resize
  get_final_Bbox         :162-194
  __getitem__            :311-316   image: 256 px INTER_LINEAR; GT image / masks: 128 px INTER_NEAREST
  transform_pre          :333-347   ToTensor + Normalize((0.485, 0.456, 0.406), (0.229, 0.224, 0.225))
                                    on the BGR array; masks / 255. (f64) -> float32
class_id_encoder_decoder.py:6-15, 43-63   id = B << 16 | G << 8 | R; bit i = (id >> (L-1-i)) & 1

cv2 is a third-party dependency absent from this image.  ``cv_resize_linear_u8`` and
``cv_resize_nearest`` restate OpenCV 4.x's generic resize (modules/imgproc/src/resize.cpp, non-IPP
path) for 8-bit data:
  * scale = 1 / (dsize / ssize) (double); exact 2x downscale with INTER_LINEAR -> INTER_AREA fast
    path: (a + b + c + d + 2) >> 2; same size -> copy
  * INTER_LINEAR: fx = float((dx + 0.5) * scale - 0.5), sx = floor(fx), fx -= sx; sx < 0 -> (0, 0);
    sx + 1 >= n -> "edge" (horizontal pass uses S[sx] * 2048 only), and sx >= n - 1 -> (n - 1, 0);
    coefficients cvRound(c * 2048) (int16); horizontal pass exact int32; vertical pass as
    VResizeLinearVec_32s8u: u8((mulhi(h0 >> 4, b0) + mulhi(h1 >> 4, b1) + 2) >> 2)
  * INTER_NEAREST: sx = min(floor(dx * (1 / (dsize / ssize))), ssize - 1)
PARITY UNPINNED against OpenCV itself (no cv2 here, no crop fixtures in the reference).  The
restatement builds the ROI array exactly as the reference does (numpy slices) and is written
independently of the HIP kernels (zebrapose_amd/csrc/zp_crop.hip), which it pins bit-exactly.
"""
from __future__ import annotations

import numpy as np

MEAN = np.array([0.485, 0.456, 0.406], dtype=np.float32)
STD = np.array([0.229, 0.224, 0.225], dtype=np.float32)


def square_roi(img, bbox):
    """crop_square_resize (:36-70) up to the resize: the zero-padded s x s ROI."""
    x1 = bbox[0]
    bw = max(bbox[2], 0)
    x2 = bbox[0] + bw
    y1 = bbox[1]
    bh = max(bbox[3], 0)
    y2 = bbox[1] + bh
    c = np.array([0.5 * (x1 + x2), 0.5 * (y1 + y2)])
    if bh > bw:
        x1 = c[0] - bh / 2
        x2 = c[0] + bh / 2
    else:
        y1 = c[1] - bw / 2
        y2 = c[1] + bw / 2
    x1, y1, x2, y2 = int(x1), int(y1), int(x2), int(y2)
    s = max(bh, bw)
    roi = np.zeros((s, s) + img.shape[2:], dtype=img.dtype)
    rx1 = max(-x1, 0)
    x1 = max(x1, 0)
    rx2 = rx1 + min(img.shape[1] - x1, x2 - x1)
    ry1 = max(-y1, 0)
    y1 = max(y1, 0)
    ry2 = ry1 + min(img.shape[0] - y1, y2 - y1)
    x2 = min(x2, img.shape[1])
    y2 = min(y2, img.shape[0])
    roi[ry1:ry2, rx1:rx2] = img[y1:y2, x1:x2]
    return roi


def _lin_taps(d, n):
    scale = 1.0 / (d / n)
    s0 = np.empty(d, np.int64)
    a = np.empty((d, 2), np.int64)
    edge = np.zeros(d, bool)
    for i in range(d):
        f = np.float32((i + 0.5) * scale - 0.5)
        s = int(np.floor(f))
        f = np.float32(f - np.float32(s))
        if s < 0:
            f, s = np.float32(0), 0
        if s + 1 >= n:
            edge[i] = True
            if s >= n - 1:
                f, s = np.float32(0), n - 1
        s0[i] = s
        a[i] = [int(np.rint((np.float32(1) - f) * np.float32(2048))), int(np.rint(f * np.float32(2048)))]
    return s0, np.minimum(s0 + 1, n - 1), a, edge


def cv_resize_linear_u8(roi, d):
    """cv2.resize(roi, (d, d), interpolation=cv2.INTER_LINEAR) for a square uint8 HxWxC roi."""
    n = roi.shape[0]
    if n == d:
        return roi.copy()
    scale = 1.0 / (d / n)
    iscale = int(np.rint(scale))
    r = roi.astype(np.int64)
    if iscale == 2 and abs(scale - iscale) < np.finfo(np.float64).eps:
        return ((r[0::2, 0::2] + r[0::2, 1::2] + r[1::2, 0::2] + r[1::2, 1::2] + 2) >> 2).astype(np.uint8)
    xs0, xs1, xa, xedge = _lin_taps(d, n)
    ys0, ys1, ya, _ = _lin_taps(d, n)
    # horizontal pass over every source row
    h = r[:, xs0] * xa[:, 0][None, :, None] + r[:, xs1] * xa[:, 1][None, :, None]
    h[:, xedge] = r[:, xs0[xedge]] * 2048
    h0 = np.clip(h[ys0] >> 4, -32768, 32767)
    h1 = np.clip(h[ys1] >> 4, -32768, 32767)
    v = ((h0 * ya[:, 0][:, None, None]) >> 16) + ((h1 * ya[:, 1][:, None, None]) >> 16)
    return np.clip((v + 2) >> 2, 0, 255).astype(np.uint8)


def cv_resize_nearest(roi, d):
    n = roi.shape[0]
    ifx = 1.0 / (d / n)
    idx = np.minimum(np.floor(np.arange(d) * ifx).astype(np.int64), n - 1)
    return roi[idx][:, idx]


def crop_image(img, bbox, S=256):
    """-> f32 [3, S, S]: ToTensor + Normalize of the 256 px INTER_LINEAR crop (BGR order kept)."""
    if max(bbox[2], 0) == 0 and max(bbox[3], 0) == 0:
        return np.zeros((3, S, S), np.float32)
    roi = cv_resize_linear_u8(square_roi(img, bbox), S)
    x = roi.astype(np.float32) / np.float32(255)
    return ((x - MEAN) / STD).transpose(2, 0, 1).astype(np.float32)


def crop_gt(gt_img, mask, entire, bbox, S=128, L=16):
    """-> (code u8 [L, S, S], mask f32 [S, S], entire f32 [S, S])."""
    if max(bbox[2], 0) == 0 and max(bbox[3], 0) == 0:
        return np.zeros((L, S, S), np.uint8), np.zeros((S, S), np.float32), np.zeros((S, S), np.float32)
    g = cv_resize_nearest(square_roi(gt_img, bbox), S).astype(np.int64)
    cid = (g[:, :, 0] << 16) + (g[:, :, 1] << 8) + g[:, :, 2]
    code = np.stack([(cid >> (L - 1 - i)) - ((cid >> (L - i)) << 1) for i in range(L)]).astype(np.uint8)
    m = (cv_resize_nearest(square_roi(mask, bbox), S) / 255.).astype(np.float32)
    e = (cv_resize_nearest(square_roi(entire, bbox), S) / 255.).astype(np.float32)
    return code, m, e
