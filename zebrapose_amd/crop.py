"""Device crop pipeline: the DataLoader worker's per-crop CPU work of
bop_dataset_pytorch.py, batched on the GPU.

The reference's ``__getitem__`` (bop_dataset_pytorch.py:280-347) reads the image, GT code image
and masks with cv2, pads the box (``padding_Bbox``), crops a zero-padded square ROI and resizes it
(``crop_square_resize``; INTER_LINEAR to 256 px for the image, INTER_NEAREST to 128 px for the GT
image and masks), turns the GT colours into 16 code planes (``RGB_image_to_class_id_image`` +
``class_id_image_to_class_code_images``), normalises the image (``transform_pre``) and returns
``get_final_Bbox``'s box.  Here the box arithmetic stays on the host (a few integer operations
per crop, same functions as the reference) and the pixel work is two kernels over a whole batch
(``zp_crop_image``, ``zp_crop_gt``, csrc/zp_crop.hip) reading images resident in HBM.
Only ``resize_method="crop_square_resize"`` (the configs' method) is on the device.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L


def padding_Bbox(Bbox, padding_ratio):
    """bop_dataset_pytorch.py:124-139."""
    x1, x2 = Bbox[0], Bbox[0] + Bbox[2]
    y1, y2 = Bbox[1], Bbox[1] + Bbox[3]
    cx, cy = 0.5 * (x1 + x2), 0.5 * (y1 + y2)
    bh, bw = y2 - y1, x2 - x1
    pbw, pbh = int(bw * padding_ratio), int(bh * padding_ratio)
    return np.array([int(cx - pbw / 2), int(cy - pbh / 2), int(pbw), int(pbh)])


def get_final_Bbox(Bbox, resize_method, max_x, max_y):
    """bop_dataset_pytorch.py:162-194 (the box the decode maps pixels back with)."""
    x1, bw = Bbox[0], Bbox[2]
    y1, bh = Bbox[1], Bbox[3]
    x2, y2 = x1 + bw, y1 + bh
    if resize_method in ("crop_square_resize", "crop_resize_by_warp_affine"):
        c = np.array([0.5 * (x1 + x2), 0.5 * (y1 + y2)])
        if bh > bw:
            x1, x2 = c[0] - bh / 2, c[0] + bh / 2
        else:
            y1, y2 = c[1] - bw / 2, c[1] + bw / 2
        x1, y1, x2, y2 = int(x1), int(y1), int(x2), int(y2)
        return np.array([x1, y1, x2 - x1, y2 - y1])
    if resize_method == "crop_resize":
        x1, y1 = int(max(x1, 0)), int(max(y1, 0))
        x2, y2 = int(min(x2, max_x)), int(min(y2, max_y))
        return np.array([x1, y1, x2 - x1, y2 - y1])
    return Bbox


def _u8(t, name, ndim):
    if t is None:
        return None
    if not (isinstance(t, torch.Tensor) and t.dtype == torch.uint8 and t.is_cuda and t.dim() == ndim):
        raise ValueError(f"{name}: expected a uint8 CUDA tensor with {ndim} dims")
    return t.contiguous()


class CropPipeline:
    """Batched square-ROI crops of device-resident images (``crop_square_resize`` path)."""

    def __init__(self, crop_size_img=256, crop_size_gt=128, code_bits=16, padding_ratio=1.5):
        self.S_img, self.S_gt = int(crop_size_img), int(crop_size_gt)
        self.L = int(code_bits)
        self.padding_ratio = padding_ratio

    def boxes(self, Bboxes, img_w, img_h):
        """Host box arithmetic for a batch of raw boxes [B, 4] -> (padded boxes int32 [B, 4] fed to
        the kernels, final boxes int64 [B, 4] for the decode).  A box of -1s (no detection) stays a
        zero box: the kernels then emit the reference's all-zero dummy crop."""
        pad, fin = [], []
        for bb in np.asarray(Bboxes).reshape(-1, 4):
            if np.any(np.isclose(bb, -1)):  # :291-298
                pad.append(np.zeros(4, np.int64))
                fin.append(np.zeros(4, np.int64))
                continue
            p = padding_Bbox(bb, self.padding_ratio)
            pad.append(p)
            fin.append(get_final_Bbox(p, "crop_square_resize", img_w, img_h))
        return np.stack(pad).astype(np.int32), np.stack(fin).astype(np.int64)

    def __call__(self, images, img_index, boxes, gt_images=None, masks=None, entire_masks=None):
        """images u8 [N, H, W, 3] (BGR, device); img_index int [B]; boxes = padded boxes int [B, 4].
        Returns dict: x f32 [B, 3, S_img, S_img] and, when the GT inputs are given, code u8
        [B, L, S_gt, S_gt], mask / entire_mask f32 [B, S_gt, S_gt]."""
        images = _u8(images, "images", 4)
        gt_images = _u8(gt_images, "gt_images", 4)
        masks = _u8(masks, "masks", 3)
        entire_masks = _u8(entire_masks, "entire_masks", 3)
        N, H, W, C = images.shape
        if C != 3:
            raise ValueError("images must be HWC with 3 channels")
        for t in (gt_images, masks, entire_masks):
            if t is not None and (t.shape[0] != N or t.shape[1] != H or t.shape[2] != W):
                raise ValueError("GT images / masks must match the image stack")
        dev = images.device
        idx = np.asarray(img_index, dtype=np.int64).reshape(-1)
        B = len(idx)
        if B == 0 or idx.min() < 0 or idx.max() >= N:
            raise ValueError("img_index out of range")
        ii = torch.from_numpy(idx.astype(np.int32)).to(dev)
        bb = torch.as_tensor(np.asarray(boxes), dtype=torch.int32).reshape(B, 4).to(dev).contiguous()
        st = L.stream_ptr()
        out = {"x": torch.empty((B, 3, self.S_img, self.S_img), dtype=torch.float32, device=dev)}
        L.call("zp_crop_image", images.data_ptr(), N, H, W, ii.data_ptr(), bb.data_ptr(), B, self.S_img,
               out["x"].data_ptr(), st)
        if gt_images is not None or masks is not None or entire_masks is not None:
            S = self.S_gt
            code = torch.empty((B, self.L, S, S), dtype=torch.uint8, device=dev) if gt_images is not None else None
            m = torch.empty((B, S, S), dtype=torch.float32, device=dev) if masks is not None else None
            e = torch.empty((B, S, S), dtype=torch.float32, device=dev) if entire_masks is not None else None
            L.call("zp_crop_gt", L.ptr(gt_images), L.ptr(masks), L.ptr(entire_masks), N, H, W, ii.data_ptr(),
                   bb.data_ptr(), B, S, self.L, L.ptr(code), L.ptr(m), L.ptr(e), st)
            out.update(code=code, mask=m, entire_mask=e)
        return out
