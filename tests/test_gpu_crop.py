"""Device crop pipeline (zp_crop_image / zp_crop_gt through zebrapose_amd.crop.CropPipeline)
against the CPU restatement (oracle/crop_ref.py), bit-exact: normalised image crops (f32),
GT code planes (u8) and masks (f32).  Boxes cover the cases the reference's crop_square_resize
meets: inside the image, partly outside on each side, tall / wide (square-ified with int()
truncation), a small box (upscale), an exact 2x downscale (INTER_AREA route), an equal-size copy,
a large downscale and the all-zero dummy crop of a missing detection.  Parity against OpenCV
itself is unpinned (cv2 absent; oracle header)."""
import numpy as np
import pytest
import torch

from oracle import crop_ref as C

pytestmark = pytest.mark.gpu

BOXES = [[100, 80, 200, 150], [-40, -30, 120, 200], [560, 400, 150, 120], [10, 10, 512, 512], [300, 200, 256, 256],
         [250, 200, 37, 23], [0, 0, 640, 480], [-100, 100, 700, 300], [0, 0, 0, 0], [620, -20, 40, 90],
         [123, 45, 255, 257], [50, 60, 1, 1]]


def test_crop_pipeline_matches_oracle(gpu):
    from zebrapose_amd.crop import CropPipeline
    rng = np.random.default_rng(0)
    N, H, W = 3, 480, 640
    imgs = rng.integers(0, 256, (N, H, W, 3), dtype=np.uint8)
    gts = rng.integers(0, 256, (N, H, W, 3), dtype=np.uint8)
    masks = rng.integers(0, 2, (N, H, W), dtype=np.uint8) * 255
    ent = rng.integers(0, 256, (N, H, W), dtype=np.uint8)
    B = len(BOXES)
    idx = rng.integers(0, N, B)
    bb = np.array(BOXES, dtype=np.int32)
    cp = CropPipeline()
    out = cp(torch.from_numpy(imgs).cuda(), idx, bb, torch.from_numpy(gts).cuda(), torch.from_numpy(masks).cuda(),
             torch.from_numpy(ent).cuda())
    x, code, m, e = (out[k].cpu().numpy() for k in ("x", "code", "mask", "entire_mask"))
    for b in range(B):
        i = idx[b]
        np.testing.assert_array_equal(x[b], C.crop_image(imgs[i], bb[b]), err_msg=f"image crop {b} {BOXES[b]}")
        rc, rm, re = C.crop_gt(gts[i], masks[i], ent[i], bb[b])
        np.testing.assert_array_equal(code[b], rc, err_msg=f"code {b}")
        np.testing.assert_array_equal(m[b], rm, err_msg=f"mask {b}")
        np.testing.assert_array_equal(e[b], re, err_msg=f"entire {b}")


def test_crop_feeds_network_and_rejects_bad_input(gpu):
    from zebrapose_amd.crop import CropPipeline
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    imgs = torch.randint(0, 256, (2, 480, 640, 3), dtype=torch.uint8, device="cuda")
    cp = CropPipeline()
    pad, fin = cp.boxes([[100, 100, 80, 60], [-1, -1, -1, -1]], 640, 480)
    out = cp(imgs, [0, 1], pad)
    assert not out["x"][1].any()  # missing detection -> the reference's zero input
    net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision="bf16").cuda().eval()
    with torch.no_grad():
        mk, cd = net(out["x"])
    assert mk.shape == (2, 1, 128, 128) and cd.shape == (2, 16, 128, 128)
    with pytest.raises(ValueError):
        cp(imgs.float(), [0], pad[:1])
    with pytest.raises(ValueError):
        cp(imgs, [5], pad[:1])


def test_gt_code_planes_match_reference_fixture(gpu, golden):
    """A15 pinned to the reference itself: zp_crop_gt's code planes on 128x128 BGR GT crops (same-size
    ROI) equal RGB_image_to_class_id_image + class_id_image_to_class_code_images + the CHW permute of
    bop_dataset_pytorch.py:311-312, 345 (tests/golden/gt_codes.npz, captured from the reference),
    including colours whose id exceeds 2^16 (the blue byte is ignored by the 16-bit split)."""
    from zebrapose_amd.crop import CropPipeline
    f = golden("gt_codes.npz")
    gt = torch.from_numpy(f["gt_bgr"]).cuda()
    n = gt.shape[0]
    img = torch.zeros((n, 128, 128, 3), dtype=torch.uint8, device="cuda")
    cp = CropPipeline()
    out = cp(img, np.arange(n), np.tile(np.array([[0, 0, 128, 128]], np.int32), (n, 1)), gt)
    np.testing.assert_array_equal(out["code"].cpu().numpy(), f["code"])
