"""CPU restatement of the OpenCV pixel operations the reference's training augmentation calls
(datasets/coco_dataset_one.py:99-126 -> utils/image_helper.py:200-217, 245-257, 378-381).

TEST INFRASTRUCTURE ONLY: the checker for csrc/augment.hip in tests/test_augment_gpu.py; the
product never imports it.  Parity unpinned: OpenCV (cv2) is absent from this image, so these
restate OpenCV's published algorithms (imgproc box filter, warpPerspective + remap bilinear
fixed point) without a golden output to pin them; numpy float64, no FMA.
"""
import numpy as np


def reflect101(i, n):
    """BORDER_REFLECT_101 index (gfedcb|abcdefgh|gfedcba), vectorised."""
    i = np.asarray(i)
    if n == 1:
        return np.zeros_like(i)
    period = 2 * n - 2
    i = np.abs(i) % period
    return np.where(i >= n, period - i, i)


def box_blur(img, k):
    """cv2.blur(img, (k, k)) for HWC uint8: anchor (k//2, k//2), BORDER_REFLECT_101, the integer
    window sum times 1/k^2 rounded half to even, saturated."""
    if k <= 1:
        return img.copy()
    H, W = img.shape[:2]
    a = k // 2
    ys = reflect101(np.arange(H)[:, None] - a + np.arange(k)[None, :], H)  # [H, k]
    xs = reflect101(np.arange(W)[:, None] - a + np.arange(k)[None, :], W)  # [W, k]
    x = img.astype(np.int64)
    s = np.zeros(img.shape, np.int64)
    for dy in range(k):
        rows = x[ys[:, dy]]
        for dx in range(k):
            s += rows[:, xs[:, dx]]
    return np.minimum(np.rint(s * (1.0 / (k * k))), 255).astype(np.uint8)


def warp_perspective(img, inv, border_replicate, bg):
    """cv2.warpPerspective(img, M, (w, h), INTER_LINEAR, border) for HWC uint8 given the inverse
    map inv = M^-1 (destination -> source): per destination pixel the block-origin double terms
    of WarpPerspectiveInvoker (64-column blocks), coordinates on the 1/32 grid (round half to
    even), 15-bit fixed-point bilinear weights, BORDER_CONSTANT / BORDER_REPLICATE."""
    H, W = img.shape[:2]
    M = np.asarray(inv, np.float64).reshape(-1)
    y, x = np.meshgrid(np.arange(H, dtype=np.float64), np.arange(W, dtype=np.float64), indexing="ij")
    xb = np.floor(x / 64) * 64
    x1 = x - xb
    X0 = M[0] * xb + M[1] * y + M[2]
    Y0 = M[3] * xb + M[4] * y + M[5]
    W0 = M[6] * xb + M[7] * y + M[8]
    w = W0 + M[6] * x1
    with np.errstate(divide="ignore"):
        w = np.where(w != 0, 32.0 / np.where(w != 0, w, 1.0), 0.0)
    fX = np.clip((X0 + M[0] * x1) * w, -2147483648.0, 2147483647.0)
    fY = np.clip((Y0 + M[3] * x1) * w, -2147483648.0, 2147483647.0)
    Xi, Yi = np.rint(fX).astype(np.int64), np.rint(fY).astype(np.int64)
    sx, sy = np.clip(Xi >> 5, -32768, 32767), np.clip(Yi >> 5, -32768, 32767)
    ax, ay = Xi & 31, Yi & 31
    wts = [(32 - ax) * (32 - ay) * 32, ax * (32 - ay) * 32, (32 - ax) * ay * 32, ax * ay * 32]
    taps = [(sx, sy), (sx + 1, sy), (sx, sy + 1), (sx + 1, sy + 1)]
    src = img.astype(np.int64)
    bgv = np.asarray(bg, np.int64)[:3]
    acc = np.zeros((H, W, 3), np.int64)
    for (tx, ty), wt in zip(taps, wts):
        ok = (tx >= 0) & (tx < W) & (ty >= 0) & (ty < H)
        v = src[np.clip(ty, 0, H - 1), np.clip(tx, 0, W - 1)]
        if not border_replicate:
            v = np.where(ok[..., None], v, bgv)
        acc += v * wt[..., None]
    out = np.clip((acc + (1 << 14)) >> 15, 0, 255)
    if not border_replicate:
        far = (sx >= W) | (sx + 1 < 0) | (sy >= H) | (sy + 1 < 0)
        out = np.where(far[..., None], bgv, out)
    return out.astype(np.uint8)
