"""ORACLE — test infrastructure only. NOT part of the product path.

CPU restatement (numpy, scalar loops: small images only) of the reference's input pipeline,
SURVEY §8(f) next-2:
  ResizeAndPadA.apply      data/transforms.py:83-120 (RGB conversion, aspect-preserving fit,
                           white canvas, alignment)
  cv2.resize INTER_LINEAR  upscaling (:78-81): OpenCV 4.x resize.cpp, generic fixed-point path
                           (11-bit coefficients, HResizeLinear / VResizeLinear + FixedPtCast)
  cv2.resize INTER_AREA    downscaling: integer factors -> resizeAreaFast (2x2: rounding shift
                           (sum + 2) >> 2 as the SIMD kernel; otherwise cvRound(sum * (1/area)));
                           other factors -> resizeArea (computeResizeAreaTab weights, float
                           accumulation in cv2's order, cvRound)
  A.Normalize(0.5, 0.5)    data/transforms.py:190, albumentations 1.3.1:
                           (float32(v) - 127.5) * float32(1 / 127.5)

PARITY UNPINNED against cv2 / albumentations: neither is installed in this image and the
reference ships no preprocessed fixtures, so this is a restatement of the published OpenCV 4.x
algorithm (scalar arithmetic). OpenCV's SIMD kernels may round differently in the last bit for
some pixels (the vertical linear pass). The HIP kernel (csrc/preprocess.hip) is held
bit-exact to THIS restatement.
Only tests/ and bench.py's cpu_baseline leg may import this module.
"""
from __future__ import annotations

import math
from typing import Tuple

import numpy as np

COEF_BITS = 11
COEF_SCALE = 1 << COEF_BITS


def _cv_round(x: float) -> int:
    """cvRound: nearest, ties to even (lrint in the default rounding mode)."""
    return int(np.rint(x))


def geometry(h: int, w: int, img_h: int, img_w: int, align_h: str = "left", align_v: str = "center"):
    """ResizeAndPadA.apply :91-118 -> (new_h, new_w, y0, x0, interp) with interp 0 = linear, 1 = area
    (Python's round(): ties to even, as the reference evaluates it)."""
    scale = min(img_h / max(h, 1), img_w / max(w, 1))
    new_w = max(1, int(round(w * scale)))
    new_h = max(1, int(round(h * scale)))
    interp = 1 if (new_h < h or new_w < w) else 0          # _interp :78-81
    x0 = 0 if align_h == "left" else (img_w - new_w if align_h == "right" else (img_w - new_w) // 2)
    y0 = 0 if align_v == "top" else (img_h - new_h if align_v == "bottom" else (img_h - new_h) // 2)
    x0 = max(0, min(x0, img_w - new_w))
    y0 = max(0, min(y0, img_h - new_h))
    return new_h, new_w, y0, x0, interp


def to_rgb(img: np.ndarray) -> np.ndarray:
    """:86-89 (GRAY2RGB replicates, RGBA2RGB drops alpha)."""
    img = np.asarray(img, dtype=np.uint8)
    if img.ndim == 2:
        return np.repeat(img[:, :, None], 3, axis=2)
    if img.shape[2] == 4:
        return img[:, :, :3]
    return img


def _linear_taps(ssize: int, dsize: int, clamp_coef: bool):
    """per destination index: (s0, s1, c0, c1) — source taps and 11-bit coefficients.
    Columns (clamp_coef): a tap left of 0 or at / right of the last column becomes a one-tap
    copy (fx = 0). Rows: the coefficients are kept and the two row indices are clamped."""
    scale = ssize / dsize
    out = []
    for d in range(dsize):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = int(math.floor(f))
        f = np.float32(f - np.float32(s))
        if clamp_coef:
            if s < 0:
                f, s = np.float32(0.0), 0
            if s >= ssize - 1:
                f, s = np.float32(0.0), ssize - 1
        c0 = _cv_round(float(np.float32(np.float32(1.0) - f) * np.float32(COEF_SCALE)))
        c1 = _cv_round(float(f * np.float32(COEF_SCALE)))
        out.append((min(max(s, 0), ssize - 1), min(max(s + 1, 0), ssize - 1), c0, c1))
    return out


def resize_linear(img: np.ndarray, new_h: int, new_w: int) -> np.ndarray:
    h, w, cn = img.shape
    xt, yt = _linear_taps(w, new_w, True), _linear_taps(h, new_h, False)
    src = img.astype(np.int64)
    out = np.empty((new_h, new_w, cn), np.uint8)
    for dy, (sy0, sy1, b0, b1) in enumerate(yt):
        for dx, (sx0, sx1, a0, a1) in enumerate(xt):
            for c in range(cn):
                r0 = src[sy0, sx0, c] * a0 + src[sy0, sx1, c] * a1       # HResizeLinear (int)
                r1 = src[sy1, sx0, c] * a0 + src[sy1, sx1, c] * a1
                v = (b0 * r0 + b1 * r1 + (1 << (2 * COEF_BITS - 1))) >> (2 * COEF_BITS)   # FixedPtCast
                out[dy, dx, c] = min(255, max(0, v))
    return out


def _area_tab(ssize: int, dsize: int):
    """computeResizeAreaTab: per destination index the list of (source index, float32 weight)."""
    scale = ssize / dsize
    tab = []
    for d in range(dsize):
        fs1 = d * scale
        fs2 = fs1 + scale
        cell = min(scale, ssize - fs1)
        s1 = int(math.ceil(fs1))
        s2 = int(math.floor(fs2))
        s2 = min(s2, ssize - 1)
        s1 = min(s1, s2)
        e = []
        if s1 - fs1 > 1e-3:
            e.append((s1 - 1, np.float32((s1 - fs1) / cell)))
        for s in range(s1, s2):
            e.append((s, np.float32(1.0 / cell)))
        if fs2 - s2 > 1e-3:
            e.append((s2, np.float32(min(min(fs2 - s2, 1.0), cell) / cell)))
        tab.append(e)
    return tab


def resize_area(img: np.ndarray, new_h: int, new_w: int) -> np.ndarray:
    h, w, cn = img.shape
    sx, sy = w / new_w, h / new_h
    ix, iy = int(round(sx)), int(round(sy))
    out = np.empty((new_h, new_w, cn), np.uint8)
    if abs(sx - ix) < np.finfo(float).eps and abs(sy - iy) < np.finfo(float).eps:   # resizeAreaFast
        area = ix * iy
        inv = np.float32(1.0) / np.float32(area)
        for dy in range(new_h):
            for dx in range(new_w):
                cellv = img[dy * iy:(dy + 1) * iy, dx * ix:(dx + 1) * ix].astype(np.int64)
                for c in range(cn):
                    s = int(cellv[:, :, c].sum())
                    v = (s + 2) >> 2 if (ix == 2 and iy == 2) else _cv_round(float(np.float32(s) * inv))
                    out[dy, dx, c] = min(255, max(0, v))
        return out
    xt, yt = _area_tab(w, new_w), _area_tab(h, new_h)
    f = img.astype(np.float32)
    for dy in range(new_h):
        for dx in range(new_w):
            for c in range(cn):
                acc = None
                for (syy, beta) in yt[dy]:
                    buf = np.float32(0.0)
                    for (sxx, alpha) in xt[dx]:
                        buf = np.float32(buf + np.float32(f[syy, sxx, c] * alpha))
                    term = np.float32(beta * buf)
                    acc = term if acc is None else np.float32(acc + term)
                out[dy, dx, c] = min(255, max(0, _cv_round(float(acc))))
    return out


def resize_and_pad(img: np.ndarray, img_h: int = 32, img_w: int = 256, align_h: str = "left",
                   align_v: str = "center") -> np.ndarray:
    """ResizeAndPadA.apply (data/transforms.py:83-120) -> [img_h, img_w, 3] uint8."""
    img = to_rgb(img)
    h, w = img.shape[:2]
    new_h, new_w, y0, x0, interp = geometry(h, w, img_h, img_w, align_h, align_v)
    if (new_h, new_w) == (h, w):
        r = img.copy()                                   # cv2.resize copies on equal sizes
    elif interp == 1:
        r = resize_area(img, new_h, new_w)
    else:
        r = resize_linear(img, new_h, new_w)
    canvas = np.full((img_h, img_w, 3), 255, np.uint8)
    canvas[y0:y0 + new_h, x0:x0 + new_w] = r
    return canvas


def normalize(canvas_u8: np.ndarray) -> np.ndarray:
    """A.Normalize(mean=0.5, std=0.5, max_pixel_value=255) + ToTensorV2 -> [3, H, W] float32."""
    den = np.float32(1.0) / np.float32(127.5)
    x = (canvas_u8.astype(np.float32) - np.float32(127.5)) * den
    return np.ascontiguousarray(x.transpose(2, 0, 1))


def preprocess(img: np.ndarray, img_h: int, img_w: int, align_h: str = "left",
               align_v: str = "center") -> Tuple[np.ndarray, np.ndarray]:
    """-> (canvas u8 [H, W, 3], normalized float32 [3, H, W])"""
    c = resize_and_pad(img, img_h, img_w, align_h, align_v)
    return c, normalize(c)
