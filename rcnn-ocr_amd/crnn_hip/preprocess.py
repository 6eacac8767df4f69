"""GPU input pipeline: ResizeAndPadA + A.Normalize(0.5, 0.5) + ToTensorV2
(data/transforms.py:62-120, :185-193) for a ragged batch of uint8 crops, on the HIP path
(csrc/preprocess.hip, crnn_preprocess).

    batch = CropBatch.upload(images, device)           # one H2D copy of all crops back to back
    x = preprocess(batch, 32, 256)                      # [B, 3, 32, 256] fp32, the reference's tensor
    x8 = preprocess(batch, 32, 256, out="encoder", dtype=torch.bfloat16)
                                                        # [B, 32, 256, 8]: the encoder's input layout,
                                                        # accepted by CRNNEngine.forward / RCNN directly
The per-crop geometry is computed here exactly as the reference computes it (Python floats and
round(), :91-118); the kernel does the resampling and normalisation.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Sequence

import numpy as np
import torch

from . import _lib as L
from ._lib import call, ptr


class _CropDesc(C.Structure):
    _fields_ = [("offset", C.c_longlong), ("h", C.c_int), ("w", C.c_int), ("c", C.c_int), ("new_h", C.c_int),
                ("new_w", C.c_int), ("y0", C.c_int), ("x0", C.c_int), ("interp", C.c_int), ("pad", C.c_int)]


def resize_geometry(h: int, w: int, img_h: int, img_w: int, align_h: str = "left", align_v: str = "center"):
    """ResizeAndPadA.apply (data/transforms.py:91-118) + _interp (:78-81) ->
    (new_h, new_w, y0, x0, interp) with interp 0 = INTER_LINEAR, 1 = INTER_AREA."""
    scale = min(img_h / max(h, 1), img_w / max(w, 1))
    new_w = max(1, int(round(w * scale)))
    new_h = max(1, int(round(h * scale)))
    interp = 1 if (new_h < h or new_w < w) else 0
    if align_h == "left":
        x0 = 0
    elif align_h == "right":
        x0 = img_w - new_w
    else:
        x0 = (img_w - new_w) // 2
    if align_v == "top":
        y0 = 0
    elif align_v == "bottom":
        y0 = img_h - new_h
    else:
        y0 = (img_h - new_h) // 2
    x0 = max(0, min(x0, img_w - new_w))
    y0 = max(0, min(y0, img_h - new_h))
    return new_h, new_w, y0, x0, interp


class CropBatch:
    """a ragged batch of uint8 HWC crops (HxW gray, HxWx3 RGB, HxWx4 RGBA) resident on the device."""

    def __init__(self, data: torch.Tensor, shapes: List[tuple], offsets: List[int]):
        self.data, self.shapes, self.offsets = data, shapes, offsets

    @classmethod
    def upload(cls, images: Sequence[np.ndarray], device) -> "CropBatch":
        shapes, offsets, flat, off = [], [], [], 0
        for im in images:
            a = np.ascontiguousarray(np.asarray(im))
            if a.dtype != np.uint8:
                raise ValueError("crops must be uint8")
            if a.ndim == 2:
                h, w, c = a.shape[0], a.shape[1], 1
            elif a.ndim == 3 and a.shape[2] in (1, 3, 4):
                h, w, c = a.shape
            else:
                raise ValueError(f"unsupported crop shape {a.shape}")
            if h <= 0 or w <= 0:
                raise ValueError("empty crop")
            shapes.append((h, w, c))
            offsets.append(off)
            flat.append(a.reshape(-1))
            off += a.size
        if not flat:
            raise ValueError("empty batch")
        host = torch.from_numpy(np.concatenate(flat))
        dev = torch.device(device)
        if dev.type != "cuda":
            raise RuntimeError("crnn_hip preprocessing runs only on a HIP device (no CPU fallback)")
        return cls(host.pin_memory().to(dev, non_blocking=True), shapes, offsets)

    def __len__(self):
        return len(self.shapes)

    def plan(self, img_h: int, img_w: int, align_h: str = "left", align_v: str = "center"):
        """device-resident crop descriptors (the reference's geometry per crop) + tap workspace,
        cached per canvas / alignment."""
        key = (img_h, img_w, align_h, align_v)
        cache = self.__dict__.setdefault("_plans", {})
        if key not in cache:
            B = len(self)
            descs = (_CropDesc * B)()
            for i, ((h, w, c), off) in enumerate(zip(self.shapes, self.offsets)):
                nh, nw, y0, x0, it = resize_geometry(h, w, img_h, img_w, align_h, align_v)
                descs[i] = _CropDesc(off, h, w, c, nh, nw, y0, x0, it, 0)
            raw = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8)
            d = raw.to(self.data.device)
            need = int(L.lib().crnn_preprocess_workspace(B, img_h, img_w))
            ws = torch.empty(need, dtype=torch.uint8, device=self.data.device)
            cache[key] = (d, ws)
        return cache[key]


def preprocess(batch: CropBatch, img_h: int = 32, img_w: int = 256, align_h: str = "left",
               align_v: str = "center", out: str = "nchw", dtype: torch.dtype = torch.float32) -> torch.Tensor:
    """out: "nchw" -> [B, 3, H, W] fp32 (get_val_transform's tensor, batched);
    "encoder" -> [B, H, W, 8] in dtype (the encoder's input layout); "u8" -> [B, H, W, 3] uint8
    canvas (before Normalize)."""
    L.require_device(batch.data)
    B = len(batch)
    d, ws = batch.plan(img_h, img_w, align_h, align_v)
    dev = batch.data.device
    if out == "nchw":
        res, kind, dt = torch.empty(B, 3, img_h, img_w, device=dev), 0, L.F32
    elif out == "encoder":
        res, kind, dt = torch.empty(B, img_h, img_w, 8, device=dev, dtype=dtype), 1, L.dtype_code(dtype)
    elif out == "u8":
        res, kind, dt = torch.empty(B, img_h, img_w, 3, device=dev, dtype=torch.uint8), 2, L.F32
    else:
        raise ValueError("out must be 'nchw', 'encoder' or 'u8'")
    call("crnn_preprocess", ptr(batch.data), ptr(d), B, img_h, img_w, kind, dt, ptr(res), ptr(ws), ws.numel(),
         L.stream_ptr())
    return res
