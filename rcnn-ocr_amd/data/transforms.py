"""Input preprocessing for the CTC path: data/transforms.py of the reference, restated on
PIL + numpy (cv2 / albumentations are not available in this image).

  load_charset            data/transforms.py:39-59 (one token per line, blank lines skipped)
  resize_and_pad          ResizeAndPadA :62-120 (aspect-preserving fit, white canvas, left/center align);
                          PIL BILINEAR for upscaling (cv2 INTER_LINEAR), BOX for downscaling (INTER_AREA)
  normalize               A.Normalize(0.5, 0.5) :190 -> (u8/255 - 0.5) / 0.5
  get_val_transform       :186-193, callable(image=HxWx3 uint8) -> {"image": [3,H,W] float tensor}
  ctc_targets             label strings -> padded id tensor + lengths (blank = 0 = <PAD>)
The resize is not bit-identical to cv2 (different resampling kernels); the rest is exact.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch


def load_charset(charset_path: str):
    itos = []
    with open(charset_path, "r", encoding="utf-8") as f:
        for line in f:
            tok = line.rstrip("\n")
            if tok == "":
                continue
            itos.append(tok)
    return itos, {s: i for i, s in enumerate(itos)}


def _to_rgb(img: np.ndarray) -> np.ndarray:
    if img.ndim == 2:
        img = np.repeat(img[:, :, None], 3, axis=2)
    elif img.shape[2] == 4:
        img = img[:, :, :3]
    return img


def resize_and_pad(img: np.ndarray, img_h: int = 32, img_w: int = 256, align_h: str = "left",
                   align_v: str = "center") -> np.ndarray:
    from PIL import Image
    img = _to_rgb(np.asarray(img))
    h, w = img.shape[:2]
    scale = min(img_h / max(h, 1), img_w / max(w, 1))
    new_w, new_h = max(1, int(round(w * scale))), max(1, int(round(h * scale)))
    resample = Image.BOX if (new_h < h or new_w < w) else Image.BILINEAR
    resized = np.asarray(Image.fromarray(img.astype(np.uint8)).resize((new_w, new_h), resample=resample))
    canvas = np.full((img_h, img_w, 3), 255, dtype=np.uint8)
    x0 = {"left": 0, "right": img_w - new_w}.get(align_h, (img_w - new_w) // 2)
    y0 = {"top": 0, "bottom": img_h - new_h}.get(align_v, (img_h - new_h) // 2)
    x0 = max(0, min(x0, img_w - new_w))
    y0 = max(0, min(y0, img_h - new_h))
    canvas[y0:y0 + new_h, x0:x0 + new_w] = resized
    return canvas


def normalize(img_u8: np.ndarray) -> torch.Tensor:
    x = torch.from_numpy(np.ascontiguousarray(img_u8)).float().permute(2, 0, 1)
    return (x / 255.0 - 0.5) / 0.5


class _ValTransform:
    def __init__(self, img_h, img_w):
        self.img_h, self.img_w = img_h, img_w

    def __call__(self, image) -> Dict[str, torch.Tensor]:
        return {"image": normalize(resize_and_pad(image, self.img_h, self.img_w))}


def get_val_transform(img_h: int, img_w: int):
    return _ValTransform(img_h, img_w)


def ctc_targets(texts: Sequence[str], stoi: Dict[str, int], max_len: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """label ids per string (unknown characters dropped, like pack_attention_targets :139-146),
    zero-padded [B, max(1, Lmax)] + lengths [B]."""
    ids: List[List[int]] = []
    for s in texts:
        row = [stoi[ch] for ch in s if ch in stoi and stoi[ch] > 2][:max_len]
        ids.append(row)
    lmax = max(1, max((len(r) for r in ids), default=1))
    out = torch.zeros(len(ids), lmax, dtype=torch.long)
    for i, r in enumerate(ids):
        if r:
            out[i, :len(r)] = torch.tensor(r)
    return out, torch.tensor([len(r) for r in ids], dtype=torch.long)


def decode_tokens(ids, itos, pad_id, eos_id, blank_id=None) -> str:
    """data/transforms.py:196-206: stop at EOS, skip PAD / BLANK, join the rest."""
    out = []
    for t in ids:
        t = int(t)
        if t == eos_id:
            break
        if t == pad_id or (blank_id is not None and t == blank_id):
            continue
        out.append(itos[t])
    return "".join(out)
