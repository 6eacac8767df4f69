"""Input preprocessing: data/transforms.py of the reference on the HIP path (cv2 / albumentations
are not available in this image; the resampling is restated in csrc/preprocess.hip).

  load_charset            data/transforms.py:39-59 (one token per line, blank lines skipped)
  ResizeAndPadA           :62-120 (aspect-preserving fit, white canvas, alignment; INTER_LINEAR up,
                          INTER_AREA down, OpenCV 4.x arithmetic) -> crnn_hip.preprocess (HIP)
  get_val_transform       :185-193, callable(image=HxW[xC] uint8) -> {"image": [3,H,W] float tensor}:
                          ResizeAndPadA + A.Normalize(0.5, 0.5) ((v - 127.5) * (1/127.5), fp32) + ToTensorV2
  preprocess_batch        the same for a ragged list of crops in one launch, optionally straight into
                          the encoder's input layout (what OCRInference.predict uses)
  pack_attention_targets  :123-157 (text_in = [SOS, ids, PAD...], target_y = [ids, EOS, PAD...])
  ctc_targets             label strings -> padded id tensor + lengths (blank = 0 = <PAD>)
There is no CPU fallback: the transforms need a HIP device (parity of the kernel with the
restatement in oracle/preprocess_oracle.py is bit-exact; with cv2 itself it is unpinned).
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


def _device(device=None):
    dev = torch.device(device if device is not None else "cuda")
    if dev.type != "cuda" or not torch.cuda.is_available():
        raise RuntimeError("data.transforms runs on the HIP device (crnn_preprocess); no CPU fallback")
    return dev


def preprocess_batch(images: Sequence[np.ndarray], img_h: int = 32, img_w: int = 256, align_h: str = "left",
                     align_v: str = "center", out: str = "nchw", dtype: torch.dtype = torch.float32, device=None):
    """ragged list of uint8 crops -> [B, 3, H, W] fp32 ("nchw"), [B, H, W, 8] dtype ("encoder") or
    [B, H, W, 3] uint8 ("u8"), on the device."""
    from crnn_hip.preprocess import CropBatch, preprocess
    batch = CropBatch.upload(list(images), _device(device))
    return preprocess(batch, img_h, img_w, align_h, align_v, out=out, dtype=dtype)


def resize_and_pad(img: np.ndarray, img_h: int = 32, img_w: int = 256, align_h: str = "left",
                   align_v: str = "center") -> np.ndarray:
    """ResizeAndPadA.apply -> [img_h, img_w, 3] uint8 (host array)."""
    return preprocess_batch([img], img_h, img_w, align_h, align_v, out="u8")[0].cpu().numpy()


class ResizeAndPadA:
    """albumentations-style callable with the reference's constructor (:62-76)."""

    def __init__(self, img_h=32, img_w=256, align_h="left", align_v="center", always_apply=True, p=1.0):
        self.img_h, self.img_w, self.align_h, self.align_v = int(img_h), int(img_w), align_h, align_v

    def __call__(self, image, **kw) -> Dict[str, np.ndarray]:
        return {"image": resize_and_pad(image, self.img_h, self.img_w, self.align_h, self.align_v)}


class _ValTransform:
    def __init__(self, img_h, img_w):
        self.img_h, self.img_w = img_h, img_w

    def __call__(self, image) -> Dict[str, torch.Tensor]:
        return {"image": preprocess_batch([image], self.img_h, self.img_w)[0].cpu()}


def get_val_transform(img_h: int, img_w: int):
    return _ValTransform(img_h, img_w)


def pack_attention_targets(texts, stoi, max_len, drop_blank=True):
    """data/transforms.py:123-157: text_in [B, max_len+1] = [SOS, ids[:L], PAD...], target_y =
    [ids[:L], EOS, PAD...], lengths = L + 1; unknown characters (and <BLANK> if drop_blank) skipped."""
    PAD, SOS, EOS = stoi["<PAD>"], stoi["<SOS>"], stoi["<EOS>"]
    BLANK = stoi.get("<BLANK>", None)
    B, T = len(texts), max_len + 1
    text_in = torch.full((B, T), PAD, dtype=torch.long)
    text_in[:, 0] = SOS
    target_y = torch.full((B, T), PAD, dtype=torch.long)
    lengths = torch.zeros(B, dtype=torch.long)
    for i, s in enumerate(texts):
        ids = [stoi[ch] for ch in s if ch in stoi and not (drop_blank and BLANK is not None and stoi[ch] == BLANK)]
        n = min(len(ids), max_len)
        if n > 0:
            text_in[i, 1:1 + n] = torch.tensor(ids[:n], dtype=torch.long)
            target_y[i, :n] = torch.tensor(ids[:n], dtype=torch.long)
        target_y[i, n] = EOS
        lengths[i] = n + 1
    return text_in, target_y, lengths


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
