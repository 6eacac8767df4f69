"""OCRInference — the reference's inference.py:12-195 API on the MI355X CTC path.

Same constructor arguments, checkpoint formats and predict() contract (single image -> str,
list -> list, optional (text, confidence)). The checkpoint picks the decoder (strict load): a
CTC checkpoint (ctc_head.*) decodes by the greedy CTC collapse (repeats merged,
blank = id 0 = <PAD> dropped) in the HIP greedy kernel, confidence = mean max-softmax over the
emitted frames; a reference checkpoint (attn.*) runs the HIP attention decoder and the
reference's decode_tokens / confidence rule (inference.py:166-190). Each batch of images goes through
the HIP input pipeline in one launch (data.transforms.preprocess_batch: ResizeAndPadA +
Normalize, inference.py:93-124 / data/transforms.py:185-193) straight into the encoder's input
layout.
"""
from __future__ import annotations

import os
from typing import List, Union

import numpy as np
import torch

from crnn_hip.ctc import ctc_greedy_decode
from data.transforms import decode_tokens, get_val_transform, load_charset, preprocess_batch
from model.model import RCNN
from training.utils import rcnn_from_state


class OCRInference:
    def __init__(self, model_path: str, charset_path: str, device: str = "auto", img_h: int = 64,
                 img_w: int = 256, compute_dtype: torch.dtype = torch.bfloat16):
        self.model_path, self.charset_path = model_path, charset_path
        self.img_h, self.img_w = img_h, img_w
        if device == "auto":
            device = "cuda" if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        self.itos, self.stoi = load_charset(charset_path)
        self.pad_id = self.stoi["<PAD>"]
        self.sos_id = self.stoi["<SOS>"]
        self.eos_id = self.stoi["<EOS>"]
        self.blank_id = self.stoi.get("<BLANK>", None)
        self.compute_dtype = compute_dtype
        self.transform = get_val_transform(img_h, img_w)
        self.model = self._load_model()

    def _load_model(self) -> RCNN:
        ckpt = torch.load(self.model_path, map_location="cpu", weights_only=True)
        if isinstance(ckpt, dict) and "config" in ckpt:
            hidden = ckpt["config"].get("hidden_size", 256)
            state = ckpt["model_state"]
        elif isinstance(ckpt, dict) and "model_state_dict" in ckpt:
            hidden = ckpt.get("hidden_size", 256)
            state = ckpt["model_state_dict"]
        else:
            hidden, state = 256, ckpt
        model = rcnn_from_state(state, len(self.itos), hidden, self.sos_id, self.eos_id, self.pad_id,
                                self.blank_id, self.compute_dtype)
        return model.to(self.device).eval()

    def _load_image(self, image) -> np.ndarray:
        """inference.py:104-119: path (read as RGB), PIL image (RGB) or array (gray / RGB / RGBA)."""
        from PIL import Image
        if isinstance(image, str):
            if not os.path.exists(image):
                raise FileNotFoundError(f"Image file not found: {image}")
            return np.asarray(Image.open(image).convert("RGB"))
        if isinstance(image, Image.Image):
            return np.asarray(image.convert("RGB"))
        if isinstance(image, np.ndarray):
            return image
        raise ValueError(f"Unsupported image type: {type(image)}")

    def _preprocess_image(self, image) -> torch.Tensor:
        """inference.py:93-124: one image -> [1, 3, H, W] on the device."""
        return preprocess_batch([self._load_image(image)], self.img_h, self.img_w, device=self.device)

    @torch.no_grad()
    def predict(self, images: Union[np.ndarray, str, "Image.Image", List], max_length: int = 25, batch_size: int = 32,
                return_confidence: bool = False):
        single = not isinstance(images, list)
        items = [images] if single else images
        results = []
        for i in range(0, len(items), batch_size):
            batch = preprocess_batch([self._load_image(im) for im in items[i:i + batch_size]], self.img_h, self.img_w,
                                     out="encoder", dtype=self.compute_dtype, device=self.device)
            logits = self.model(batch, is_train=False, batch_max_length=max_length)   # [B, T, C]
            if self.model.decoder == "attn":
                results.extend(self._attn_texts(logits, return_confidence))
                continue
            seqs = ctc_greedy_decode(logits)
            if return_confidence:
                probs = torch.softmax(logits.float(), dim=-1).max(dim=-1)
                best, arg = probs.values.cpu(), probs.indices.cpu()
            for j, seq in enumerate(seqs):
                text = "".join(self.itos[t] for t in seq[:max_length])
                if return_confidence:
                    a = arg[j]
                    keep = (a != 0) & torch.cat([torch.ones(1, dtype=torch.bool), a[1:] != a[:-1]])
                    conf = float(best[j][keep].mean()) if bool(keep.any()) else 0.0
                    results.append((text, conf))
                else:
                    results.append(text)
        return results[0] if single else results

    def _attn_texts(self, logits, return_confidence):
        """inference.py:166-190 for the reference's attention decoder: argmax per step ->
        decode_tokens (stop at <EOS>, skip <PAD> / <BLANK>); confidence = mean max-softmax over the
        steps that are neither <PAD> nor <EOS>."""
        pred = logits.argmax(dim=-1).cpu()
        if return_confidence:
            best = torch.softmax(logits.float(), dim=-1).max(dim=-1).values.cpu()
        out = []
        for j, row in enumerate(pred):
            text = decode_tokens(row, self.itos, pad_id=self.pad_id, eos_id=self.eos_id, blank_id=self.blank_id)
            if return_confidence:
                keep = (row != self.pad_id) & (row != self.eos_id)
                out.append((text, float(best[j][keep].mean()) if bool(keep.any()) else 0.0))
            else:
                out.append(text)
        return out
