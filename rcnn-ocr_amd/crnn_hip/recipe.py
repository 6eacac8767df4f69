"""Deterministic, seed-only weight + input recipes.

Golden fixtures (tests/golden/) store seeds and outputs, never 55M-parameter
state dicts: every consumer (the golden generator that drives the reference,
the oracle, the HIP path's tests, bench.py) rebuilds the same tensors from the
same seed with torch's CPU generator.

The key layout is the reference's state_dict (model/model.py:166-221,
model/seresnet31.py:70-187 of sherstpasha/RCNN-OCR) plus the CTC head
`ctc_head.{weight,bias}` this build adds.
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, Tuple

import torch


def _u(gen: torch.Generator, shape, lo: float, hi: float) -> torch.Tensor:
    return torch.rand(shape, generator=gen, dtype=torch.float64).mul_(hi - lo).add_(lo).float()


def recipe_tensor(name: str, shape: Tuple[int, ...], seed: int, index: int,
                  head_gain: float = 1.0) -> torch.Tensor:
    """One state-dict entry from (seed, position in key order)."""
    gen = torch.Generator().manual_seed(int(seed) * 100003 + int(index))
    shape = tuple(int(s) for s in shape)
    if name.endswith("num_batches_tracked"):
        return torch.zeros((), dtype=torch.long)
    if name.endswith("running_mean"):
        return torch.zeros(shape)
    if name.endswith("running_var"):
        return torch.ones(shape)
    is_bn = (".bn" in name or name.startswith("cnn.conv0.1") or name.startswith("cnn.conv0.4")
             or ".downsample.1." in name or name.startswith("cnn.conv_out.1")
             or name.startswith("cnn.conv_out.4"))
    if is_bn and name.endswith("weight"):
        return _u(gen, shape, 0.8, 1.2)
    if is_bn and name.endswith("bias"):
        return _u(gen, shape, -0.1, 0.1)
    if ".rnn." in name:
        hidden = shape[0] // 4
        k = 1.0 / math.sqrt(hidden)
        return _u(gen, shape, -k, k)
    if name.startswith("ctc_head"):
        fan_in = shape[-1] if name.endswith("weight") else 1
        k = head_gain * math.sqrt(3.0 / max(1, fan_in))
        if name.endswith("bias"):
            return _u(gen, shape, -0.1, 0.1)
        return _u(gen, shape, -k, k)
    if name.endswith("bias"):
        return _u(gen, shape, -0.05, 0.05)
    # conv / linear / SE weights: uniform with variance 2/fan_in (kaiming, ReLU gain)
    fan_in = 1
    for s in shape[1:]:
        fan_in *= s
    k = math.sqrt(6.0 / max(1, fan_in))
    return _u(gen, shape, -k, k)


def recipe_state_dict(shapes: Iterable[Tuple[str, Tuple[int, ...]]], seed: int,
                      head_gain: float = 1.0) -> Dict[str, torch.Tensor]:
    """state dict for `shapes` (ordered (name, shape) pairs)."""
    out = {}
    for i, (name, shape) in enumerate(shapes):
        out[name] = recipe_tensor(name, tuple(shape), seed, i, head_gain=head_gain)
    return out


def synthetic_batch(batch: int, img_h: int, img_w: int, seq_len: int, num_classes: int,
                    seed: int = 1234, max_label: int | None = None, first_token: int = 3):
    """SURVEY.md §8(d) synthetic inputs.

    Crops are uint8 pixels normalised like data/transforms.py:190
    ((u8/255-0.5)/0.5 in [-1,1]); columns past a per-sample content width
    U{W/4..W} are white padding (+1.0), as ResizeAndPadA pads
    (data/transforms.py:100-120). Labels: L ~ U{1..T/2}, ids U{first_token..C-1}.
    Returns (images float32 [B,3,H,W], pixels uint8 [B,3,H,W], targets int64 [B,Lmax]
    zero-padded, target_lengths int64 [B]).
    """
    gen = torch.Generator().manual_seed(int(seed))
    pix = torch.randint(0, 256, (batch, 3, img_h, img_w), generator=gen, dtype=torch.int64)
    widths = torch.randint(max(1, img_w // 4), img_w + 1, (batch,), generator=gen)
    cols = torch.arange(img_w).view(1, 1, 1, img_w)
    pix = torch.where(cols < widths.view(batch, 1, 1, 1), pix, torch.full_like(pix, 255))
    pix = pix.to(torch.uint8)
    images = (pix.float() / 255.0 - 0.5) / 0.5
    lmax = max_label if max_label is not None else max(1, seq_len // 2)
    lengths = torch.randint(1, lmax + 1, (batch,), generator=gen)
    targets = torch.randint(first_token, num_classes, (batch, lmax), generator=gen)
    mask = torch.arange(lmax).view(1, lmax) < lengths.view(batch, 1)
    targets = torch.where(mask, targets, torch.zeros_like(targets))
    return images, pix, targets, lengths
