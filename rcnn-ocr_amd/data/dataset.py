"""OCRDatasetAttn of the reference (data/dataset.py:23-156) for the HIP training loop: the CSV / TSV
reader, header detection, label / file-name normalisation, charset and max-length filtering and the
file-index path resolution, with the same constructor arguments and skip reasons.

What differs, by design: items are the decoded uint8 RGB crops (host arrays) plus their label
strings. The resize / pad / normalise of a whole batch runs in ONE HIP launch
(data.transforms.preprocess_batch -> crnn_preprocess) instead of per item on the CPU, so `transform`
is not applied per item; albumentations augmentation is out of scope. Images are decoded
with PIL (cv2 is absent here): `.convert("RGB")` equals cv2.IMREAD_COLOR + BGR2RGB for 8-bit gray,
RGB, RGBA (alpha dropped, not composited) and palette PNG / BMP / TIFF; JPEG decoders may differ by
rounding.
"""
from __future__ import annotations

import csv
import os
import random
from collections import Counter, defaultdict
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .transforms import pack_attention_targets

IMAGE_EXTS = {".png", ".jpg", ".jpeg", ".bmp", ".tif", ".tiff"}
HEADER_WORDS = {"file", "filename", "image", "path", "img", "name"}


def build_file_index(roots, exts=IMAGE_EXTS):
    """basename (lower case) -> paths under the roots (data/transforms.py:12-26)."""
    if isinstance(roots, str):
        roots = [roots]
    index = defaultdict(list)
    for root in roots:
        if not os.path.isdir(root):
            continue
        for dirpath, _, filenames in os.walk(root):
            for fn in filenames:
                if exts and os.path.splitext(fn)[1].lower() not in exts:
                    continue
                index[fn.lower()].append(os.path.join(dirpath, fn))
    return index


def imread_rgb(path: str) -> np.ndarray:
    """data/transforms.py:29-36 (imread_cv2): HxWx3 uint8 RGB."""
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("RGB"))


class OCRDatasetAttn:
    def __init__(self, csv_path: str, images_dir, stoi: dict, img_height: int = 32, img_max_width: int = 128,
                 encoding: str = "utf-8", transform=None, num_workers: int = -1, delimiter: Optional[str] = None,
                 has_header: Optional[bool] = None, strict_charset: bool = True, validate_image: bool = True,
                 max_len: Optional[int] = None, strict_max_len: bool = True):
        self.images_dir = images_dir
        self.img_h, self.img_w = img_height, img_max_width
        self.stoi = stoi
        self.transform = transform
        self._file_index = build_file_index(images_dir)
        self._delimiter = delimiter if delimiter is not None else ("\t" if csv_path.lower().endswith(".tsv") else ",")
        self._strict_charset = strict_charset
        self._max_len = max_len
        self._strict_max_len = strict_max_len
        self.reasons = Counter()
        self.missing_chars = Counter()
        with open(csv_path, newline="", encoding=encoding) as f:
            rows = list(csv.reader(f, delimiter=self._delimiter))
        # header detection (:169-180): the first cell names a file column
        if has_header is None and rows:
            has_header = str(rows[0][0]).strip().lower() in HEADER_WORDS
        if has_header and rows:
            rows = rows[1:]
        self.samples: List[Tuple[str, str]] = []
        for row in rows:
            r = self._validate_row(row)
            if r is not None:
                self.samples.append(r)
        self._invalid = [False] * len(self.samples)
        if not self.samples:
            raise RuntimeError(f"no valid samples left in {csv_path}")

    @staticmethod
    def _norm_label(s: str) -> str:
        return s.replace(" ", " ").strip().replace("﻿", "")

    @staticmethod
    def _norm_fname(s: str) -> str:
        return s.strip().replace("﻿", "").replace("\\", "/")

    def _resolve_path(self, fname: str) -> Optional[str]:
        """:186-207: absolute path, root-relative path, then the basename index"""
        if os.path.isabs(fname) and os.path.exists(fname):
            return fname
        roots = [self.images_dir] if isinstance(self.images_dir, str) else list(self.images_dir)
        for root in roots:
            p = os.path.join(root, fname)
            if os.path.exists(p):
                return p
        cands = self._file_index.get(os.path.basename(fname).lower(), [])
        if len(cands) > 1:
            self.reasons["ambiguous"] += 1
        return cands[0] if cands else None

    def _validate_row(self, row) -> Optional[Tuple[str, str]]:
        """:214-261: the reference's skip reasons, in its order"""
        if len(row) < 2:
            self.reasons["bad_row"] += 1
            return None
        fname, label = self._norm_fname(row[0]), self._norm_label(row[1])
        if not fname:
            self.reasons["empty_fname"] += 1
            return None
        if label == "":
            self.reasons["empty_label"] += 1
            return None
        if self._strict_charset:
            missing = [c for c in label if c not in self.stoi]
            if missing:
                self.reasons["charset"] += 1
                self.missing_chars.update(missing)
                return None
        if self._strict_max_len and self._max_len is not None:
            eff = sum(1 for c in label if c in self.stoi) if self._strict_charset else len(label)
            if eff > self._max_len:
                self.reasons["too_long"] += 1
                return None
        path = self._resolve_path(fname)
        if not path or not os.path.exists(path):
            self.reasons["missing_path"] += 1
            return None
        return path, label

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, idx) -> Tuple[np.ndarray, str]:
        """(HxWx3 uint8 RGB, label); an unreadable image is marked and a random valid one taken
        instead (the reference's lazy validation, :101-129)."""
        if not 0 <= idx < len(self.samples):
            raise IndexError(idx)
        cur = idx
        for _ in range(8):
            path, label = self.samples[cur]
            if not self._invalid[cur]:
                try:
                    return imread_rgb(path), label
                except Exception:
                    self._invalid[cur] = True
                    self.reasons["readfail"] += 1
            cands = [i for i, bad in enumerate(self._invalid) if not bad and i != cur]
            if not cands:
                break
            cur = random.choice(cands)
        raise RuntimeError("Failed to fetch a valid sample after lazy validation retries.")

    @staticmethod
    def make_collate_attn(stoi, max_len: int, drop_blank: bool = True):
        """:147-156: (crops, text_in, target_y, lengths); crops stay a ragged list of uint8 arrays
        (the HIP preprocess takes the whole batch in one launch)."""
        def collate(batch):
            imgs, labels = zip(*batch)
            text_in, target_y, lengths = pack_attention_targets(labels, stoi=stoi, max_len=max_len,
                                                                 drop_blank=drop_blank)
            return list(imgs), text_in, target_y, lengths
        return collate


def random_split_indices(n: int, n_val: int, seed: int) -> Tuple[List[int], List[int]]:
    """torch.utils.data.random_split(ds, [n - n_val, n_val]) with a seeded generator: (train, val)."""
    import torch
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(seed)).tolist()
    return perm[:n - n_val], perm[n - n_val:]


def batches(indices: Sequence[int], batch_size: int, shuffle: bool, seed: int):
    """index batches of a DataLoader(batch_size, shuffle) over `indices` (last batch ragged)."""
    import torch
    order = list(indices)
    if shuffle:
        perm = torch.randperm(len(order), generator=torch.Generator().manual_seed(seed)).tolist()
        order = [order[i] for i in perm]
    for i in range(0, len(order), batch_size):
        yield order[i:i + batch_size]
