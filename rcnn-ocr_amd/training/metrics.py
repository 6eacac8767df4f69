"""training/metrics.py of the reference (CER via Levenshtein, WER via jiwer, exact-match
accuracy), restated without the python-Levenshtein / jiwer dependencies (absent here)."""
from __future__ import annotations

from typing import List, Sequence


def _edit_distance(a: Sequence, b: Sequence) -> int:
    if len(a) < len(b):
        a, b = b, a
    prev = list(range(len(b) + 1))
    for i, x in enumerate(a, 1):
        cur = [i]
        for j, y in enumerate(b, 1):
            cur.append(min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (x != y)))
        prev = cur
    return prev[-1]


def character_error_rate(reference: str, hypothesis: str) -> float:
    """CER = char edit distance / len(reference) (training/metrics.py:5-14)."""
    if len(reference) == 0:
        return float("inf") if len(hypothesis) > 0 else 0.0
    return _edit_distance(reference, hypothesis) / len(reference)


def word_error_rate(reference: str, hypothesis: str) -> float:
    """WER = word edit distance / #reference words (jiwer.wer semantics, training/metrics.py:17-22)."""
    r, h = reference.split(), hypothesis.split()
    if len(r) == 0:
        return float("inf") if len(h) > 0 else 0.0
    return _edit_distance(r, h) / len(r)


def compute_accuracy(references: List[str], hypotheses: List[str]) -> float:
    """exact-match accuracy (training/metrics.py:25-32)."""
    total = len(references)
    if total == 0:
        return 0.0
    return sum(1 for r, h in zip(references, hypotheses) if r == h) / total
