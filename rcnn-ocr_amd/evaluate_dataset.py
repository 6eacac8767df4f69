"""evaluate_dataset.py of the reference (sherstpasha/RCNN-OCR evaluate_dataset.py:18-199) on the HIP
path: OCRInference over a labelled CSV (`filename,text` columns), exact-match accuracy, mean CER and
WER (training/metrics.py restated), the top-5 errors, and a per-sample CSV report.

    python evaluate_dataset.py --model model.pth --charset charset.txt --csv labels.csv --root images/

evaluate_model() also RETURNS the metrics (the reference only prints them), so tools and tests can
use it: {"samples", "accuracy", "cer", "wer", "cer_min", "cer_max", "cer_median", "wer_min",
"wer_max", "wer_median", "report"}.
"""
from __future__ import annotations

import argparse
import os
from typing import Dict, List, Optional, Tuple

import numpy as np

from training.metrics import character_error_rate, compute_accuracy, word_error_rate

EXTS = [".png", ".jpg", ".jpeg", ".bmp", ".tiff"]


def load_dataset(csv_path: str, root_path: str) -> Tuple[List[str], List[str]]:
    """:18-56: `filename` and `text` columns; a filename without extension is tried with the usual
    image extensions; rows whose image is missing are reported and skipped."""
    import pandas as pd
    if not os.path.exists(csv_path):
        raise FileNotFoundError(f"CSV not found: {csv_path}")
    if not os.path.exists(root_path):
        raise FileNotFoundError(f"image directory not found: {root_path}")
    df = pd.read_csv(csv_path, keep_default_na=False, dtype={"text": str})
    if "filename" not in df.columns or "text" not in df.columns:
        raise ValueError("the CSV must have 'filename' and 'text' columns")
    paths, texts = [], []
    for fn, text in zip(df["filename"], df["text"]):
        p = os.path.join(root_path, fn)
        if not os.path.exists(p):
            p = next((os.path.join(root_path, fn + e) for e in EXTS if os.path.exists(os.path.join(root_path, fn + e))),
                     p)
        if os.path.exists(p):
            paths.append(p)
            texts.append(str(text))
        else:
            print(f"image not found: {fn}")
    return paths, texts


def evaluate_model(model_path, charset_path, csv_path, root_path, batch_size=16, max_samples: Optional[int] = None,
                   img_h=32, img_w=128, report_path: Optional[str] = None, verbose: bool = True) -> Optional[Dict]:
    """:59-158"""
    from inference import OCRInference
    ocr = OCRInference(model_path, charset_path, device="auto", img_h=img_h, img_w=img_w)
    paths, truth = load_dataset(csv_path, root_path)
    if max_samples:
        paths, truth = paths[:max_samples], truth[:max_samples]
    if not paths:
        print("no samples to evaluate")
        return None
    pred: List[str] = []
    for i in range(0, len(paths), batch_size):
        pred.extend(ocr.predict(paths[i:i + batch_size], batch_size=batch_size))
    acc = compute_accuracy(truth, pred)
    cers = [character_error_rate(t, p) for t, p in zip(truth, pred)]
    wers = []
    for t, p in zip(truth, pred):
        try:
            wers.append(word_error_rate(t, p))
        except Exception:      # the reference counts a failing WER as 1.0 (:107-111)
            wers.append(1.0)
    out = {"samples": len(paths), "accuracy": acc, "cer": float(np.mean(cers)), "wer": float(np.mean(wers)),
           "cer_min": float(min(cers)), "cer_max": float(max(cers)), "cer_median": float(np.median(cers)),
           "wer_min": float(min(wers)), "wer_max": float(max(wers)), "wer_median": float(np.median(wers))}
    if verbose:
        print(f"samples: {out['samples']}  accuracy (exact match): {acc:.4f}  CER: {out['cer']:.4f}  "
              f"WER: {out['wer']:.4f}")
        worst = sorted(zip(truth, pred, cers), key=lambda r: r[2], reverse=True)[:5]
        for i, (t, p, c) in enumerate(worst):
            print(f"{i + 1}. CER={c:.3f}  true: {t!r}  predicted: {p!r}")
    import pandas as pd
    report = pd.DataFrame({"image_path": [os.path.basename(p) for p in paths], "true_text": truth,
                           "predicted_text": pred, "cer": cers, "wer": wers,
                           "exact_match": [t == p for t, p in zip(truth, pred)]})
    report_path = report_path or f"evaluation_results_{os.path.basename(model_path)}.csv"
    report.to_csv(report_path, index=False, encoding="utf-8")
    out["report"] = report_path
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="OCR model evaluation on a labelled dataset")
    ap.add_argument("--model", required=True)
    ap.add_argument("--charset", required=True)
    ap.add_argument("--csv", required=True)
    ap.add_argument("--root", required=True)
    ap.add_argument("--batch-size", type=int, default=16)
    ap.add_argument("--max-samples", type=int, default=None)
    ap.add_argument("--img-h", type=int, default=32)
    ap.add_argument("--img-w", type=int, default=128)
    a = ap.parse_args(argv)
    for p, what in ((a.model, "model"), (a.charset, "charset")):
        if not os.path.exists(p):
            print(f"{what} not found: {p}")
            return 1
    try:
        evaluate_model(a.model, a.charset, a.csv, a.root, a.batch_size, a.max_samples, a.img_h, a.img_w)
    except Exception as e:
        print(f"error: {e}")
        return 1
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
