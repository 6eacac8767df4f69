"""Trains the CTC model of the word-accuracy fixture ON THE MI355X with this path's own
training.train.run_training, at the bench configuration: RCNN(decoder="ctc"), hidden 512,
2 BiLSTM layers, 32x256 crops, C = 194 (tests/golden/charset.txt), bf16, the whole model trained (the CNN
included), AdamW + cosine schedule, enc_dropout 0.1, on N rendered lines (tests/golden/make_lines.py's
renderer, written as PNG + labels.csv in the reference's dataset format, training/train.py:179-782).

Output: gpurun_out/refmodel3_weights.npz: the best-validation-accuracy weights, every tensor of more than one
dimension as int8 per output row + fp32 scale (the dequantized values are the model both sides evaluate; the
file must fit gpurun's 64 MiB merge), everything else fp32. tests/golden/make_refmodel3.py (build container)
records the reference's predictions for it on held-out lines.

    python tools/train_refmodel_ctc.py [n_lines] [epochs]
"""
import csv
import json
import os
import random
import sys
import time
from multiprocessing import Pool

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rcnn-ocr_amd"))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))

SEED = 6161
WORK = os.environ.get("RM3_WORK", "/tmp/rm3")


def render_chunk(args):
    from make_lines import render, words
    lo, hi, root = args
    rows = []
    for i in range(lo, hi):
        rng = random.Random(SEED * 1_000_003 + i)
        t = words(rng)
        fn = f"l{i:06d}.png"
        render(t, rng).save(os.path.join(root, fn))
        rows.append((fn, t))
    return rows


def quantize(w):
    """int8 per row (dim 0) with an fp32 scale (as tests/golden/make_refmodel.py)"""
    w2 = w.reshape(w.shape[0], -1)
    s = np.maximum(np.abs(w2).max(axis=1, keepdims=True) / 127.0, 1e-12).astype(np.float32)
    q = np.clip(np.round(w2 / s), -127, 127).astype(np.int8)
    return q.reshape(w.shape), s.reshape(-1)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
    epochs = int(sys.argv[2]) if len(sys.argv) > 2 else 24
    t0 = time.time()
    root = os.path.join(WORK, "lines")
    os.makedirs(root, exist_ok=True)
    step = 1000
    with Pool(min(16, os.cpu_count() or 1)) as pool:
        parts = pool.map(render_chunk, [(lo, min(n, lo + step), root) for lo in range(0, n, step)])
    rows = [r for p in parts for r in p]
    with open(os.path.join(WORK, "labels.csv"), "w", newline="", encoding="utf-8") as f:
        w = csv.writer(f)
        w.writerow(["filename", "text"])
        w.writerows(rows)
    print(f"rendered {len(rows)} lines ({time.time() - t0:.0f} s)", flush=True)

    import torch
    from training.train import Config, run_training
    cfg_d = {"train_csvs": [os.path.join(WORK, "labels.csv")], "train_roots": [root],
             "charset_path": os.path.join(REPO, "tests", "golden", "charset.txt"),
             "img_h": 32, "img_w": 256, "hidden_size": 512, "num_rnn_layers": 2, "batch_size": 128,
             "epochs": epochs, "lr": 1e-3, "optimizer": "AdamW", "weight_decay": 1e-4,
             "scheduler": "CosineAnnealingLR", "val_size": 2000, "eval_every": 1, "max_len": 25, "decoder": "ctc",
             "dtype": "bf16", "enc_dropout_p": 0.1, "seed": SEED, "exp_dir": os.path.join(WORK, "exp")}
    with open(os.path.join(WORK, "config.json"), "w") as f:
        json.dump(cfg_d, f)
    res = run_training(Config(os.path.join(WORK, "config.json")), device="cuda")
    print(f"run_training: {res} ({time.time() - t0:.0f} s)", flush=True)
    ck = torch.load(os.path.join(res["exp_dir"], "best_acc_ckpt.pth"), map_location="cpu", weights_only=True)
    sd = ck["model_state"]
    out = {"val_acc": np.float64(ck.get("best_val_acc", res["val_acc"])), "seed": np.int64(SEED),
           "n_train_lines": np.int64(n), "epochs": np.int64(epochs), "img_h": np.int64(32), "img_w": np.int64(256),
           "hidden": np.int64(512), "max_len": np.int64(25)}
    for k, v in sd.items():
        a = v.detach().float().cpu().numpy() if v.is_floating_point() else v.cpu().numpy()
        if v.is_floating_point() and a.ndim > 1:
            q, s = quantize(a)
            out["q::" + k], out["s::" + k] = q, s
        else:
            out["f::" + k] = a
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    path = os.path.join(REPO, "gpurun_out", os.environ.get("RM3_OUT", "refmodel3_weights.npz"))
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) / 2 ** 20:.1f} MiB), best val acc {float(out['val_acc']):.4f}",
          flush=True)


if __name__ == "__main__":
    main()
