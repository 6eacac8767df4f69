"""Word accuracy / CER / WER of the CTC path on rendered text lines (VERDICT r02
next 9): renders seeded DejaVu text lines into the reference's CSV format, trains a CTC model with
training.train.run_training on the HIP path (bf16), then runs evaluate_dataset.evaluate_model on a
held-out rendered set. Parity unpinned: the reference ships no CTC model and no data to compare
against, so this measures the path's own accuracy, not agreement with the reference.

    python tools/accuracy_run.py --out gpurun_out/acc [--train 12000 --test 2000 --epochs 15]
"""
import argparse
import csv
import json
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("rcnn-ocr_amd",):
    sys.path.insert(0, os.path.join(REPO, sub))

FONTS = ["/usr/share/fonts/truetype/dejavu/DejaVuSans.ttf", "/usr/share/fonts/truetype/dejavu/DejaVuSansMono.ttf",
         "/usr/share/fonts/truetype/dejavu/DejaVuSerif.ttf", "/usr/share/fonts/truetype/dejavu/DejaVuSans-Bold.ttf"]


def alphabet(charset, which):
    from data.transforms import load_charset
    itos, _ = load_charset(charset)
    chars = [t for t in itos[3:] if len(t) == 1 and t != " "]
    if which == "full":   # every single character of the reference charset (Latin, Cyrillic, digits,
        return chars      # punctuation): Latin / Cyrillic look-alikes make it ambiguous to read
    return [c for c in chars if c in "abcdefghijklmnopqrstuvwxyz0123456789"]


def render_set(root, n, rng, chars, max_chars):
    from PIL import Image, ImageDraw, ImageFont
    os.makedirs(root, exist_ok=True)
    fonts = {}
    rows = []
    for i in range(n):
        words = [("".join(rng.choice(chars) for _ in range(rng.randint(1, 7)))) for _ in range(rng.randint(1, 2))]
        text = " ".join(words)[:max_chars].strip() or "a"
        fp, size = rng.choice(FONTS), rng.randint(20, 26)
        font = fonts.setdefault((fp, size), ImageFont.truetype(fp, size))
        x0, y0, x1, y1 = font.getbbox(text)
        h = 32 + rng.randint(0, 8)
        img = Image.new("L", (x1 + 10 + rng.randint(0, 12), h), color=rng.randint(200, 255))
        ImageDraw.Draw(img).text((4 + rng.randint(0, 4), (h - (y1 - y0)) // 2 - y0), text, fill=rng.randint(0, 60),
                                 font=font)
        fn = f"{i:06d}.png"
        img.save(os.path.join(root, fn))
        rows.append((fn, text))
    with open(os.path.join(root, "labels.csv"), "w", newline="", encoding="utf-8") as f:
        w = csv.writer(f)
        w.writerow(["filename", "text"])
        w.writerows(rows)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/acc")
    ap.add_argument("--train", type=int, default=60000)
    ap.add_argument("--test", type=int, default=2000)
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--alphabet", default="latin", choices=["latin", "full"],
                    help="latin: lowercase Latin + digits (unambiguous glyphs); full: the whole reference charset")
    a = ap.parse_args()
    charset = os.path.join(REPO, "tests", "golden", "charset.txt")
    chars = alphabet(charset, a.alphabet)
    rng = random.Random(20261017)
    t0 = time.time()
    for name, n in (("train", a.train), ("val", 1000), ("test", a.test)):
        render_set(os.path.join(a.out, name), n, rng, chars, 16)
    t_render = time.time() - t0
    cfg_d = {"train_csvs": [os.path.join(a.out, "train", "labels.csv")], "train_roots": [os.path.join(a.out, "train")],
             "val_csvs": [os.path.join(a.out, "val", "labels.csv")], "val_roots": [os.path.join(a.out, "val")],
             "charset_path": charset, "img_h": 32, "img_w": 256, "max_len": 16, "hidden_size": a.hidden,
             "batch_size": a.batch, "epochs": a.epochs, "lr": a.lr, "optimizer": "Adam",
             "scheduler": "CosineAnnealingLR", "weight_decay": 1.95e-5, "seed": 42, "eval_every": 5,
             "exp_dir": os.path.join(a.out, "exp"), "decoder": "ctc", "dtype": "bf16", "enc_dropout_p": 0.1}
    with open(os.path.join(a.out, "config.json"), "w") as f:
        json.dump(cfg_d, f)
    from training.train import Config, run_training
    t1 = time.time()
    res = run_training(Config(os.path.join(a.out, "config.json")), device="cuda")
    t_train = time.time() - t1
    from evaluate_dataset import evaluate_model
    ev = evaluate_model(os.path.join(res["exp_dir"], "best_acc_ckpt.pth"), charset,
                        os.path.join(a.out, "test", "labels.csv"), os.path.join(a.out, "test"), batch_size=256,
                        img_h=32, img_w=256, report_path=os.path.join(a.out, "test_report.csv"), verbose=True)
    out = {"what": "CTC path (bf16, HIP) trained by training.train.run_training on rendered DejaVu lines, evaluated "
                   "by evaluate_dataset.evaluate_model on a held-out rendered set; parity UNPINNED (the reference "
                   "ships no CTC model or data)",
           "train_samples": a.train, "test_samples": ev["samples"], "epochs": a.epochs, "hidden": a.hidden,
           "batch": a.batch, "val_acc_best": res["val_acc"], "test_accuracy": ev["accuracy"], "test_cer": ev["cer"],
           "test_wer": ev["wer"], "render_s": round(t_render, 1), "train_s": round(t_train, 1),
           "alphabet": a.alphabet, "alphabet_size": len(chars), "lr": a.lr}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
