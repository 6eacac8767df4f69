"""A briefly TRAINED reference RCNN (attention head) and its own predictions on held-out lines, as
fixtures for the word-accuracy parity test (north_star: "word-accuracy within
0.1 % of reference"; tests/test_gpu_refmodel.py).

Runs only in the build container: it imports the reference (/root/reference: model/model.py,
model/seresnet31.py; torchvision.ops.DropBlock2d stubbed, never constructed at dropblock_p = 0) and
trains it on CPU. Nothing of the reference is stored — only data:

  * the model: the reference's RCNN(num_classes=194, hidden_size=256, blank_id=None) — the reference's
    configs/config.json hidden size and train.py's blank rule. Its CNN is the
    seed-only recipe (crnn_hip/recipe.py) with BatchNorm running statistics calibrated on training
    lines (stored, 30k floats), frozen; the BiLSTM encoder and the attention decoder are trained here
    with the reference's own modules and its teacher-forced cross-entropy step (training/train.py:
    493-508: CrossEntropyLoss(ignore_index=PAD), Adam; the reference's enc_dropout 0.1 and attention
    dropout 0.1, and 2^-7 relative noise on the frozen CNN features, so that the fitted model is not
    balanced on the fp32 values of a random feature map) and stored as int8 with a per-row fp32 scale
    (~4 MB; the dequantized values ARE the model both sides evaluate);
  * lines rendered with DejaVu fonts (tests/golden/make_lines.py's renderer): 3000 training lines,
    1000 held-out lines; stored as uint8 pixels (ragged widths): the held-out lines and the first 1000
    training lines (the model, its CNN a frozen random recipe, reads the lines it was fitted on — 95+ %
    exact match — but hardly any held-out line, so the fitted lines carry the accuracy comparison);
  * the reference model's greedy predictions on both sets: RCNN.forward(is_train=False,
    batch_max_length=16) -> argmax -> decode_tokens (data/transforms.py:196-206, restated: the module
    imports cv2 / albumentations, absent here), i.e. inference.py:166-175, and their accuracy.

The reference's input pipeline (cv2 resize + pad + Normalize) is absent here; its restatement
oracle/preprocess_oracle.py (bit-exact to the HIP preprocess kernel) prepares the reference's input.

    python tests/golden/make_refmodel.py        # ~60 min on 8 cores -> tests/golden/refmodel_attn.npz
    python tests/golden/make_refmodel.py --eval-only   # predictions again, from the stored model
"""
from __future__ import annotations

import os
import random
import sys
import time

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "rcnn-ocr_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, HERE)

from make_goldens import _import_reference, load_charset  # noqa: E402  (the reference import + stub)
from make_lines import render, words  # noqa: E402
from crnn_hip.recipe import recipe_state_dict  # noqa: E402
import preprocess_oracle as P  # noqa: E402

SEED = 4242
IMG_H, IMG_W, MAX_LEN, HIDDEN = 32, 128, 16, 256
N_TRAIN, N_VAL, N_CAL = 3000, 1000, 64
TRAINED = ("enc_rnn.", "attn.")
EPOCHS, BATCH, LR = 150, 32, 2e-3
NOISE = 2.0 ** -7
OUT = os.path.join(HERE, "refmodel_attn.npz")


def lines(n, seed):
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        t = words(rng)
        out.append((np.asarray(render(t, rng).convert("RGB")), t))
    return out


def batch_tensor(imgs):
    return torch.from_numpy(np.stack([P.preprocess(im, IMG_H, IMG_W)[1] for im in imgs]))


def attention_targets(texts, stoi, max_len):
    """pack_attention_targets (data/transforms.py:123-157) restated: text_in = <SOS> + ids (+ PAD),
    target_y = ids + <EOS> (+ PAD), both [B, max_len + 1]"""
    sos, eos, pad = stoi["<SOS>"], stoi["<EOS>"], stoi["<PAD>"]
    B = len(texts)
    ti = torch.full((B, max_len + 1), pad, dtype=torch.long)
    ty = torch.full((B, max_len + 1), pad, dtype=torch.long)
    for i, s in enumerate(texts):
        ids = [stoi[c] for c in s if c in stoi][:max_len]
        ti[i, 0] = sos
        ti[i, 1:1 + len(ids)] = torch.tensor(ids, dtype=torch.long) if ids else ti[i, 1:1]
        ty[i, :len(ids)] = torch.tensor(ids, dtype=torch.long) if ids else ty[i, :0]
        ty[i, len(ids)] = eos
    return ti, ty


def quantize(w: torch.Tensor):
    """int8 per row (last dim) with an fp32 scale: q = round(w / s), s = max|row| / 127"""
    w2 = w.reshape(w.shape[0], -1) if w.dim() > 1 else w.reshape(1, -1)
    s = (w2.abs().amax(dim=1, keepdim=True) / 127.0).clamp_min(1e-12)
    q = torch.round(w2 / s).clamp(-127, 127).to(torch.int8)
    return q.reshape(w.shape), s.reshape(-1).float()


def dequantize(q: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    """the fixture's weights: q * s per row (tests/test_gpu_refmodel.py rebuilds them the same way)"""
    q2 = q.reshape(q.shape[0], -1) if q.dim() > 1 else q.reshape(1, -1)
    return (q2.float() * s.reshape(-1, 1)).reshape(q.shape)


def decode_tokens(ids, itos, pad_id, eos_id, blank_id=None):
    """data/transforms.py:196-206 restated"""
    out = []
    for t in ids:
        t = int(t)
        if t == eos_id:
            break
        if t == pad_id or (blank_id is not None and t == blank_id):
            continue
        out.append(itos[t])
    return "".join(out)


def main():
    torch.set_num_threads(os.cpu_count() or 8)
    RCNN, _, _ = _import_reference()
    itos = load_charset(os.path.join(HERE, "charset.txt"))
    stoi = {s: i for i, s in enumerate(itos)}
    C = len(itos)
    torch.manual_seed(SEED)
    m = RCNN(num_classes=C, hidden_size=HIDDEN, sos_id=stoi["<SOS>"], eos_id=stoi["<EOS>"], pad_id=stoi["<PAD>"],
             blank_id=stoi.get("<BLANK>"), enc_dropout_p=0.0)
    shapes = [(k, tuple(v.shape)) for k, v in m.state_dict().items() if not k.startswith("attn.")]
    m.load_state_dict(recipe_state_dict(shapes, SEED), strict=False)
    t0 = time.time()
    train, val = lines(N_TRAIN, SEED + 1), lines(N_VAL, SEED + 2)
    print(f"rendered {len(train)} + {len(val)} lines ({time.time() - t0:.0f} s)", flush=True)
    # BatchNorm running statistics: one train-mode pass over N_CAL training lines with momentum 1
    bns = [b for b in m.modules() if isinstance(b, nn.BatchNorm2d)]
    for b in bns:
        b.momentum = 1.0
    m.train()
    with torch.no_grad():
        m.cnn(batch_tensor([im for im, _ in train[:N_CAL]]))
    for b in bns:
        b.momentum = 0.1
    m.eval()
    # frozen CNN: its output sequence for every training line, once
    with torch.no_grad():
        feats = []
        for i in range(0, N_TRAIN, 100):
            f = m.cnn(batch_tensor([im for im, _ in train[i:i + 100]]))
            feats.append(m.pool(f).squeeze(2).permute(0, 2, 1))
        feats = torch.cat(feats)
    print(f"encoder features {tuple(feats.shape)} ({time.time() - t0:.0f} s)", flush=True)
    params = [p for k, p in m.named_parameters() if k.startswith(TRAINED)]
    for k, p in m.named_parameters():
        p.requires_grad_(k.startswith(TRAINED))
    opt = torch.optim.Adam(params, lr=LR)
    crit = nn.CrossEntropyLoss(ignore_index=stoi["<PAD>"])
    texts = [t for _, t in train]
    g = torch.Generator().manual_seed(SEED + 3)
    m.enc_rnn.train()
    m.attn.train()
    for ep in range(EPOCHS):
        perm = torch.randperm(N_TRAIN, generator=g).tolist()
        tot = 0.0
        for i in range(0, N_TRAIN - BATCH + 1, BATCH):
            idx = perm[i:i + BATCH]
            ti, ty = attention_targets([texts[j] for j in idx], stoi, MAX_LEN)
            # robustness to the storage rounding of a bf16 deployment: the frozen CNN's features
            # perturbed by ~2^-7 relative noise, and the reference's enc_dropout (p = 0.1, its default)
            f = feats[idx]
            f = f * (1.0 + NOISE * torch.randn(f.shape, generator=g))
            enc = torch.nn.functional.dropout(m.enc_rnn(f), p=0.1, training=True)
            logits = m.attn(enc, text=ti, is_train=True, batch_max_length=MAX_LEN)
            loss = crit(logits.reshape(-1, C), ty.reshape(-1))
            opt.zero_grad()
            loss.backward()
            opt.step()
            tot += float(loss.detach())
        print(f"epoch {ep + 1}: loss {tot / (N_TRAIN // BATCH):.4f} ({time.time() - t0:.0f} s)", flush=True)
    # the stored (int8 with a per-row fp32 scale) weights are the model
    q8 = {}
    with torch.no_grad():
        for k, p in m.named_parameters():
            if k.startswith(TRAINED):
                q, sc = quantize(p.detach())
                q8[k] = (q, sc)
                p.copy_(dequantize(q, sc))
    weights = {}
    for k, v in m.state_dict().items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            weights["bn::" + k] = v.numpy()
        elif k in q8:
            weights["q::" + k] = q8[k][0].numpy()
            weights["s::" + k] = q8[k][1].numpy()
    evaluate(m, itos, stoi, train, val, weights)


def predict(m, itos, stoi, lines_):
    preds = []
    with torch.no_grad():
        for i in range(0, len(lines_), 50):
            out = m(batch_tensor([im for im, _ in lines_[i:i + 50]]), is_train=False, batch_max_length=MAX_LEN)
            for row in out.argmax(-1):
                preds.append(decode_tokens(row, itos, stoi["<PAD>"], stoi["<EOS>"], stoi.get("<BLANK>")))
    return preds


def evaluate(m, itos, stoi, train, val, weights):
    """the reference model's greedy predictions on the held-out lines and on the first N_VAL training
    lines (which the briefly trained model reads: the held-out accuracy of a model whose CNN is a
    frozen random recipe is near 0), with their exact-match accuracies"""
    m.eval()
    out = dict(seed=np.int64(SEED), img_h=np.int64(IMG_H), img_w=np.int64(IMG_W), max_len=np.int64(MAX_LEN),
               hidden=np.int64(HIDDEN), **weights)
    for name, lines_ in (("val", val), ("fit", train[:N_VAL])):
        preds = predict(m, itos, stoi, lines_)
        truth = [t for _, t in lines_]
        acc = float(np.mean([p == t for p, t in zip(preds, truth)]))
        print(f"reference exact-match accuracy on the {name} lines: {acc:.4f}", flush=True)
        out.update({f"{name}_widths": np.array([im.shape[1] for im, _ in lines_], dtype=np.int32),
                    f"{name}_pixels": np.concatenate([im.reshape(-1) for im, _ in lines_]),
                    f"{name}_truth": np.array(truth), f"{name}_ref_pred": np.array(preds),
                    f"{name}_ref_accuracy": np.float64(acc)})
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT} ({os.path.getsize(OUT) / 1e6:.1f} MB)")


def eval_only():
    """rebuild the reference model from the stored fixture (recipe CNN + stored BN statistics +
    dequantized BiLSTM / decoder) and recompute the predictions"""
    RCNN, _, _ = _import_reference()
    itos = load_charset(os.path.join(HERE, "charset.txt"))
    stoi = {s: i for i, s in enumerate(itos)}
    z = np.load(OUT)
    torch.manual_seed(SEED)
    m = RCNN(num_classes=len(itos), hidden_size=HIDDEN, sos_id=stoi["<SOS>"], eos_id=stoi["<EOS>"],
             pad_id=stoi["<PAD>"], blank_id=stoi.get("<BLANK>"), enc_dropout_p=0.0)
    shapes = [(k, tuple(v.shape)) for k, v in m.state_dict().items() if not k.startswith("attn.")]
    sd = dict(m.state_dict())
    sd.update(recipe_state_dict(shapes, SEED))
    weights = {k: z[k] for k in z.files if k[:3] in ("bn:", "q::", "s::")}
    for k in z.files:
        if k.startswith("bn::"):
            sd[k[4:]] = torch.from_numpy(z[k])
        elif k.startswith("q::"):
            sd[k[3:]] = dequantize(torch.from_numpy(z[k]), torch.from_numpy(z["s::" + k[3:]]))
    m.load_state_dict(sd)
    train, val = lines(N_TRAIN, SEED + 1), lines(N_VAL, SEED + 2)
    evaluate(m, itos, stoi, train, val, weights)


if __name__ == "__main__":
    eval_only() if sys.argv[1:] == ["--eval-only"] else main()
