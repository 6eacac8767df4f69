"""Generate golden fixtures by running the REFERENCE (sherstpasha/RCNN-OCR) on CPU.

Runs only in the build container, where /root/reference exists. The reference is
imported read-only (model/model.py, model/seresnet31.py, training/utils.py); its
only missing dependency on this path, torchvision.ops.DropBlock2d, is stubbed:
it is constructed only when dropblock_p > 0 (model/seresnet31.py:49-53), never here.

Everything written under tests/golden/ is data (seeds, inputs, expected outputs):
    python tests/golden/make_goldens.py

Fixtures:
  charset.txt            the reference's configs/charset.txt token list (data; C=194)
  encode_eval_<case>.npz eval-mode RCNN.encode + CTC head logits (model/model.py:215-221)
  train_<case>.npz       train-mode fwd (BN batch stats, dropout 0) + F.ctc_loss + backward
  ctc_cases.npz          F.ctc_loss(blank=0, mean, zero_infinity) values + grads, incl. infeasible labels
  decode.npz/.json       training/utils.py:122-150 ctc_greedy_decoder strings at T < B
  decode_b8_t16.npz/.json  BASELINE configs[0]'s decode shape, B=8 / T=16 (T > B: the reference's
                         layout heuristic would swap the axes there): the reference's
                         decoder run on the 8 samples padded with 17 extra rows to B=25 > T, so its
                         heuristic reads the intended (B, T, C) layout; only the 8 real rows are kept
  bilstm_stack.npz       4 x BidirectionalLSTM(768) stack (model/model.py:151-163)
  attn_decoder.npz       the attention decoder (model/model.py:23-148) on a
                         fixed encoder output: eval greedy decode (incl. blank masking) and
                         teacher-forced logits, with its (seeded, generator-scaled) weights
Only some:  python tests/golden/make_goldens.py attn | decode_b8
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, os.path.join(REPO, "rcnn-ocr_amd"))

from crnn_hip.recipe import recipe_state_dict, synthetic_batch  # noqa: E402


def _import_reference():
    tv = types.ModuleType("torchvision")
    ops = types.ModuleType("torchvision.ops")

    class DropBlock2d:  # never constructed at dropblock_p=0
        def __init__(self, *a, **k):
            raise RuntimeError("DropBlock2d stub")

    ops.DropBlock2d = DropBlock2d
    tv.ops = ops
    sys.modules.setdefault("torchvision", tv)
    sys.modules.setdefault("torchvision.ops", ops)
    sys.path.insert(0, REF)
    from model.model import RCNN, BidirectionalLSTM  # noqa
    from training.utils import ctc_greedy_decoder  # noqa
    return RCNN, BidirectionalLSTM, ctc_greedy_decoder


RCNN, BidirectionalLSTM, ctc_greedy_decoder = _import_reference()


def load_charset(path):
    # restatement of data/transforms.py:39-59 (cv2/albumentations absent here)
    itos = []
    with open(path, "r", encoding="utf-8") as f:
        for line in f:
            tok = line.rstrip("\n")
            if tok == "":
                continue
            itos.append(tok)
    return itos


class CTCModel(nn.Module):
    """reference RCNN encoder + the CTC head this build adds."""

    def __init__(self, num_classes, hidden):
        super().__init__()
        self.rcnn = RCNN(num_classes=num_classes, hidden_size=hidden, blank_id=None)
        self.ctc_head = nn.Linear(hidden, num_classes)

    def forward(self, x):
        return self.ctc_head(self.rcnn.encode(x))


def build(num_classes, hidden, seed, head_gain):
    m = CTCModel(num_classes, hidden)
    shapes = model_shapes(m)
    sd = recipe_state_dict(shapes, seed, head_gain=head_gain)
    m.load_state_dict(to_wrapped(sd), strict=False)
    return m, sd


def model_shapes(m):
    """(key, shape) in build order: encoder keys (reference names) then ctc_head."""
    out = []
    for k, v in m.state_dict().items():
        if k.startswith("rcnn.attn."):
            continue
        name = k[len("rcnn."):] if k.startswith("rcnn.") else k
        out.append((name, tuple(v.shape)))
    return out


def to_wrapped(sd):
    return {("rcnn." + k if not k.startswith("ctc_head") else k): v for k, v in sd.items()}


def calibrate(m, images):
    """BN running-stat calibration: one train-mode pass with momentum 1."""
    bns = [mod for mod in m.modules() if isinstance(mod, nn.BatchNorm2d)]
    saved = [b.momentum for b in bns]
    for b in bns:
        b.momentum = 1.0
    m.train()
    with torch.no_grad():
        m(images)
    for b, mo in zip(bns, saved):
        b.momentum = mo
    m.eval()
    return {k[len("rcnn."):]: v.detach().clone() for k, v in m.state_dict().items()
            if k.endswith("running_mean") or k.endswith("running_var")}


def sample_idx(n, count=512):
    if n <= count:
        return np.arange(n)
    return np.linspace(0, n - 1, count).astype(np.int64)


CASES_EVAL = [
    # name, B, H, W, hidden, seed, head_gain
    ("b4_32x128_h256", 4, 32, 128, 256, 11, 6.0),
    ("b4_32x256_h512", 4, 32, 256, 512, 12, 6.0),
    ("b2_64x256_h256", 2, 64, 256, 256, 13, 6.0),
]

CASES_TRAIN = [
    ("b4_32x128_h256", 4, 32, 128, 256, 21, 1.0),
    ("b3_32x256_h512", 3, 32, 256, 512, 22, 1.0),
]


def gen_eval(itos):
    C = len(itos)
    for name, B, H, W, hid, seed, gain in CASES_EVAL:
        torch.manual_seed(0)
        m, sd = build(C, hid, seed, gain)
        T = W // 8
        calib, _, _, _ = synthetic_batch(8, H, W, T, C, seed=seed + 500)
        stats = calibrate(m, calib)
        images, pix, _, _ = synthetic_batch(B, H, W, T, C, seed=seed + 1000)
        with torch.no_grad():
            f = m.rcnn.cnn(images)
            seq = m.rcnn.pool(f).squeeze(2).permute(0, 2, 1)
            enc = m.rcnn.encode(images)
            logits = m.ctc_head(enc)
        out = dict(pixels=pix.numpy(), seed=np.int64(seed), head_gain=np.float64(gain),
                   hidden=np.int64(hid), calib_seed=np.int64(seed + 500),
                   cnn_out=f.numpy(), seq=seq.numpy(), enc=enc.numpy(), logits=logits.numpy())
        for k, v in stats.items():
            out["bn::" + k] = v.numpy()
        np.savez_compressed(os.path.join(HERE, f"encode_eval_{name}.npz"), **out)
        print("wrote encode_eval", name, logits.shape, float(logits.abs().max()))


def gen_train(itos):
    C = len(itos)
    for name, B, H, W, hid, seed, gain in CASES_TRAIN:
        torch.manual_seed(0)
        m, sd = build(C, hid, seed, gain)
        m.rcnn.enc_dropout.p = 0.0
        m.train()
        T = W // 8
        images, pix, targets, lengths = synthetic_batch(B, H, W, T, C, seed=seed + 1000)
        logits = m(images)
        logits.retain_grad()
        lp = F.log_softmax(logits, dim=-1).permute(1, 0, 2)
        loss = F.ctc_loss(lp, targets, torch.full((B,), T, dtype=torch.long), lengths,
                          blank=0, reduction="mean", zero_infinity=True)
        loss.backward()
        out = dict(pixels=pix.numpy(), targets=targets.numpy(), target_lengths=lengths.numpy(),
                   seed=np.int64(seed), head_gain=np.float64(gain), hidden=np.int64(hid),
                   logits=logits.detach().numpy(), loss=np.float64(loss.item()),
                   dlogits=logits.grad.numpy())
        names = []
        for k, p in m.named_parameters():
            if k.startswith("rcnn.attn."):
                continue
            key = k[len("rcnn."):] if k.startswith("rcnn.") else k
            g = p.grad.detach().reshape(-1).numpy().astype(np.float64)
            idx = sample_idx(g.size)
            out["gnorm::" + key] = np.float64(np.sqrt((g * g).sum()))
            out["gsum::" + key] = np.float64(g.sum())
            out["gidx::" + key] = idx
            out["gval::" + key] = g[idx].astype(np.float32)
            names.append(key)
        for k, v in m.state_dict().items():
            if k.endswith("running_mean") or k.endswith("running_var"):
                out["bnrun::" + k[len("rcnn."):]] = v.numpy()
        out["param_names"] = np.array(names)
        np.savez_compressed(os.path.join(HERE, f"train_{name}.npz"), **out)
        print("wrote train", name, "loss", loss.item())


def gen_ctc():
    g = torch.Generator().manual_seed(77)
    T, B, C = 20, 6, 12
    logits = torch.randn(T, B, C, generator=g, dtype=torch.float64).float() * 2.0
    # includes repeats, max length (T/2 with repeats), an infeasible label (zero_infinity), len-1
    tl = [3, 5, 1, 10, 12, 4]
    labels = torch.zeros(B, 12, dtype=torch.long)
    rows = [
        [1, 2, 3], [4, 4, 5, 5, 6], [7], [1, 1, 1, 1, 1, 1, 1, 1, 1, 1],
        [2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2], [3, 9, 3, 9],
    ]
    for b, r in enumerate(rows):
        labels[b, :len(r)] = torch.tensor(r)
    out = {}
    for red in ["mean", "sum", "none"]:
        for zi in [True, False]:
            x = logits.clone().requires_grad_(True)
            lp = F.log_softmax(x, dim=-1)
            loss = F.ctc_loss(lp, labels, torch.full((B,), T, dtype=torch.long),
                              torch.tensor(tl), blank=0, reduction=red, zero_infinity=zi)
            s = loss.sum()
            if torch.isfinite(s):
                s.backward()
                gr = x.grad.numpy()
            else:
                gr = np.full(x.shape, np.nan, np.float32)
            out[f"loss_{red}_{int(zi)}"] = loss.detach().numpy()
            out[f"grad_{red}_{int(zi)}"] = gr
    out.update(logits=logits.numpy(), labels=labels.numpy(), target_lengths=np.array(tl))
    # a bigger case at the bench geometry (T=32, C=194) with mean + zero_infinity
    T2, B2, C2 = 32, 16, 194
    l2 = torch.randn(T2, B2, C2, generator=g, dtype=torch.float64).float() * 3.0
    tl2 = torch.randint(1, 17, (B2,), generator=g)
    lab2 = torch.randint(3, C2, (B2, 16), generator=g)
    x = l2.clone().requires_grad_(True)
    loss = F.ctc_loss(F.log_softmax(x, -1), lab2, torch.full((B2,), T2, dtype=torch.long), tl2,
                      blank=0, reduction="mean", zero_infinity=True)
    loss.backward()
    out.update(big_logits=l2.numpy(), big_labels=lab2.numpy(), big_tl=tl2.numpy(),
               big_loss=loss.detach().numpy(), big_grad=x.grad.numpy())
    np.savez_compressed(os.path.join(HERE, "ctc_cases.npz"), **out)
    print("wrote ctc_cases")


def gen_decode(itos):
    alphabet = "".join(itos[1:]) if all(len(t) == 1 for t in itos[3:]) else None
    # alphabet[p-1] indexing (training/utils.py:146): alphabet = itos[1:], as a list
    alpha_list = itos[1:]
    g = torch.Generator().manual_seed(91)
    B, T, C = 40, 32, len(itos)
    logits = torch.randn(B, T, C, generator=g)
    # make blanks and repeats frequent
    boost = torch.randint(0, 3, (B, T), generator=g)
    logits[..., 0] += (boost == 0).float() * 4.0
    texts, seqs = ctc_greedy_decoder(logits, alpha_list, blank=0)
    np.savez_compressed(os.path.join(HERE, "decode.npz"), logits=logits.numpy())
    with open(os.path.join(HERE, "decode.json"), "w", encoding="utf-8") as f:
        json.dump({"texts": texts, "seqs": seqs, "layout": "BTC", "B": B, "T": T,
                   "alphabet_is_str": alphabet is not None}, f, ensure_ascii=False)
    print("wrote decode", texts[:3])


def gen_decode_b8(itos):
    """B=8, T=16 (configs[0]): explicit (B, T, C) strings from the reference's decoder itself."""
    alpha_list = itos[1:]
    g = torch.Generator().manual_seed(92)
    B, T, C, PAD_B = 8, 16, len(itos), 25
    logits = torch.randn(B, T, C, generator=g)
    boost = torch.randint(0, 3, (B, T), generator=g)
    logits[..., 0] += (boost == 0).float() * 4.0
    rep = torch.randint(0, 2, (B, T), generator=g).bool()       # frequent repeats of the previous argmax
    for t in range(1, T):
        logits[:, t][rep[:, t]] = logits[:, t - 1][rep[:, t]]
    padded = torch.cat([logits, torch.zeros(PAD_B - B, T, C)], 0)   # B=25 > T=16: no axis swap
    texts, seqs = ctc_greedy_decoder(padded, alpha_list, blank=0)
    # what the heuristic does with the bare B=8 batch (for the record: it decodes the wrong axis)
    texts_bare, _ = ctc_greedy_decoder(logits, alpha_list, blank=0)
    np.savez_compressed(os.path.join(HERE, "decode_b8_t16.npz"), logits=logits.numpy())
    with open(os.path.join(HERE, "decode_b8_t16.json"), "w", encoding="utf-8") as f:
        json.dump({"texts": texts[:B], "seqs": seqs[:B], "layout": "BTC", "B": B, "T": T,
                   "padded_to": PAD_B, "heuristic_on_bare_batch_rows": len(texts_bare)}, f, ensure_ascii=False)
    print("wrote decode_b8_t16", texts[:2], "bare heuristic rows:", len(texts_bare))


def gen_bilstm_stack():
    torch.manual_seed(0)
    layers = [BidirectionalLSTM(512, 768, 768)] + [BidirectionalLSTM(768, 768, 768) for _ in range(3)]
    stack = nn.Sequential(*layers)
    shapes = [(k, tuple(v.shape)) for k, v in stack.state_dict().items()]
    sd = recipe_state_dict([("enc_rnn." + k, s) for k, s in shapes], 31)
    stack.load_state_dict({k: sd["enc_rnn." + k] for k, _ in shapes})
    g = torch.Generator().manual_seed(32)
    x = torch.randn(2, 16, 512, generator=g).requires_grad_(True)
    proj = torch.randn(2, 16, 768, generator=g)
    y = stack(x)
    (y * proj).sum().backward()
    np.savez_compressed(os.path.join(HERE, "bilstm_stack.npz"), x=x.detach().numpy(),
                        proj=proj.numpy(), y=y.detach().numpy(), dx=x.grad.numpy(),
                        seed=np.int64(31))
    print("wrote bilstm_stack", y.shape)


def gen_attn():
    """reference Attention decoder, eval mode (dropout off): greedy decode and teacher forcing.
    The generator is scaled x30 so the greedy argmax margins survive fp32 reordering."""
    from model.model import Attention  # noqa (reference, read-only)
    B, T, H, V, steps = 4, 16, 64, 194, 11
    torch.manual_seed(41)
    dec = Attention(input_size=H, hidden_size=H, num_classes=V, sos_id=1, eos_id=2, pad_id=0, blank_id=3,
                    dropout_p=0.1, sampling_prob=0.0)
    with torch.no_grad():
        dec.generator.weight.mul_(30.0)
        dec.generator.bias.mul_(30.0)
    dec.eval()
    g = torch.Generator().manual_seed(42)
    enc = torch.randn(B, T, H, generator=g)
    text = torch.randint(4, V, (B, steps), generator=g)
    text[:, 0] = 1
    with torch.no_grad():
        probs = dec(enc, is_train=False, batch_max_length=steps - 1)
        logits = dec(enc, text=text, is_train=True, batch_max_length=steps - 1)
    top2 = probs.topk(2, dim=-1).values
    margin = float((top2[..., 0] - top2[..., 1]).min())
    out = {k: v.detach().numpy() for k, v in dec.state_dict().items()}
    out.update(enc=enc.numpy(), text=text.numpy(), probs=probs.numpy(), logits=logits.numpy(),
               greedy=probs.argmax(-1).numpy(), min_margin=np.float64(margin))
    np.savez_compressed(os.path.join(HERE, "attn_decoder.npz"), **out)
    print("wrote attn_decoder", probs.shape, "min greedy margin", margin)


def main():
    if sys.argv[1:] == ["attn"]:
        gen_attn()
        return
    itos = load_charset(os.path.join(REF, "configs", "charset.txt"))
    if sys.argv[1:] == ["decode_b8"]:
        gen_decode_b8(itos)
        return
    with open(os.path.join(HERE, "charset.txt"), "w", encoding="utf-8") as f:
        for t in itos:
            f.write(t + "\n")
    torch.set_num_threads(8)
    gen_ctc()
    gen_decode(itos)
    gen_decode_b8(itos)
    gen_bilstm_stack()
    gen_eval(itos)
    gen_train(itos)
    gen_attn()


if __name__ == "__main__":
    main()
