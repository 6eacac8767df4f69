"""The reference's predictions for a CTC model that READS, at the bench configuration (VERDICT r05 next 2;
north_star "word-accuracy within 0.1 % of reference", "identical greedy-decoded strings").

The model: RCNN(decoder="ctc"), hidden 512, 2 BiLSTM layers, 32x256 crops, C = 194, trained WHOLE (CNN
included) on the MI355X by this path's own training.train.run_training (tools/train_refmodel_ctc.py ->
gpurun_out/refmodel3_weights.npz: int8 per row + fp32 scale for every tensor of more than one dimension, fp32
for the rest; the dequantized values are the model both sides evaluate).

Runs only in the build container: it imports the reference (/root/reference: model/model.py,
model/seresnet31.py, training/utils.py; torchvision.ops.DropBlock2d stubbed, never constructed at
dropblock_p = 0). Nothing of the reference is stored — only data:
  * the weights (as above);
  * 10 000 held-out lines rendered with DejaVu fonts (tests/golden/make_lines.py's renderer, a seed the
    training lines never used), grayscale uint8 at their 32-px height (ragged widths);
  * the reference's greedy predictions on them: RCNN.encode (model/model.py:215-221) -> the CTC head
    (Linear 512 -> 194, the path's SURVEY D1 addition, with the trained weights) -> ctc_greedy_decoder
    (training/utils.py:122-150, alphabet[p-1] with alphabet = charset[1:], blank 0), on the restated input
    pipeline oracle/preprocess_oracle.py (bit-exact to the HIP preprocess kernel; cv2 / albumentations are
    absent here), and their exact-match accuracy.

    python tests/golden/make_refmodel3.py [gpurun_out/refmodel3_weights.npz]   # ~5 min on 8 cores
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
import preprocess_oracle as P  # noqa: E402

N_TEST = 10000
TEST_SEED = 7373   # the training lines use tools/train_refmodel_ctc.py's SEED (6161) streams
OUT = os.path.join(HERE, "refmodel3_ctc.npz")


def dequantize(q, s):
    q2 = q.reshape(q.shape[0], -1).astype(np.float32)
    return (q2 * s.reshape(-1, 1)).reshape(q.shape)


def state_dict_of(z):
    sd = {}
    for k in z.files:
        if k.startswith("q::"):
            sd[k[3:]] = torch.from_numpy(dequantize(z[k], z["s::" + k[3:]]))
        elif k.startswith("f::"):
            sd[k[3:]] = torch.from_numpy(np.array(z[k]))
    return sd


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out", "refmodel3_weights.npz")
    torch.set_num_threads(os.cpu_count() or 8)
    RCNN, _, ctc_greedy_decoder = _import_reference()
    z = np.load(src)
    sd = state_dict_of(z)
    itos = load_charset(os.path.join(HERE, "charset.txt"))
    stoi = {s: i for i, s in enumerate(itos)}
    C, hidden, H, W = len(itos), int(z["hidden"]), int(z["img_h"]), int(z["img_w"])
    m = RCNN(num_classes=C, hidden_size=hidden, sos_id=stoi["<SOS>"], eos_id=stoi["<EOS>"], pad_id=stoi["<PAD>"],
             blank_id=stoi.get("<BLANK>"), enc_dropout_p=0.1)
    head = nn.Linear(hidden, C)
    ref_keys = set(m.state_dict().keys())
    enc = {k: v for k, v in sd.items() if k in ref_keys}
    missing = [k for k in ref_keys if k not in enc and not k.startswith("attn.")]
    assert not missing, missing[:5]
    m.load_state_dict(enc, strict=False)
    head.load_state_dict({"weight": sd["ctc_head.weight"], "bias": sd["ctc_head.bias"]})
    m.eval()
    head.eval()
    t0 = time.time()
    test = []
    for i in range(N_TEST):
        rng = random.Random(TEST_SEED * 1_000_003 + i)
        t = words(rng)
        test.append((np.asarray(render(t, rng).convert("L")), t))
    print(f"rendered {len(test)} held-out lines ({time.time() - t0:.0f} s)", flush=True)
    alphabet = list(itos[1:])   # alphabet[p - 1] = itos[p] (training/utils.py:146)
    preds = []
    with torch.no_grad():
        for i in range(0, N_TEST, 100):
            x = torch.from_numpy(np.stack([P.preprocess(np.repeat(im[:, :, None], 3, axis=2), H, W)[1]
                                           for im, _ in test[i:i + 100]]))
            logits = head(m.encode(x))                    # [B, T, C]
            texts, _ = ctc_greedy_decoder(logits, alphabet, blank=0)
            preds += list(texts)
            if i % 2000 == 0:
                print(f"  {i}/{N_TEST} ({time.time() - t0:.0f} s)", flush=True)
    truth = [t for _, t in test]
    acc = float(np.mean([p == t for p, t in zip(preds, truth)]))
    print(f"reference exact-match accuracy on the {N_TEST} held-out lines: {acc:.4f} "
          f"(training-side validation accuracy {float(z['val_acc']):.4f})", flush=True)
    out = {k: z[k] for k in z.files}
    out.update(test_widths=np.array([im.shape[1] for im, _ in test], dtype=np.int32),
               test_pixels=np.concatenate([im.reshape(-1) for im, _ in test]),
               test_truth=np.array(truth), test_ref_pred=np.array(preds), test_ref_accuracy=np.float64(acc),
               test_seed=np.int64(TEST_SEED))
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT} ({os.path.getsize(OUT) / 1e6:.1f} MB)", flush=True)


if __name__ == "__main__":
    main()
