"""Which bf16 stage flips the reference model's strings? On the fitted set of
tests/golden/refmodel_attn.npz (tests/test_gpu_refmodel.py), the same fp32 attention decoder runs on
encoder outputs made four ways:
  fp32      the fp32 engine (CNN + BiLSTM in fp32): the reference's strings (the parity claim);
  out16     the fp32 encoder output rounded to bf16 once (only the output store in bf16);
  cnn16     the bf16 engine's CNN sequence (crnn_hpool output, bf16) through an fp32 BiLSTM (the oracle's
            restatement, oracle/crnn_oracle.py bilstm, on the GPU in fp32 torch ops: diagnostic only);
  bf16      the bf16 engine (CNN + BiLSTM in bf16, the performance mode).
For each: strings that differ from the reference's, and the net accuracy change.
    python tools/refmodel_trace.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("rcnn-ocr_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, sub))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from helpers import GOLDEN  # noqa: E402


def load(tmp):
    from test_gpu_refmodel import dequantize
    from crnn_hip.recipe import recipe_state_dict
    from data.transforms import load_charset
    from model.model import RCNN
    z = np.load(os.path.join(GOLDEN, "refmodel_attn.npz"))
    hid, seed = int(z["hidden"]), int(z["seed"])
    m = RCNN(num_classes=194, hidden_size=hid, blank_id=None, decoder="attn")
    shapes = [(k, tuple(v.shape)) for k, v in m.state_dict().items() if not k.startswith("attn.")]
    sd = dict(m.state_dict())
    sd.update(recipe_state_dict(shapes, seed))
    for k in z.files:
        if k.startswith("bn::"):
            sd[k[4:]] = torch.from_numpy(z[k])
        elif k.startswith("q::"):
            sd[k[3:]] = dequantize(torch.from_numpy(z[k]), torch.from_numpy(z["s::" + k[3:]]))
    itos, stoi = load_charset(os.path.join(GOLDEN, "charset.txt"))
    H, W = int(z["img_h"]), int(z["img_w"])
    widths, flat = z["fit_widths"], z["fit_pixels"]
    imgs, off = [], 0
    for w in widths.tolist():
        imgs.append(flat[off:off + H * w * 3].reshape(H, w, 3))
        off += H * w * 3
    return sd, itos, stoi, imgs, [str(t) for t in z["fit_truth"]], [str(t) for t in z["fit_ref_pred"]], H, W, \
        int(z["max_len"]), hid


def main():
    from data.transforms import decode_tokens, preprocess_batch
    from model.model import RCNN
    import crnn_oracle as O
    sd, itos, stoi, imgs, truth, ref, H, W, max_len, hid = load(None)
    dev = torch.device("cuda")
    models = {}
    for name, dt in (("fp32", torch.float32), ("bf16", torch.bfloat16)):
        m = RCNN(num_classes=194, hidden_size=hid, blank_id=None, decoder="attn", compute_dtype=dt,
                 sos_id=stoi["<SOS>"], eos_id=stoi["<EOS>"], pad_id=stoi["<PAD>"])
        m.load_state_dict(sd)
        models[name] = m.to(dev).eval()
    p32 = {k: v.to(dev).float() for k, v in sd.items()}
    dec = models["fp32"]._attn_decoder(dev)
    outs = {k: [] for k in ("fp32", "out16", "cnn16", "bf16")}
    encerr = {k: [] for k in outs}
    for i in range(0, len(imgs), 256):
        batch = [imgs[j] for j in range(i, min(len(imgs), i + 256))]
        x32 = preprocess_batch(batch, H, W, out="encoder", dtype=torch.float32, device=dev)
        x16 = preprocess_batch(batch, H, W, out="encoder", dtype=torch.bfloat16, device=dev)
        e32 = models["fp32"].encode(x32)
        e16 = models["bf16"].encode(x16)
        seq16 = models["bf16"]._engine.ws.bufs["seq"].float()          # the bf16 CNN's sequence features
        ec = seq16
        for l in range(2):
            ec = O.bilstm(ec, p32, f"enc_rnn.{l}")
        encs = {"fp32": e32, "out16": e32.bfloat16().float(), "cnn16": ec, "bf16": e16}
        for k, e in encs.items():
            encerr[k].append(float((e - e32).norm() / e32.norm()))
            logits = dec.run(e.contiguous(), max_len + 1)
            for row in logits.argmax(-1).cpu():
                outs[k].append(decode_tokens(row, itos, pad_id=stoi["<PAD>"], eos_id=stoi["<EOS>"],
                                             blank_id=None))
    acc_ref = np.mean([r == t for r, t in zip(ref, truth)])
    for k, got in outs.items():
        diff = [i for i, (g, r) in enumerate(zip(got, ref)) if g != r]
        acc = np.mean([g == t for g, t in zip(got, truth)])
        print(f"{k:6s}: enc rel err vs fp32 {np.mean(encerr[k]):.2e}; {len(diff)} of {len(ref)} strings differ from the "
              f"reference's; accuracy {acc:.4f} (reference {acc_ref:.4f}, {acc - acc_ref:+.4f}); lines {diff[:12]}",
              flush=True)


if __name__ == "__main__":
    main()
