"""Word accuracy pinned to the reference's OWN trained model (north_star:
"word-accuracy within 0.1 % of reference").

tests/golden/make_refmodel.py trained the reference RCNN (attention head; its CNN the seed recipe,
frozen; its BiLSTM encoder and decoder trained with the reference's modules and CE step on CPU, with
feature noise and dropout) and recorded the reference's own greedy predictions on two sets of 1000
rendered lines: 1000 of the lines it was fitted on (reference exact-match accuracy 98.4 %) and 1000
held-out lines (0.0 %: a frozen random CNN fitted on 3000 lines does not generalise, so that set only
checks that the same strings come out). Here the same weights go through the reference's checkpoint
format into this path's reference API — training.utils.load_crnn and inference.OCRInference.predict
(HIP preprocess -> engine -> HIP attention decoder -> decode_tokens):
  * fp32: the reference's strings, line for line, on both sets (the parity claim);
  * bf16 (the performance mode), fitted lines: the reference's string on at least 99 % of the lines
    and exact-match accuracy within 0.3 % of the reference's. Measured (profiles/r04k_refmodel.log):
    8 of 1000 strings differ, accuracy 98.6 % vs 98.4 %. That is +0.2 %, so bf16 does NOT meet the
    north star's 0.1 % at this sample: one line in 1000 is the resolution, and 8 flips give a net
    change of order sqrt(8) lines. The held-out set's bf16 agreement (47 %) is printed, not asserted:
    this memorising model's outputs on unseen lines change under any perturbation of the features.

r05: tests/golden/make_refmodel2.py trains the same architecture on 40 000 lines so that it
READS unseen lines, and records the reference's predictions on 10 000 held-out lines (refmodel2_attn.npz). On that
set the bar is the north star's: fp32 gives the reference's strings, and bf16 exact-match accuracy is within
0.001 of the reference's (10 lines in 10 000).
r06: that model reads only 17 % of its lines, with an attention head on a frozen random CNN at
hidden 256. tests/golden/make_refmodel3.py pins the bench's own configuration instead: RCNN(decoder="ctc"), hidden
512, 2 BiLSTM layers, 32x256 crops, C = 194, trained WHOLE (CNN included) on the MI355X by this path's own
training.train.run_training (tools/train_refmodel_ctc.py), and the reference's predictions for it on 10 000
held-out lines (RCNN.encode + the CTC head + the reference's ctc_greedy_decoder, training/utils.py:122-150). Bars:
fp32 gives the reference's strings line for line; bf16 exact-match accuracy within 0.001 of the reference's AND the
reference's string on nearly every line (the bound below, set from the measurement).
Reference: inference.py:126-195, training/utils.py:70-119, model/model.py:166-227."""
import os

import numpy as np
import pytest
import torch

from helpers import GOLDEN

pytestmark = pytest.mark.gpu
CHARSET = os.path.join(GOLDEN, "charset.txt")


def dequantize(q, s):
    q2 = q.reshape(q.shape[0], -1) if q.dim() > 1 else q.reshape(1, -1)
    return (q2.float() * s.reshape(-1, 1)).reshape(q.shape)


def _checkpoint(z, path, best_acc):
    """the fixture's weights in the reference's save_checkpoint format (training/utils.py)"""
    from crnn_hip.recipe import recipe_state_dict
    from model.model import RCNN
    hid, seed = int(z["hidden"]), int(z["seed"])
    m = RCNN(num_classes=194, hidden_size=hid, blank_id=None, decoder="attn")
    shapes = [(k, tuple(v.shape)) for k, v in m.state_dict().items() if not k.startswith("attn.")]
    sd = dict(m.state_dict())                      # every key of the reference's attention model
    sd.update(recipe_state_dict(shapes, seed))     # the CNN (and the BiLSTM, overwritten below): the recipe
    for k in z.files:
        if k.startswith("bn::"):
            sd[k[4:]] = torch.from_numpy(z[k])
        elif k.startswith("q::"):
            name = k[3:]
            sd[name] = dequantize(torch.from_numpy(z[k]), torch.from_numpy(z["s::" + name]))
    assert all(("q::" + k) in z.files for k in sd if k.startswith("attn.") or k.startswith("enc_rnn."))
    from data.transforms import load_charset
    itos, stoi = load_charset(CHARSET)
    ck = {"epoch": 1, "global_step": 0, "model_state": sd, "optimizer_state": None, "scheduler_state": None,
          "itos": itos, "stoi": stoi, "scaler_state": None, "best_val_loss": 0.0, "best_val_acc": best_acc,
          "config": {"hidden_size": hid, "img_h": int(z["img_h"]), "img_w": int(z["img_w"]),
                     "max_len": int(z["max_len"])}}
    torch.save(ck, path)


@pytest.fixture(scope="module")
def refmodel2(tmp_path_factory):
    """the generalising model (make_refmodel2.py): checkpoint path, (gray lines as 3-channel arrays, truth,
    reference predictions, reference accuracy) for 10 000 held-out lines, max_len, (img_h, img_w)"""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    z = np.load(os.path.join(GOLDEN, "refmodel2_attn.npz"))
    path = str(tmp_path_factory.mktemp("refmodel2") / "ref_ckpt.pth")
    _checkpoint(z, path, float(z["test_ref_accuracy"]))
    H = int(z["img_h"])
    widths, flat = z["test_widths"], z["test_pixels"]
    imgs, off = [], 0
    for w in widths.tolist():
        g = flat[off:off + H * w].reshape(H, w)
        imgs.append(np.repeat(g[:, :, None], 3, axis=2))   # as the generator fed the reference
        off += H * w
    assert off == flat.size and len(imgs) >= 5000
    test = (imgs, [str(t) for t in z["test_truth"]], [str(t) for t in z["test_ref_pred"]],
            float(z["test_ref_accuracy"]))
    return path, {"test": test}, int(z["max_len"]), (H, int(z["img_w"]))


@pytest.fixture(scope="module")
def refmodel3(tmp_path_factory):
    """the bench-configuration CTC model (make_refmodel3.py): checkpoint path in the reference's save_checkpoint
    format, (gray lines as 3-channel arrays, truth, reference predictions, reference accuracy), (img_h, img_w)"""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    z = np.load(os.path.join(GOLDEN, "refmodel3_ctc.npz"))
    sd = {}
    for k in z.files:
        if k.startswith("q::"):
            sd[k[3:]] = dequantize(torch.from_numpy(z[k]), torch.from_numpy(z["s::" + k[3:]]))
        elif k.startswith("f::"):
            sd[k[3:]] = torch.from_numpy(np.array(z[k]))
    from data.transforms import load_charset
    itos, stoi = load_charset(CHARSET)
    H, W = int(z["img_h"]), int(z["img_w"])
    ck = {"epoch": int(z["epochs"]), "global_step": 0, "model_state": sd, "optimizer_state": None,
          "scheduler_state": None, "itos": itos, "stoi": stoi, "scaler_state": None, "best_val_loss": 0.0,
          "best_val_acc": float(z["val_acc"]),
          "config": {"hidden_size": int(z["hidden"]), "img_h": H, "img_w": W, "max_len": int(z["max_len"]),
                     "decoder": "ctc"}}
    path = str(tmp_path_factory.mktemp("refmodel3") / "ctc_ckpt.pth")
    torch.save(ck, path)
    widths, flat = z["test_widths"], z["test_pixels"]
    imgs, off = [], 0
    for w in widths.tolist():
        imgs.append(np.repeat(flat[off:off + H * w].reshape(H, w)[:, :, None], 3, axis=2))
        off += H * w
    assert off == flat.size and len(imgs) == 10000
    test = (imgs, [str(t) for t in z["test_truth"]], [str(t) for t in z["test_ref_pred"]],
            float(z["test_ref_accuracy"]))
    return path, {"test": test}, int(z["max_len"]), (H, W)


@pytest.fixture(scope="module")
def refmodel(tmp_path_factory):
    """(checkpoint path in the reference's save_checkpoint format, {set: (images, truth, reference
    predictions, reference accuracy)} for the fitted and the held-out lines, max_len, (img_h, img_w))"""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    z = np.load(os.path.join(GOLDEN, "refmodel_attn.npz"))
    path = str(tmp_path_factory.mktemp("refmodel") / "ref_ckpt.pth")
    _checkpoint(z, path, float(z["val_ref_accuracy"]))
    H = int(z["img_h"])
    sets = {}
    for name in ("fit", "val"):
        widths, flat = z[f"{name}_widths"], z[f"{name}_pixels"]
        imgs, off = [], 0
        for w in widths.tolist():
            n = H * w * 3
            imgs.append(flat[off:off + n].reshape(H, w, 3))
            off += n
        assert off == flat.size
        sets[name] = (imgs, [str(t) for t in z[f"{name}_truth"]], [str(t) for t in z[f"{name}_ref_pred"]],
                      float(z[f"{name}_ref_accuracy"]))
    return path, sets, int(z["max_len"]), (H, int(z["img_w"]))


def _predict(refmodel, dtype, name, decoder="attn"):
    from inference import OCRInference
    path, sets, max_len, (H, W) = refmodel
    ocr = OCRInference(path, CHARSET, device="cuda", img_h=H, img_w=W, compute_dtype=dtype)
    assert ocr.model.decoder == decoder
    return ocr.predict(sets[name][0], max_length=max_len, batch_size=256)


@pytest.mark.parametrize("name", ["fit", "val"])
def test_refmodel_fp32_reproduces_reference_strings(refmodel, name):
    _, truth, ref, ref_acc = refmodel[1][name]
    got = _predict(refmodel, torch.float32, name)
    diff = [(i, r, g) for i, (r, g) in enumerate(zip(ref, got)) if r != g]
    acc = float(np.mean([g == t for g, t in zip(got, truth)]))
    print(f"{name} fp32: {len(diff)} of {len(ref)} strings differ from the reference's; accuracy {acc:.4f} "
          f"(reference {ref_acc:.4f}); first differences {diff[:5]}")
    assert not diff
    assert acc == ref_acc


@pytest.mark.parametrize("name", ["fit", "val"])
def test_refmodel_bf16_agreement(refmodel, name):
    """r04's memorising model: bf16 keeps the reference's string on >= 99 % of its fitted lines (printed for the
    held-out ones; the accuracy bar lives in test_refmodel_bf16_accuracy on the generalising model)"""
    _, truth, ref, ref_acc = refmodel[1][name]
    got = _predict(refmodel, torch.bfloat16, name)
    same = float(np.mean([g == r for g, r in zip(got, ref)]))
    acc = float(np.mean([g == t for g, t in zip(got, truth)]))
    print(f"{name} bf16: exact-match accuracy {acc:.4f} vs reference {ref_acc:.4f}; the reference's string on "
          f"{same:.4f} of the lines")
    if name == "fit":
        assert same >= 0.99


def test_refmodel2_fp32_reproduces_reference_strings(refmodel2):
    """fp32 on 10 000 held-out lines: the reference's strings, line for line"""
    _, truth, ref, ref_acc = refmodel2[1]["test"]
    got = _predict(refmodel2, torch.float32, "test")
    diff = [(i, r, g) for i, (r, g) in enumerate(zip(ref, got)) if r != g]
    acc = float(np.mean([g == t for g, t in zip(got, truth)]))
    print(f"held-out fp32: {len(diff)} of {len(ref)} strings differ from the reference's; accuracy {acc:.4f} "
          f"(reference {ref_acc:.4f}); first differences {diff[:5]}")
    assert not diff
    assert acc == ref_acc


def test_refmodel_bf16_accuracy(refmodel2):
    """the north star's bar: bf16 (the performance mode) exact-match word accuracy within 0.1 % of the
    reference's on 10 000 held-out lines (a resolution of 0.01 %)"""
    _, truth, ref, ref_acc = refmodel2[1]["test"]
    got = _predict(refmodel2, torch.bfloat16, "test")
    same = float(np.mean([g == r for g, r in zip(got, ref)]))
    acc = float(np.mean([g == t for g, t in zip(got, truth)]))
    print(f"held-out bf16: exact-match accuracy {acc:.4f} vs reference {ref_acc:.4f} (diff {acc - ref_acc:+.4f}); "
          f"the reference's string on {same:.4f} of {len(ref)} lines")
    assert abs(acc - ref_acc) <= 0.001 + 1e-9


def test_refmodel_load_crnn(refmodel):
    """training.utils.load_crnn (training/utils.py:70-119) on the same checkpoint: the attention
    model with the checkpoint's weights, eval mode"""
    from training.utils import load_crnn
    path = refmodel[0]
    m = load_crnn(path, hidden_size=256, device="cuda")
    assert m.decoder == "attn" and not m.training
    sd = torch.load(path, map_location="cpu", weights_only=True)["model_state"]
    got = m.state_dict()
    for k in ("attn.generator.weight", "enc_rnn.1.rnn.weight_hh_l0", "cnn.layer4.2.bn2.running_var"):
        assert torch.equal(got[k].cpu(), sd[k]), k


def test_refmodel3_reads(refmodel3):
    """the fixture is a model that reads: the reference's own exact-match accuracy on the held-out lines"""
    assert refmodel3[1]["test"][3] >= 0.85


def test_refmodel3_fp32_reproduces_reference_strings(refmodel3):
    """fp32, the bench's CTC model, 10 000 held-out lines: the reference's greedy-decoded strings, line for line
    (north_star "identical greedy-decoded strings")"""
    _, truth, ref, ref_acc = refmodel3[1]["test"]
    got = _predict(refmodel3, torch.float32, "test", decoder="ctc")
    diff = [(i, r, g) for i, (r, g) in enumerate(zip(ref, got)) if r != g]
    acc = float(np.mean([g == t for g, t in zip(got, truth)]))
    print(f"CTC held-out fp32: {len(diff)} of {len(ref)} strings differ from the reference's; accuracy {acc:.4f} "
          f"(reference {ref_acc:.4f}); first differences {diff[:5]}")
    assert not diff
    assert acc == ref_acc


REFMODEL3_BF16_AGREEMENT = 0.999  # bound on the bf16 string agreement (measured value there)


def test_refmodel3_bf16_accuracy_and_agreement(refmodel3):
    """bf16 (the performance mode) on the bench's CTC model: exact-match accuracy within 0.001 of the reference's
    on 10 000 held-out lines, and the reference's string on at least REFMODEL3_BF16_AGREEMENT of them"""
    _, truth, ref, ref_acc = refmodel3[1]["test"]
    got = _predict(refmodel3, torch.bfloat16, "test", decoder="ctc")
    same = float(np.mean([g == r for g, r in zip(got, ref)]))
    acc = float(np.mean([g == t for g, t in zip(got, truth)]))
    print(f"CTC held-out bf16: exact-match accuracy {acc:.4f} vs reference {ref_acc:.4f} (diff {acc - ref_acc:+.4f}); "
          f"the reference's string on {same:.4f} of {len(ref)} lines")
    assert abs(acc - ref_acc) <= 0.001 + 1e-9
    assert same >= REFMODEL3_BF16_AGREEMENT
