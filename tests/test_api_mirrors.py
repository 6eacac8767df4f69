"""Reference-API mirrors around the hot path: data/transforms, training/metrics, training/utils
checkpoint round trip (CPU), and OCRInference end to end on the HIP path (GPU)."""
import os

import numpy as np
import pytest
import torch

import crnn_oracle as O
from helpers import GOLDEN, case_params, load, pixels_to_images


@pytest.mark.gpu
def test_val_transform_is_identity_resize_plus_normalize():
    """a crop already at the target size is only normalised, with albumentations' arithmetic
    (v - 127.5) * (1/127.5) (data/transforms.py:186-193): exactly the oracle's, and within 1 ulp
    of the goldens' (x/255 - 0.5)/0.5 (pixels_to_images)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import preprocess_oracle as P
    from data.transforms import get_val_transform
    z = load("encode_eval_b4_32x128_h256.npz")
    pix = np.asarray(z["pixels"])            # [B, 3, H, W] uint8
    tf = get_val_transform(pix.shape[2], pix.shape[3])
    got = torch.stack([tf(image=p.transpose(1, 2, 0))["image"] for p in pix])
    want = torch.stack([torch.from_numpy(P.normalize(p.transpose(1, 2, 0))) for p in pix])
    assert torch.equal(got, want)
    assert float((got - pixels_to_images(pix)).abs().max()) <= 1.2e-7


@pytest.mark.gpu
def test_resize_and_pad_geometry():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from data.transforms import resize_and_pad
    img = np.zeros((20, 50, 3), np.uint8)
    out = resize_and_pad(img, 32, 256)
    assert out.shape == (32, 256, 3)
    # 20x50 -> scale min(32/20, 256/50) = 1.6 -> 32x80 at the left, white elsewhere
    assert (out[:, :80] == 0).all() and (out[:, 80:] == 255).all()


def test_pack_attention_targets():
    """data/transforms.py:123-157 semantics: SOS-prefixed inputs, EOS-terminated targets, truncation
    at max_len, unknown characters and <BLANK> dropped."""
    from data.transforms import pack_attention_targets, load_charset
    itos, stoi = load_charset(os.path.join(GOLDEN, "charset.txt"))
    a, b = itos[5], itos[9]
    ti, ty, ln = pack_attention_targets([a + b + "\u2603" + a, "", a * 40], stoi, max_len=25)
    assert ti.shape == (3, 26) and ty.shape == (3, 26)
    assert ti[0, :4].tolist() == [stoi["<SOS>"], 5, 9, 5] and ti[0, 4:].eq(stoi["<PAD>"]).all()
    assert ty[0, :4].tolist() == [5, 9, 5, stoi["<EOS>"]] and ln[0] == 4
    assert ti[1, 0] == stoi["<SOS>"] and ty[1, 0] == stoi["<EOS>"] and ln[1] == 1
    assert ti[2, 1:].eq(5).all() and ty[2, :25].eq(5).all() and ty[2, 25] == stoi["<EOS>"] and ln[2] == 26


def test_metrics():
    from training.metrics import character_error_rate, compute_accuracy, word_error_rate
    assert character_error_rate("abcd", "abed") == 0.25
    assert character_error_rate("", "") == 0.0
    assert word_error_rate("a b c", "a x c") == pytest.approx(1 / 3)
    assert compute_accuracy(["a", "b"], ["a", "c"]) == 0.5


def test_charset_and_decode_tokens():
    from data.transforms import decode_tokens, load_charset
    itos, stoi = load_charset(os.path.join(GOLDEN, "charset.txt"))
    assert itos[:3] == ["<PAD>", "<SOS>", "<EOS>"] and len(itos) == 194   # <PAD> = CTC blank
    ids = [stoi[c] for c in "ab"] + [stoi["<PAD>"], stoi["<EOS>"], stoi["c"]]
    assert decode_tokens(ids, itos, stoi["<PAD>"], stoi["<EOS>"]) == "ab"


def test_checkpoint_round_trip(tmp_path):
    from model.model import RCNN
    from training.utils import load_checkpoint, save_checkpoint
    z = load("encode_eval_b4_32x128_h256.npz")
    sd, hidden = case_params(z)
    m = RCNN(num_classes=194, hidden_size=hidden, blank_id=None, compute_dtype=torch.float32)
    m.load_state_dict(sd, strict=False)
    path = tmp_path / "ck.pth"
    save_checkpoint(str(path), m, None, None, None, 3, 17, 1.5, 0.25, ["a"], {"a": 0}, {"hidden_size": hidden}, "x")
    m2 = RCNN(num_classes=194, hidden_size=hidden, blank_id=None, compute_dtype=torch.float32)
    ck = load_checkpoint(str(path), m2, map_location="cpu")
    assert ck["epoch"] == 3 and ck["global_step"] == 17 and ck["config"]["hidden_size"] == hidden
    for k, v in m.state_dict().items():
        assert torch.equal(v, m2.state_dict()[k]), k


@pytest.mark.gpu
def test_ocr_inference_predicts_golden_strings(tmp_path):
    """inference.py:126-195 contract on the HIP path: a checkpoint in the reference's format,
    predict() on raw HxWx3 crops -> the strings the oracle decodes from the golden logits."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from inference import OCRInference
    from model.model import RCNN
    z = load("encode_eval_b4_32x128_h256.npz")
    sd, hidden = case_params(z)
    m = RCNN(num_classes=194, hidden_size=hidden, blank_id=None, compute_dtype=torch.float32)
    m.load_state_dict(sd, strict=False)
    ck = tmp_path / "model.pth"
    torch.save({"config": {"hidden_size": hidden}, "model_state": m.state_dict()}, ck)
    ocr = OCRInference(str(ck), os.path.join(GOLDEN, "charset.txt"), img_h=32, img_w=128,
                       compute_dtype=torch.float32)
    crops = [p.transpose(1, 2, 0) for p in np.asarray(z["pixels"])]
    itos = ocr.itos
    want = ["".join(itos[t] for t in s) for s in O.greedy_decode(z["logits"])]
    assert ocr.predict(crops) == want
    assert ocr.predict(crops[0]) == want[0]
    texts_conf = ocr.predict(crops, return_confidence=True)
    assert [t for t, _ in texts_conf] == want
    assert all(0.0 <= c <= 1.0 for _, c in texts_conf)
