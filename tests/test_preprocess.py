"""Input pipeline: ResizeAndPadA + A.Normalize(0.5, 0.5) + ToTensorV2
(data/transforms.py:62-120, :185-193).

CPU: the oracle restatement (oracle/preprocess_oracle.py; parity with cv2 itself UNPINNED — cv2
and albumentations are not installed and the reference ships no preprocessed fixtures) checked
on properties cv2's resize has by construction, and the product's host-side geometry
(crnn_hip/preprocess.resize_geometry) against the oracle's restatement of :91-118.
GPU: crnn_preprocess bit-exact against the oracle on ragged batches (gray / RGB / RGBA, up- and
downscaling by integer and fractional factors, equal size, every alignment), and the encoder-layout
output feeding the model gives the same logits as the NCHW tensor."""
import numpy as np
import pytest
import torch

import preprocess_oracle as P

SIZES = [(20, 60), (32, 256), (64, 512), (13, 41), (100, 900), (48, 100), (33, 10), (1, 1), (16, 2000),
         (200, 30), (31, 255), (96, 768), (45, 333), (7, 3)]


def test_geometry_matches_reference_restatement():
    from crnn_hip.preprocess import resize_geometry
    for h, w in SIZES + [(h, w) for h in range(1, 80, 7) for w in range(1, 900, 37)]:
        for ah in ("left", "center", "right"):
            for av in ("top", "center", "bottom"):
                assert resize_geometry(h, w, 32, 256, ah, av) == P.geometry(h, w, 32, 256, ah, av), (h, w, ah, av)


def test_oracle_resize_properties():
    rng = np.random.default_rng(1)
    for h, w in [(13, 41), (100, 900), (20, 60), (64, 512), (45, 333)]:
        k = np.full((h, w, 3), 77, np.uint8)
        c = P.resize_and_pad(k, 32, 256)
        nh, nw, y0, x0, _ = P.geometry(h, w, 32, 256)
        assert (c[y0:y0 + nh, x0:x0 + nw] == 77).all()                     # constants are preserved
        assert (c[:y0] == 255).all() and (c[y0 + nh:] == 255).all() and (c[:, x0 + nw:] == 255).all()
    img = rng.integers(0, 256, (32, 200, 3), dtype=np.uint8)
    assert (P.resize_and_pad(img, 32, 256)[:, :200] == img).all()             # equal size: a copy
    img = rng.integers(0, 256, (64, 512, 3), dtype=np.uint8)                # 2x2 area: rounding shift
    c = P.resize_and_pad(img, 32, 256).astype(int)
    ref = (img[0::2, 0::2].astype(int) + img[1::2, 0::2] + img[0::2, 1::2] + img[1::2, 1::2] + 2) >> 2
    assert (c == ref).all()
    g = np.tile(np.array([0, 255], np.uint8)[None, :, None], (16, 1, 3))     # linear upscale, monotone
    c = P.resize_and_pad(g, 32, 256)
    row = c[16, :, 0].astype(int)
    nh, nw, _, _, it = P.geometry(16, 2, 32, 256)
    assert it == 0 and (np.diff(row[:nw]) >= 0).all() and row[0] == 0 and row[nw - 1] == 255
    gray = rng.integers(0, 256, (20, 60), dtype=np.uint8)                     # GRAY2RGB, RGBA2RGB
    assert (P.resize_and_pad(gray) == P.resize_and_pad(np.repeat(gray[:, :, None], 3, 2))).all()
    rgba = rng.integers(0, 256, (20, 60, 4), dtype=np.uint8)
    assert (P.resize_and_pad(rgba) == P.resize_and_pad(rgba[:, :, :3])).all()
    n = P.normalize(np.array([[[0, 255, 128]]], np.uint8))
    assert n.shape == (3, 1, 1) and n[0, 0, 0] == -1.0 and n[1, 0, 0] == 1.0


def _batch(rng):
    ims = []
    for i, (h, w) in enumerate(SIZES):
        c = (3, 1, 4)[i % 3]
        shape = (h, w) if c == 1 else (h, w, c)
        ims.append(rng.integers(0, 256, shape, dtype=np.uint8))
    return ims


@pytest.mark.gpu
@pytest.mark.parametrize("align", [("left", "center"), ("center", "top"), ("right", "bottom")])
@pytest.mark.parametrize("hw", [(32, 256), (64, 256)])
def test_preprocess_bit_exact_vs_oracle(align, hw):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from crnn_hip.preprocess import CropBatch, preprocess
    rng = np.random.default_rng(hash(align) % 1000 + hw[0])
    ims = _batch(rng)
    b = CropBatch.upload(ims, "cuda")
    u8 = preprocess(b, hw[0], hw[1], *align, out="u8").cpu().numpy()
    x = preprocess(b, hw[0], hw[1], *align, out="nchw").cpu().numpy()
    bad = []
    for i, im in enumerate(ims):
        c, n = P.preprocess(im, hw[0], hw[1], *align)
        if not (u8[i] == c).all():
            bad.append((i, im.shape, int((u8[i] != c).sum())))
        assert np.array_equal(x[i], n), i
    assert not bad, bad
    for dt in (torch.float32, torch.bfloat16):
        e = preprocess(b, hw[0], hw[1], *align, out="encoder", dtype=dt).cpu()
        want = torch.zeros(len(ims), hw[0], hw[1], 8, dtype=dt)
        want[..., :3] = torch.from_numpy(x).permute(0, 2, 3, 1).to(dt)
        assert torch.equal(e, want)


@pytest.mark.gpu
def test_preprocessed_encoder_input_feeds_the_model():
    """RCNN on crnn_preprocess(out="encoder") == RCNN on the NCHW tensor (same logits, fp32 and bf16)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import crnn_oracle as O
    from crnn_hip.preprocess import CropBatch, preprocess
    from crnn_hip.recipe import recipe_state_dict
    from model.model import RCNN
    rng = np.random.default_rng(3)
    ims = _batch(rng)[:6]
    b = CropBatch.upload(ims, "cuda")
    for dt in (torch.float32, torch.bfloat16):
        m = RCNN(num_classes=194, hidden_size=256, blank_id=None, compute_dtype=dt)
        m.load_state_dict(recipe_state_dict(O.param_shapes(256, 194), 5), strict=False)
        m = m.cuda().eval()
        with torch.no_grad():
            a = m(preprocess(b, 32, 256, out="nchw")).clone()
            e = m(preprocess(b, 32, 256, out="encoder", dtype=dt)).clone()
        assert torch.equal(a, e)
