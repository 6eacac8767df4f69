"""Training-loop correctness around the hot path: optimizer state in checkpoints (resume ==
uninterrupted run, torch AdamW format), decoder-aware strict checkpoint loading (CTC vs the
reference's attention head), the saved-activation generation guard, and the persistent
BiLSTM's sticky status word."""
import os

import numpy as np
import pytest
import torch

import crnn_oracle as O
from helpers import GOLDEN, case_params, load, pixels_to_images


class _FlatModel(torch.nn.Module):
    """stand-in for RCNN's flat-buffer layout (parameters are views of one fp32 buffer)"""

    def __init__(self, shapes, seed=0):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.randn(*s, generator=g)) for s in shapes])
        n = sum(p.numel() for p in self.ps)
        self._flat_param = torch.empty(n)
        self._flat_grad = torch.zeros(n)
        off = 0
        for p in self.ps:
            k = p.numel()
            self._flat_param[off:off + k].copy_(p.data.reshape(-1))
            p.data = self._flat_param[off:off + k].view_as(p)
            off += k


def test_fused_adamw_loads_torch_adamw_state():
    """torch.optim.AdamW's state_dict (the reference's optimizer, training/train.py:294-295) loads
    into FusedAdamW's flat moments and round-trips back out in the same format."""
    from crnn_hip.optim import FusedAdamW
    shapes = [(3, 4), (5,), (2, 2, 2)]
    ref = _FlatModel(shapes)
    opt_t = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.05)
    g = torch.Generator().manual_seed(3)
    for _ in range(3):
        for p in ref.parameters():
            p.grad = torch.randn(p.shape, generator=g)
        opt_t.step()
    sd = opt_t.state_dict()
    m = _FlatModel(shapes, seed=1)
    opt = FusedAdamW(m, lr=1e-2, weight_decay=0.05)
    opt.load_state_dict(sd)
    assert opt.step_count == 3
    want_m = torch.cat([sd["state"][i]["exp_avg"].reshape(-1) for i in range(3)])
    want_v = torch.cat([sd["state"][i]["exp_avg_sq"].reshape(-1) for i in range(3)])
    assert torch.equal(opt._m, want_m) and torch.equal(opt._v, want_v)
    out = opt.state_dict()
    assert set(out["state"]) == {0, 1, 2}
    for i in range(3):
        assert int(float(out["state"][i]["step"])) == 3
        assert torch.equal(out["state"][i]["exp_avg"], sd["state"][i]["exp_avg"])
        assert torch.equal(out["state"][i]["exp_avg_sq"], sd["state"][i]["exp_avg_sq"])
    # a torch AdamW accepts FusedAdamW's state_dict
    opt_t2 = torch.optim.AdamW(_FlatModel(shapes).parameters(), lr=1e-2, weight_decay=0.05)
    opt_t2.load_state_dict(out)
    assert torch.equal(opt_t2.state_dict()["state"][1]["exp_avg"], sd["state"][1]["exp_avg"])


def test_fused_adamw_load_before_flat_buffers_defers():
    from crnn_hip.optim import FusedAdamW
    shapes = [(4,), (2, 3)]
    src = _FlatModel(shapes)
    o = FusedAdamW(src)
    o.step_count = 5
    o._bufs = [torch.arange(10.0), torch.arange(10.0) * 2]
    sd = o.state_dict()
    m = _FlatModel(shapes)
    flat = m._flat_param
    m._flat_param = None          # the RCNN case before its first device forward
    o2 = FusedAdamW(m)
    o2.load_state_dict(sd)
    assert o2._m is None and o2.step_count == 5
    o2._alloc_state(flat)
    assert torch.equal(o2._m, torch.arange(10.0)) and torch.equal(o2._v, torch.arange(10.0) * 2)


def _attn_state(hidden=64):
    from crnn_hip.recipe import recipe_state_dict
    z = load("attn_decoder.npz")
    sd = {k: v for k, v in recipe_state_dict(O.param_shapes(hidden, 194), 17).items() if not k.startswith("ctc_head.")}
    for k in z.files:
        if k.startswith(("attention_cell.", "generator.")):
            sd["attn." + k] = torch.from_numpy(z[k])
    return sd


def test_checkpoint_decoder_is_chosen_by_keys_and_loaded_strictly():
    """a reference checkpoint (attn.*, no ctc_head.*) builds the attention model and
    loads strictly; a CTC checkpoint builds the CTC model; a checkpoint with neither raises."""
    from training.utils import rcnn_from_state
    sd = _attn_state()
    m = rcnn_from_state(sd, 194, 64, 1, 2, 0, None, torch.float32)
    assert m.decoder == "attn" and m.ctc_head is None
    assert set(m.state_dict()) == set(sd)
    for k, v in sd.items():
        assert torch.equal(m.state_dict()[k], v), k
    z = load("encode_eval_b4_32x128_h256.npz")
    sd_ctc, hidden = case_params(z)
    m = rcnn_from_state(sd_ctc, 194, hidden, 1, 2, 0, None, torch.float32)
    assert m.decoder == "ctc"
    with pytest.raises(ValueError, match="neither"):
        rcnn_from_state({k: v for k, v in sd.items() if not k.startswith("attn.")}, 194, 64, 1, 2, 0, None)
    bad = dict(sd)
    bad.pop("attn.generator.bias")
    with pytest.raises(RuntimeError, match="Missing key"):
        rcnn_from_state(bad, 194, 64, 1, 2, 0, None)


# ---------------------------------------------------------------------------------- GPU
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


@pytest.mark.gpu
def test_resume_equals_uninterrupted_training(tmp_path):
    """save_checkpoint after 2 steps -> fresh model + FusedAdamW -> load_checkpoint -> step 3
    gives the parameters of 3 uninterrupted steps (bitwise: same kernels, same inputs)."""
    _gpu()
    from crnn_hip.ctc import ctc_loss
    from crnn_hip.optim import FusedAdamW
    from crnn_hip.recipe import recipe_state_dict, synthetic_batch
    from model.model import RCNN
    from training.utils import load_checkpoint, save_checkpoint
    sd = recipe_state_dict(O.param_shapes(256, 194), 5)
    x, _, tg, tl = synthetic_batch(16, 32, 128, 16, 194, seed=9)
    x = x.cuda()

    def fresh():
        m = RCNN(num_classes=194, hidden_size=256, blank_id=None, compute_dtype=torch.bfloat16, enc_dropout_p=0.0)
        m.load_state_dict(sd, strict=False)
        m = m.cuda().train()
        return m, FusedAdamW(m, lr=1e-3, weight_decay=1e-2)

    def step(m, opt):
        opt.zero_grad()
        ctc_loss(m(x), tg, tl).backward()
        opt.step()

    a, oa = fresh()
    for _ in range(3):
        step(a, oa)
    b, ob = fresh()
    for _ in range(2):
        step(b, ob)
    path = str(tmp_path / "ck.pth")
    save_checkpoint(path, b, ob, None, None, 0, 2, 0.0, 0.0, ["a"], {"a": 0}, {"hidden_size": 256}, "x")
    c, oc = fresh()
    load_checkpoint(path, c, oc, map_location="cuda")
    assert oc.step_count == 2
    step(c, oc)
    torch.cuda.synchronize()
    for (k, pa), (_, pc) in zip(a.named_parameters(), c.named_parameters()):
        assert torch.equal(pa, pc), k
    # BN running statistics resume too
    for (k, ba), (_, bc) in zip(a.named_buffers(), c.named_buffers()):
        assert torch.equal(ba, bc), k


@pytest.mark.gpu
def test_second_forward_before_backward_raises():
    """the engine keeps one forward's activations; a backward through an older
    forward must fail loudly instead of differentiating the newer batch."""
    _gpu()
    from crnn_hip.ctc import ctc_loss
    from crnn_hip.recipe import recipe_state_dict, synthetic_batch
    from model.model import RCNN
    m = RCNN(num_classes=194, hidden_size=256, blank_id=None, compute_dtype=torch.bfloat16, enc_dropout_p=0.0)
    m.load_state_dict(recipe_state_dict(O.param_shapes(256, 194), 5), strict=False)
    m = m.cuda().train()
    x1, _, tg, tl = synthetic_batch(16, 32, 128, 16, 194, seed=9)
    x2, _, _, _ = synthetic_batch(16, 32, 128, 16, 194, seed=10)
    l1 = ctc_loss(m(x1.cuda()), tg, tl)
    l2 = ctc_loss(m(x2.cuda()), tg, tl)
    with pytest.raises(RuntimeError, match="forward #"):
        (l1 + l2).backward()
    # the latest forward alone still differentiates
    l3 = ctc_loss(m(x2.cuda()), tg, tl)
    l3.backward()
    assert all(torch.isfinite(p.grad).all() for p in m.parameters())


@pytest.mark.gpu
def test_seq_status_word_is_sticky_and_polled():
    """the persistent BiLSTM's error words are ORed into a sticky word; check_status() raises on
    it and the per-call non-blocking poll raises once its copy has landed."""
    _gpu()
    from crnn_hip import _lib as L
    from crnn_hip.ctc import ctc_loss
    from crnn_hip.optim import FusedAdam, FusedAdamW, FusedSGD
    from crnn_hip.recipe import recipe_state_dict, synthetic_batch
    from model.model import RCNN
    m = RCNN(num_classes=194, hidden_size=256, blank_id=None, compute_dtype=torch.bfloat16, enc_dropout_p=0.0)
    m.load_state_dict(recipe_state_dict(O.param_shapes(256, 194), 5), strict=False)
    m = m.cuda().train()
    x, _, tg, tl = synthetic_batch(16, 32, 128, 16, 194, seed=9)
    x = x.cuda()
    ctc_loss(m(x), tg, tl).backward()
    eng = m._engine
    assert eng._seq_used, "B=16, H=256 bf16 should run the persistent BiLSTM kernels"
    eng.check_status()                     # clean
    ws = eng.ws.bufs["rnn.seq_ws"]
    # the library's layout, not a hard-coded one
    assert eng._sticky_index == L.lib().crnn_lstm_seq_status_offset(16) // 4
    ws[eng._sticky_index] = 1             # as if a sweep had timed out
    with pytest.raises(RuntimeError, match="timed out"):
        eng.check_status()
    # the optimizer kernels read the sticky word and leave weights and moments untouched (ADVICE r02:
    # a timed-out sweep's NaN gradients must not reach a checkpoint)
    for make in (lambda: FusedAdam(m, lr=1e-2, weight_decay=1e-2), lambda: FusedAdamW(m, lr=1e-2),
                 lambda: FusedSGD(m, lr=1e-2, momentum=0.9)):
        opt = make()
        before = m._flat_param.clone()
        m._flat_grad.fill_(float("nan"))
        opt.step()
        torch.cuda.synchronize()
        assert torch.equal(m._flat_param, before)
        assert all(torch.count_nonzero(b) == 0 for b in opt._bufs)
    with pytest.raises(RuntimeError, match="timed out"):
        for _ in range(4):
            ctc_loss(m(x), tg, tl).backward()
            torch.cuda.synchronize()


@pytest.mark.gpu
def test_ocr_inference_with_reference_attention_checkpoint(tmp_path):
    """a reference-format checkpoint (attn.*, no ctc_head.*) is served by the attention
    decoder: predict() returns the oracle's greedy attention decode through decode_tokens."""
    _gpu()
    from data.transforms import decode_tokens
    from inference import OCRInference
    sd = _attn_state()
    ck = tmp_path / "ref_attn.pth"
    torch.save({"config": {"hidden_size": 64}, "model_state": sd}, ck)
    ocr = OCRInference(str(ck), os.path.join(GOLDEN, "charset.txt"), img_h=32, img_w=128,
                       compute_dtype=torch.float32)
    assert ocr.model.decoder == "attn"
    z = load("encode_eval_b4_32x128_h256.npz")
    pix = np.asarray(z["pixels"])
    crops = [p.transpose(1, 2, 0) for p in pix]
    p = {k: v.float() for k, v in sd.items()}
    enc = O.encode(pixels_to_images(pix), p, O.Ctx(train=False))
    pa = {k[5:]: v for k, v in p.items() if k.startswith("attn.")}
    ref = O.attn_greedy(pa, enc, 26, ocr.sos_id, ocr.blank_id, 194)
    want = [decode_tokens(r, ocr.itos, ocr.pad_id, ocr.eos_id, ocr.blank_id) for r in ref.argmax(-1)]
    assert ocr.predict(crops, max_length=25) == want
    tc = ocr.predict(crops, max_length=25, return_confidence=True)
    assert [t for t, _ in tc] == want and all(0.0 <= c <= 1.0 for _, c in tc)
