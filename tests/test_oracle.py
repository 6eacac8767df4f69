"""Pin the oracle (oracle/) against the reference-generated goldens (CPU only)."""
import json
import os

import numpy as np
import pytest
import torch

import crnn_oracle as O
from ctc_oracle import ctc_loss_and_grad
from helpers import case_params, load, pixels_to_images, GOLDEN

torch.set_num_threads(min(8, os.cpu_count() or 1))


@pytest.mark.parametrize("case", ["b4_32x128_h256", "b4_32x256_h512", "b2_64x256_h256"])
def test_oracle_encode_eval(case):
    z = load(f"encode_eval_{case}.npz")
    p, hidden = case_params(z)
    x = pixels_to_images(z["pixels"])
    ctx = O.Ctx(train=False, record=True)
    with torch.no_grad():
        enc = O.encode(x, p, ctx)
        logits = O.head(enc, p)
    np.testing.assert_allclose(ctx.acts["cnn_out"].numpy(), z["cnn_out"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(enc.numpy(), z["enc"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(logits.numpy(), z["logits"], rtol=1e-4, atol=1e-4)
    assert O.greedy_decode(logits.numpy()) == O.greedy_decode(z["logits"])


@pytest.mark.parametrize("case", ["b4_32x128_h256", "b3_32x256_h512"])
def test_oracle_train_grads(case):
    z = load(f"train_{case}.npz")
    p, hidden = case_params(z, with_running=False)
    p = {k: (v.clone().requires_grad_(True) if v.is_floating_point() and "running" not in k else v)
         for k, v in p.items()}
    x = pixels_to_images(z["pixels"])
    ctx = O.Ctx(train=True)
    logits = O.head(O.encode(x, p, ctx), p)
    logits.retain_grad()
    loss = O.ctc_loss(logits, torch.from_numpy(z["targets"]), torch.from_numpy(z["target_lengths"]))
    loss.backward()
    assert abs(float(loss.detach()) - float(z["loss"])) < 1e-4 * max(1.0, abs(float(z["loss"])))
    np.testing.assert_allclose(logits.grad.numpy(), z["dlogits"], rtol=1e-3, atol=1e-6)
    for name in z["param_names"]:
        name = str(name)
        g = p[name].grad.reshape(-1).double().numpy()
        ref_norm = float(z["gnorm::" + name])
        assert abs(np.sqrt((g * g).sum()) - ref_norm) <= 2e-3 * ref_norm + 1e-7, name
        idx = z["gidx::" + name]
        ref = z["gval::" + name].astype(np.float64)
        err = np.linalg.norm(g[idx] - ref) / max(np.linalg.norm(ref), 1e-12)
        assert err < 2e-3, (name, err)
    for k, v in ctx.running.items():
        np.testing.assert_allclose(v.numpy(), z["bnrun::" + k], rtol=1e-4, atol=1e-5)


def test_oracle_ctc_cases():
    z = load("ctc_cases.npz")
    logits_btc = np.transpose(z["logits"], (1, 0, 2))
    for red in ["mean", "sum", "none"]:
        for zi in [True, False]:
            loss, grad = ctc_loss_and_grad(logits_btc, z["labels"], z["target_lengths"],
                                           reduction=red, zero_infinity=zi)
            ref = z[f"loss_{red}_{int(zi)}"]
            np.testing.assert_allclose(np.asarray(loss, dtype=np.float64), ref, rtol=1e-5, atol=1e-5)
            refg = z[f"grad_{red}_{int(zi)}"]
            if np.all(np.isfinite(refg)) and np.all(np.isfinite(np.asarray(loss))):
                np.testing.assert_allclose(np.transpose(grad, (1, 0, 2)), refg, rtol=1e-4, atol=1e-6)
    loss, grad = ctc_loss_and_grad(np.transpose(z["big_logits"], (1, 0, 2)), z["big_labels"], z["big_tl"])
    np.testing.assert_allclose(loss, z["big_loss"], rtol=1e-5)
    np.testing.assert_allclose(np.transpose(grad, (1, 0, 2)), z["big_grad"], rtol=1e-4, atol=1e-7)


def test_oracle_decode(itos):
    z = load("decode.npz")
    with open(os.path.join(GOLDEN, "decode.json"), encoding="utf-8") as f:
        ref = json.load(f)
    seqs = O.greedy_decode(z["logits"])
    assert seqs == ref["seqs"]
    assert O.ids_to_text(seqs, itos) == ref["texts"]
    # B=8 / T=16 (configs[0]; T > B): the reference's strings from a batch padded past T
    z = load("decode_b8_t16.npz")
    with open(os.path.join(GOLDEN, "decode_b8_t16.json"), encoding="utf-8") as f:
        ref = json.load(f)
    assert ref["B"] == 8 and ref["T"] == 16 and z["logits"].shape == (8, 16, 194)
    seqs = O.greedy_decode(z["logits"])
    assert seqs == ref["seqs"]
    assert O.ids_to_text(seqs, itos) == ref["texts"]


def test_oracle_bilstm_stack():
    z = load("bilstm_stack.npz")
    from crnn_hip.recipe import recipe_state_dict
    shapes = []
    for l in range(4):
        ind = 512 if l == 0 else 768
        for sfx in ["", "_reverse"]:
            shapes += [(f"enc_rnn.{l}.rnn.weight_ih_l0{sfx}", (3072, ind)),
                       (f"enc_rnn.{l}.rnn.weight_hh_l0{sfx}", (3072, 768)),
                       (f"enc_rnn.{l}.rnn.bias_ih_l0{sfx}", (3072,)),
                       (f"enc_rnn.{l}.rnn.bias_hh_l0{sfx}", (3072,))]
        shapes += [(f"enc_rnn.{l}.linear.weight", (768, 1536)), (f"enc_rnn.{l}.linear.bias", (768,))]
    p = recipe_state_dict(shapes, int(z["seed"]))
    x = torch.from_numpy(z["x"]).requires_grad_(True)
    y = x
    for l in range(4):
        y = O.bilstm(y, p, f"enc_rnn.{l}")
    np.testing.assert_allclose(y.detach().numpy(), z["y"], rtol=1e-4, atol=1e-5)
    (y * torch.from_numpy(z["proj"])).sum().backward()
    np.testing.assert_allclose(x.grad.numpy(), z["dx"], rtol=1e-3, atol=1e-5)


def test_forced_decisions_reproduce_own_decisions():
    """crnn_oracle.relu / maxpool2 with forced decisions equal to the oracle's own give the
    unforced result (the forced fp64 reference used by the GPU train-step tests)."""
    import torch.nn.functional as F
    g = torch.Generator().manual_seed(5)
    u = torch.randn(2, 8, 6, 10, generator=g, dtype=torch.float64)
    own = O.Ctx(train=True)
    forced = O.Ctx(train=True, force={"r": u > 0})
    assert torch.equal(O.relu(own, "r", u), O.relu(forced, "r", u))
    x = torch.relu(u)
    ref, idx = F.max_pool2d(x, 2, 2, return_indices=True)
    # flat index h*W + w -> window element t = 2*dh + dw
    W = x.shape[-1]
    t = 2 * ((idx // W) % 2) + (idx % W) % 2
    got = O.maxpool2(O.Ctx(train=True, force={"stem.pool": t}), "stem.pool", x)
    assert torch.equal(got, ref)
    assert torch.equal(O.maxpool2(own, "stem.pool", x), ref)


def test_oracle_attn_decoder():
    """attention decoder restatement vs the reference's own outputs (attn_decoder.npz): greedy
    decode logits incl. blank masking, the greedy sequence, and teacher-forced logits."""
    z = load("attn_decoder.npz")
    p = {k: torch.from_numpy(z[k]) for k in z.files if k.startswith(("attention_cell.", "generator."))}
    enc = torch.from_numpy(z["enc"])
    text = torch.from_numpy(z["text"]).long()
    steps, V = z["probs"].shape[1], z["probs"].shape[2]
    probs = O.attn_greedy(p, enc, steps, 1, 3, V)
    np.testing.assert_allclose(probs.numpy(), z["probs"], rtol=1e-5, atol=1e-4)
    assert np.array_equal(probs.argmax(-1).numpy(), z["greedy"])
    logits = O.attn_teacher(p, enc, text, steps, 3, V)
    np.testing.assert_allclose(logits.numpy(), z["logits"], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("geo", [(2, 3, 8, 12, 0.3, 5), (3, 4, 5, 5, 0.5, 5), (2, 1, 3, 9, 0.4, 5), (1, 2, 6, 7, 0.2, 3)])
def test_dropblock_keep_definition(geo):
    """crnn_oracle.dropblock_keep (torchvision's drop_block2d structure: pad + bs x bs max-pool of the
    seed map) against the direct definition: a seed at (i, j) of the (H-bs+1) x (W-bs+1) grid drops
    rows i..i+bs-1, cols j..j+bs-1; seeds are the splitmix hash of the flat NCHW seed index below
    gamma * 2^32."""
    B, C, H, W, p, bsz = geo
    seed = 99
    keep = O.dropblock_keep(seed, B, C, H, W, p, bsz)
    bs = min(bsz, H, W)
    Hs, Ws = H - bs + 1, W - bs + 1
    gamma = p * H * W / (bs * bs * Hs * Ws)
    thr = int(gamma * 4294967296.0)
    h = O._splitmix_hash(seed, np.arange(B * C * Hs * Ws)).reshape(B, C, Hs, Ws)
    want = np.ones((B, C, H, W), np.uint8)
    for n in range(B):
        for c in range(C):
            for i in range(Hs):
                for j in range(Ws):
                    if int(h[n, c, i, j]) < thr:
                        want[n, c, i:i + bs, j:j + bs] = 0
    assert np.array_equal(keep, want)
    m = O.dropblock_mult(keep)
    assert np.isclose(float(m.sum()), keep.size if keep.any() else 0.0, rtol=1e-5)


def test_dropblock_keep_rate_and_even_block():
    """the drop share is near p (gamma compensates for the block area; overlaps make it a little
    lower), and an even effective block raises like the reference's broadcast failure."""
    keep = O.dropblock_keep(5, 8, 16, 16, 64, 0.1, 5)
    share = 1.0 - keep.mean()
    assert 0.07 < share < 0.11, share
    with pytest.raises(ValueError):
        O.dropblock_keep(5, 2, 8, 4, 32, 0.1, 5)


def _oracle_reads(fixture, sets, gray, n=24):
    """the oracle's eval encode + attention greedy decode on the first n lines of each set of a reference-model
    fixture, on the preprocess restatement's input: the reference's own strings"""
    import preprocess_oracle as P
    from crnn_hip.recipe import recipe_state_dict
    z = np.load(os.path.join(GOLDEN, fixture))
    hid, seed, H, W, L = (int(z[k]) for k in ("hidden", "seed", "img_h", "img_w", "max_len"))
    with open(os.path.join(GOLDEN, "charset.txt"), encoding="utf-8") as f:
        itos = [l.rstrip("\n") for l in f if l.rstrip("\n") != ""]
    stoi = {s: i for i, s in enumerate(itos)}
    enc_shapes = [(k, s) for k, s in O.param_shapes(hid, len(itos)) if not k.startswith("ctc_head")]
    p = recipe_state_dict(enc_shapes, seed)
    for k in z.files:
        if k.startswith("bn::"):
            p[k[4:]] = torch.from_numpy(z[k])
        elif k.startswith("q::"):
            q, s = torch.from_numpy(z[k]), torch.from_numpy(z["s::" + k[3:]])
            q2 = q.reshape(q.shape[0], -1) if q.dim() > 1 else q.reshape(1, -1)
            p[k[3:] if not k[3:].startswith("attn.") else k[3 + 5:]] = (q2.float() * s.reshape(-1, 1)).reshape(q.shape)
    ch = 1 if gray else 3
    for name in sets:
        widths, flat = z[f"{name}_widths"], z[f"{name}_pixels"]
        imgs, off = [], 0
        for w in widths.tolist()[:n]:
            im = flat[off:off + H * w * ch].reshape(H, w, ch)
            imgs.append(np.repeat(im, 3, axis=2) if gray else im)
            off += H * w * ch
        x = torch.from_numpy(np.stack([P.preprocess(im, H, W)[1] for im in imgs]))
        with torch.no_grad():
            enc = O.encode(x, p, O.Ctx(train=False))
            lg = O.attn_greedy(p, enc, L + 1, stoi["<SOS>"], None, len(itos))
        got = []
        for row in lg.argmax(-1):
            s = ""
            for t in row.tolist():
                if t == stoi["<EOS>"]:
                    break
                if t != stoi["<PAD>"]:
                    s += itos[t]
            got.append(s)
        ref = [str(t) for t in z[f"{name}_ref_pred"][:n]]
        assert got == ref, (name, [(g, r) for g, r in zip(got, ref) if g != r][:4])


def test_oracle_reads_like_the_trained_reference_model():
    """tests/golden/refmodel_attn.npz (make_refmodel.py: the reference RCNN with a trained BiLSTM +
    attention decoder and its own greedy predictions): the oracle gives the reference's strings on a sample of
    the fitted and the held-out lines (the fixture and the oracle pin each other; the GPU test
    tests/test_gpu_refmodel.py runs all 2 x 1000 lines on the HIP path)."""
    _oracle_reads("refmodel_attn.npz", ("fit", "val"), gray=False)


def test_oracle_reads_like_the_generalising_reference_model():
    """tests/golden/refmodel2_attn.npz (make_refmodel2.py: trained on 40 000 lines, reads unseen ones): the
    oracle gives the reference's strings on the first 24 of its 10 000 held-out lines (the GPU test runs all
    10 000 on the HIP path and bounds the bf16 accuracy change at 0.1 %)."""
    _oracle_reads("refmodel2_attn.npz", ("test",), gray=True)


def test_oracle_reads_like_the_bench_configuration_ctc_model():
    """tests/golden/refmodel3_ctc.npz (make_refmodel3.py: RCNN(decoder="ctc") at hidden 512, 32x256, trained whole
    by run_training on the MI355X; the reference's greedy strings on 10 000 held-out lines, 99.6 % correct): the
    oracle's encode + CTC head + greedy collapse gives the reference's strings on the first 48 lines (the GPU test
    runs all 10 000 on the HIP path in fp32 and bf16)."""
    import preprocess_oracle as P
    z = np.load(os.path.join(GOLDEN, "refmodel3_ctc.npz"))
    assert float(z["test_ref_accuracy"]) >= 0.85
    with open(os.path.join(GOLDEN, "charset.txt"), encoding="utf-8") as f:
        itos = [l.rstrip("\n") for l in f if l.rstrip("\n") != ""]
    p = {}
    for k in z.files:
        if k.startswith("q::"):
            q, s = torch.from_numpy(z[k]), torch.from_numpy(z["s::" + k[3:]])
            p[k[3:]] = (q.reshape(q.shape[0], -1).float() * s.reshape(-1, 1)).reshape(q.shape)
        elif k.startswith("f::"):
            p[k[3:]] = torch.from_numpy(np.array(z[k]))
    H, W, n = int(z["img_h"]), int(z["img_w"]), 48
    widths, flat = z["test_widths"], z["test_pixels"]
    imgs, off = [], 0
    for w in widths.tolist()[:n]:
        imgs.append(np.repeat(flat[off:off + H * w].reshape(H, w)[:, :, None], 3, axis=2))
        off += H * w
    x = torch.from_numpy(np.stack([P.preprocess(im, H, W)[1] for im in imgs]))
    with torch.no_grad():
        lg = O.head(O.encode(x, p, O.Ctx(train=False)), p)
    got = ["".join(itos[t] for t in seq) for seq in O.greedy_decode(lg.numpy())]   # training/utils.py:122-150
    ref = [str(t) for t in z["test_ref_pred"][:n]]
    assert got == ref, [(g, r) for g, r in zip(got, ref) if g != r][:4]
