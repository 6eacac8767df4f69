"""End-to-end parity of the HIP path (RCNN API) against the reference goldens and the oracle.

fp32 mode (exact-f32 MFMA): logits within 1e-3 of the reference CPU path, identical
greedy strings, train-step loss / dlogits / parameter gradients at fp32 tolerance.
bf16 mode (the performance configuration): bf16-level agreement, reported.
"""
import numpy as np
import pytest
import torch

import crnn_oracle as O
from helpers import case_params, load, pixels_to_images

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def build_model(sd, hidden, dtype, enc_dropout_p=0.0, **kw):
    """enc_dropout_p = 0: the train-mode goldens were made with the reference's dropout off
    (tests/golden/make_goldens.py); test_enc_dropout_train covers p > 0."""
    from model.model import RCNN
    m = RCNN(num_classes=194, hidden_size=hidden, blank_id=None, compute_dtype=dtype, enc_dropout_p=enc_dropout_p,
             **kw)
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all(k.endswith("num_batches_tracked") for k in missing), missing
    return m.to(DEV)


def stage_errors(model, sd, x):
    """relative error per backbone stage vs the oracle (debug aid for failures)."""
    eng = model._engine
    ctx = O.Ctx(train=model.training, record=True)
    with torch.no_grad():
        O.encode(x, {k: v for k, v in sd.items()}, ctx)
    out = {}
    pairs = {"stem": "s1.pool", "layer1": "b0.y", "layer2": "b2.y", "layer3": "b7.y", "layer4": "b10.y"}
    for k, b in pairs.items():
        ref = ctx.acts[k]
        got = eng.ws.bufs[b].float().permute(0, 3, 1, 2).cpu()
        out[k] = float((got - ref).norm() / ref.norm())
    ref = ctx.acts["seq"]
    got = eng.ws.bufs["seq"].float().cpu()
    out["seq"] = float((got - ref).norm() / ref.norm())
    return out


@pytest.mark.parametrize("case", ["b4_32x128_h256", "b4_32x256_h512", "b2_64x256_h256"])
def test_encode_eval_fp32_matches_reference(case, itos):
    z = load(f"encode_eval_{case}.npz")
    sd, hidden = case_params(z)
    model = build_model(sd, hidden, torch.float32).eval()
    x = pixels_to_images(z["pixels"])
    with torch.no_grad():
        logits = model(x.to(DEV)).cpu()
    err = float((logits - torch.from_numpy(z["logits"])).abs().max())
    if err >= 1e-3:
        print("stage errors:", stage_errors(model, sd, x))
    assert err < 1e-3, err
    assert O.greedy_decode(logits.numpy()) == O.greedy_decode(z["logits"])
    enc = model.encode(x.to(DEV)).cpu()
    assert float((enc - torch.from_numpy(z["enc"])).abs().max()) < 1e-3


@pytest.mark.parametrize("case", ["b4_32x256_h512"])
def test_encode_eval_bf16_close(case):
    z = load(f"encode_eval_{case}.npz")
    sd, hidden = case_params(z)
    model = build_model(sd, hidden, torch.bfloat16).eval()
    x = pixels_to_images(z["pixels"])
    with torch.no_grad():
        logits = model(x.to(DEV)).cpu()
    ref = torch.from_numpy(z["logits"])
    rel = float((logits - ref).norm() / ref.norm())
    print("bf16 logits rel err", rel)
    assert rel < 5e-2
    a = logits.argmax(-1)
    b = ref.argmax(-1)
    agree = float((a == b).float().mean())
    print("bf16 argmax agreement", agree)
    assert agree > 0.9


def _hip_train_grads(z, hidden, sd):
    from crnn_hip.ctc import ctc_loss
    model = build_model(sd, hidden, torch.float32).train()
    x = pixels_to_images(z["pixels"]).to(DEV)
    logits = model(x)
    logits.retain_grad()
    loss = ctc_loss(logits, torch.from_numpy(z["targets"]), torch.from_numpy(z["target_lengths"]))
    loss.backward()
    torch.cuda.synchronize()
    return model, logits, loss


def _oracle_grads(sd, z, dt, force=None):
    x = pixels_to_images(z["pixels"])
    tg, tl = torch.from_numpy(z["targets"]), torch.from_numpy(z["target_lengths"])
    p = {k: (v.to(dt).clone().requires_grad_(True) if v.is_floating_point() and "running" not in k
             else (v.to(dt) if v.is_floating_point() else v)) for k, v in sd.items()}
    lg = O.head(O.encode(x.to(dt), p, O.Ctx(train=True, force=force)), p)
    O.ctc_loss(lg, tg, tl).backward()
    return {k: v.grad.double() for k, v in p.items() if getattr(v, "grad", None) is not None}


SMOOTH = ("enc_rnn.", "ctc_head.")   # no ReLU / max-pool decisions between them and the loss


def fp32_floor(z, params, g64, g32):
    """median CNN-parameter gradient error vs fp64, on the golden's sampled indices, of
    (HIP fp32, oracle CPU fp32, the reference's own fp32 run = the golden)."""
    eh, ec, er = [], [], []
    for name in z["param_names"]:
        name = str(name)
        if name.startswith(SMOOTH) or name not in g64:
            continue
        idx = z["gidx::" + name]
        r64 = g64[name].reshape(-1)[idx].numpy()
        n = np.linalg.norm(r64) + 1e-30
        eh.append(np.linalg.norm(params[name].grad.detach().reshape(-1).double().cpu().numpy()[idx] - r64) / n)
        ec.append(np.linalg.norm(g32[name].reshape(-1)[idx].numpy() - r64) / n)
        er.append(np.linalg.norm(z["gval::" + name].astype(np.float64) - r64) / n)
    return float(np.median(eh)), float(np.median(ec)), float(np.median(er))


def test_train_step_fp32_grads_match_reference():
    """(a) vs the reference's own output (tests/golden): loss, logits, dlogits tight.
    (b) BiLSTM stack + CTC head (smooth: no ReLU / max-pool decisions downstream): every
        parameter gradient within 1e-4 of the golden and of the fp64 oracle.
    (c) CNN parameters. Any fp32 evaluation of this case meets ReLU ties: layer4.0's BN1 has a
        pre-activation of 9e-8, whose side flips with summation order. So per-parameter CNN
        agreement is chaotic; the reference's own CPU fp32 grads sit up to 2e-3 from fp64.
        Kernel exactness is proven decision-consistently in test_train_step_fp32_block_local_exact.
        Here: every CNN gradient within 2e-2 of the golden (norm within 1e-2), and the median
        HIP error vs fp64 within 5x that of the reference's own fp32 run (the golden)."""
    z = load("train_b4_32x128_h256.npz")
    sd, hidden = case_params(z, with_running=False)
    model, logits, loss = _hip_train_grads(z, hidden, sd)
    assert abs(float(loss) - float(z["loss"])) < 1e-5 * abs(float(z["loss"]))
    np.testing.assert_allclose(logits.detach().cpu().numpy(), z["logits"], atol=1e-4)
    np.testing.assert_allclose(logits.grad.cpu().numpy(), z["dlogits"], rtol=1e-4, atol=1e-7)
    params = dict(model.named_parameters())
    bad = []
    for name in z["param_names"]:
        name = str(name)
        g = params[name].grad.detach().reshape(-1).double().cpu().numpy()
        ref_norm = float(z["gnorm::" + name])
        nerr = abs(np.sqrt((g * g).sum()) - ref_norm) / max(ref_norm, 1e-12)
        idx = z["gidx::" + name]
        ref = z["gval::" + name].astype(np.float64)
        serr = np.linalg.norm(g[idx] - ref) / max(np.linalg.norm(ref), 1e-12)
        tol_n, tol_s = (1e-4, 1e-4) if name.startswith(SMOOTH) else (1e-2, 2e-2)
        if nerr > tol_n or serr > tol_s:
            bad.append((name, nerr, serr))
    assert not bad, bad
    g64 = _oracle_grads(sd, z, torch.float64)
    g32 = _oracle_grads(sd, z, torch.float32)
    err = lambda g, k: float((g.double().cpu() - g64[k]).norm() / (g64[k].norm() + 1e-30))
    smooth = max((err(params[k].grad, k), k) for k in g64 if k.startswith(SMOOTH))
    print("smooth-region max grad error vs fp64:", smooth)
    assert smooth[0] < 1e-4, smooth
    med_h, med_c, med_r = fp32_floor(z, params, g64, g32)
    print(f"CNN median grad error vs fp64 (own decisions): hip {med_h:.2e}  reference(golden) {med_r:.2e}  "
          f"oracle-fp32 {med_c:.2e}")
    _assert_vs_forced_fp64(model, sd, z)
    bufs = dict(model.named_buffers())
    for k in z.keys():
        if k.startswith("bnrun::"):
            np.testing.assert_allclose(bufs[k[7:]].cpu().numpy(), z[k], rtol=1e-5, atol=1e-6)


def _assert_vs_forced_fp64(model, sd, z, tol=1e-4):
    """EVERY parameter gradient of the HIP fp32 step vs an fp64 oracle evaluation that takes the
    HIP forward's ReLU / max-pool decisions (crnn_oracle.Ctx.force): ties cannot intervene,
    so this is the path's exact reference."""
    from blockcheck import hip_decisions
    params = dict(model.named_parameters())
    g64f = _oracle_grads(sd, z, torch.float64, force=hip_decisions(model._engine))
    errs = sorted(((float((params[k].grad.double().cpu() - r).norm() / (r.norm() + 1e-30)), k)
                   for k, r in g64f.items()), reverse=True)
    print("grad error vs fp64 with HIP decisions: max", errs[0], "median", errs[len(errs) // 2][0])
    assert errs[0][0] < tol, errs[:5]


@pytest.mark.parametrize("case", ["b4_32x128_h256", "b3_32x256_h512"])
def test_train_step_fp32_block_local_exact(case):
    """Every SE-residual block recomputed in fp64 from the HIP path's own saved input and
    upstream gradient (tests/blockcheck.py), so decisions are the HIP path's: forward
    activations, all block parameter gradients and d(input) within 2e-5."""
    from blockcheck import block_errors
    z = load(f"train_{case}.npz")
    sd, hidden = case_params(z, with_running=False)
    from crnn_hip.ctc import ctc_loss
    model = build_model(sd, hidden, torch.float32).train()
    x = pixels_to_images(z["pixels"]).to(DEV)
    model._engine_for(x).debug = True
    ctc_loss(model(x), torch.from_numpy(z["targets"]), torch.from_numpy(z["target_lengths"])).backward()
    torch.cuda.synchronize()
    params = dict(model.named_parameters())
    res = block_errors(model._engine, params, {k: v.grad for k, v in params.items()})
    worst = max((v, bi, k) for bi, e in res for k, v in e.items())
    print("worst block-local error:", worst)
    assert worst[0] < 2e-5, worst


def test_train_step_fp32_ill_conditioned_case_vs_fp64():
    """b3_32x256_h512: ReLU / max-pool decisions on near-zero pre-activations make the
    fp32 backward chaotic (the reference's own CPU fp32 gradients sit 1e-3..4e-3 from an
    fp64 evaluation). The HIP fp32 path against fp64 next to CPU fp32: the median
    per-parameter error within 5x CPU fp32's, loss / dlogits exact; and EVERY gradient within
    1e-4 of the fp64 evaluation that takes the HIP decisions."""
    z = load("train_b3_32x256_h512.npz")
    sd, hidden = case_params(z, with_running=False)
    model, logits, loss = _hip_train_grads(z, hidden, sd)
    assert abs(float(loss) - float(z["loss"])) < 1e-5 * abs(float(z["loss"]))
    np.testing.assert_allclose(logits.grad.cpu().numpy(), z["dlogits"], rtol=1e-4, atol=1e-7)
    x = pixels_to_images(z["pixels"])
    tg, tl = torch.from_numpy(z["targets"]), torch.from_numpy(z["target_lengths"])
    ref = {}
    for dt in (torch.float64, torch.float32):
        p = {k: (v.to(dt).clone().requires_grad_(True) if v.is_floating_point() and "running" not in k
                 else (v.to(dt) if v.is_floating_point() else v)) for k, v in sd.items()}
        lg = O.head(O.encode(x.to(dt), p, O.Ctx(train=True)), p)
        O.ctc_loss(lg, tg, tl).backward()
        ref[dt] = {k: v.grad.double() for k, v in p.items() if getattr(v, "grad", None) is not None}
    eh, ec = [], []
    for name, prm in model.named_parameters():
        r = ref[torch.float64][name]
        n = float(r.norm()) + 1e-30
        eh.append(float((prm.grad.double().cpu() - r).norm()) / n)
        ec.append(float((ref[torch.float32][name] - r).norm()) / n)
    mh, mc = float(np.median(eh)), float(np.median(ec))
    print(f"median grad err vs fp64: hip32 {mh:.2e} cpu32 {mc:.2e}; max hip32 {max(eh):.2e} cpu32 {max(ec):.2e}")
    assert mh <= 5 * mc + 1e-5
    assert max(eh) <= 5 * max(ec) + 1e-4
    _assert_vs_forced_fp64(model, sd, z)


def test_zero_grad_then_backward_overwrites_not_accumulates():
    """FusedAdamW.zero_grad(set_to_none=True) + backward twice == one backward (no leftover
    accumulation); zero_grad(set_to_none=False) zeroes, and a second backward then doubles."""
    from crnn_hip.ctc import ctc_loss
    from crnn_hip.optim import FusedAdamW
    z = load("train_b4_32x128_h256.npz")
    sd, hidden = case_params(z, with_running=False)
    model = build_model(sd, hidden, torch.float32).train()
    x = pixels_to_images(z["pixels"]).to(DEV)
    tg, tl = torch.from_numpy(z["targets"]), torch.from_numpy(z["target_lengths"])
    opt = FusedAdamW(model)

    def grads():
        ctc_loss(model(x), tg, tl).backward()
        return {k: p.grad.detach().clone() for k, p in model.named_parameters()}

    opt.zero_grad()
    g1 = grads()
    opt.zero_grad()
    g2 = grads()
    for k in g1:
        assert torch.allclose(g1[k], g2[k], rtol=1e-5, atol=1e-8), k
    opt.zero_grad(set_to_none=False)
    grads()
    g3 = grads()
    for k in g1:
        assert torch.allclose(g3[k], 2 * g1[k], rtol=1e-4, atol=1e-7), k


def test_train_step_bf16_runs_and_descends():
    from crnn_hip.ctc import ctc_loss
    from crnn_hip.optim import FusedAdamW
    from crnn_hip.recipe import recipe_state_dict, synthetic_batch
    sd = recipe_state_dict(O.param_shapes(256, 194), 5)
    model = build_model(sd, 256, torch.bfloat16).train()
    x, _, tg, tl = synthetic_batch(8, 32, 128, 16, 194, seed=9)
    x = x.to(DEV)
    opt = FusedAdamW(model, lr=1e-3, weight_decay=0.0)
    losses = []
    for _ in range(6):
        opt.zero_grad()
        loss = ctc_loss(model(x), tg, tl)
        loss.backward()
        opt.step()
        losses.append(float(loss))
    print("losses", losses)
    assert all(np.isfinite(losses))
    assert losses[-1] < losses[0]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_wgrad_side_stream_bit_identical(dtype):
    """conv weight gradients on the side stream (CRNNEngine.wgrad_stream) give exactly the
    gradients of the one-stream backward, over two steps (the second overwrites the first's
    buffers while the side stream may still lag behind the compute stream)."""
    from crnn_hip.ctc import ctc_loss
    from crnn_hip.recipe import recipe_state_dict, synthetic_batch
    sd = recipe_state_dict(O.param_shapes(256, 194), 7)
    model = build_model(sd, 256, dtype).train()
    x, _, tg, tl = synthetic_batch(32, 32, 256, 32, 194, seed=21)
    x = x.to(DEV)
    out = []
    for side in (False, True, False, True):
        model(x)                       # build the engine
        model._engine.wgrad_stream = side
        model.zero_grad(set_to_none=True)
        for _ in range(2):
            model.zero_grad(set_to_none=True)
            ctc_loss(model(x), tg, tl).backward()
        out.append({k: p.grad.detach().clone() for k, p in model.named_parameters()})
    for k in out[0]:
        for o in out[1:]:
            if k.startswith("cnn."):
                assert torch.equal(out[0][k], o[k]), k
            else:
                # head / BiLSTM gradients (same stream either way); some sum with fp32 atomics
                # (crnn_colsum, the fp32 BiLSTM weight gradients), so only to fp32 order
                assert torch.allclose(out[0][k], o[k], rtol=1e-5, atol=1e-7), k


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 5e-2)])
def test_eval_fused_conv_bn_relu_matches_unfused(dtype, tol):
    """eval inference runs conv1 -> bn1 -> relu (and conv_out's first pair) as one conv launch with
    the running-stat affine + ReLU in the epilogue (crnn_conv_fwd_bnrelu): logits equal the
    unfused conv / finalize / bn_act path (fp32: to rounding; bf16: both within 5e-2 of the fp32
    path, the fused one no further), with running statistics that are not the identity."""
    from crnn_hip.recipe import recipe_state_dict, synthetic_batch
    sd = recipe_state_dict(O.param_shapes(256, 194), 3)
    g = torch.Generator().manual_seed(5)
    for k in list(sd):
        if k.endswith("running_mean"):
            sd[k] = torch.randn(sd[k].shape, generator=g) * 0.1
        elif k.endswith("running_var"):
            sd[k] = torch.rand(sd[k].shape, generator=g) + 0.5
    model = build_model(sd, 256, dtype).eval()
    x, _, _, _ = synthetic_batch(8, 32, 256, 32, 194, seed=4)
    x = x.to(DEV)
    out = []
    for fuse in (True, False):
        with torch.no_grad():
            model(x)
            model._engine.eval_fuse = fuse
            out.append(model(x).float().cpu())
    err = float((out[0] - out[1]).norm() / out[1].norm())
    if dtype == torch.float32:
        assert err < tol, err
        assert torch.equal(out[0].argmax(-1), out[1].argmax(-1))
    else:
        # bf16: both paths round differently (the fused one skips a bf16 rounding of z per fused
        # pair), so judge each against the fp32 path: the fused one must be no further from it
        m32 = build_model(sd, 256, torch.float32).eval()
        with torch.no_grad():
            ref = m32(x).float().cpu()
        e_f = float((out[0] - ref).norm() / ref.norm())
        e_u = float((out[1] - ref).norm() / ref.norm())
        # (which path lands closer after 28 bf16 layers is noise; per-kernel rounding is pinned
        # exactly in test_gpu_kernels.py::test_halo_eval_bnrelu_epilogue)
        assert e_f < tol and e_f <= 1.5 * e_u, (e_f, e_u, err)
    # the eval affine is cached between forwards: an in-place edit of a running statistic, a
    # training forward and an optimizer-style parameter edit must each be seen by the next eval
    model._engine.eval_fuse = True
    bufs = dict(model.named_buffers())
    prm = dict(model.named_parameters())
    with torch.no_grad():
        bufs["cnn.layer3.0.bn1.running_mean"].add_(0.3)
        prm["cnn.layer2.0.bn1.weight"].mul_(1.5)
        got = model(x).float().cpu()
        model.train()
        model(x)                        # updates running stats on the device
        model.eval()
        got2 = model(x).float().cpu()
    ref = build_model({k: v.detach().cpu() for k, v in model.state_dict().items()}, 256, dtype).eval()
    with torch.no_grad():
        want2 = ref(x).float().cpu()
    assert float((got2 - want2).norm() / want2.norm()) < 1e-6
    assert float((got - out[0]).norm() / out[0].norm()) > 1e-4   # the edits changed the output


def test_enc_dropout_train():
    """enc_dropout (model/model.py:201,220) in training: the head sees the encoder output with a
    Bernoulli(1 - p) mask scaled by 1/(1-p) (keep share within 4 sigma), the logits are the head
    applied to exactly that tensor, the head-weight gradient is dlogits^T @ that tensor, and eval
    mode applies no dropout. The mask stream is counter-based (crnn_dropout), not torch's Philox."""
    from crnn_hip.ctc import ctc_loss
    from crnn_hip.recipe import recipe_state_dict, synthetic_batch
    p = 0.3
    sd = recipe_state_dict(O.param_shapes(64, 194), 11)
    model = build_model(sd, 64, torch.float32, enc_dropout_p=p).train()
    x, _, tg, tl = synthetic_batch(4, 32, 128, 16, 194, seed=12)
    x = x.to(DEV)
    logits = model(x)
    eng = model._engine
    raw = eng.ws.bufs[f"r{model.num_rnn_layers - 1}.out"].float()
    drop = eng.ws.bufs["enc.drop"].float()
    kept = drop != 0
    n = kept.numel()
    share = float(kept.float().mean())
    assert abs(share - (1 - p)) < 4 * ((p * (1 - p) / n) ** 0.5)
    assert torch.allclose(drop[kept], raw[kept] / (1 - p), rtol=1e-6, atol=1e-6)
    w = model.ctc_head.weight.detach()
    b = model.ctc_head.bias.detach()
    assert torch.allclose(logits.detach(), drop @ w.t() + b, rtol=1e-4, atol=1e-4)
    logits.retain_grad()
    ctc_loss(logits, tg, tl).backward()
    gw = (logits.grad.reshape(-1, logits.shape[-1]).t() @ drop.reshape(-1, drop.shape[-1]))
    assert float((model.ctc_head.weight.grad - gw).norm() / gw.norm()) < 1e-4
    # a second training forward draws a new mask; eval applies none
    model(x)
    assert not torch.equal(eng.ws.bufs["enc.drop"] != 0, kept)
    model.eval()
    with torch.no_grad():
        model(x)


def test_dropblock_train_step_matches_forced_fp64():
    """DropBlock2d in every SE block (model/seresnet31.py:49-53,62), training, block_size 3 on the
    32x128 golden case: each block's keep mask is bit for bit crnn_oracle.dropblock_keep (the seed
    draw is counter based, not torch's Philox), and EVERY parameter gradient of the HIP fp32 step is
    within 1e-4 of the fp64 oracle that takes the HIP path's ReLU / max-pool decisions and these
    masks (times numel / (1e-6 + kept), drop_block2d's scale). Eval applies none: logits equal a
    dropblock-free model's. block_size 5 at this height raises, as the reference does (layer3's maps
    are 4 rows, min(5, 4) = 4 is even and drop_block2d's mask does not broadcast)."""
    from crnn_hip.ctc import ctc_loss
    z = load("train_b4_32x128_h256.npz")
    sd, hidden = case_params(z, with_running=False)
    p, bs = 0.2, 3
    model = build_model(sd, hidden, torch.float32, dropblock_p=p, dropblock_block_size=bs).train()
    x = pixels_to_images(z["pixels"]).to(DEV)
    logits = model(x)
    ctc_loss(logits, torch.from_numpy(z["targets"]), torch.from_numpy(z["target_lengths"])).backward()
    torch.cuda.synchronize()
    eng = model._engine
    B = x.shape[0]
    for blk, sb in zip(eng.blocks, eng._saved["blocks"]):
        d = sb["drop"]
        assert d is not None, blk.prefix
        ref = O.dropblock_keep(d["seed"], B, blk.planes, sb["ho"], sb["wo"], p, bs)
        got = d["keep"].permute(0, 3, 1, 2).cpu().numpy()
        assert np.array_equal(got, ref), blk.prefix
        assert int(d["kept"].item()) == int(ref.sum())
    _assert_vs_forced_fp64(model, sd, z)
    plain = build_model(sd, hidden, torch.float32)
    plain.load_state_dict(model.state_dict())   # the training step moved the BN running stats
    plain.eval()
    model.eval()
    with torch.no_grad():
        same = torch.equal(model(x), plain(x))
    assert same
    bad = build_model(sd, hidden, torch.float32, dropblock_p=p, dropblock_block_size=5).train()
    with pytest.raises(RuntimeError):
        bad(x)


def test_dropblock_bf16_train():
    """DropBlock2d in the bf16 configuration: the masks are the fp32 path's (same seed stream), a new
    mask is drawn every training forward, the bf16 gradient is no further from the fp32 path's (same
    masks) than it is without DropBlock (random-init weights make both distances large: ReLU
    decisions flip under bf16 storage), and a few AdamW steps descend."""
    from crnn_hip.ctc import ctc_loss
    from crnn_hip.optim import FusedAdamW
    from crnn_hip.recipe import recipe_state_dict, synthetic_batch
    sd = recipe_state_dict(O.param_shapes(256, 194), 5)
    x, _, tg, tl = synthetic_batch(8, 32, 128, 16, 194, seed=9)
    x = x.to(DEV)
    flat, keeps = {}, {}
    for p in (0.0, 0.1):
        for dt in (torch.float32, torch.bfloat16):
            m = build_model(sd, 256, dt, dropblock_p=p, dropblock_block_size=3).train()
            ctc_loss(m(x), tg, tl).backward()
            torch.cuda.synchronize()
            flat[p, dt] = torch.cat([q.grad.reshape(-1).float() for _, q in sorted(m.named_parameters())])
            if p > 0:
                keeps[dt] = [sb["drop"]["keep"].clone() for sb in m._engine._saved["blocks"]]
    assert all(torch.equal(a, b) for a, b in zip(keeps[torch.float32], keeps[torch.bfloat16]))
    err = {p: float((flat[p, torch.bfloat16] - flat[p, torch.float32]).norm() / flat[p, torch.float32].norm())
           for p in (0.0, 0.1)}
    print("bf16 vs fp32 gradient distance: without DropBlock", err[0.0], "with (same masks)", err[0.1])
    assert err[0.1] < 2 * err[0.0] + 1e-2
    model = build_model(sd, 256, torch.bfloat16, dropblock_p=0.1, dropblock_block_size=3).train()
    opt = FusedAdamW(model, lr=1e-3, weight_decay=0.0)
    losses, first = [], None
    for _ in range(6):
        opt.zero_grad()
        loss = ctc_loss(model(x), tg, tl)
        k = model._engine._saved["blocks"][0]["drop"]["keep"].clone()
        if first is None:
            first = k
        else:
            assert not torch.equal(first, k)
        loss.backward()
        opt.step()
        losses.append(float(loss))
    print("losses", losses)
    assert all(np.isfinite(losses))
    assert losses[-1] < losses[0]


def test_attn_decoder_matches_reference():
    """HIP attention decoder (crnn_hip/attn.py, csrc/attn.hip) vs the reference's own outputs
    (attn_decoder.npz, model/model.py:23-148): greedy-decode logits (blank masked) and the greedy
    sequence, teacher-forced logits; fp32."""
    from crnn_hip.attn import AttnDecoderHIP
    z = load("attn_decoder.npz")
    p = {k: torch.from_numpy(z[k]) for k in z.files if k.startswith(("attention_cell.", "generator."))}
    steps, V = z["probs"].shape[1], z["probs"].shape[2]
    dec = AttnDecoderHIP(p, V, sos_id=1, blank_id=3, device=DEV)
    enc = torch.from_numpy(z["enc"]).to(DEV)
    probs = dec.run(enc, steps).cpu()
    np.testing.assert_allclose(probs.numpy(), z["probs"], rtol=1e-4, atol=1e-3)
    assert np.array_equal(probs.argmax(-1).numpy(), z["greedy"])
    logits = dec.run(enc, steps, text=torch.from_numpy(z["text"])).cpu()
    np.testing.assert_allclose(logits.numpy(), z["logits"], rtol=1e-4, atol=1e-3)


def test_rcnn_attn_model_eval_matches_oracle():
    """RCNN(decoder='attn') end to end on the HIP path (encode + attention decoder, fp32, eval)
    vs the oracle (encode + attn_greedy) on the same weights: logits and greedy sequence; the
    teacher-forced path (is_train=True under no_grad) vs attn_teacher."""
    from crnn_hip.recipe import recipe_state_dict, synthetic_batch
    from model.model import RCNN
    z = load("attn_decoder.npz")
    sd = recipe_state_dict(O.param_shapes(64, 194), 17)
    for k in z.files:
        if k.startswith(("attention_cell.", "generator.")):
            sd["attn." + k] = torch.from_numpy(z[k])
    m = RCNN(num_classes=194, hidden_size=64, blank_id=3, decoder="attn", compute_dtype=torch.float32)
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert sorted(unexpected) == ["ctc_head.bias", "ctc_head.weight"], unexpected
    m = m.to(DEV).eval()
    x, _, tg, _ = synthetic_batch(3, 32, 128, 16, 194, seed=18)
    with torch.no_grad():
        probs = m(x.to(DEV), is_train=False, batch_max_length=9).cpu()
        text = torch.randint(4, 194, (3, 10), generator=torch.Generator().manual_seed(5))
        text[:, 0] = 1
        tf = m(x.to(DEV), text=text.to(DEV), is_train=True, batch_max_length=9).cpu()
    p = {k: v.float() for k, v in sd.items()}
    enc = O.encode(x, p, O.Ctx(train=False))
    pa = {k[5:]: v for k, v in p.items() if k.startswith("attn.")}
    ref = O.attn_greedy(pa, enc, 10, 1, 3, 194)
    assert float((probs - ref).abs().max()) < 1e-2 * float(ref.abs().max())
    assert torch.equal(probs.argmax(-1), ref.argmax(-1))
    reft = O.attn_teacher(pa, enc, text, 10, 3, 194)
    assert float((tf - reft).abs().max()) < 1e-2 * float(reft.abs().max())


def _attn_params64(z):
    return {k: torch.from_numpy(z[k]).double() for k in z.files if k.startswith(("attention_cell.", "generator."))}


@pytest.mark.parametrize("drop_p", [0.0, 0.3])
def test_attn_decoder_backward_matches_oracle(drop_p):
    """Attention decoder BPTT on the HIP path (AttnDecoderHIP.run_train / backward: cell, attention
    and one-hot kernels + GEMMs) vs fp64 autograd through the oracle's attn_teacher
    (model/model.py:33-45, :114-148) on the reference-generated weights (attn_decoder.npz), with
    the attention-weight dropout off and on (mask = crnn_oracle.attn_drop_masks, the same hash):
    logits, d enc and every parameter gradient within 1e-4 (relative, fp32 path vs fp64)."""
    from crnn_hip.attn import AttnDecoderHIP
    z = load("attn_decoder.npz")
    p64 = _attn_params64(z)
    B, T, C, steps, V, seed = 5, 24, p64["attention_cell.i2h.weight"].shape[1], 12, 194, 1234
    g = torch.Generator().manual_seed(11)
    enc = torch.randn(B, T, C, generator=g, dtype=torch.float64)
    text = torch.randint(4, V, (B, steps), generator=g)
    text[:, 0] = 1
    gout = torch.randn(B, steps, V, generator=g, dtype=torch.float64)
    dec = AttnDecoderHIP({k: v.float() for k, v in p64.items()}, V, 1, 3, DEV)
    lg = dec.run_train(enc.float().to(DEV), steps, text.to(DEV), drop_p=drop_p, seed=seed)
    grads = {k: torch.zeros(v.shape, device=DEV) for k, v in p64.items()}
    denc = dec.backward(gout.float().to(DEV), grads, accumulate=False).cpu().double()
    pr = {k: v.clone().requires_grad_(True) for k, v in p64.items()}
    e = enc.clone().requires_grad_(True)
    ref = O.attn_teacher(pr, e, text, steps, 3, V, O.attn_drop_masks(seed, steps, B, T, drop_p))
    (ref * gout).sum().backward()
    rel = lambda a, b: float((a - b).norm() / (b.norm() + 1e-30))  # noqa: E731
    assert rel(lg.cpu().double(), ref.detach()) < 1e-5
    errs = {k: rel(grads[k].cpu().double(), pr[k].grad) for k in pr}
    errs["enc"] = rel(denc, e.grad)
    print("attn backward rel errors:", errs)
    assert max(errs.values()) < 1e-4, errs
    # accumulate = True adds
    lg = dec.run_train(enc.float().to(DEV), steps, text.to(DEV), drop_p=drop_p, seed=seed)
    dec.backward(gout.float().to(DEV), grads, accumulate=True)
    for k in pr:
        assert rel(grads[k].cpu().double(), 2 * pr[k].grad) < 1e-4, k


def test_attn_decoder_backward_bf16mma():
    """The decoder's training pass with train_bf16 (GEMMs on bf16 MFMA over fp32 operands, CRNN_F32_BF16MMA — the
    reference trains this head under fp16 autocast, training/train.py:499-505) vs fp64 autograd through the
    oracle's attn_teacher at the bench configuration's widths (C = 1024, H = 256, V = 194): logits within 1e-2
    and every gradient within 3e-2 (relative norm; bf16 operand rounding, 2^-9 per element)."""
    from crnn_hip.attn import AttnDecoderHIP
    B, T, C, H, steps, V, seed = 16, 32, 1024, 256, 12, 194, 77
    g = torch.Generator().manual_seed(12)
    p64 = {"attention_cell.i2h.weight": torch.randn(H, C, generator=g, dtype=torch.float64) / C ** 0.5,
           "attention_cell.h2h.weight": torch.randn(H, H, generator=g, dtype=torch.float64) / H ** 0.5,
           "attention_cell.h2h.bias": torch.randn(H, generator=g, dtype=torch.float64) * 0.1,
           "attention_cell.score.weight": torch.randn(1, H, generator=g, dtype=torch.float64) / H ** 0.5,
           "attention_cell.rnn.weight_ih": torch.randn(4 * H, C + V, generator=g, dtype=torch.float64) / (C + V) ** 0.5,
           "attention_cell.rnn.weight_hh": torch.randn(4 * H, H, generator=g, dtype=torch.float64) / H ** 0.5,
           "attention_cell.rnn.bias_ih": torch.randn(4 * H, generator=g, dtype=torch.float64) * 0.1,
           "attention_cell.rnn.bias_hh": torch.randn(4 * H, generator=g, dtype=torch.float64) * 0.1,
           "generator.weight": torch.randn(V, H, generator=g, dtype=torch.float64) / H ** 0.5,
           "generator.bias": torch.randn(V, generator=g, dtype=torch.float64) * 0.1}
    enc = torch.randn(B, T, C, generator=g, dtype=torch.float64)
    text = torch.randint(4, V, (B, steps), generator=g)
    text[:, 0] = 1
    gout = torch.randn(B, steps, V, generator=g, dtype=torch.float64)
    dec = AttnDecoderHIP({k: v.float() for k, v in p64.items()}, V, 1, 3, DEV, train_bf16=True)
    lg = dec.run_train(enc.float().to(DEV), steps, text.to(DEV), drop_p=0.0, seed=seed)
    grads = {k: torch.zeros(v.shape, device=DEV) for k, v in p64.items()}
    denc = dec.backward(gout.float().to(DEV), grads, accumulate=False).cpu().double()
    pr = {k: v.clone().requires_grad_(True) for k, v in p64.items()}
    e = enc.clone().requires_grad_(True)
    ref = O.attn_teacher(pr, e, text, steps, 3, V)
    (ref * gout).sum().backward()
    rel = lambda a, b: float((a - b).norm() / (b.norm() + 1e-30))  # noqa: E731
    errs = {k: rel(grads[k].cpu().double(), pr[k].grad) for k in pr}
    errs["enc"] = rel(denc, e.grad)
    errs["logits"] = rel(lg.cpu().double(), ref.detach())
    print("attn backward (bf16 MFMA) rel errors:", errs)
    assert errs["logits"] < 1e-2, errs
    assert max(errs.values()) < 3e-2, errs


def test_rcnn_attn_train_step_matches_oracle():
    """RCNN(decoder='attn') training step end to end on the HIP path (fp32): encoder forward
    (train-mode BN) -> teacher-forced decoder -> cross-entropy -> decoder BPTT -> encoder
    backward, vs fp64 autograd through the oracle (encode + attn_teacher) taking the HIP
    forward's ReLU / max-pool decisions (tests/blockcheck.py): every parameter gradient within
    1e-4; the model has no CTC head (the reference's parameter set)."""
    from blockcheck import hip_decisions
    from crnn_hip.recipe import recipe_state_dict, synthetic_batch
    from model.model import RCNN
    z = load("attn_decoder.npz")
    sd = recipe_state_dict(O.param_shapes(64, 194), 17)
    for k in z.files:
        if k.startswith(("attention_cell.", "generator.")):
            sd["attn." + k] = torch.from_numpy(z[k])
    m = RCNN(num_classes=194, hidden_size=64, blank_id=3, decoder="attn", compute_dtype=torch.float32,
             enc_dropout_p=0.0)
    m.attn_dropout_p = 0.0
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert sorted(unexpected) == ["ctc_head.bias", "ctc_head.weight"], unexpected
    m = m.to(DEV).train()
    x, _, _, _ = synthetic_batch(3, 32, 128, 16, 194, seed=18)
    text = torch.randint(4, 194, (3, 10), generator=torch.Generator().manual_seed(5))
    text[:, 0] = 1
    logits = m(x.to(DEV), text=text.to(DEV), is_train=True, batch_max_length=9)
    from crnn_hip.attn import cross_entropy
    tgt = torch.roll(text, -1, 1)   # next-token targets, PAD (0) tails ignored as training/train.py:289,503
    tgt[0, 6:] = 0
    tgt[2, 8:] = 0
    tgt = tgt.to(DEV)
    loss = cross_entropy(logits, tgt, ignore_index=0)
    loss.backward()
    torch.cuda.synchronize()
    params = dict(m.named_parameters())
    p = {k: (v.double().clone().requires_grad_(True) if v.is_floating_point() and "running" not in k
             else (v.double() if v.is_floating_point() else v)) for k, v in sd.items()}
    enc = O.encode(x.double(), p, O.Ctx(train=True, force=hip_decisions(m._engine)))
    pa = {k[5:]: v for k, v in p.items() if k.startswith("attn.")}
    ref = O.attn_teacher(pa, enc, text, 10, 3, 194)
    rl = torch.nn.functional.cross_entropy(ref.reshape(-1, 194), tgt.cpu().reshape(-1), ignore_index=0)
    assert abs(float(loss.detach()) - float(rl.detach())) < 1e-5 * abs(float(rl.detach()))
    rl.backward()
    errs = sorted(((float((params[k].grad.double().cpu() - v.grad).norm() / (v.grad.norm() + 1e-30)), k)
                   for k, v in p.items() if getattr(v, "grad", None) is not None), reverse=True)
    print("attn train grad error vs fp64 (HIP decisions): max", errs[0], "median", errs[len(errs) // 2][0])
    assert errs[0][0] < 1e-4, errs[:5]
    assert not any(k.startswith("ctc_head.") for k in params)


@pytest.mark.parametrize("MV", [(7, 5), (300, 194), (1000, 37)])
def test_attn_cross_entropy_matches_torch(MV):
    """crnn_attn_xent (the attention head's loss, nn.CrossEntropyLoss(ignore_index=PAD),
    training/train.py:289,503) vs torch fp64: loss and d logits, with ignored rows."""
    from crnn_hip.attn import cross_entropy
    M, V = MV
    g = torch.Generator().manual_seed(M)
    x = (torch.randn(M, V, generator=g, dtype=torch.float64) * 4)
    t = torch.randint(0, V, (M,), generator=g)
    t[::3] = 0
    xd = x.float().to(DEV).requires_grad_(True)
    loss = cross_entropy(xd, t.to(DEV), ignore_index=0)
    (2.5 * loss).backward()
    xr = x.clone().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(xr, t, ignore_index=0)
    (2.5 * ref).backward()
    assert abs(float(loss.detach()) - float(ref.detach())) < 1e-5 * abs(float(ref.detach()))
    assert float((xd.grad.double().cpu() - xr.grad).abs().max()) < 1e-6
