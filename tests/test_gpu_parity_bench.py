"""Parity at the BENCHMARKED kernel selection (VERDICT r02 "what's weak" 1, "next" 1-2).

The bench runs bf16 at B=256 (train, configs[2]) and B=256 inference (configs[1]); at those sizes
the persistent BiLSTM sweeps (bf16, B % 16 == 0), the 256-row LDS-DMA conv GEMMs (M*Co >= 256*256*128
for the deep layers, which needs B >= 128 at 32x256), the halo stem kernels and, in eval, the fused
conv+BN+ReLU(+pool) epilogues and the greedy-decode kernel run — none of which the B <= 8 golden
tests reach. Here the HIP path runs exactly that selection and is compared with the fp32 oracle
(oracle/crnn_oracle.py, itself pinned to the reference's goldens) on the same seeded inputs.

The error bar is principled, not a fixed tolerance: the same oracle evaluated with bf16 storage
(bf16 weights, and every tensor the HIP path keeps in bf16 between kernels rounded to bf16 —
crnn_oracle.Ctx.store) is the bf16 model of the computation. The HIP path must be no further from
fp32 than that model is (logit error, frame argmax agreement, greedy-string agreement), up to a
factor for the independent rounding noise. configs[4] (4 x 768 BiLSTM, 32x1024) runs end to end in
fp32 (logits within 1e-3 of the oracle, identical greedy strings) and bf16 (against the bar), and the
engine's BiLSTM stack reproduces the reference's own 4 x 768 stack golden (bilstm_stack.npz).
"""
import numpy as np
import pytest
import torch

import crnn_oracle as O
from crnn_hip.recipe import recipe_state_dict, synthetic_batch
from helpers import load

pytestmark = pytest.mark.gpu
DEV = "cuda"
C = 194
HEAD_GAIN = 6.0   # as the reference-generated eval goldens (tests/golden/make_goldens.py): logit margins
                  # large enough that a greedy string is a meaningful target


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.set_num_threads(min(16, torch.get_num_threads()))


def bf16(t):
    return t.to(torch.bfloat16).to(t.dtype)


def bf16_weights(sd):
    """the tensors the HIP engine packs to bf16 (engine.pack): conv, LSTM, BiLSTM-linear and head
    weights; BN / SE parameters and all biases stay fp32"""
    out = {}
    for k, v in sd.items():
        rnd = v.is_floating_point() and (
            (k.startswith("cnn.") and k.endswith(".weight") and v.dim() == 4)
            or ".rnn.weight_" in k or k.endswith(".linear.weight") or k == "ctc_head.weight")
        out[k] = bf16(v) if rnd else v
    return out


def oracle_logits(sd, x, train, layers=2, store=None, grads=False, targets=None):
    """oracle logits [B,T,C] (fp32); store=bf16 -> the bf16-storage model. grads: also the CTC loss,
    d loss / d logits and every parameter gradient (store rounds the backward's stored gradients too)"""
    p = bf16_weights(sd) if store is not None else dict(sd)
    st = store
    if grads and store is not None:
        class _R(torch.autograd.Function):
            @staticmethod
            def forward(ctx, t):
                return bf16(t)

            @staticmethod
            def backward(ctx, g):
                return bf16(g)
        st = _R.apply
    if grads:
        p = {k: (v.clone().requires_grad_(True) if v.is_floating_point() and "running" not in k else v)
             for k, v in p.items()}
    ctx = O.Ctx(train=train, store=st)
    with torch.set_grad_enabled(grads):
        lg = O.head(O.encode(x, p, ctx, layers), p)
        if not grads:
            return lg
        lg.retain_grad()
        loss = O.ctc_loss(lg, *targets)
        loss.backward()
    g = {k: v.grad for k, v in p.items() if getattr(v, "grad", None) is not None}
    return lg.detach(), float(loss.detach()), lg.grad, g


def rel(a, b):
    return float((a.double() - b.double()).norm() / (b.double().norm() + 1e-30))


def hip_model(sd, hidden, dtype, layers=2):
    from model.model import RCNN
    m = RCNN(num_classes=C, hidden_size=hidden, blank_id=None, compute_dtype=dtype, enc_dropout_p=0.0,
             num_rnn_layers=layers)
    m.load_state_dict(sd, strict=False)
    return m.to(DEV)


def agreement(lg, ref):
    """(frame argmax agreement, greedy-string agreement) of logits lg vs ref ([B,T,C])"""
    a, b = lg.argmax(-1), ref.argmax(-1)
    frames = float((a == b).float().mean())
    sa, sb = O.greedy_decode(lg.numpy()), O.greedy_decode(ref.numpy())
    return frames, float(np.mean([x == y for x, y in zip(sa, sb)]))


def assert_within_bar(name, hip, emu, ref):
    """HIP bf16 vs the fp32 oracle, no further than the bf16-storage model (x1.5 for independent
    rounding noise, plus one frame / one string of slack for the agreement rates)"""
    e_h, e_e = rel(hip, ref), rel(emu, ref)
    f_h, s_h = agreement(hip, ref)
    f_e, s_e = agreement(emu, ref)
    B, T = ref.shape[:2]
    print(f"{name}: logits rel err hip {e_h:.3e} vs bf16-model {e_e:.3e}; frame argmax agreement hip {f_h:.4f} "
          f"vs {f_e:.4f}; greedy strings hip {s_h:.4f} vs {s_e:.4f}")
    assert e_h <= 1.5 * e_e + 1e-4, (e_h, e_e)
    assert 1 - f_h <= 1.5 * (1 - f_e) + 1.0 / (B * T), (f_h, f_e)
    assert 1 - s_h <= 1.5 * (1 - s_e) + 1.0 / B, (s_h, s_e)
    return dict(err=e_h, err_model=e_e, frames=f_h, frames_model=f_e, strings=s_h, strings_model=s_e)


def _kernel_selection(eng, B, H, W):
    """the bench's kernels are the ones this batch runs (else the test would not pin them)"""
    import ctypes
    from crnn_hip import _lib as L
    assert eng._seq_ok(B), "persistent BiLSTM must run at this batch"
    bm, bn = ctypes.c_int(0), ctypes.c_int(0)
    d = eng.blocks[-1].conv2.desc(B, H // 8, W // 8)   # layer4: 4 x 32 at 32x256
    L.lib().crnn_conv_fwd_tile(L.BF16, ctypes.byref(d), ctypes.byref(bm), ctypes.byref(bn))
    assert bm.value == 256, "layer4 must run on the 256-row GEMM"


GRAD_FLOOR = 2e-3   # per-parameter slack: two bf16 roundings' worth (2^-8) of independent noise


def test_train_step_bf16_b256_bench_selection():
    """configs[2]'s train step in bf16 at the bench's B=256 (persistent BiLSTM fwd + BPTT, 256-row
    conv fwd / dgrad / wgrad, halo stem, stride-2 class-group dgrads): logits, loss and d logits
    against the fp32 oracle within the bf16-storage bar, and EVERY parameter's gradient within twice
    its own bf16-storage-model error plus GRAD_FLOOR (a single broken gradient — an SE weight, a BN
    scale — fails the test; r03 bounded only the median)."""
    from crnn_hip.ctc import ctc_loss
    B, H, W, hid = 256, 32, 256, 512
    sd = recipe_state_dict(O.param_shapes(hid, C), 41, head_gain=HEAD_GAIN)
    x, _, tg, tl = synthetic_batch(B, H, W, W // 8, C, seed=42)
    m = hip_model(sd, hid, torch.bfloat16).train()
    logits = m(x.to(DEV))
    logits.retain_grad()
    loss = ctc_loss(logits, tg, tl)
    loss.backward()
    torch.cuda.synchronize()
    _kernel_selection(m._engine, B, H, W)
    ref_lg, ref_loss, ref_dl, ref_g = oracle_logits(sd, x, True, grads=True, targets=(tg, tl))
    emu_lg, emu_loss, emu_dl, emu_g = oracle_logits(sd, x, True, store=bf16, grads=True, targets=(tg, tl))
    hip_lg = logits.detach().float().cpu()
    assert_within_bar("train B=256 logits", hip_lg, emu_lg, ref_lg)
    e_l, e_le = abs(float(loss) - ref_loss) / abs(ref_loss), abs(emu_loss - ref_loss) / abs(ref_loss)
    print(f"loss rel err hip {e_l:.2e} vs bf16-model {e_le:.2e}")
    assert e_l <= 1.5 * e_le + 1e-4
    e_d, e_de = rel(logits.grad.cpu(), ref_dl), rel(emu_dl, ref_dl)
    print(f"dlogits rel err hip {e_d:.2e} vs bf16-model {e_de:.2e}")
    assert e_d <= 1.5 * e_de + 1e-4
    params = dict(m.named_parameters())
    eh = {k: rel(params[k].grad.cpu(), r) for k, r in ref_g.items()}
    ee = {k: rel(emu_g[k], r) for k, r in ref_g.items()}
    mh, me = float(np.median(list(eh.values()))), float(np.median(list(ee.values())))
    worst = sorted(eh.items(), key=lambda kv: -kv[1])[:3]
    print(f"param grads vs fp32 oracle: median rel err hip {mh:.3e} vs bf16-model {me:.3e}; worst hip {worst}")
    ratio = sorted(((eh[k] / (2.0 * ee[k] + GRAD_FLOOR), k, eh[k], ee[k]) for k in eh), reverse=True)
    print("tightest parameters (hip / bar, hip err, model err):", [(k, round(r, 3), f"{a:.2e}", f"{b:.2e}")
                                                                  for r, k, a, b in ratio[:6]])
    bad = [(k, a, b) for r, k, a, b in ratio if r > 1.0]
    assert not bad, f"{len(bad)} parameter gradients outside 2x their bf16-model error + {GRAD_FLOOR}: {bad[:6]}"
    assert len(eh) == len(dict(m.named_parameters())), "every parameter must have an oracle gradient"


def test_inference_bf16_b256_bench_selection():
    """configs[1] exactly: B=256 eval inference in bf16 (fused conv+BN+ReLU / +max-pool epilogues,
    SE squeeze from the epilogue sums, persistent BiLSTM without saved state) + the on-device greedy
    decode kernel, against the fp32 oracle within the bf16-storage bar; running statistics from a
    calibration batch (momentum 1, as the reference-generated goldens)."""
    from crnn_hip import _lib as L
    B, H, W, hid = 256, 32, 256, 512
    sd = recipe_state_dict(O.param_shapes(hid, C), 43, head_gain=HEAD_GAIN)
    cal, _, _, _ = synthetic_batch(32, H, W, W // 8, C, seed=44)
    ctx = O.Ctx(train=True, momentum=1.0)
    with torch.no_grad():
        O.encode(cal, sd, ctx)
    sd.update(ctx.running)
    x, _, _, _ = synthetic_batch(B, H, W, W // 8, C, seed=45)
    m = hip_model(sd, hid, torch.bfloat16).eval()
    with torch.no_grad():
        m(x.to(DEV))                    # the engine forward, then the bench's decode launch on its logits
        eng = m._engine
        lg = eng.logits_padded()
        T = W // 8
        ids = torch.empty(B, T, dtype=torch.int32, device=DEV)
        lens = torch.empty(B, dtype=torch.int32, device=DEV)
        L.call("crnn_ctc_greedy", lg.data_ptr(), lg.shape[-1], B, T, C, ids.data_ptr(), lens.data_ptr(),
               L.stream_ptr())
        torch.cuda.synchronize()
    _kernel_selection(eng, B, H, W)
    hip_lg = lg[:, :, :C].float().cpu()
    ref = oracle_logits(sd, x, False)
    emu = oracle_logits(sd, x, False, store=bf16)
    assert_within_bar("inference B=256 logits", hip_lg, emu, ref)
    # the decode kernel's strings are the oracle's decode of the same (HIP) logits, exactly
    got = [r[:n] for r, n in zip(ids.cpu().tolist(), lens.cpu().tolist())]
    assert got == O.greedy_decode(hip_lg.numpy())


@pytest.mark.parametrize("dtype,B", [(torch.float32, 16), (torch.bfloat16, 16), (torch.float32, 64),
                                     (torch.bfloat16, 64)])
def test_long_line_config4_end_to_end(dtype, B):
    """BASELINE configs[4] shapes on the HIP path: 4 x 768 BiLSTM (model/model.py:151-163 stacked,
    SURVEY D4) on 32x1024 crops (T = 128), B = 16 and the configuration's own B = 64 per GPU (persistent
    BiLSTM in bf16), train-mode forward + CTC + backward. fp32: logits within 1e-3 of the oracle, identical
    greedy strings, loss to 1e-4; bf16: within the bf16-storage bar."""
    from crnn_hip.ctc import ctc_loss
    H, W, hid, nl = 32, 1024, 768, 4
    sd = recipe_state_dict(O.param_shapes(hid, C, nl), 47, head_gain=HEAD_GAIN)
    x, _, tg, tl = synthetic_batch(B, H, W, W // 8, C, seed=48)
    m = hip_model(sd, hid, dtype, nl).train()
    logits = m(x.to(DEV))
    loss = ctc_loss(logits, tg, tl)
    loss.backward()
    torch.cuda.synchronize()
    assert all(torch.isfinite(p.grad).all() for p in m.parameters())
    hip_lg = logits.detach().float().cpu()
    with torch.no_grad():
        ref = oracle_logits(sd, x, True, nl)
        ref_loss = float(O.ctc_loss(ref, tg, tl))
    if dtype == torch.float32:
        err = float((hip_lg - ref).abs().max())
        print("config4 fp32 max |logit err|", err)
        assert err < 1e-3, err
        assert O.greedy_decode(hip_lg.numpy()) == O.greedy_decode(ref.numpy())
        assert abs(float(loss) - ref_loss) < 1e-4 * abs(ref_loss)
    else:
        assert m._engine._seq_ok(B)
        with torch.no_grad():
            emu = oracle_logits(sd, x, True, nl, store=bf16)
        assert_within_bar("config4 bf16 logits", hip_lg, emu, ref)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_engine_bilstm_stack_matches_reference_golden(dtype):
    """the engine's BiLSTM stack (CRNNEngine.bilstm_stack: the kernels and workspace of the full
    forward / backward) on the reference's own 4 x 768 stack golden (tests/golden/bilstm_stack.npz,
    model/model.py:151-163 stacked 4x): output and d input within 1e-4 / 1e-3 (fp32); bf16 within
    the bf16-storage bar."""
    from model.model import RCNN
    z = load("bilstm_stack.npz")
    shapes = [(k, s) for k, s in O.param_shapes(768, C, 4) if k.startswith("enc_rnn.")]
    p = recipe_state_dict(shapes, int(z["seed"]))
    m = RCNN(num_classes=C, hidden_size=768, num_rnn_layers=4, compute_dtype=dtype, blank_id=None)
    m.load_state_dict(p, strict=False)
    m = m.to(DEV).train()
    m.flatten_parameters_()
    dummy = torch.zeros(1, 3, 32, 8, device=DEV)
    eng = m._engine_for(dummy)
    grads, _, _ = m._grad_views()
    x = torch.from_numpy(z["x"])
    proj = torch.from_numpy(z["proj"])
    y, dx = eng.bilstm_stack(x.to(DEV), proj.to(DEV), grads)
    y, dx = y.cpu(), dx.cpu()
    if dtype == torch.float32:
        np.testing.assert_allclose(y.numpy(), z["y"], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(dx.numpy(), z["dx"], rtol=1e-3, atol=1e-5)
        # one parameter gradient against oracle autograd
        pr = {k: v.clone().requires_grad_(True) for k, v in p.items()}
        yr = x
        for l in range(4):
            yr = O.bilstm(yr, pr, f"enc_rnn.{l}")
        (yr * proj).sum().backward()
        for k in ("enc_rnn.0.rnn.weight_hh_l0", "enc_rnn.3.linear.weight", "enc_rnn.2.rnn.bias_ih_l0_reverse"):
            assert rel(grads[k].cpu(), pr[k].grad) < 1e-4, k
    else:
        yref = torch.from_numpy(z["y"])
        pe = bf16_weights(p)
        ye = bf16(x)
        with torch.no_grad():
            for l in range(4):
                ye = O.bilstm(ye, pe, f"enc_rnn.{l}", bf16)
        e_h, e_e = rel(y, yref), rel(ye, yref)
        print(f"4x768 stack bf16: rel err hip {e_h:.3e} vs bf16-model {e_e:.3e}")
        assert e_h <= 1.5 * e_e + 1e-4
