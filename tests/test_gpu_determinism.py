"""Run-to-run determinism UNDER UNEVEN LOAD: while a side stream keeps a
CU-occupying compute kernel (hipBLASLt GEMMs through torch.matmul) and large copies running, the
same inputs must give bit-identical results launch after launch.

r01-r03's BN finalize handed its chunk partials to the last workgroup of a channel group through a
ticket with 4-byte sc1 stores / loads — a form the MI355X guide measures valid only at ONE workgroup
per CU (MI355X_MICROARCH.md, visibility table, first row); with other work sharing the CUs its
last block could read stale chunk results, and the SE blocks' BN2 sums (and everything below them)
then differed run to run (profiles/r03zw_det_load_origin.log). The finalize is now one launch with no
inter-workgroup hand-off (bn.hip fin_one_kernel), and the bias column sums no longer use fp32
atomics (linear.hip colsum_kernel).

Reference math: /root/reference/model/seresnet31.py:16-20,55-67 (SE block), model/model.py:215-227."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from crnn_hip import _lib as L
    L.lib()
    yield


class SideLoad:
    """a side stream of CU-occupying GEMMs + HBM copies, issued asynchronously before each launch
    under test so that its workgroups share the CUs with ours"""

    def __init__(self, n=2048, copies=16 << 20):
        g = torch.Generator().manual_seed(99)
        self.s = torch.cuda.Stream()
        self.a = torch.randn(n, n, generator=g).to(DEV, torch.bfloat16)
        self.b = torch.randn(n, n, generator=g).to(DEV, torch.bfloat16)
        self.c = torch.empty(n, n, device=DEV, dtype=torch.bfloat16)
        self.x = torch.empty(copies, device=DEV)
        self.y = torch.empty_like(self.x)

    def issue(self, k):
        self.s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.s):
            for i in range(k):
                torch.matmul(self.a, self.b, out=self.c)
                if i % 2 == 0:
                    self.y.copy_(self.x)


@pytest.mark.parametrize("rows,C", [(256, 256), (256, 512), (128, 512), (1024, 256), (2048, 128)])
def test_bn_finalize_bit_identical_under_load(rows, C):
    """crnn_bn_bwd_finalize / crnn_bn_finalize at the engine's row counts (SE blocks: B = 256 rows;
    conv epilogue partials: 128-1024; backward reduces: up to 1024) under a CU-occupying side stream:
    every launch bit-identical to the first, and equal to fp64 sums."""
    from crnn_hip import _lib as L
    g = torch.Generator().manual_seed(rows + C)
    pg = torch.randn(rows, C, generator=g).to(DEV)
    pgx = torch.randn(rows, C, generator=g).to(DEV)
    fws = torch.zeros((L.lib().crnn_bn_finalize_workspace(512) + 3) // 4, device=DEV)
    st = L.stream_ptr()
    load = SideLoad()
    outs = [torch.empty(C, device=DEV) for _ in range(4)]
    fwd = [torch.empty(C, device=DEV) for _ in range(4)]
    gamma, beta = torch.rand(C, generator=g).to(DEV) + 0.5, torch.randn(C, generator=g).to(DEV)
    psum = (torch.randn(rows, C, generator=g) * 64 + 3).to(DEV)
    pm2 = (torch.rand(rows, C, generator=g) * 64).to(DEV)
    ref = None
    for i in range(40):
        load.issue(3)
        L.call("crnn_bn_bwd_finalize", pg.data_ptr(), pgx.data_ptr(), rows, C, rows * 64, outs[0].data_ptr(),
               outs[1].data_ptr(), outs[2].data_ptr(), outs[3].data_ptr(), 0, fws.data_ptr(), st)
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        L.call("crnn_bn_finalize", psum.data_ptr(), pm2.data_ptr(), rows, 64, C, rows * 64, gamma.data_ptr(),
               beta.data_ptr(), rm.data_ptr(), rv.data_ptr(), 0.1, 1e-5, 1, fwd[0].data_ptr(), fwd[1].data_ptr(),
               fwd[2].data_ptr(), fwd[3].data_ptr(), fws.data_ptr(), st)
        got = [t.clone() for t in outs + fwd] + [rv.clone()]
        if ref is None:
            torch.cuda.synchronize()
            ref = got
            continue
        for k, (a, b) in enumerate(zip(got, ref)):
            assert torch.equal(a, b), f"launch {i}: output {k} differs from the first launch"
    torch.cuda.synchronize()
    assert torch.allclose(ref[1].double(), pg.double().sum(0), rtol=1e-6, atol=1e-4)
    assert torch.allclose(ref[0].double(), pgx.double().sum(0), rtol=1e-6, atol=1e-4)
    mean64 = psum.double().sum(0) / (rows * 64)
    assert torch.allclose(ref[4].double(), mean64, rtol=1e-6, atol=1e-6)


def test_colsum_bit_identical_under_load():
    """crnn_colsum (the CTC head / BiLSTM linear bias gradients) in a fixed order: bit-identical
    under load, ragged column counts included (the head's C = 194 inside a 200-column row)."""
    from crnn_hip import _lib as L
    g = torch.Generator().manual_seed(5)
    st = L.stream_ptr()
    load = SideLoad()
    for dt, M, N, ld in [(L.F32, 8192, 194, 200), (L.BF16, 8192, 512, 512), (L.F32, 1000, 37, 37)]:
        x = torch.randn(M, ld, generator=g).to(DEV, torch.float32 if dt == L.F32 else torch.bfloat16)
        out = torch.empty(N, device=DEV)
        ref = None
        for i in range(20):
            load.issue(2)
            L.call("crnn_colsum", dt, x.data_ptr(), ld, M, N, out.data_ptr(), 0, 1 if dt == L.F32 else 0, st)
            if ref is None:
                torch.cuda.synchronize()
                ref = out.clone()
                want = x[:, :N].double().sum(0)
                assert torch.allclose(ref.double().cpu(), want.cpu(), rtol=1e-5, atol=1e-3), (M, N)
            else:
                assert torch.equal(out, ref), f"{(M, N)} launch {i} differs"
        # accumulate = 1 adds onto out
        base = out.clone()
        L.call("crnn_colsum", dt, x.data_ptr(), ld, M, N, out.data_ptr(), 1, 1 if dt == L.F32 else 0, st)
        torch.cuda.synchronize()
        assert torch.allclose(out, base + ref, rtol=1e-6, atol=1e-5)


@pytest.mark.parametrize("persistent_lstm", [True, False])
def test_train_step_gradients_bit_identical_under_load(persistent_lstm):
    """The bench configuration's train step (configs[2]: B = 256, 32x256, hidden 512, bf16) repeated
    on the same batch while a side stream runs GEMMs across the CUs: every parameter gradient and the
    loss bit-identical to the first step's (no optimizer step, enc_dropout off: the inputs of every
    step are equal). The SE block chain (se_bn_bwd_reduce -> se_mlp_bwd_partials -> BN2 finalize ->
    apply -> conv2 dgrad with BN1 sums -> ...) at every layer shape runs inside."""
    import crnn_oracle as O
    from crnn_hip.ctc import ctc_loss
    from crnn_hip.recipe import recipe_state_dict, synthetic_batch
    from model.model import RCNN
    B, H, W, hid = 256, 32, 256, 512
    m = RCNN(num_classes=194, hidden_size=hid, blank_id=None, compute_dtype=torch.bfloat16, enc_dropout_p=0.0)
    m.load_state_dict(recipe_state_dict(O.param_shapes(hid, 194), 5), strict=False)
    m = m.cuda().train()
    x, _, tg, tl = synthetic_batch(B, H, W, W // 8, 194, seed=100)
    x = x.cuda()
    m(x)
    m._engine.use_seq = persistent_lstm
    load = SideLoad(n=4096)
    ref = None
    steps = 6
    for i in range(steps):
        m.zero_grad(set_to_none=True)
        load.issue(4)
        loss = ctc_loss(m(x), tg, tl)
        load.issue(12)            # the GEMMs overlap the backward
        loss.backward()
        torch.cuda.synchronize()
        g = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
        g["loss"] = loss.detach().clone().reshape(1)
        if ref is None:
            ref = g
            continue
        bad = sorted(k for k in g if not torch.equal(g[k], ref[k]))
        assert not bad, f"step {i}: {len(bad)} gradients differ from step 0, e.g. {bad[:6]}"


def _bench_model(seed, use_seq):
    import crnn_oracle as O
    from crnn_hip.recipe import recipe_state_dict, synthetic_batch
    from model.model import RCNN
    m = RCNN(num_classes=194, hidden_size=512, blank_id=None, compute_dtype=torch.bfloat16, enc_dropout_p=0.0)
    m.load_state_dict(recipe_state_dict(O.param_shapes(512, 194), seed), strict=False)
    m = m.cuda().train()
    x, _, tg, tl = synthetic_batch(256, 32, 256, 32, 194, seed=100 + seed)
    x = x.cuda()
    m(x)
    m._engine.use_seq = use_seq
    return m, x, tg, tl


def _grads(m, x, tg, tl):
    from crnn_hip.ctc import ctc_loss
    m.zero_grad(set_to_none=True)
    ctc_loss(m(x), tg, tl).backward()


@pytest.mark.parametrize("victim_seq", [False, True])
def test_train_steps_bit_identical_beside_this_librarys_step(victim_seq):
    """the side load is THIS library's own bf16 train step (a second model with its
    own engine and batch: the 256-row LDS-DMA conv GEMMs, the W-halo and halo stem convs, the BN / SE
    chain, the per-step BiLSTM) on a side stream, overlapping a victim model's step at the bench
    configuration (B = 256, 32x256, hidden 512). Both models' every gradient must be bit-identical to the
    one each computed on an idle device, over 40 overlapped iterations.
    Found with this set-up (tools/cohab_model.py, profiles/r05*_cohab*): the SE chain's small reductions
    (se_wgrad, the SE-MLP backward's dpool) returned different outputs from identical inputs in 4-25 % of
    the iterations — single low halves of packed fp32 pairs (the v_pk_add_f32 / v_pk_fma_f32 results) — and
    in none of 200 with the device code built without packed fp32 VALU ops (csrc/Makefile NOPK)."""
    vm, vx, vtg, vtl = _bench_model(5, victim_seq)
    am, ax, atg, atl = _bench_model(6, False)   # the persistent sweeps need the whole chip: one at a time
    _grads(vm, vx, vtg, vtl)
    torch.cuda.synchronize()
    vref = {k: p.grad.detach().clone() for k, p in vm.named_parameters()}
    _grads(am, ax, atg, atl)
    torch.cuda.synchronize()
    aref = {k: p.grad.detach().clone() for k, p in am.named_parameters()}
    side = torch.cuda.Stream()
    for i in range(40):
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):
                _grads(am, ax, atg, atl)
        _grads(vm, vx, vtg, vtl)
        torch.cuda.synchronize()
        vbad = [k for k, p in vm.named_parameters() if not torch.equal(p.grad, vref[k])]
        abad = [k for k, p in am.named_parameters() if not torch.equal(p.grad, aref[k])]
        assert not vbad and not abad, (f"iteration {i}: victim {len(vbad)} gradients differ {vbad[-3:]}, "
                                       f"side model {len(abad)} {abad[-3:]}")
