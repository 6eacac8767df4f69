"""Fused optimizers (csrc/ctc.hip crnn_adam_step / crnn_sgd_step) against torch.optim on the CPU:
the reference picks Adam (its default, coupled L2 decay), AdamW or SGD by name
(training/train.py:219,292-301). Several steps with weight decay and a DP grad scale; fp32."""
import pytest
import torch

pytestmark = pytest.mark.gpu


class _DevFlat(torch.nn.Module):
    """parameters as views of one flat fp32 device buffer (RCNN.flatten_parameters_'s layout)"""

    def __init__(self, shapes, seed, device):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        ps = [torch.randn(*s, generator=g) for s in shapes]
        n = sum(p.numel() for p in ps)
        self._flat_param = torch.empty(n, device=device)
        self._flat_grad = torch.zeros(n, device=device)
        self.ps = torch.nn.ParameterList()
        off = 0
        for p in ps:
            k = p.numel()
            self._flat_param[off:off + k].copy_(p.reshape(-1))
            self.ps.append(torch.nn.Parameter(self._flat_param[off:off + k].view_as(p)))
            off += k
        self._engine = None

    def mark_params_changed(self):
        pass


SHAPES = [(37, 11), (5,), (3, 4, 9), (1001,)]   # odd sizes: the vector kernel's tail and the scalar kernel


@pytest.mark.parametrize("name,kw", [("Adam", dict(weight_decay=0.0)), ("Adam", dict(weight_decay=0.05)),
                                     ("AdamW", dict(weight_decay=0.05)), ("SGD", dict(momentum=0.9, weight_decay=1e-3)),
                                     ("SGD", dict(momentum=0.0, weight_decay=0.0))])
@pytest.mark.parametrize("grad_scale", [1.0, 0.125])
def test_fused_optimizer_matches_torch(name, kw, grad_scale):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from crnn_hip.optim import make_optimizer
    lr = 3e-3
    m = _DevFlat(SHAPES, 1, "cuda")
    ref = [torch.nn.Parameter(p.detach().cpu().clone()) for p in m.parameters()]
    opt = make_optimizer(name, m, lr=lr, **kw)
    topt = {"Adam": torch.optim.Adam, "AdamW": torch.optim.AdamW, "SGD": torch.optim.SGD}[name](ref, lr=lr, **kw)
    g = torch.Generator().manual_seed(7)
    for _ in range(5):
        grads = [torch.randn(p.shape, generator=g) for p in ref]
        for p, gr in zip(ref, grads):
            p.grad = gr * grad_scale
        topt.step()
        m._flat_grad.copy_(torch.cat([gr.reshape(-1) for gr in grads]).cuda())
        opt.step(grad_scale=grad_scale)
    torch.cuda.synchronize()
    got = m._flat_param.cpu()
    want = torch.cat([p.detach().reshape(-1) for p in ref])
    err = float((got - want).abs().max() / want.abs().max())
    assert err < 2e-6, err
    # torch-format state round trip (what save_checkpoint writes)
    sd = opt.state_dict()
    tsd = topt.state_dict()
    for i in range(len(SHAPES)):
        for k, v in tsd["state"].get(i, {}).items():   # SGD without momentum keeps no state
            if torch.is_tensor(v) and v.numel() > 1:
                assert torch.allclose(sd["state"][i][k].cpu(), v, rtol=1e-5, atol=1e-7), (i, k)
