import os, sys, torch
sys.path.insert(0, "rcnn-ocr_amd")
from crnn_hip import _lib as L
for (B, T, H) in [(256, 32, 512), (64, 128, 768)]:
    g = torch.Generator().manual_seed(3)
    dev = "cuda"
    whh = (torch.randn(2, 4 * H, H, generator=g) / H ** 0.5).to(dev, torch.bfloat16)
    whh_t = whh.transpose(1, 2).contiguous()
    gsv = torch.rand(2, T, B, 4 * H, generator=g).to(dev, torch.bfloat16)
    csv = (torch.randn(2, T, B, H, generator=g) * 0.5).to(dev)
    dh = (torch.randn(B, T, 2 * H, generator=g) * 0.5).to(dev, torch.bfloat16)
    st = L.stream_ptr()
    outs = []
    for mode in (0, 1, 0, 1):
        L.call("crnn_set_option", 13, mode)
        dg = torch.full((2, T, B, 4 * H), 3.0, dtype=torch.bfloat16, device=dev)
        ws = torch.zeros(L.lib().crnn_lstm_seq_workspace(B) // 4, dtype=torch.int32, device=dev)
        L.call("crnn_lstm_seq_bwd", dh.data_ptr(), whh_t.data_ptr(), gsv.data_ptr(), csv.data_ptr(), dg.data_ptr(), ws.data_ptr(), B, T, H, st)
        torch.cuda.synchronize()
        outs.append((dg.clone(), int(ws[2 * (B // 16 + 1)].item())))
    print(B, T, H, "err words", [o[1] for o in outs], "plain==sc1:", torch.equal(outs[0][0], outs[1][0]), torch.equal(outs[2][0], outs[3][0]), torch.equal(outs[0][0], outs[2][0]))
L.call("crnn_set_option", 13, 0)
