"""Which XCD each persistent-BiLSTM workgroup ran on (the per-launch XCC table of seq_group_local,
read back from the workspace), grouped by (direction, batch slice): shows whether the groups are
XCD-local (the fast hand-off) or split (write-through).   python tools/lstm_xcc_map.py [B T H]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rcnn-ocr_amd"))
from crnn_hip import _lib as L  # noqa: E402

B, T, H = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (256, 32, 512)
dev = "cuda"
g = torch.Generator().manual_seed(0)
xg = (torch.randn(B, T, 2, 4 * H, generator=g) * 0.5).to(dev, torch.bfloat16)
whh = (torch.randn(2, 4 * H, H, generator=g) / H ** 0.5).to(dev, torch.bfloat16)
whh_t = whh.transpose(1, 2).contiguous()
hseq = torch.zeros(B, T, 2 * H, device=dev, dtype=torch.bfloat16)
gsv = torch.zeros(2, T, B, 4 * H, device=dev, dtype=torch.bfloat16)
csv = torch.zeros(2, T, B, H, device=dev)
dg = torch.zeros(2, T, B, 4 * H, device=dev, dtype=torch.bfloat16)
ws = torch.zeros(L.lib().crnn_lstm_seq_workspace(B) // 4, dtype=torch.int32, device=dev)
tab = ((2 * (B // 16 + 1) + 1 + 63) // 64 * 256) // 4
st = L.stream_ptr()
import ctypes
for kind in ("fwd", "bwd"):
    S, U = ctypes.c_int(0), ctypes.c_int(0)
    L.lib().crnn_lstm_seq_config(B, H, int(kind == "bwd"), ctypes.byref(S), ctypes.byref(U))
    S, U = S.value, U.value
    if kind == "fwd":
        L.call("crnn_lstm_seq_fwd", xg.data_ptr(), whh.data_ptr(), hseq.data_ptr(), gsv.data_ptr(), csv.data_ptr(),
               ws.data_ptr(), B, T, H, st)
    else:
        L.call("crnn_lstm_seq_bwd", hseq.data_ptr(), whh_t.data_ptr(), gsv.data_ptr(), csv.data_ptr(), dg.data_ptr(),
               ws.data_ptr(), B, T, H, st)
    torch.cuda.synchronize()
    nsl, ng = H // U, 2 * (B // S)
    x = ws[tab: tab + ng * nsl].view(ng, nsl).cpu() - 1
    local = sum(int((r == r[0]).all()) for r in x)
    print(f"{kind} B={B} H={H} tile {S}x{U}: {local}/{ng} groups on one XCD; first groups:",
          [r.tolist() for r in x[:4]])
