"""Window-attention fwd+bwd at the C3 shape through the library in MMNI_LIB; saves the table,
q/k/v gradients to the given .pt file (precision comparisons between kernel variants)."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_neuroimage_amd import functional as MF

out_path = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
dev = torch.device("cuda:0")
S, C, heads = 96, 12, 6
geom = MF.WindowGeometry(B, (S, S, S), (6, 6, 6), (3, 3, 3))
g = torch.Generator(device=dev).manual_seed(0)
qkv = torch.randn(geom.tokens, 3 * C, device=dev, generator=g).requires_grad_(True)
table = (torch.randn(geom.table_rows, heads, device=dev, generator=g) * 0.02).requires_grad_(True)
dy = torch.randn(geom.tokens, C, device=dev, generator=g)
out = MF.window_attention_self(qkv, table, geom, heads)
out.backward(dy)
torch.save(dict(dtable=table.grad.cpu(), dqkv=qkv.grad.cpu(), out=out.detach().cpu()), out_path)
print("saved", out_path)
