import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", ".."), os.path.join(os.path.dirname(__file__), "..", "..", "f5-tts_amd")]
import torch
from f5_tts_amd.engine import op_attention
torch.manual_seed(0)
for (S, H, N) in [(1, 1, 64), (1, 1, 128), (1, 1, 192), (1, 1, 256), (2, 2, 300)]:
    Q, K, V = (torch.randn(S, H, N, 64, device="cuda") for _ in range(3))
    O = op_attention(Q, K, V, None, compute="bf16")
    ref = torch.nn.functional.scaled_dot_product_attention(Q, K, V).transpose(1, 2).reshape(S, N, H * 64)
    d = (O - ref).abs()
    print(S, H, N, "max err", d.max().item(), "err dh<32", d[..., :32].max().item(), "dh>=32", d[..., 32:64].max().item(),
          "q<32", d[:, :32].max().item(), "by 32-q block", [round(d[:, i:i+32].max().item(), 3) for i in range(0, N, 32)])
