"""A/B: DC-AE multiscale attention with branch outputs written into one buffer (current forward) vs
the concat form, interleaved in one process at the decoder's three EfficientViT shapes."""
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402
from hyperscalees_t2i_amd.dcae import MultiscaleLinearAttention  # noqa: E402
from tools.gemm_probe_util import bench  # noqa: E402


def concat_forward(m, x):
    B, H, W, C = x.shape
    qkv = F.linear(x, m.w_qkv)

    def att(br):
        flat = br.reshape(B * H * W, -1)
        return K.linear_attention(flat, flat[:, m.hd:], flat[:, 2 * m.hd:], B, H * W, m.heads, 3 * m.hd,
                                  relu_qk=True).view(B, H, W, -1)
    outs = [att(qkv)]
    for ks, wdw, wpw in zip(m.scales, m.ms_dw, m.ms_pw):
        d = K.dwconv_nhwc(qkv, wdw, None, ks, pre_silu=False, glu=False)
        g = d.view(B * H * W, 3 * m.heads, m.hd).transpose(0, 1)
        p = torch.bmm(g, wpw.transpose(1, 2)).transpose(0, 1).reshape(B, H, W, -1)
        outs.append(att(p))
    return m.norm_out(F.linear(torch.cat(outs, dim=-1), m.w_out), res=x)


dev = torch.device("cuda:0")
with torch.no_grad():
    for c, hw in ((512, 128), (1024, 64), (1024, 32)):
        m = MultiscaleLinearAttention(c).to(dev)
        for prm in m.parameters():
            prm.copy_((torch.randn_like(prm, dtype=torch.float32) * 0.05).to(prm.dtype))
        x = torch.randn(8, hw, hw, c, device=dev).to(torch.bfloat16)
        a, b = [], []
        for _ in range(5):
            a.append(bench(lambda: m(x)))
            b.append(bench(lambda: concat_forward(m, x)))
        ya, yb = m(x).float(), concat_forward(m, x).float()
        print(f"  max|diff| {(ya - yb).abs().max().item():.3g}  max|y| {yb.abs().max().item():.3g}", flush=True)
        print(f"c{c} {hw}x{hw}: buffer {min(a):.3f} ms  concat {min(b):.3f} ms", flush=True)
