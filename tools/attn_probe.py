"""Time cross-attention formulations at the Sana shape (q [B,20,1024,112], kv [B,20,300,112])."""
import sys
import torch
import torch.nn.functional as F

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
H, N, L, d = 20, 1024, 300, 112
dev = "cuda"
q = torch.randn(B, N, H, d, device=dev, dtype=torch.bfloat16).transpose(1, 2)
k = torch.randn(B, L, H, d, device=dev, dtype=torch.bfloat16).transpose(1, 2)
v = torch.randn(B, L, H, d, device=dev, dtype=torch.bfloat16).transpose(1, 2)
mask = torch.zeros(B, 1, 1, L, device=dev, dtype=torch.bfloat16)
mask[:, :, :, 200:] = -10000.0


def t(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


flops = 4 * B * H * N * L * d
ref = F.scaled_dot_product_attention(q, k, v, attn_mask=mask)


def manual():
    s = torch.matmul(q, k.transpose(-1, -2)) * d ** -0.5 + mask
    p = torch.softmax(s.float(), dim=-1).to(torch.bfloat16)
    return torch.matmul(p, v)


def padded():
    qp, kp, vp = (F.pad(x, (0, 16)) for x in (q, k, v))
    return F.scaled_dot_product_attention(qp, kp, vp, attn_mask=mask, scale=d ** -0.5)[..., :d]


qc, kc, vc = q.contiguous(), k.contiguous(), v.contiguous()
cands = {
    "sdpa_default": lambda: F.scaled_dot_product_attention(q, k, v, attn_mask=mask),
    "sdpa_contig": lambda: F.scaled_dot_product_attention(qc, kc, vc, attn_mask=mask),
    "sdpa_nomask": lambda: F.scaled_dot_product_attention(q, k, v),
    "manual_bmm": manual,
    "pad128": padded,
}
for name, fn in cands.items():
    try:
        ms = t(fn)
        err = (fn().float() - ref.float()).abs().max().item()
        print(f"{name:14s} {ms:8.3f} ms  {flops / ms / 1e9:8.1f} TF/s  maxdiff {err:.3g}", flush=True)
    except Exception as ex:  # noqa: BLE001
        print(name, "failed", type(ex).__name__, str(ex)[:200], flush=True)
for be in ("MATH", "EFFICIENT_ATTENTION", "FLASH_ATTENTION"):
    try:
        from torch.nn.attention import SDPBackend, sdpa_kernel
        with sdpa_kernel(getattr(SDPBackend, be)):
            ms = t(lambda: F.scaled_dot_product_attention(q, k, v, attn_mask=mask if be != "FLASH_ATTENTION" else None))
        print(f"backend {be:20s} {ms:8.3f} ms  {flops / ms / 1e9:8.1f} TF/s", flush=True)
    except Exception as ex:  # noqa: BLE001
        print("backend", be, "failed", type(ex).__name__, str(ex)[:150], flush=True)
