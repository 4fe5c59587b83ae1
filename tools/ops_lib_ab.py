"""A/B of two or more builds of libeggroll through the package's own op wrappers (kernels.py): the
global library handle is swapped between bound builds, each op's outputs are compared bitwise with the
first build's, then timed interleaved (median of rounds, HIP events on the launch stream).  Ops: the
epoch's row norms (Sana AdaLN on the fp32 stream with fp32 modulation, C = 2240; bf16 rows, C = 2240;
DC-AE RMSNorm + bias + fp32 residual, C = 512 and 1024), resid_layernorm (CLIP towers), the Z-Image q/k
norm + RoPE and the DC-AE decoder head.
usage: python tools/ops_lib_ab.py <libA.so> <libB.so> [...]"""
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import _lib  # noqa: E402
from hyperscalees_t2i_amd import kernels as K  # noqa: E402
from es_lib_ab import bind, timed  # noqa: E402


def cases(dev, g):
    r = lambda *s, dt=torch.bfloat16, sc=1.0: (torch.randn(*s, device=dev, generator=g) * sc).to(dt)  # noqa: E731
    out = {}
    # Sana AdaLN: fp32 stream x [131072, 2240], fp32 (1 + scale) / shift per image (1024 rows each)
    x32 = r(131072, 2240, dt=torch.float32)
    ms, mh = r(128, 2240, dt=torch.float32, sc=0.1), r(128, 2240, dt=torch.float32, sc=0.1)
    out["adaln f32 131072x2240"] = lambda: K.rownorm(x32, 1e-6, layer=True, mscale=ms, mshift=mh, rows_per_group=1024)
    xb = r(131072, 2240)
    wb = r(2240, sc=0.5)
    out["rms bf16 131072x2240 +w"] = lambda: K.rownorm(xb, 1e-6, w=wb)
    for C, rows in ((512, 8 * 256 * 256), (512, 8 * 128 * 128), (1024, 8 * 128 * 128)):
        xc, wc, bc = r(rows, C), r(C, sc=0.5), r(C, sc=0.1)
        res0 = r(rows, C, dt=torch.float32)
        res = res0.clone()

        def f(xc=xc, wc=wc, bc=bc, res=res, res0=res0):
            res.copy_(res0)
            return K.rownorm(xc, 1e-5, w=wc, b=bc, res=res)
        out[f"dcae rms+res32 {rows}x{C}"] = f
        o32, sh = torch.empty_like(res0), torch.empty(rows, C, device=dev, dtype=torch.bfloat16)

        def f2(xc=xc, wc=wc, bc=bc, res0=res0, o32=o32, sh=sh):   # the product form, out of place (no copy timed)
            return K.rownorm(xc, 1e-5, w=wc, b=bc, res=res0, out=o32, shadow=sh)
        out[f"dcae rms+res32+shadow {rows}x{C}"] = f2
    # linear attention: Sana attn1 (separate q / k / v [B*N, 2240], 70 heads) and DC-AE planar [Q|K|V]
    qs, ks, vs = r(128 * 1024, 2240), r(128 * 1024, 2240), r(128 * 1024, 2240)
    out["linear_attention sana 128x1024 h70"] = lambda: K.linear_attention(qs, ks, vs, 128, 1024, 70, 32, False)
    for Bd, N, hd in ((8, 16384, 16), (8, 4096, 32), (8, 1024, 32)):
        flat = r(Bd * N, 3 * hd * 32)
        inner = hd * 32
        out[f"linear_attention dcae {Bd}x{N} h{hd}"] = (lambda flat=flat, inner=inner, Bd=Bd, N=N, hd=hd:
            K.linear_attention(flat, flat[:, inner:], flat[:, 2 * inner:], Bd, N, hd, 32, True))
    # DC-AE ResBlock conv2 + RMSNorm + residual (halo kernel, NORM epilogue): 128 ch at 1024^2, 256 ch at 512^2
    for Bc, Hc, Cc in ((8, 1024, 128), (8, 512, 256)):
        xc = r(Bc, Hc, Hc, Cc, sc=0.5)
        wpk = r(Cc, 9 * Cc, sc=(9 * Cc) ** -0.5)
        nwc, nbc, resc = r(Cc, sc=0.5), r(Cc, sc=0.1), r(Bc, Hc, Hc, Cc)
        out[f"conv3x3_rmsnorm {Bc}x{Hc}^2x{Cc}"] = (lambda xc=xc, wpk=wpk, nwc=nwc, nbc=nbc, resc=resc:
            K.conv3x3_rmsnorm_nhwc(xc, wpk, None, 1, 1e-6, nwc, nbc, resc))
    # flash attention (head dim 128): Z-Image's joint sequence (4 images x 4096+512 tokens x 30 heads) and a
    # ragged one (a partial key block, Nq not a multiple of the query tile)
    for Bf, Nf, Hf in ((4, 4608, 30), (2, 1000, 8)):
        qf, kf, vf = (r(Bf, Nf, Hf, 128, sc=0.5) for _ in range(3))
        out[f"flash_attention {Bf}x{Nf} h{Hf}"] = (lambda qf=qf, kf=kf, vf=vf:
            K.flash_attention(qf, kf, vf, 128 ** -0.5))
    # DC-AE up-blocks: 2x2 phase conv + sub-pixel interleave + bias + shortcut in one launch (the four product
    # shapes, 8 images; the 512->1024 one also on the fp32 stream with its bf16 shadow)
    from hyperscalees_t2i_amd.dcae import subpixel_phase_weights
    for Hs, Cin, Cout, f32 in ((512, 256, 128, False), (256, 512, 256, False), (128, 512, 512, False),
                               (64, 1024, 512, False), (64, 1024, 512, True)):
        xs = r(8, Hs, Hs, Cin, sc=0.5)
        w4 = subpixel_phase_weights(torch.randn(Cout, Cin, 3, 3, device=dev, generator=g) / (9 * Cin) ** 0.5)
        w4p = K.pack_conv3x3_weight(w4.to(torch.bfloat16).contiguous(memory_format=torch.channels_last), 1)
        bs = r(Cout, sc=0.1)
        if f32:
            src = r(8, Hs, Hs, Cin, dt=torch.float32)
            sh = torch.empty(8, 2 * Hs, 2 * Hs, Cout, device=dev, dtype=torch.bfloat16)
            out[f"conv2x2_subpixel f32 8x{Hs}^2 {Cin}->{Cout}"] = (lambda xs=xs, w4p=w4p, src=src, bs=bs, sh=sh:
                torch.cat([K.conv2x2_subpixel(xs, w4p, src, bias=bs, shadow=sh).flatten(), sh.float().flatten()]))
        else:
            out[f"conv2x2_subpixel 8x{Hs}^2 {Cin}->{Cout}"] = (lambda xs=xs, w4p=w4p, bs=bs:
                K.conv2x2_subpixel(xs, w4p, xs, bias=bs))
    # DC-AE multi-scale branch: 5x5 depthwise + grouped 1x1 (the three product shapes)
    for Hd, Cd in ((128, 1536), (64, 3072), (32, 3072)):
        xd = r(8, Hd, Hd, Cd, sc=0.5)
        wd = r(25, Cd, sc=0.2)
        pwd = r(Cd // 32, 32, 32, sc=1 / 6)
        out[f"~dwconv_pw5 8x{Hd}^2x{Cd}"] = lambda xd=xd, wd=wd, pwd=pwd: K.dwconv_pw_nhwc(xd, wd, pwd, 5)
    h0 = r(16 * 257, 1280, dt=torch.float32)
    h = h0.clone()
    y, w2, b2 = r(16 * 257, 1280), r(1280, sc=0.5), r(1280, sc=0.1)

    def rl():
        h.copy_(h0)
        return torch.cat([K.resid_layernorm_(h, y, w2, b2, 1e-5).float().flatten(), h.flatten()])
    out["resid_layernorm 4112x1280"] = rl
    return out


def main(paths, rounds=7, only=None):
    libs = [bind(p) for p in paths]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    res = {}
    for name, fn in cases(dev, g).items():
        if only and only not in name:
            continue
        outs = []
        for lib in libs:
            _lib._lib = lib
            outs.append(fn().clone())
        torch.cuda.synchronize()
        same = [torch.equal(outs[0], o) for o in outs[1:]]
        us = [[] for _ in libs]
        for _ in range(rounds):
            for i, lib in enumerate(libs):
                _lib._lib = lib
                us[i].append(timed(fn))
        res[name] = {"bitwise_equal_to_A": same, **{Path(p).name: round(statistics.median(u), 1)
                                                     for p, u in zip(paths, us)}}
        if name.startswith("~"):   # a numerics-changing A/B: report the largest relative difference instead
            res[name]["max_rel_diff_to_A"] = [float((o.float() - outs[0].float()).abs().max() /
                                                    outs[0].float().abs().max().clamp_min(1e-30)) for o in outs[1:]]
        print(json.dumps({name: res[name]}), flush=True)
        assert all(same) or name.startswith("~"), name
    print(json.dumps(res))


if __name__ == "__main__":
    only = next((a[7:] for a in sys.argv[1:] if a.startswith("--only=")), None)
    main([a for a in sys.argv[1:] if not a.startswith("--only=")], only=only)
