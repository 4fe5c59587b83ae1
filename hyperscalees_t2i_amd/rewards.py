"""Reward contract of the reference (rewards.py:164-268), batched over all images of all local
members and kept on the GPU (no PIL round trip, no per-image model calls).

Per image the reference computes (compute_all_rewards, called once per image at
unifed_es.py:175-191):
  clip_aesthetic = (cos(img, AESTHETIC_TEXT) + 1) / 2           CLIP ViT-B/32
  clip_text      = (cos(img, prompt) + 1) / 2                   CLIP ViT-B/32
  no_artifacts   = 1 - (cos(img, NEGATIVE_TEXT) + 1) / 2        CLIP ViT-B/32
  pickscore      = exp(logit_scale) * cos(text_emb, img_emb)    PickScore_v1 (CLIP ViT-H/14)
  combined       = w_aes*aes + w_txt*txt + w_noart*noart + w_pick*pick
Images reach the reward models as the reference's PIL path would deliver them: VAE output ->
(x/2+0.5).clamp(0,1) -> *255 rounded to uint8 (PixArtImageProcessor.postprocess) -> CLIP fast
processor (PIL backend): Pillow's fixed-point bicubic resize of the shortest edge to 224 -> center
crop -> /255 -> CLIP mean/std normalisation.  Done here as tensor ops on the device, bit-exact
with Pillow's resampling (tests/test_checkpoint_rewards.py).

Weights: the hub checkpoints (openai/clip-vit-base-patch32, yuvalkirstain/PickScore_v1) are not
available offline, so both models are built from their published configs with seeded random
init (architecture- and FLOP-exact, scores meaningless); tokenisation is a deterministic
synthetic word hash (no CLIP BPE vocab offline).  Reward-value parity is therefore UNPINNED;
the reward *contract* (dict keys, per-image scalars, combination, S aggregation) is exact.
"""
from __future__ import annotations

import ctypes
import zlib
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

AESTHETIC_TEXT = "a high quality, professional, beautiful, aesthetically pleasing image"
NEGATIVE_TEXT = "blurry, low resolution, noisy, pixelated, washed out colors, oversaturated "
CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)

CLIP_B32 = dict(
    text_config=dict(hidden_size=512, intermediate_size=2048, num_hidden_layers=12, num_attention_heads=8,
                     max_position_embeddings=77, vocab_size=49408, hidden_act="quick_gelu"),
    vision_config=dict(hidden_size=768, intermediate_size=3072, num_hidden_layers=12, num_attention_heads=12,
                       image_size=224, patch_size=32, hidden_act="quick_gelu"),
    projection_dim=512)
CLIP_H14 = dict(  # laion/CLIP-ViT-H-14-laion2B-s32B-b79K == PickScore_v1 architecture
    text_config=dict(hidden_size=1024, intermediate_size=4096, num_hidden_layers=24, num_attention_heads=16,
                     max_position_embeddings=77, vocab_size=49408, hidden_act="gelu"),
    vision_config=dict(hidden_size=1280, intermediate_size=5120, num_hidden_layers=32, num_attention_heads=16,
                       image_size=224, patch_size=14, hidden_act="gelu"),
    projection_dim=1024)
CLIP_TINY = dict(  # test-size config
    text_config=dict(hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
                     max_position_embeddings=77, vocab_size=49408, hidden_act="quick_gelu"),
    vision_config=dict(hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
                       image_size=224, patch_size=32, hidden_act="quick_gelu"),
    projection_dim=32)


def synthetic_tokenize(texts: Sequence[str], max_length: int = 77) -> Tuple[torch.Tensor, torch.Tensor]:
    """Deterministic stand-in for the CLIP BPE tokenizer: BOS + crc32(word) ids + EOS, padded."""
    ids = torch.zeros(len(texts), max_length, dtype=torch.long)
    mask = torch.zeros(len(texts), max_length, dtype=torch.long)
    for i, t in enumerate(texts):
        toks = [49406] + [1 + zlib.crc32(w.encode()) % 49000 for w in t.lower().split()][: max_length - 2] + [49407]
        ids[i, :len(toks)] = torch.tensor(toks)
        mask[i, :len(toks)] = 1
        ids[i, len(toks):] = 49407
    return ids, mask


def postprocess_uint8(images: torch.Tensor) -> torch.Tensor:
    """PixArtImageProcessor.postprocess(output_type='pil') pixel values, as float tensor of ints."""
    return torch.round((images.float() / 2 + 0.5).clamp(0, 1) * 255.0)


_PIL_PRECISION_BITS = 32 - 8 - 2  # Pillow's Resample.c fixed point for 8-bit images
_COEF_CACHE: Dict[tuple, torch.Tensor] = {}


def _pil_bicubic_coeffs(in_size: int, out_size: int) -> np.ndarray:
    """Pillow's precompute_coeffs + normalize_coeffs_8bpc for the BICUBIC filter (a = -0.5):
    the integer (22-bit fixed-point) weights as a dense [out_size, in_size] matrix."""
    def bicubic(x):
        a = -0.5
        x = abs(x)
        if x < 1.0:
            return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
        if x < 2.0:
            return (((x - 5) * x + 8) * x - 4) * a
        return 0.0
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 2.0 * filterscale
    mat = np.zeros((out_size, in_size), np.float64)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = [bicubic((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = sum(w)
        for x in range(xmax):
            k = w[x] / ww if ww != 0.0 else w[x]
            mat[xx, xmin + x] = int(-0.5 + k * (1 << _PIL_PRECISION_BITS)) if k < 0 else \
                int(0.5 + k * (1 << _PIL_PRECISION_BITS))
    return mat


def _pil_pass(x: torch.Tensor, coeffs: torch.Tensor) -> torch.Tensor:
    """One separable 8-bit pass over the last dim: clip8(sum(in * k_int) + 2^21) >> 22.  fp64
    holds every partial sum exactly (|sum| < 2^36), so the dense matmul is the integer result."""
    acc = torch.matmul(x, coeffs.t()) + float(1 << (_PIL_PRECISION_BITS - 1))
    return torch.floor(acc / float(1 << _PIL_PRECISION_BITS)).clamp_(0.0, 255.0)


def pil_bicubic_resize(u8: torch.Tensor, out_h: int, out_w: int) -> torch.Tensor:
    """PIL Image.resize((out_w, out_h), BICUBIC) of uint8-valued images [n, c, H, W] (any float dtype),
    bit-exact: horizontal pass first, each pass rounded and clipped to 8 bits (Resample.c)."""
    n, c, h, w = u8.shape
    x = u8.to(torch.float64)
    for dim_in, dim_out, horiz in ((w, out_w, True), (h, out_h, False)):
        if dim_in == dim_out:
            continue
        key = (dim_in, dim_out, str(x.device))
        cf = _COEF_CACHE.get(key)
        if cf is None:
            cf = _COEF_CACHE[key] = torch.from_numpy(_pil_bicubic_coeffs(dim_in, dim_out)).to(x.device)
        x = _pil_pass(x, cf) if horiz else _pil_pass(x.transpose(-1, -2), cf).transpose(-1, -2)
    return x


def clip_preprocess(u8: torch.Tensor, size: int = 224) -> torch.Tensor:
    """transformers CLIPImageProcessor (PIL backend, rewards.py:86-90 / 133-147) on uint8-valued
    images [n,3,H,W] -> normalized [n,3,224,224]: BICUBIC resize of the short edge to `size`
    (bit-exact Pillow resampling), center crop, /255, CLIP mean/std."""
    n, c, h, w = u8.shape
    # transformers get_resize_output_image_size(default_to_square=False): the short edge becomes
    # `size`, the long edge int(size * long / short) (truncation)
    if h <= w:
        nh, nw = size, int(size * w / h)
    else:
        nh, nw = int(size * h / w), size
    x = pil_bicubic_resize(u8, nh, nw).float()
    top, left = (nh - size) // 2, (nw - size) // 2
    x = x[:, :, top:top + size, left:left + size] / 255.0
    mean = torch.tensor(CLIP_MEAN, device=x.device).view(1, 3, 1, 1)
    std = torch.tensor(CLIP_STD, device=x.device).view(1, 3, 1, 1)
    return (x - mean) / std


_TAP_CACHE: Dict[tuple, Tuple[torch.Tensor, int]] = {}


def pil_tap_table(in_size: int, out_size: int, device) -> Tuple[torch.Tensor, int]:
    """Pillow's bicubic 8-bit taps as the int32 table eggroll_clip_preprocess reads: [out][1 + KT] =
    {first input index, KT taps} (identity taps when the size is unchanged: Pillow skips that pass)."""
    key = (in_size, out_size, str(device))
    if key not in _TAP_CACHE:
        mat = (np.eye(in_size) * float(1 << _PIL_PRECISION_BITS) if in_size == out_size
               else _pil_bicubic_coeffs(in_size, out_size))
        nz = [np.nonzero(r)[0] for r in mat]
        KT = max(int(z[-1] - z[0] + 1) for z in nz)
        tab = np.zeros((out_size, 1 + KT), np.int64)
        for o, z in enumerate(nz):
            first = int(min(z[0], in_size - KT))          # keep every tap index inside the row
            tab[o, 0] = first
            tab[o, 1 + z[0] - first: 1 + z[-1] - first + 1] = mat[o, z[0]:z[-1] + 1]
        _TAP_CACHE[key] = (torch.from_numpy(tab.astype(np.int32)).to(device), KT)
    return _TAP_CACHE[key]


def clip_pixels(images: torch.Tensor, pil_mode: int = 0, size: int = 224) -> torch.Tensor:
    """Decoder images [n,3,H,W] (bf16, any strides) -> CLIP pixel values [n,3,size,size] fp32 on the
    HIP path (eggroll_clip_preprocess): the uint8 PIL conversion of the backend (pil_mode 0: PixArt
    postprocess, rounding; 1: the VAR PIL path, fp16 + truncation), Pillow's bicubic resize of the
    short edge, center crop, CLIP normalisation — bitwise equal to
    clip_preprocess(postprocess_uint8(images)) / clip_preprocess(quantize_uint8_var(images))."""
    from . import _lib
    from .kernels import _stream
    if images.device.type != "cuda" or images.dtype != torch.bfloat16:
        raise _lib.EggrollError("clip_pixels: expected a bf16 ROCm tensor (no CPU fallback)")
    n, c, h, w = images.shape
    if c != 3:
        raise ValueError(f"clip_pixels: expected 3 channels, got {c}")
    nh, nw = (size, int(size * w / h)) if h <= w else (int(size * h / w), size)
    tw, ktw = pil_tap_table(w, nw, images.device)
    th, kth = pil_tap_table(h, nh, images.device)
    out = torch.empty((n, 3, size, size), dtype=torch.float32, device=images.device)
    tmp = torch.empty((max(n * 3 * h * size, 1),), dtype=torch.uint8, device=images.device)
    mean = (ctypes.c_float * 3)(*CLIP_MEAN)
    std = (ctypes.c_float * 3)(*CLIP_STD)
    sn, sc, sh, sw = images.stride()
    _lib.call("eggroll_clip_preprocess", images.data_ptr(), n, h, w, sn, sc, sh, sw, int(pil_mode), tw.data_ptr(),
              th.data_ptr(), ktw, kth, nw, nh, size, ctypes.cast(mean, ctypes.c_void_p),
              ctypes.cast(std, ctypes.c_void_p), tmp.data_ptr(), out.data_ptr(), _stream(images.device))
    return out


def build_clip(cfg: dict, device, seed: int, dtype=torch.bfloat16):
    from transformers import CLIPConfig, CLIPModel
    torch.manual_seed(seed)
    with torch.device(device):
        model = CLIPModel(CLIPConfig(**cfg))
    return model.to(dtype).eval().requires_grad_(False)


def _image_features(model, pixels: torch.Tensor) -> torch.Tensor:
    out = model.vision_model(pixel_values=pixels.to(model.dtype))
    return model.visual_projection(out.pooler_output).float()


def _text_features(model, ids: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    out = model.text_model(input_ids=ids, attention_mask=mask)
    return model.text_projection(out.pooler_output).float()


@dataclass
class _TextOnly:
    """text_model + text_projection of a CLIPModel (what _text_features reads)."""
    text_model: object
    text_projection: object


def split_mix_weights(mix_weights) -> Tuple[float, float, float, float]:
    """rewards.py:247-253: (w_aes, w_align, w_noart) with w_pick = 0, or all four; else ValueError."""
    w = tuple(float(x) for x in mix_weights)
    if len(w) == 3:
        return w + (0.0,)
    if len(w) == 4:
        return w
    raise ValueError(f"mix_weights must have length 3 or 4, got {len(w)}")


@dataclass
class RewardModels:
    clip: object
    pick: object
    mix_weights: Tuple[float, ...] = (0.0, 0.0, 0.0, 1.0)  # unifed_es.py:360-363 defaults (length 3 or 4)
    image_batch: int = 256
    fp32_residual: bool = True     # towers carry their residual stream / norms in fp32 (clip_tower.py)
    text_graphs: bool = True       # replay the per-epoch text towers as one HIP graph per prompt count
    _towers: Optional[tuple] = None
    _text32: Optional[tuple] = None
    _tgraphs: Optional[dict] = None

    def towers(self):
        if self._towers is None or self._towers[0].fp32_residual != self.fp32_residual:
            from .clip_tower import CLIPVisionTower
            self._towers = (CLIPVisionTower(self.clip, fp32_residual=self.fp32_residual),
                            CLIPVisionTower(self.pick, fp32_residual=self.fp32_residual))
        return self._towers

    def text_models(self):
        """The text towers + projections the prompt features come from: fp32 copies (once per epoch
        for a handful of prompts, so the reference's fp32 precision costs nothing) unless the towers
        run in plain bf16."""
        if not self.fp32_residual:
            return self.clip, self.pick
        if self._text32 is None:
            import copy
            self._text32 = tuple(_TextOnly(copy.deepcopy(m.text_model).float(),
                                           copy.deepcopy(m.text_projection).float()) for m in (self.clip, self.pick))
        return self._text32

    @classmethod
    def build(cls, device, mix_weights=(0.0, 0.0, 0.0, 1.0), tiny: bool = False, seed: int = 7):
        split_mix_weights(mix_weights)
        clip = build_clip(CLIP_TINY if tiny else CLIP_B32, device, seed)
        pick = build_clip(CLIP_TINY if tiny else CLIP_H14, device, seed + 1)
        return cls(clip=clip, pick=pick, mix_weights=tuple(mix_weights))

    def _text_eager(self, ids: torch.Tensor, mask: torch.Tensor) -> Dict[str, torch.Tensor]:
        tc_model, tp_model = self.text_models()
        t_clip = _text_features(tc_model, ids, mask)
        t_clip = t_clip / t_clip.norm(dim=-1, keepdim=True).clamp_min(1e-6)   # rewards.py:100
        t_pick = _text_features(tp_model, ids[2:], mask[2:])
        t_pick = t_pick / t_pick.norm(dim=-1, keepdim=True)                   # rewards.py:153
        return {"clip_aes": t_clip[0], "clip_neg": t_clip[1], "clip_prompt": t_clip[2:], "pick_prompt": t_pick}

    def _text_graphed(self, ids: torch.Tensor, mask: torch.Tensor) -> Dict[str, torch.Tensor]:
        """The same kernels as _text_eager, captured once per prompt count into a HIP graph and replayed:
        the fp32 text towers are ~690 small launches per epoch whose host-side dispatch (not their
        7.5 ms of GPU work) set the pace.  The inputs are copied into the graph's static buffers."""
        if self._tgraphs is None:
            self._tgraphs = {}
        key = tuple(ids.shape)
        ent = self._tgraphs.get(key)
        if ent is None:
            sid, smask = ids.clone(), mask.clone()
            side = torch.cuda.Stream(device=ids.device)
            side.wait_stream(torch.cuda.current_stream(ids.device))
            with torch.cuda.stream(side):
                self._text_eager(sid, smask)   # warm-up off the capture (library handles, kernel selection)
            torch.cuda.current_stream(ids.device).wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                out = self._text_eager(sid, smask)
            ent = self._tgraphs[key] = (graph, sid, smask, out)
        graph, sid, smask, out = ent
        sid.copy_(ids)
        smask.copy_(mask)
        graph.replay()
        return {k: v.clone() for k, v in out.items()}

    @torch.no_grad()
    def prompt_features(self, prompts: Sequence[str]) -> Dict[str, torch.Tensor]:
        """Text features once per epoch (members share prompts: common random numbers)."""
        dev = next(self.clip.parameters()).device
        ids, mask = synthetic_tokenize([AESTHETIC_TEXT, NEGATIVE_TEXT] + list(prompts))
        ids, mask = ids.to(dev), mask.to(dev)
        if self.text_graphs and dev.type == "cuda":
            try:
                return self._text_graphed(ids, mask)
            except RuntimeError:   # a capture-incompatible op: run the same towers eagerly from now on
                torch.cuda.synchronize(dev)
                self.text_graphs, self._tgraphs = False, None
        return self._text_eager(ids, mask)

    @torch.no_grad()
    def score(self, images: torch.Tensor, prompt_index: torch.Tensor, feats: Dict[str, torch.Tensor],
              pil_mode: int = 0) -> Dict[str, torch.Tensor]:
        """images: decoder outputs [n,3,H,W] in [-1,1] (bf16); prompt_index [n] into feats' prompt
        rows; pil_mode: the backend's image -> PIL conversion (0 Sana: PixArt postprocess, rounding;
        1 VAR: models/VAR.py:245-259, fp16 + truncation).  Returns per-image fp32 tensors with the
        compute_all_rewards keys."""
        n = images.shape[0]
        t_clip, t_pick = self.towers()
        e_clip, e_pick = [], []
        for s in range(0, n, self.image_batch):
            px = clip_pixels(images[s:s + self.image_batch].to(torch.bfloat16), pil_mode)
            e_clip.append(t_clip(px))
            e_pick.append(t_pick(px))
        ic = torch.cat(e_clip)
        ic = ic / ic.norm(dim=-1, keepdim=True).clamp_min(1e-6)  # rewards.py:99
        ip = torch.cat(e_pick)
        ip = ip / ip.norm(dim=-1, keepdim=True)                   # rewards.py:150
        aes = (ic @ feats["clip_aes"] + 1.0) / 2.0
        txt = ((ic * feats["clip_prompt"][prompt_index]).sum(-1) + 1.0) / 2.0
        neg = (ic @ feats["clip_neg"] + 1.0) / 2.0
        noart = 1.0 - neg
        pick = self.pick.logit_scale.float().exp() * (ip * feats["pick_prompt"][prompt_index]).sum(-1)
        w_aes, w_txt, w_no, w_pick = split_mix_weights(self.mix_weights)
        comb = w_aes * aes + w_txt * txt + w_no * noart + w_pick * pick
        return {"clip_aesthetic": aes, "clip_text": txt, "no_artifacts": noart, "pickscore": pick, "combined": comb}
