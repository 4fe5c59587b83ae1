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

Weights (rewards.py:32-60 loads openai/clip-vit-base-patch32 and yuvalkirstain/PickScore_v1 + the
laion CLIP-ViT-H-14 processor by hub name): `RewardModels.build(clip_path=..., pickscore_path=...)`
loads LOCAL copies of those repos with transformers (`CLIPModel.from_pretrained(local_files_only)`,
the CLIP BPE tokenizer from the directory's vocab.json / merges.txt or tokenizer.json, and its
preprocessor_config.json, checked against what the device preprocessing implements).  Without
local weights (none exist in this container) `synthetic=True` builds both models from their
published configs with seeded random init (architecture- and FLOP-exact, scores meaningless) and
tokenises with a deterministic word hash; anything else raises FileNotFoundError.  Reward-value
parity is UNPINNED (no real weights here); the reward *contract* (dict keys, per-image scalars,
combination, S aggregation) is exact.
"""
from __future__ import annotations

import ctypes
import json
import zlib
from dataclasses import dataclass
from pathlib import Path
from typing import Callable, Dict, List, Optional, Sequence, Tuple

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


def clip_pixels(images: torch.Tensor, pil_mode: int = 0, size: int = 224, mean: Sequence[float] = CLIP_MEAN,
                std: Sequence[float] = CLIP_STD) -> torch.Tensor:
    """Decoder images [n,3,H,W] (bf16, any strides) -> CLIP pixel values [n,3,size,size] fp32 on the
    HIP path (eggroll_clip_preprocess): the uint8 PIL conversion of the backend (pil_mode 0: PixArt
    postprocess, rounding; 1: the VAR PIL path, fp16 + truncation; 2: Infinity's, bf16 + truncation), Pillow's bicubic resize of the
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
    mean = (ctypes.c_float * 3)(*mean)
    std = (ctypes.c_float * 3)(*std)
    sn, sc, sh, sw = images.stride()
    _lib.call("eggroll_clip_preprocess", images.data_ptr(), n, h, w, sn, sc, sh, sw, int(pil_mode), tw.data_ptr(),
              th.data_ptr(), ktw, kth, nw, nh, size, ctypes.cast(mean, ctypes.c_void_p),
              ctypes.cast(std, ctypes.c_void_p), tmp.data_ptr(), out.data_ptr(), _stream(images.device))
    return out


class ClipTokenizer:
    """The CLIP BPE tokenizer of a local model / processor directory (vocab.json + merges.txt or
    tokenizer.json), called as the reference's processors are (rewards.py:87, 131-137: truncation at
    77 tokens) but always padded to 77: the text towers are causal and read the [EOS] position, so
    padding past it does not change the features, and a fixed shape lets the text graph replay."""

    def __init__(self, path, max_length: int = 77):
        from transformers import AutoTokenizer
        p = Path(path)
        if not ((p / "vocab.json").is_file() and (p / "merges.txt").is_file()) and not (p / "tokenizer.json").is_file():
            raise FileNotFoundError(f"{p}: no CLIP tokenizer files (vocab.json + merges.txt or tokenizer.json)")
        self.tok = AutoTokenizer.from_pretrained(str(p), local_files_only=True)
        self.max_length = max_length
        self.path = str(p)

    def __call__(self, texts: Sequence[str]) -> Tuple[torch.Tensor, torch.Tensor]:
        enc = self.tok(list(texts), padding="max_length", truncation=True, max_length=self.max_length,
                       return_tensors="pt")
        return enc["input_ids"].long(), enc["attention_mask"].long()


@dataclass(frozen=True)
class PixelSpec:
    """What eggroll_clip_preprocess does for one reward model: short edge -> size (Pillow bicubic),
    center crop size x size, /255, (x - mean) / std."""
    size: int = 224
    mean: Tuple[float, float, float] = CLIP_MEAN
    std: Tuple[float, float, float] = CLIP_STD


def pixel_spec_from_processor(path) -> PixelSpec:
    """A CLIPImageProcessor preprocessor_config.json -> PixelSpec; NotImplementedError for anything
    the device preprocessing does not restate (it is bit-exact for exactly this pipeline)."""
    p = Path(path) / "preprocessor_config.json"
    if not p.is_file():
        raise FileNotFoundError(f"{p} not found")
    c = json.loads(p.read_text())
    size = c.get("size", {})
    short = size.get("shortest_edge") if isinstance(size, dict) else size
    crop = c.get("crop_size", short)
    crop = (crop.get("height"), crop.get("width")) if isinstance(crop, dict) else (crop, crop)
    ok = (c.get("do_resize", True) and c.get("do_center_crop", True) and c.get("do_rescale", True)
          and c.get("do_normalize", True) and int(c.get("resample", 3)) == 3 and short is not None
          and crop == (short, short) and abs(float(c.get("rescale_factor", 1 / 255)) - 1 / 255) < 1e-12)
    if not ok:
        raise NotImplementedError(f"{p}: only the CLIP pipeline (bicubic short-edge resize, square center crop "
                                  f"of the same size, /255, mean/std) is implemented on the device")
    return PixelSpec(int(short), tuple(float(x) for x in c.get("image_mean", CLIP_MEAN)),
                     tuple(float(x) for x in c.get("image_std", CLIP_STD)))


def load_clip(path, device, dtype=torch.bfloat16):
    """A local transformers CLIPModel directory (openai/clip-vit-base-patch32, yuvalkirstain/PickScore_v1
    layouts) -> (model in `dtype`, fp32 _TextOnly copy of its text tower taken BEFORE the cast)."""
    import copy
    from transformers import CLIPModel
    p = Path(path)
    if not (p / "config.json").is_file():
        raise FileNotFoundError(f"{p}: not a local CLIPModel directory (config.json missing; no hub downloads)")
    m32 = CLIPModel.from_pretrained(str(p), local_files_only=True, dtype=torch.float32)
    text32 = _TextOnly(copy.deepcopy(m32.text_model).to(device).eval().requires_grad_(False),
                       copy.deepcopy(m32.text_projection).to(device).eval().requires_grad_(False))
    return m32.to(device=device, dtype=dtype).eval().requires_grad_(False), text32


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
    clip_tok: Optional[Callable] = None   # texts -> (ids, mask); None: synthetic_tokenize (synthetic models)
    pick_tok: Optional[Callable] = None
    clip_px: PixelSpec = PixelSpec()
    pick_px: PixelSpec = PixelSpec()
    source: str = "synthetic"
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
        run in plain bf16.  Loaded checkpoints keep the fp32 copies taken before the bf16 cast."""
        if not self.fp32_residual:
            return self.clip, self.pick
        if self._text32 is None:
            import copy
            self._text32 = tuple(_TextOnly(copy.deepcopy(m.text_model).float(),
                                           copy.deepcopy(m.text_projection).float()) for m in (self.clip, self.pick))
        return self._text32

    @classmethod
    def build(cls, device, mix_weights=(0.0, 0.0, 0.0, 1.0), tiny: bool = False, seed: int = 7,
              clip_path: Optional[str] = None, pickscore_path: Optional[str] = None,
              pickscore_processor_path: Optional[str] = None, synthetic: bool = False):
        """rewards.py:32-60.  clip_path / pickscore_path: local copies of openai/clip-vit-base-patch32 and
        yuvalkirstain/PickScore_v1 (CLIPModel directories); pickscore_processor_path: the local
        laion/CLIP-ViT-H-14-laion2B-s32B-b79K processor (tokenizer + preprocessor_config) the reference
        pairs with PickScore — default: the PickScore directory's own files, else the CLIP-B/32
        tokenizer (the same BPE vocabulary).  Without local weights, synthetic=True (or tiny=True, the
        test-size config) builds seeded random towers; otherwise FileNotFoundError."""
        split_mix_weights(mix_weights)
        if clip_path is not None or pickscore_path is not None:
            if clip_path is None or pickscore_path is None:
                raise ValueError("RewardModels.build: pass both clip_path and pickscore_path")
            clip, t_clip = load_clip(clip_path, device)
            pick, t_pick = load_clip(pickscore_path, device)
            clip_tok = ClipTokenizer(clip_path)
            proc = pickscore_processor_path or pickscore_path
            try:
                pick_tok = ClipTokenizer(proc)
            except FileNotFoundError:
                if pickscore_processor_path is not None:
                    raise
                pick_tok = clip_tok
            pick_px_dir = proc if (Path(proc) / "preprocessor_config.json").is_file() else clip_path
            rm = cls(clip=clip, pick=pick, mix_weights=tuple(mix_weights), clip_tok=clip_tok, pick_tok=pick_tok,
                     clip_px=pixel_spec_from_processor(clip_path), pick_px=pixel_spec_from_processor(pick_px_dir),
                     source=f"local({clip_path}, {pickscore_path})")
            rm._text32 = (t_clip, t_pick)
            return rm
        if not (synthetic or tiny):
            raise FileNotFoundError("RewardModels.build: no local CLIP / PickScore weights given (clip_path, "
                                    "pickscore_path; no hub downloads offline) — pass synthetic=True for seeded "
                                    "random towers")
        clip = build_clip(CLIP_TINY if tiny else CLIP_B32, device, seed)
        pick = build_clip(CLIP_TINY if tiny else CLIP_H14, device, seed + 1)
        return cls(clip=clip, pick=pick, mix_weights=tuple(mix_weights), source=f"synthetic(seed={seed})")

    def tokenize(self, prompts: Sequence[str]):
        """(clip ids, clip mask) of [AESTHETIC, NEGATIVE, *prompts] and (pick ids, pick mask) of prompts."""
        texts = [AESTHETIC_TEXT, NEGATIVE_TEXT] + list(prompts)
        if self.clip_tok is None:
            ids, mask = synthetic_tokenize(texts)
            return ids, mask, ids[2:], mask[2:]
        ids_c, mask_c = self.clip_tok(texts)
        ids_p, mask_p = self.pick_tok(list(prompts))
        return ids_c, mask_c, ids_p, mask_p

    def _text_eager(self, ids_c, mask_c, ids_p, mask_p) -> Dict[str, torch.Tensor]:
        tc_model, tp_model = self.text_models()
        t_clip = _text_features(tc_model, ids_c, mask_c)
        t_clip = t_clip / t_clip.norm(dim=-1, keepdim=True).clamp_min(1e-6)   # rewards.py:100
        t_pick = _text_features(tp_model, ids_p, mask_p)
        t_pick = t_pick / t_pick.norm(dim=-1, keepdim=True)                   # rewards.py:153
        return {"clip_aes": t_clip[0], "clip_neg": t_clip[1], "clip_prompt": t_clip[2:], "pick_prompt": t_pick}

    def _text_graphed(self, *toks) -> Dict[str, torch.Tensor]:
        """The same kernels as _text_eager, captured once per (token shapes, tower precision) into a HIP
        graph and replayed: the fp32 text towers are ~690 small launches per epoch whose host-side
        dispatch (not their 7.5 ms of GPU work) set the pace.  The inputs are copied into the graph's
        static buffers.  The key includes fp32_residual: a graph captured on the fp32 text towers must
        not be replayed after a switch to the bf16 ones."""
        if self._tgraphs is None:
            self._tgraphs = {}
        key = (tuple(tuple(t.shape) for t in toks), bool(self.fp32_residual))
        ent = self._tgraphs.get(key)
        dev = toks[0].device
        if ent is None:
            static = [t.clone() for t in toks]
            side = torch.cuda.Stream(device=dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                self._text_eager(*static)   # warm-up off the capture (library handles, kernel selection)
            torch.cuda.current_stream(dev).wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                out = self._text_eager(*static)
            ent = self._tgraphs[key] = (graph, static, out)
        graph, static, out = ent
        for dst, src in zip(static, toks):
            dst.copy_(src)
        graph.replay()
        return {k: v.clone() for k, v in out.items()}

    @torch.no_grad()
    def prompt_features(self, prompts: Sequence[str]) -> Dict[str, torch.Tensor]:
        """Text features once per epoch (members share prompts: common random numbers)."""
        dev = next(self.clip.parameters()).device
        toks = [t.to(dev) for t in self.tokenize(prompts)]
        if self.text_graphs and dev.type == "cuda":
            try:
                return self._text_graphed(*toks)
            except RuntimeError:   # a capture-incompatible op: run the same towers eagerly from now on
                torch.cuda.synchronize(dev)
                self.text_graphs, self._tgraphs = False, None
        return self._text_eager(*toks)

    @torch.no_grad()
    def score(self, images: torch.Tensor, prompt_index: torch.Tensor, feats: Dict[str, torch.Tensor],
              pil_mode: int = 0) -> Dict[str, torch.Tensor]:
        """images: decoder outputs [n,3,H,W] in [-1,1] (bf16); prompt_index [n] into feats' prompt
        rows; pil_mode: the backend's image -> PIL conversion (0 Sana: PixArt postprocess, rounding;
        1 VAR: models/VAR.py:245-259, fp16 + truncation).  Returns per-image fp32 tensors with the
        compute_all_rewards keys."""
        n = images.shape[0]
        t_clip, t_pick = self.towers()
        same_px = self.clip_px == self.pick_px
        e_clip, e_pick = [], []
        for s in range(0, n, self.image_batch):
            im = images[s:s + self.image_batch].to(torch.bfloat16)
            px = clip_pixels(im, pil_mode, self.clip_px.size, self.clip_px.mean, self.clip_px.std)
            e_clip.append(t_clip(px))
            if not same_px:
                px = clip_pixels(im, pil_mode, self.pick_px.size, self.pick_px.mean, self.pick_px.std)
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
