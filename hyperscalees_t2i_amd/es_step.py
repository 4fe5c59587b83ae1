"""One EGGROLL ES epoch (unifed_es.py:89-314 `es_step_unified`), population-batched and
member-sharded over ranks.

Per epoch, on every rank (seed = epoch, unifed_es.py:766):
  1. sampling info (bit-exact prompt ids, es_backend.py:234-263)
  2. noise factors for ALL base samples (Philox, regenerated inside perturb / update — never stored or
     communicated)                                                                     kernel (1)
  3. theta_k = theta + sigma*eps_k for the rank's members [lo, hi)                    perturb
  4. one batched Sana one-step forward + VAE decode for all local members             kernel (2) inside
  5. batched rewards -> S_local [n_local, m] (mean over repeats, unifed_es.py:208-215)
  6. all-gather S over ranks (RCCL over xGMI; the only collective)
  7. promptnorm -> finite mask -> z-score -> ranks                                    kernel (3)
  8. theta' = caps(theta + lr_scale*sigma*mean_k f_k eps_k), identical on every rank  kernel (4)
The reference evaluates members sequentially with a host sync per member; here the only host
sync is the final stats copy.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Dict, List, Optional, Tuple

import torch

from . import kernels as K
from .es import EggRollNoiser, unflatten_to_params
from .rewards import RewardModels, split_mix_weights


# ---------------------------------------------------------------------------------------
# member sharding + the one collective
# ---------------------------------------------------------------------------------------


def member_shard(pop: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous member block of `rank` (first pop % world ranks get one extra member)."""
    base, extra = divmod(pop, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    group: Any = None

    @classmethod
    def from_env(cls) -> "DistInfo":
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return cls(dist.get_rank(), dist.get_world_size(), None)
        return cls()


def all_gather_members(local: torch.Tensor, pop: int, info: DistInfo) -> torch.Tensor:
    """Gather per-member rows [n_local, ...] of every rank into [pop, ...] in member order."""
    if info.world == 1:
        return local
    import torch.distributed as dist
    shards = [member_shard(pop, r, info.world) for r in range(info.world)]
    width = max(hi - lo for lo, hi in shards)
    pad = local.new_zeros((width,) + tuple(local.shape[1:]))
    pad[: local.shape[0]] = local
    outs = [torch.empty_like(pad) for _ in range(info.world)]
    dist.all_gather(outs, pad.contiguous(), group=info.group)
    return torch.cat([outs[r][: hi - lo] for r, (lo, hi) in enumerate(shards)])


def theta_checksum(theta: torch.Tensor) -> torch.Tensor:
    """Order-independent bit checksum of fp32 theta: int64 sums of its words and of the words
    weighted by (index mod 65521 + 1), so a swap or a one-ulp change on any element shows."""
    w = theta.detach().contiguous().view(torch.int32).to(torch.int64)
    idx = torch.arange(w.numel(), device=w.device, dtype=torch.int64) % 65521 + 1
    return torch.stack([w.sum(), (w * idx).sum()])


def verify_theta_replicas(theta: torch.Tensor, info: DistInfo) -> None:
    """Debug check of SURVEY §8(e) "theta checksum allReduce": every rank runs the same fitness and
    update kernels on the same gathered S, so theta' must be bit-identical on every rank.  Two
    all-reduces (MIN, MAX) of the checksum; raises on every rank if any replica diverged."""
    if info.world == 1:
        return
    import torch.distributed as dist
    c = theta_checksum(theta)
    lo, hi = c.clone(), c.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=info.group)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=info.group)
    if not torch.equal(lo, hi):
        raise RuntimeError(f"theta replicas diverged across ranks (checksum min {lo.tolist()} != max {hi.tolist()}, "
                           f"rank {info.rank} has {c.tolist()})")


# ---------------------------------------------------------------------------------------
# S aggregation (unifed_es.py:165-215)
# ---------------------------------------------------------------------------------------

RAW_KEYS = ("combined", "clip_aesthetic", "clip_text", "no_artifacts", "pickscore")


def aggregate_member_rewards(rew: Dict[str, torch.Tensor], flat_ids: List[int], pid_to_j: Dict[int, int],
                             n_members: int, m: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-image rewards of n_members members (member-major, each member's images in flat_ids order)
    -> S [n, m] with S[k, j] = mean over member k's images of unique prompt j, in flat order
    (per_prompt_comb[pid_to_j[pid]] then torch.stack(...).mean(), unifed_es.py:175-209), and the
    raw per-member means [n, 5] over ALL its images (unifed_es.py:211-215), columns RAW_KEYS.
    The image -> prompt mapping comes from pid_to_j, not from an assumed repeat order."""
    B = len(flat_ids)
    comb = rew["combined"].float().view(n_members, B)
    groups: List[List[int]] = [[] for _ in range(m)]
    for idx, pid in enumerate(flat_ids):
        groups[pid_to_j[int(pid)]].append(idx)
    if any(not g for g in groups):
        raise ValueError("every unique prompt needs at least one image (per_prompt_comb[j] empty)")
    if len({len(g) for g in groups}) == 1:   # equal repeats (repeat_batches): one gather + mean
        idx = torch.tensor(groups, device=comb.device)                        # [m, R]
        S = comb[:, idx].mean(dim=-1)
    else:                                    # ragged: one mean per prompt
        S = torch.stack([comb[:, torch.tensor(g, device=comb.device)].mean(dim=-1) for g in groups], dim=1)
    raw = torch.stack([rew[k].float().view(n_members, B).mean(dim=1) for k in RAW_KEYS], 1)
    return S.contiguous(), raw


# ---------------------------------------------------------------------------------------
# engine
# ---------------------------------------------------------------------------------------


@dataclass
class ESConfig:
    pop_size: int = 8
    sigma: float = 1e-2
    lr_scale: float = 1e-1
    egg_rank: int = 1
    use_antithetic: bool = True
    promptnorm: bool = True
    theta_max_norm: float = 40.0
    max_step_norm: float = 0.0
    max_log_batches: int = 1
    verify_replicas: bool = False   # debug: theta checksum all-reduce after every update (N > 1)
    regenerate_noise: bool = True   # factors regenerated in perturb / update from the epoch seed (False: stored)


class ESEngine:
    def log_imgs(self, info) -> int:
        """unifed_es.py:132-135: logged images per member from the max_log_batches ARGUMENT."""
        repeats = int(len(info["flat_ids"]) // max(1, info["m"]))
        return int(max(0, min(int(self.cfg.max_log_batches), repeats))) * info["m"]

    def __init__(self, backend, rewards: RewardModels, noiser: EggRollNoiser, cfg: ESConfig, device,
                 dist_info: Optional[DistInfo] = None):
        self.backend, self.rewards, self.noiser, self.cfg = backend, rewards, noiser, cfg
        self.device = torch.device(device)
        self.dist = dist_info or DistInfo()
        self.lo, self.hi = member_shard(cfg.pop_size, self.dist.rank, self.dist.world)
        self.theta_pop = torch.empty((max(self.hi - self.lo, 1), noiser.layout.D), dtype=torch.float32,
                                     device=self.device)
        self.timings: Dict[str, float] = {}
        self.last_images: Optional[torch.Tensor] = None

    def member_passes(self) -> List[Tuple[int, int]]:
        """This rank's members in passes of the backend's pass size, as local [c0, c1) ranges.  Pass
        boundaries sit on GLOBAL member indices (multiples of members_per_pass from member 0 of the
        population), so a member is evaluated in the same batch whichever rank holds it whenever the
        shard boundaries are themselves multiples of the pass size (pop 64 over 8 ranks at 8 per pass);
        a shard that starts mid-pass evaluates the part of that global pass it holds."""
        nl = self.hi - self.lo
        per = self.backend.members_per_pass() if hasattr(self.backend, "members_per_pass") else None
        if not per:
            return [(0, nl)] if nl else []
        out, c0 = [], 0
        while c0 < nl:
            g0 = self.lo + c0
            c1 = min(nl, (g0 // per + 1) * per - self.lo)
            out.append((c0, c1))
            c0 = c1
        return out

    @torch.no_grad()
    def evaluate_local(self, theta: torch.Tensor, seed: int, guidance_scale: float, *, keep_images: bool = False,
                       mark=lambda name: None):
        """Steps 1-5: this rank's members -> (S_local [n_local, m], raw_local [n_local, 5], factors, info)."""
        nz, pop, nl = self.noiser, self.cfg.pop_size, self.hi - self.lo
        info = self.backend.step_sampling_info(seed=seed)
        m, flat_ids = info["m"], info["flat_ids"]
        R = len(flat_ids) // max(1, m)
        # (1): the epoch's factors as its seed, regenerated inside perturb / update (no factor buffer);
        # regenerate_noise=False stores them with the noise kernel first (the same bits)
        factors = (nz.epoch_noise(pop, seed=seed) if self.cfg.regenerate_noise
                   else nz.sample_factors(pop, self.device, seed=seed))
        mark("noise")
        tp = nz.perturb(theta, factors, pop, self.lo, self.hi, out=self.theta_pop[:nl])  # theta_k
        mark("perturb")
        if nl == 0:
            return torch.empty((0, m), device=self.device), torch.empty((0, 5), device=self.device), factors, info
        S_parts, raw_parts, logs = [], [], []
        feats = None
        for c0, c1 in self.member_passes():
            imgs = self.backend.generate_population(flat_ids, seed, guidance_scale, tp[c0:c1])      # (2) inside
            mark("generate")
            if feats is None:
                feats = self.rewards.prompt_features(info["unique_texts"])
            j_of_img = torch.tensor([info["pid_to_j"][p] for p in flat_ids], device=self.device).repeat(c1 - c0)
            rew = self.rewards.score(imgs, j_of_img, feats, pil_mode=getattr(self.backend, "image_pil_mode", 0))
            S_c, raw_c = aggregate_member_rewards(rew, flat_ids, info["pid_to_j"], c1 - c0, m)
            S_parts.append(S_c)
            raw_parts.append(raw_c)
            if keep_images:
                n_log = self.log_imgs(info)
                logs.append(imgs.view(c1 - c0, len(flat_ids), *imgs.shape[1:])[:, :n_log])
            del imgs
            mark("reward")
        S_local = S_parts[0] if len(S_parts) == 1 else torch.cat(S_parts)
        raw_local = raw_parts[0] if len(raw_parts) == 1 else torch.cat(raw_parts)
        if keep_images:
            self.last_images = logs[0] if len(logs) == 1 else torch.cat(logs)
        return S_local, raw_local, factors, info

    @torch.no_grad()
    def finish(self, theta: torch.Tensor, S: torch.Tensor, raw: torch.Tensor, factors, info, seed: int,
               mark=lambda name: None):
        """Steps 7-8 on the gathered S (identical on every rank)."""
        fit = K.fitness(S, self.cfg.promptnorm)                                            # (3)
        mark("fitness")
        theta_new = self.noiser.update_from_factors(theta, factors, fit, self.cfg.pop_size, self.cfg.max_step_norm,
                                                    self.cfg.theta_max_norm)               # (4)
        mark("update")
        return theta_new, self._stats(S, raw, fit, info, seed)

    @torch.no_grad()
    def step(self, theta: torch.Tensor, seed: int, guidance_scale: float, *, timing: bool = False,
             keep_images: bool = False) -> Tuple[torch.Tensor, Dict[str, Any]]:
        ev = []

        def mark(name):
            if timing:
                e = torch.cuda.Event(enable_timing=True)
                e.record()
                ev.append((name, e))

        mark("start")
        S_local, raw_local, factors, info = self.evaluate_local(theta, seed, guidance_scale, keep_images=keep_images,
                                                                mark=mark)
        m = info["m"]
        both = all_gather_members(torch.cat([S_local, raw_local], dim=1).contiguous(), self.cfg.pop_size,
                                  self.dist)                                               # (6)
        S, raw = both[:, :m].contiguous(), both[:, m:]
        mark("allgather")
        theta_new, stats = self.finish(theta, S, raw, factors, info, seed, mark=mark)
        if self.cfg.verify_replicas:
            verify_theta_replicas(theta_new, self.dist)
        if timing:
            torch.cuda.synchronize()
            self.timings = {}
            for i in range(1, len(ev)):   # a phase marked once per member pass sums over the passes
                self.timings[ev[i][0]] = self.timings.get(ev[i][0], 0.0) + ev[i - 1][1].elapsed_time(ev[i][1])
        return theta_new, stats

    def _stats(self, S, raw, fit, info, seed) -> Dict[str, Any]:
        """unifed_es.py:283-310 from one host copy."""
        h = {k: v.detach().cpu() for k, v in fit.items()}
        S_h, raw_h = S.detach().cpu(), raw.detach().cpu()
        fin = h["finite"].bool()
        m = info["m"]
        pn = self.cfg.promptnorm
        st: Dict[str, Any] = {"_fitness": h, "_S": S_h, "_raw": raw_h}
        if not fin.any():
            st["summary/mean_reward"] = float("nan")
            return st
        sc = h["scores"][fin]
        rf = raw_h[fin]
        st.update({
            "summary/mean_reward": float(sc.mean()), "summary/max_reward": float(sc.max()),
            "summary/min_reward": float(sc.min()), "std_reward": float(sc.std()) if sc.numel() > 1 else 0.0,
            "raw/combined_mean": float(rf[:, 0].mean()),
            "raw/combined_std": float(rf[:, 0].std()) if rf.shape[0] > 1 else 0.0,
            "aesthetic_mean": float(rf[:, 1].mean()), "clip_text_mean": float(rf[:, 2].mean()),
            "no_artifacts_mean": float(rf[:, 3].mean()), "pickscore_mean": float(rf[:, 4].mean()),
            "promptnorm/enabled": float(pn), "promptnorm/sigma_bar": float(h["stats"][0]) if pn else float("nan"),
            "epoch/seed": int(seed), "epoch/m_unique": int(m),
            "epoch/repeats": int(len(info["flat_ids"]) // max(1, m)),
            "epoch/logged_repeats": int(self.log_imgs(info) // max(1, m)),
            "epoch/logged_imgs_per_indiv": int(self.log_imgs(info)),
            "epoch/total_imgs_per_indiv": int(info["total_imgs_per_indiv"]),
        })
        for j in range(m):
            st[f"prompt_{j}/mu_over_pop"] = float(h["mu"][j])
            st[f"prompt_{j}/raw_mean_over_pop"] = float(S_h[:, j].mean())
            st[f"prompt_{j}/raw_std_over_pop"] = float(S_h[:, j].std()) if S_h.shape[0] > 1 else 0.0
        if fin.all():
            order = h["order"]
            st["_worst_best_median"] = (int(order[0]), int(order[-1]), int(order[len(order) // 2]))
        return st


def es_step_unified(*, theta, backend, lora_params, lora_shapes, clip_model, clip_processor=None, pick_model=None,
                    pickscore_processor=None, noiser: EggRollNoiser, mix_weights, seed: int, guidance_scale: float,
                    pop_size: int, promptnorm_enabled: bool, theta_max_norm: float, max_step_norm: float,
                    max_log_batches: int, save_dir: Optional[Path] = None, epoch: int = 0,
                    dist_info: Optional[DistInfo] = None):
    """Signature of unifed_es.py:90-111.  `clip_model` carries a RewardModels (CLIP-B/32 +
    PickScore); the processor/pick_model slots are accepted for call compatibility.
    Returns (theta_after, stats, img_dict, rewards_for_hist, unique_texts)."""
    if not isinstance(clip_model, RewardModels):
        raise TypeError("clip_model must be a hyperscalees_t2i_amd.rewards.RewardModels")
    split_mix_weights(mix_weights)           # rewards.py:247-253: length 3 or 4, else ValueError
    clip_model.mix_weights = tuple(mix_weights)
    cfg = ESConfig(pop_size=pop_size, sigma=noiser.sigma, lr_scale=noiser.lr_scale, egg_rank=noiser.rank,
                   use_antithetic=noiser.use_antithetic, promptnorm=promptnorm_enabled, theta_max_norm=theta_max_norm,
                   max_step_norm=max_step_norm, max_log_batches=max_log_batches)
    key = (pop_size, id(noiser), promptnorm_enabled, theta_max_norm, max_step_norm, max_log_batches)
    eng = getattr(backend, "_es_engine", None)
    if eng is None or getattr(backend, "_es_engine_key", None) != key:
        eng = ESEngine(backend, clip_model, noiser, cfg, theta.device, dist_info)
        backend._es_engine, backend._es_engine_key = eng, key
    want_imgs = save_dir is not None and max_log_batches > 0 and eng.dist.world == 1
    theta_after, stats = eng.step(theta, seed, guidance_scale, keep_images=want_imgs)
    img_dict = {"best": None, "median": None, "worst": None}
    if want_imgs and "_worst_best_median" in stats:
        from .pipeline import to_pil
        w, b, md = stats["_worst_best_median"]
        d = Path(save_dir) / f"epoch_{epoch:04d}"
        d.mkdir(parents=True, exist_ok=True)
        for name, k in (("best", b), ("median", md), ("worst", w)):
            strip = torch.cat(list(eng.last_images[k]), dim=-1)[None]
            img = to_pil(strip)[0]
            img.save(d / f"{name}.png")
            img_dict[name] = img
    fin = stats["_fitness"]["finite"].bool()
    rewards_for_hist = stats["_raw"][fin, 0] if fin.any() else None
    unique_texts = backend.step_sampling_info(seed)["unique_texts"]
    return theta_after, stats, img_dict, rewards_for_hist, unique_texts


def save_latest_checkpoint(*, theta, backend, lora_params, lora_shapes, save_dir: Path, meta_path: Path, epoch: int,
                           stats: Dict[str, Any], extra_meta: Dict[str, Any]):
    """es_backend.py:1025-1054: theta -> params, adapters, meta .pt with theta_latest."""
    Path(save_dir).mkdir(parents=True, exist_ok=True)
    unflatten_to_params(theta, lora_params, lora_shapes)
    backend.save_lora(Path(save_dir))
    payload = {"theta_latest": theta.detach().cpu(), "epoch": epoch,
               "summary_mean_reward": stats.get("summary/mean_reward", float("nan")), "backend": backend.name,
               **extra_meta}
    torch.save(payload, meta_path)


def load_latest_checkpoint(meta_path: Path, device=None) -> Tuple[torch.Tensor, Dict[str, Any]]:
    """Resume (new; the reference only writes checkpoints): the meta .pt written by
    save_latest_checkpoint, loaded with torch.load(weights_only=True) — nothing in the file is
    executed.  Returns (theta_latest on `device`, the rest of the payload)."""
    meta = torch.load(Path(meta_path), map_location="cpu", weights_only=True)
    theta = meta.pop("theta_latest")
    if not torch.is_tensor(theta) or theta.ndim != 1:
        raise ValueError(f"{meta_path}: theta_latest must be a 1-D tensor")
    return (theta.to(device) if device is not None else theta), meta
