"""Histogram gradient-boosted trees on torch tensors (the engine behind ``XGBoostEstimator``).

The reference delegates to xgboost-ray (``python/raydp/xgboost/estimator.py:54-81``: an
``XGBoostTrainer`` whose workers run XGBoost's ``hist`` method and all-reduce gradient
histograms over Rabit). XGBoost is not installed here, so this module implements the same
algorithm natively:

* features are quantised once into ``max_bin`` quantile bins (bin 0 = missing), cut points
  agreed across workers from an all-gathered sample;
* trees grow level-wise to ``max_depth``; each level builds one (node, feature, bin) histogram
  of (gradient, hessian) in fixed point (int32 per row, power-of-two scale per tree agreed across
  workers; int64 sums, so histograms are exact, order-independent and identical on CPU and GPU)
  -- one launch of the gfx950 kernel ``csrc/hip/gbdt_hist.hip`` on a GPU (LDS-privatised 64-bit
  integer atomics), one ``index_add_`` on the CPU -- all-reduces it
  (``torch.distributed`` – RCCL on MI355X, gloo on CPU) exactly like Rabit's histogram
  all-reduce, and evaluates every split with XGBoost's gain
  ``G_L²/(H_L+λ) + G_R²/(H_R+λ) − G²/(H+λ)`` including the learned default direction for
  missing values, ``min_child_weight`` and ``gamma`` pruning;
* leaves get ``−η·G/(H+λ)`` (clipped by ``max_delta_step``); prediction walks all trees in a
  vectorised loop (``x < split_cond`` goes left, XGBoost's convention).

Supported objectives: ``reg:squarederror``, ``reg:logistic``, ``binary:logistic``,
``binary:logitraw``, ``count:poisson``, ``multi:softmax``, ``multi:softprob``.
"""
import json
import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

DEFAULTS = {"eta": 0.3, "max_depth": 6, "lambda": 1.0, "alpha": 0.0, "gamma": 0.0, "min_child_weight": 1.0,
            "max_bin": 256, "objective": "reg:squarederror", "subsample": 1.0, "colsample_bytree": 1.0,
            "max_delta_step": 0.0, "num_class": 1, "seed": 0, "base_score": None}
_ALIASES = {"learning_rate": "eta", "reg_lambda": "lambda", "reg_alpha": "alpha", "min_split_loss": "gamma"}


def normalize_params(params: Optional[Dict]) -> Dict:
    p = dict(DEFAULTS)
    for k, v in (params or {}).items():
        p[_ALIASES.get(k, k)] = v
    if p["objective"].startswith("multi:") and int(p["num_class"]) < 2:
        raise ValueError("multi-class objectives need num_class >= 2")
    if not 2 <= int(p["max_bin"]) <= 32000:
        raise ValueError(f"max_bin must be in [2, 32000] (bins are stored as int16), got {p['max_bin']}")
    return p


class DMatrix:
    """Feature matrix + label (subset of ``xgboost.DMatrix``)."""

    def __init__(self, data, label=None, weight=None, feature_names: Optional[Sequence[str]] = None,
                 missing: float = float("nan")):
        import pandas as pd
        if isinstance(data, pd.DataFrame):
            feature_names = feature_names or [str(c) for c in data.columns]
            data = data.to_numpy(dtype=np.float32, na_value=np.nan)
        x = torch.as_tensor(np.asarray(data, dtype=np.float32))
        if x.dim() == 1:
            x = x[:, None]
        if not math.isnan(missing):
            x = torch.where(x == missing, torch.full_like(x, float("nan")), x)
        self.data = x
        self.label = None if label is None else torch.as_tensor(np.asarray(label, dtype=np.float32)).reshape(-1)
        self.weight = None if weight is None else torch.as_tensor(np.asarray(weight, dtype=np.float32)).reshape(-1)
        self.feature_names = list(feature_names) if feature_names else [f"f{i}" for i in range(x.shape[1])]

    def num_row(self):
        return self.data.shape[0]

    def num_col(self):
        return self.data.shape[1]

    def get_label(self):
        return None if self.label is None else self.label.numpy()


# --------------------------------------------------------------------------- objectives ----
def _grad_hess(obj: str, margin: torch.Tensor, y: torch.Tensor, p: Dict):
    if obj == "reg:squarederror":
        return margin - y, torch.ones_like(margin)
    if obj in ("reg:logistic", "binary:logistic", "binary:logitraw"):
        pr = torch.sigmoid(margin)
        return pr - y, torch.clamp(pr * (1 - pr), min=1e-16)
    if obj == "count:poisson":
        mds = float(p["max_delta_step"]) or 0.7
        return torch.exp(margin) - y, torch.exp(margin + mds)
    if obj.startswith("multi:"):
        k = int(p["num_class"])
        pr = torch.softmax(margin, dim=1)
        oh = torch.nn.functional.one_hot(y.long(), k).to(pr.dtype)
        return pr - oh, torch.clamp(2.0 * pr * (1 - pr), min=1e-16)
    raise ValueError(f"unsupported objective {obj}")


def _transform(obj: str, margin: torch.Tensor) -> torch.Tensor:
    if obj in ("reg:logistic", "binary:logistic"):
        return torch.sigmoid(margin)
    if obj == "count:poisson":
        return torch.exp(margin)
    if obj == "multi:softprob":
        return torch.softmax(margin, dim=1)
    if obj == "multi:softmax":
        return margin.argmax(dim=1).to(margin.dtype)
    return margin


def _base_margin(obj: str, y: torch.Tensor, base_score, world) -> float:
    if obj.startswith("multi:"):
        return 0.0
    if base_score is None:
        s = torch.tensor([float(y.sum()), float(y.numel())], dtype=torch.float64)
        world.allreduce(s)
        base_score = float(s[0] / max(float(s[1]), 1.0))
        if obj in ("reg:logistic", "binary:logistic", "binary:logitraw"):
            base_score = min(max(base_score, 1e-6), 1 - 1e-6)
        if obj == "count:poisson":
            base_score = max(base_score, 1e-6)
    if obj in ("reg:logistic", "binary:logistic", "binary:logitraw"):
        return math.log(base_score / (1 - base_score))
    if obj == "count:poisson":
        return math.log(base_score)
    return float(base_score)


def eval_metric(name: str, obj: str, margin: torch.Tensor, y: torch.Tensor, world) -> float:
    """Globally reduced metric (sum/count all-reduced across workers)."""
    pred = _transform(obj if obj != "multi:softmax" else "multi:softprob", margin)
    if name == "rmse":
        s = ((pred - y) ** 2).sum()
    elif name == "mae":
        s = (pred - y).abs().sum()
    elif name == "logloss":
        pr = pred.clamp(1e-7, 1 - 1e-7)
        s = -(y * pr.log() + (1 - y) * (1 - pr).log()).sum()
    elif name == "error":
        s = ((pred > 0.5).to(y.dtype) != y).sum()
    elif name == "mlogloss":
        s = -pred.clamp_min(1e-7).log().gather(1, y.long()[:, None]).sum()
    elif name == "merror":
        s = (pred.argmax(1) != y.long()).sum()
    elif name == "poisson-nloglik":
        s = (pred - y * pred.clamp_min(1e-16).log() + torch.lgamma(y + 1)).sum()
    else:
        raise ValueError(f"unsupported eval_metric {name}")
    t = torch.tensor([float(s), float(y.shape[0])], dtype=torch.float64)
    world.allreduce(t)
    v = float(t[0] / max(float(t[1]), 1.0))
    return math.sqrt(v) if name == "rmse" else v


def default_metric(obj: str) -> str:
    return {"reg:squarederror": "rmse", "reg:logistic": "rmse", "binary:logistic": "logloss",
            "binary:logitraw": "logloss", "count:poisson": "poisson-nloglik", "multi:softmax": "mlogloss",
            "multi:softprob": "mlogloss"}[obj]


# ------------------------------------------------------------------------- collectives ----
class World:
    """All-reduce / all-gather over ``torch.distributed`` when a process group is up."""

    def __init__(self):
        import torch.distributed as dist
        self.dist = dist if dist.is_available() and dist.is_initialized() else None
        self.size = self.dist.get_world_size() if self.dist else 1

    def allreduce(self, t: torch.Tensor, op: str = "sum"):
        if self.dist is not None and self.size > 1:
            rop = self.dist.ReduceOp.MAX if op == "max" else self.dist.ReduceOp.SUM
            dev = self._comm_device(t)
            if dev != t.device:
                c = t.to(dev)
                self.dist.all_reduce(c, op=rop)
                t.copy_(c.to(t.device))
            else:
                self.dist.all_reduce(t, op=rop)
        return t

    def _comm_device(self, t: torch.Tensor) -> torch.device:
        """RCCL (backend "nccl") only moves device tensors: stage CPU tensors through the
        rank's current GPU; gloo keeps them where they are."""
        if self.dist.get_backend() == "nccl" and t.device.type != "cuda":
            return torch.device("cuda", torch.cuda.current_device())
        return t.device

    def allgather_rows(self, t: torch.Tensor) -> torch.Tensor:
        if self.dist is None or self.size == 1:
            return t
        home = t.device
        dev = self._comm_device(t)
        n = torch.tensor([t.shape[0]], dtype=torch.int64, device=dev)
        ns = [torch.zeros_like(n) for _ in range(self.size)]
        self.dist.all_gather(ns, n)
        counts = [int(x) for x in torch.cat(ns).cpu()]
        m = max(counts)
        pad = torch.full((m, t.shape[1]), float("nan"), dtype=t.dtype, device=dev)
        pad[:t.shape[0]] = t.to(dev)
        outs = [torch.empty_like(pad) for _ in range(self.size)]
        self.dist.all_gather(outs, pad)
        return torch.cat([o[:k] for o, k in zip(outs, counts)]).to(home)


# ---------------------------------------------------------------------------- binning ----
def compute_cuts(x: torch.Tensor, max_bin: int, world: World, sample: int = 200_000, seed: int = 0,
                 device: Optional[torch.device] = None) -> List[torch.Tensor]:
    """Per-feature cut points from (all-gathered) quantiles; identical on every worker.

    One column-wise sort of the sample (on ``device`` when given, e.g. the GPU) serves every
    feature: distinct-value counts come from the sorted columns' steps, quantiles from linear
    interpolation between order statistics (``torch.quantile``'s default), NaNs sort last.
    """
    g = torch.Generator().manual_seed(seed)
    xs = x if x.shape[0] <= sample else x[torch.randperm(x.shape[0], generator=g)[:sample]]
    xs = world.allgather_rows(xs.float().cpu())
    if xs.shape[1] == 0:
        return []
    srt = torch.sort(xs.to(device or "cpu").double(), dim=0).values          # NaN last
    m = (~torch.isnan(srt)).sum(0)                                             # non-NaN rows per feature
    step = (srt[1:] != srt[:-1]) & ~torch.isnan(srt[1:])
    distinct = torch.where(m > 0, 1 + step.sum(0), torch.zeros_like(m))
    qs = torch.linspace(0, 1, max_bin - 1, dtype=torch.float64, device=srt.device)[1:-1]
    posq = qs[:, None] * (m.clamp_min(1) - 1).double()[None, :]               # (Q, F)
    lo = posq.floor().long()
    hi = posq.ceil().long()
    a_lo, a_hi = srt.gather(0, lo), srt.gather(0, hi)
    quant = a_lo + (a_hi - a_lo) * (posq - lo.double())
    last = srt.gather(0, (m.clamp_min(1) - 1)[None, :])[0]                     # per-feature max
    srt, quant, m, distinct, last = (t.cpu() for t in (srt, quant, m, distinct, last))
    cuts = []
    for f in range(xs.shape[1]):
        if int(m[f]) == 0:
            cuts.append(torch.empty(0))
            continue
        top = last[f:f + 1]
        pad = top + torch.clamp(top.abs() * 1e-6, min=1e-6)
        if int(distinct[f]) <= max_bin - 2:
            # all distinct values: cut between neighbours so every value gets its own bin
            u = torch.unique_consecutive(srt[:int(m[f]), f])
            c = (u[1:] + u[:-1]) / 2 if u.numel() > 1 else u[:0]
        else:
            c = torch.unique(quant[:, f])
        cuts.append(torch.cat([c, pad]).float())
    return cuts


def bin_matrix(x: torch.Tensor, cuts: List[torch.Tensor]) -> torch.Tensor:
    """uint8/int16 bins: 0 = missing, 1 + #cuts <= x otherwise."""
    n, f = x.shape
    out = torch.empty((n, f), dtype=torch.int16, device=x.device)
    for j in range(f):
        col = x[:, j]
        c = cuts[j].to(x.device)
        b = torch.searchsorted(c, col.contiguous(), right=True) + 1
        out[:, j] = torch.where(torch.isnan(col), torch.zeros_like(b), b).to(torch.int16)
    return out


# ------------------------------------------------------------------------------- trees ----
class Tree:
    """Flat arrays; node 0 is the root. ``feature < 0`` marks a leaf holding ``value``."""

    def __init__(self):
        self.feature: List[int] = []
        self.cond: List[float] = []
        self.left: List[int] = []
        self.right: List[int] = []
        self.default_left: List[bool] = []
        self.value: List[float] = []
        self.gain: List[float] = []
        self.cover: List[float] = []

    def add(self, value=0.0, cover=0.0) -> int:
        self.feature.append(-1)
        self.cond.append(0.0)
        self.left.append(-1)
        self.right.append(-1)
        self.default_left.append(True)
        self.value.append(value)
        self.gain.append(0.0)
        self.cover.append(cover)
        return len(self.feature) - 1

    def to_json(self) -> Dict:
        return {k: getattr(self, k) for k in ("feature", "cond", "left", "right", "default_left", "value",
                                              "gain", "cover")}

    @classmethod
    def from_json(cls, d: Dict) -> "Tree":
        t = cls()
        for k, v in d.items():
            setattr(t, k, list(v))
        return t

    def tensors(self, device):
        return (torch.tensor(self.feature, dtype=torch.long, device=device),
                torch.tensor(self.cond, dtype=torch.float32, device=device),
                torch.tensor(self.left, dtype=torch.long, device=device),
                torch.tensor(self.right, dtype=torch.long, device=device),
                torch.tensor(self.default_left, dtype=torch.bool, device=device),
                torch.tensor(self.value, dtype=torch.float32, device=device))

    def predict(self, x: torch.Tensor) -> torch.Tensor:
        feat, cond, left, right, dleft, value = self.tensors(x.device)
        node = torch.zeros(x.shape[0], dtype=torch.long, device=x.device)
        for _ in range(64):
            f = feat[node]
            active = f >= 0
            if not bool(active.any()):
                break
            v = x.gather(1, f.clamp_min(0)[:, None])[:, 0]
            go_left = torch.where(torch.isnan(v), dleft[node], v < cond[node])
            nxt = torch.where(go_left, left[node], right[node])
            node = torch.where(active, nxt, node)
        return value[node]

    def dump(self, names: Sequence[str]) -> str:
        lines = []

        def rec(i, depth):
            pad = "\t" * depth
            if self.feature[i] < 0:
                lines.append(f"{pad}{i}:leaf={self.value[i]:.6g}")
                return
            miss = self.left[i] if self.default_left[i] else self.right[i]
            lines.append(f"{pad}{i}:[{names[self.feature[i]]}<{self.cond[i]:.6g}] yes={self.left[i]},"
                         f"no={self.right[i]},missing={miss}")
            rec(self.left[i], depth + 1)
            rec(self.right[i], depth + 1)
        rec(0, 0)
        return "\n".join(lines) + "\n"


def _pick_splits(sc: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(K, F, 4) per-feature candidates -> best gain (K,) and (feature, threshold, default_left)
    rows, with the tensor path's order: dl = 1 first, dl = 0 only if strictly better, lowest
    feature on ties."""
    g1, g0 = sc[:, :, 0], sc[:, :, 2]
    f1 = torch.argmax(g1, 1) if g1.shape[1] else torch.zeros(sc.shape[0], dtype=torch.long)
    f0 = torch.argmax(g0, 1) if g0.shape[1] else torch.zeros(sc.shape[0], dtype=torch.long)
    r = torch.arange(sc.shape[0])
    b1, b0 = g1[r, f1], g0[r, f0]
    use0 = b0 > b1
    gain = torch.where(use0, b0, b1)
    feat = torch.where(use0, f0, f1)
    thr = torch.where(use0, sc[r, f0, 3], sc[r, f1, 1]).long()
    return gain, torch.stack([feat, thr, (~use0).long()], 1)


def grow_tree(bins: torch.Tensor, cuts: List[torch.Tensor], g: torch.Tensor, h: torch.Tensor, p: Dict,
              world: World, feat_mask: Optional[torch.Tensor] = None,
              bins_t: Optional[torch.Tensor] = None) -> Tuple[Tree, torch.Tensor]:
    """One tree on binned data; returns the tree and each row's leaf value (for margin update).

    On a GPU each level's histogram is one launch of the gfx950 kernel
    (:func:`raydp_amd.ops.gbdt_ops.level_histogram`) over ``bins_t`` (column-major bins,
    transposed here if the caller did not pass them); on the CPU it is ``index_add_``.
    """
    from raydp_amd.ops.gbdt_ops import quant_scale, quantise, soft, torch_split_candidates
    dev = bins.device
    n, F = bins.shape
    B = int(max(c.numel() for c in cuts) + 2) if cuts else 2
    lam, alpha, gamma = float(p["lambda"]), float(p["alpha"]), float(p["gamma"])
    mcw, eta, mds = float(p["min_child_weight"]), float(p["eta"]), float(p["max_delta_step"])
    tree = Tree()
    tree.add()
    pos = torch.zeros(n, dtype=torch.long, device=dev)     # index into the current level's node list
    level = [0]                                            # tree node ids of this level
    leaf_of_row = torch.zeros(n, dtype=torch.long, device=dev)
    feat_off = (torch.arange(F, device=dev) * B)[None, :]
    bins_l = bins.long()
    on_gpu = dev.type == "cuda"
    # fixed-point gradients: one power-of-two scale per tree from the global max |g|, |h| (max is
    # order-independent, so every worker and both devices derive the same scale)
    mx = torch.stack([g.abs().max(), h.abs().max()]).double() if n else torch.zeros(2, dtype=torch.float64,
                                                                                      device=dev)
    world.allreduce(mx, op="max")
    mxc = mx.cpu()
    sg_, sh_ = quant_scale(float(mxc[0])), quant_scale(float(mxc[1]))
    inv_g, inv_h = 1.0 / sg_, 1.0 / sh_
    gq, hq = quantise(g, sg_).contiguous(), quantise(h, sh_).contiguous()
    if on_gpu:
        from raydp_amd.ops.gbdt_ops import level_histogram
        if bins_t is None:
            bins_t = bins.t().contiguous()
        from raydp_amd.ops.gbdt_ops import partition_rows_, split_candidates
        ncuts32 = torch.tensor([c.numel() for c in cuts], dtype=torch.int32, device=dev)
        fmask_u8 = feat_mask.to(device=dev, dtype=torch.uint8).contiguous() if feat_mask is not None else None
    else:
        gh = torch.stack([gq, hq], 1).long()
    ncuts = torch.tensor([c.numel() for c in cuts], device=dev)

    def build(slot, nslots):
        """(nslots, F, B, 2) int64 histogram of the rows with slot >= 0, all-reduced over workers."""
        if on_gpu:
            hs = level_histogram(bins_t, slot, gq, hq, nslots, B)
        else:
            sel = slot >= 0
            idx = (slot.clamp_min(0)[:, None] * (F * B) + feat_off + bins_l)
            hs = torch.zeros(nslots * F * B, 2, dtype=torch.int64, device=dev)
            hs.index_add_(0, idx[sel].reshape(-1), gh[sel].repeat_interleave(F, dim=0))
        world.allreduce(hs)
        return hs.view(nslots, F, B, 2)

    pair_parent: List[int] = []                            # level-k pairs (2j, 2j+1) split from parent k'
    prev_hist = None
    for depth in range(int(p["max_depth"]) + 1):
        K = len(level)
        act = pos >= 0
        if prev_hist is None:
            hist = build(pos, K)
        else:
            # sibling subtraction (XGBoost's hist trick): build only the child with fewer rows
            # (global counts, so every worker picks the same one), derive the other from the
            # parent -- exact in integers
            cnt = torch.bincount(pos[act], minlength=K).double()
            world.allreduce(cnt)
            cnt = cnt.cpu()
            small = [2 * j + int(cnt[2 * j + 1] < cnt[2 * j]) for j in range(K // 2)]
            slot_of = torch.full((K + 1,), -1, dtype=torch.long)
            slot_of[torch.tensor(small, dtype=torch.long)] = torch.arange(K // 2)
            slot_of = slot_of.to(dev)
            hs = build(slot_of[torch.where(act, pos, torch.full_like(pos, K))], K // 2)
            large = torch.tensor([s ^ 1 for s in small], dtype=torch.long, device=dev)
            hist = torch.empty((K, F, B, 2), dtype=torch.int64, device=dev)
            hist[torch.tensor(small, dtype=torch.long, device=dev)] = hs
            hist[large] = prev_hist[torch.tensor(pair_parent, dtype=torch.long, device=dev)] - hs
        tot = hist[:, 0, :, :].sum(1)                         # (K, 2) exact node totals
        tc = tot.cpu()                                         # one device->host copy per level
        Gc, Hc = tc[:, 0].double() * inv_g, tc[:, 1].double() * inv_h
        den = Hc + lam
        wc = torch.where(den > 0, -soft(Gc, alpha) / torch.where(den > 0, den, torch.ones_like(den)),
                         torch.zeros_like(den))
        if mds > 0:
            wc = torch.clamp(wc, -mds, mds)
        for k, nid in enumerate(level):
            tree.cover[nid] = float(Hc[k])
            tree.value[nid] = float(wc[k]) * eta
        if depth == int(p["max_depth"]):
            break
        # per (node, feature): best threshold for both default directions -- one wave per
        # (node, feature) on a GPU, the tensor formulation on the CPU; the cross-feature choice
        # happens on the host copy (first feature wins ties). Same integers in, same gains out.
        if on_gpu:
            sc = split_candidates(hist, tot, ncuts32, fmask_u8, inv_g, inv_h, lam, alpha, mcw).cpu()
        else:
            sc = torch_split_candidates(hist, tot, ncuts, feat_mask, inv_g, inv_h, lam, alpha, mcw)
        best_gain, best = _pick_splits(sc)
        # split bookkeeping on the host, shipped to the device in one copy per table
        prev_hist, pair_parent = hist, []
        new_level, remap = [], torch.full((K,), -1, dtype=torch.long)
        split_feat = torch.full((K,), -1, dtype=torch.long)
        split_bin = torch.zeros((K,), dtype=torch.long)
        split_dl = torch.zeros((K,), dtype=torch.bool)
        bg, bb = best_gain.cpu(), best.cpu()
        for k, nid in enumerate(level):
            if float(bg[k]) <= max(gamma, 1e-6):
                continue
            f, t, dl = int(bb[k, 0]), int(bb[k, 1]), bool(bb[k, 2])
            tree.feature[nid] = f
            tree.cond[nid] = float(cuts[f][t])                  # bins <= t+1  <=>  x < cuts[t]
            tree.default_left[nid] = dl
            tree.gain[nid] = float(bg[k])
            tree.left[nid] = tree.add()
            tree.right[nid] = tree.add()
            remap[k] = len(new_level)
            pair_parent.append(k)
            new_level += [tree.left[nid], tree.right[nid]]
            split_feat[k], split_bin[k], split_dl[k] = f, t + 1, dl
        if on_gpu:
            # one fused launch: leaf bookkeeping + child routing for every row (in place)
            table = torch.stack([remap, split_feat, split_bin, split_dl.long(),
                                 torch.tensor(level, dtype=torch.long)], 1)
            partition_rows_(bins_t, table, pos, leaf_of_row)
            if not new_level:
                level = []
                break
        else:
            remap, split_feat, split_bin, split_dl = (t.to(dev) for t in (remap, split_feat, split_bin, split_dl))
            # rows in nodes that became leaves keep their leaf id; others move down
            cur = pos.clamp_min(0)
            node_ids = torch.tensor(level, dtype=torch.long, device=dev)
            leaf_rows = act & (remap[cur] < 0)
            leaf_of_row = torch.where(leaf_rows, node_ids[cur], leaf_of_row)
            if not new_level:
                pos = torch.full_like(pos, -1)
                level = []
                break
            f = split_feat[cur]
            b = bins_l.gather(1, f.clamp_min(0)[:, None])[:, 0]
            go_left = torch.where(b == 0, split_dl[cur], b <= split_bin[cur])
            child = remap[cur] + (~go_left).long()
            pos = torch.where(act & (remap[cur] >= 0), child, torch.full_like(pos, -1))
        level = new_level
    if level:
        node_ids = torch.tensor(level, dtype=torch.long, device=dev)
        act = pos >= 0
        leaf_of_row = torch.where(act, node_ids[pos.clamp_min(0)], leaf_of_row)
    values = torch.tensor(tree.value, dtype=torch.float32, device=dev)
    return tree, values[leaf_of_row]


# ----------------------------------------------------------------------------- booster ----
class Booster:
    """Trained ensemble (subset of ``xgboost.Booster``)."""

    def __init__(self, params: Optional[Dict] = None, model_file: Optional[str] = None):
        self.params = normalize_params(params)
        self.trees: List[List[Tree]] = []        # per round, one tree per output group
        self.base_margin = 0.0
        self.feature_names: Optional[List[str]] = None
        self.evals_result: Dict = {}
        if model_file is not None:
            self.load_model(model_file)

    @property
    def num_group(self) -> int:
        return int(self.params["num_class"]) if self.params["objective"].startswith("multi:") else 1

    def num_boosted_rounds(self) -> int:
        return len(self.trees)

    def num_features(self) -> int:
        return len(self.feature_names or [])

    def _margin(self, x: torch.Tensor, iteration_range=None) -> torch.Tensor:
        lo, hi = iteration_range if iteration_range else (0, len(self.trees))
        k = self.num_group
        m = torch.full((x.shape[0], k), self.base_margin, dtype=torch.float32, device=x.device)
        for rnd in self.trees[lo:hi]:
            for j, t in enumerate(rnd):
                m[:, j] += t.predict(x)
        return m if k > 1 else m[:, 0]

    def predict(self, data, output_margin: bool = False, iteration_range=None):
        x = data.data if isinstance(data, DMatrix) else torch.as_tensor(np.asarray(data, dtype=np.float32))
        if x.dim() == 1:
            x = x[None, :]
        m = self._margin(x, iteration_range)
        out = m if output_margin else _transform(self.params["objective"], m)
        return out.cpu().numpy()

    def inplace_predict(self, data, iteration_range=None, predict_type: str = "value"):
        import pandas as pd
        if isinstance(data, pd.DataFrame):
            data = data.to_numpy(dtype=np.float32, na_value=np.nan)
        return self.predict(np.asarray(data, dtype=np.float32), output_margin=predict_type == "margin",
                            iteration_range=iteration_range)

    def get_dump(self, with_stats: bool = False) -> List[str]:
        names = self.feature_names or [f"f{i}" for i in range(1000)]
        return [t.dump(names) for rnd in self.trees for t in rnd]

    def get_score(self, importance_type: str = "weight") -> Dict[str, float]:
        names = self.feature_names or []
        acc: Dict[str, List[float]] = {}
        for rnd in self.trees:
            for t in rnd:
                for f, gn, cv in zip(t.feature, t.gain, t.cover):
                    if f >= 0:
                        v = {"weight": 1.0, "gain": gn, "total_gain": gn, "cover": cv, "total_cover": cv}[importance_type]
                        acc.setdefault(names[f] if f < len(names) else f"f{f}", []).append(v)
        if importance_type in ("gain", "cover"):
            return {k: float(np.mean(v)) for k, v in acc.items()}
        return {k: float(np.sum(v)) for k, v in acc.items()}

    def save_model(self, fname: str):
        with open(fname, "w") as f:
            json.dump(self.to_json(), f)

    def to_json(self) -> Dict:
        return {"format": "raydp-gbdt-1", "params": self.params, "base_margin": self.base_margin,
                "feature_names": self.feature_names, "trees": [[t.to_json() for t in rnd] for rnd in self.trees]}

    def load_model(self, fname: str):
        with open(fname) as f:
            d = json.load(f)
        self.params = normalize_params(d["params"])
        self.base_margin = float(d["base_margin"])
        self.feature_names = d.get("feature_names")
        self.trees = [[Tree.from_json(t) for t in rnd] for rnd in d["trees"]]
        return self

    def save_raw(self) -> bytes:
        return json.dumps(self.to_json()).encode()


def _binned(dtrain: DMatrix, p: Dict, world: World, dev: torch.device):
    """Quantile cuts + bin matrix (and its column-major copy on a GPU) of ``dtrain``, computed
    once per (max_bin, seed, device, world size) and kept on the DMatrix -- as XGBoost keeps the
    quantised ``DMatrix`` across ``train`` calls -- so repeated training on the same data (warm
    starts, benchmarks, CV) re-bins nothing."""
    key = (int(p["max_bin"]), int(p["seed"]), str(dev), world.size)
    cache = dtrain.__dict__.setdefault("_binned_cache", {})
    if key not in cache:
        cuts = compute_cuts(dtrain.data, int(p["max_bin"]), world, seed=int(p["seed"]), device=dev)
        bins = bin_matrix(dtrain.data.to(dev), cuts)
        bins_t = bins.t().contiguous() if dev.type == "cuda" else None   # coalesced per-feature reads
        cache.clear()
        cache[key] = (cuts, bins, bins_t)
    return cache[key]


def train(params: Dict, dtrain: DMatrix, num_boost_round: int = 10, evals: Sequence = (),
          evals_result: Optional[Dict] = None, device: Optional[str] = None, verbose_eval: bool = False,
          callback=None) -> Booster:
    """Boost ``num_boost_round`` rounds; histograms all-reduced when a process group is up."""
    p = normalize_params(params)
    if "num_boost_round" in (params or {}):
        num_boost_round = int(params["num_boost_round"])
    world = World()
    dev = torch.device(device) if device else (torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
    obj = p["objective"]
    k = int(p["num_class"]) if obj.startswith("multi:") else 1
    x = dtrain.data
    y = dtrain.label.to(dev)
    cuts, bins, bins_t = _binned(dtrain, p, world, dev)
    bst = Booster(p)
    bst.feature_names = dtrain.feature_names
    bst.base_margin = _base_margin(obj, dtrain.label, p["base_score"], world)
    margin = torch.full((x.shape[0], k), bst.base_margin, dtype=torch.float32, device=dev)
    if k == 1:
        margin = margin[:, 0]
    ev = [(d.data.to(dev), d.label.to(dev), name) for d, name in evals]
    ev_margin = [torch.full((d[0].shape[0], k) if k > 1 else (d[0].shape[0],), bst.base_margin, device=dev)
                 for d in ev]
    metrics = p.get("eval_metric") or default_metric(obj)
    metrics = [metrics] if isinstance(metrics, str) else list(metrics)
    res = evals_result if evals_result is not None else {}
    for _, _, name in ev:
        res.setdefault(name, {m: [] for m in metrics})
    gen = torch.Generator(device="cpu").manual_seed(int(p["seed"]))
    for rnd in range(num_boost_round):
        g, h = _grad_hess(obj, margin, y, p)
        if dtrain.weight is not None:
            w = dtrain.weight.to(dev)
            g, h = (g * w[:, None], h * w[:, None]) if k > 1 else (g * w, h * w)
        if float(p["subsample"]) < 1.0:
            keep = (torch.rand(x.shape[0], generator=gen) < float(p["subsample"])).to(dev)
            keep = keep[:, None] if k > 1 else keep
            g, h = g * keep, h * keep
        fmask = None
        if float(p["colsample_bytree"]) < 1.0:
            nf = max(1, int(round(float(p["colsample_bytree"]) * x.shape[1])))
            fmask = torch.zeros(x.shape[1], dtype=torch.bool)
            fmask[torch.randperm(x.shape[1], generator=gen)[:nf]] = True
            fmask = fmask.to(dev)
        rtrees = []
        for j in range(k):
            gj, hj = (g[:, j], h[:, j]) if k > 1 else (g, h)
            tree, leaf_vals = grow_tree(bins, cuts, gj, hj, p, world, fmask, bins_t)
            rtrees.append(tree)
            if k > 1:
                margin[:, j] += leaf_vals
            else:
                margin += leaf_vals
            for i, (xe, _, _) in enumerate(ev):
                if k > 1:
                    ev_margin[i][:, j] += tree.predict(xe)
                else:
                    ev_margin[i] += tree.predict(xe)
        bst.trees.append(rtrees)
        for i, (_, ye, name) in enumerate(ev):
            for m in metrics:
                res[name][m].append(eval_metric(m, obj, ev_margin[i], ye, world))
        if verbose_eval and ev:
            print(f"[{rnd}] " + "\t".join(f"{n}-{m}:{res[n][m][-1]:.5f}" for _, _, n in ev for m in metrics))
        if callback is not None:
            callback(rnd, bst, res)
    bst.evals_result = res
    return bst
