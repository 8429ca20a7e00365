"""Host side of the fused MLP trainer (``csrc/hip/fused_mlp.hip``).

``FusedMLPTrainer`` owns the device state of one MLP replica: the flat fp32 master
parameters, gradients and optimizer moments, the bf16 ``W``/``Wt`` weight images the kernel
reads, the BatchNorm running buffers, the LDS layout and the per-step scratch. An epoch is a
single native call that enqueues ``fused fwd/bwd kernel → [all-reduce] → optimizer kernel``
per batch with no host synchronisation; metrics accumulate on the device and are read back
once per epoch (the reference syncs on ``loss.item()`` every step,
``python/raydp/torch/estimator.py:280``).
"""
import ctypes
import os
import math
from typing import Callable, Dict, List, Optional

import numpy as np
import torch
import torch.nn as nn

from raydp_amd.models.mlp_spec import MlpSpec
from raydp_amd.ops import _hip

_LOSSES = {nn.MSELoss: 0, nn.SmoothL1Loss: 1, nn.L1Loss: 2}


# words after the per-step stamps of a persistent epoch's stamp buffer: the middle step's
# intra-layer shader-clock stamps (csrc/hip/mlp_persist.h RX_PS_LAYER_STAMPS)
_PS_LAYER_STAMPS = 96

def _ru(x, m):
    return (x + m - 1) // m * m


def loss_code(loss) -> Optional[tuple]:
    """(code, beta) for a supported mean-reduced loss (MSE 0, SmoothL1 1, L1 2, BCE-with-logits
    3, weighted cross entropy 4), else None."""
    if isinstance(loss, type) and issubclass(loss, nn.Module):
        try:
            loss = loss()
        except TypeError:
            return None
    for cls, code in _LOSSES.items():
        if type(loss) is cls and getattr(loss, "reduction", "mean") == "mean":
            return code, float(getattr(loss, "beta", 1.0))
    # BCEWithLogitsLoss() (mean, no weight / pos_weight): code 3, in the last layer's epilogue
    if type(loss) is nn.BCEWithLogitsLoss and loss.reduction == "mean" and loss.weight is None \
            and loss.pos_weight is None:
        return 3, 1.0
    # CrossEntropyLoss(weight=w) over class-index labels (mean, no label smoothing): code 4 --
    # the engine feeds w[y]-weighted one-hot label rows (fused_labels)
    if type(loss) is nn.CrossEntropyLoss and loss.reduction == "mean" and float(loss.label_smoothing) == 0.0:
        w = loss.weight
        if w is not None and (w.dim() != 1 or not bool((w > 0).all())):
            return None
        return 4, 1.0
    return None


def fused_labels(loss, labels: torch.Tensor, classes: int) -> torch.Tensor:
    """The label matrix the fused kernel reads for ``loss``: the ingested column as is, or for
    cross entropy the ``[N, classes]`` one-hot rows scaled by the class weight (an
    ``ignore_index`` row is all zeros: it adds nothing to the loss or the weight sum, as in
    torch)."""
    if type(loss) is not nn.CrossEntropyLoss:
        return labels
    y = labels.reshape(-1).round().long()
    w = loss.weight.to(labels.device, torch.float32) if loss.weight is not None else \
        torch.ones(classes, device=labels.device)
    valid = (y >= 0) & (y < classes)
    out = torch.zeros(y.numel(), classes, dtype=torch.float32, device=labels.device)
    idx = torch.arange(y.numel(), device=labels.device)[valid]
    out[idx, y[valid]] = w[y[valid]]
    return out.contiguous()


def optimizer_config(opt) -> Optional[dict]:
    if opt is None or len(opt.param_groups) != 1:
        return None
    g = opt.param_groups[0]
    if isinstance(opt, torch.optim.AdamW):
        if g.get("amsgrad"):
            return None
        return dict(algo=1, lr=g["lr"], b1=g["betas"][0], b2=g["betas"][1], eps=g["eps"],
                    wd=g["weight_decay"], maximize=g.get("maximize", False))
    if isinstance(opt, torch.optim.Adam):
        if g.get("amsgrad") or g.get("decoupled_weight_decay", False):
            return None
        return dict(algo=0, lr=g["lr"], b1=g["betas"][0], b2=g["betas"][1], eps=g["eps"],
                    wd=g["weight_decay"], maximize=g.get("maximize", False))
    if isinstance(opt, torch.optim.SGD):
        return dict(algo=2, lr=g["lr"], momentum=g["momentum"], dampening=g["dampening"],
                    wd=g["weight_decay"], nesterov=g["nesterov"], maximize=g.get("maximize", False))
    return None


def jit_enabled() -> bool:
    """Per-model specialised step kernels (``raydp_amd.ops.mlp_jit``); RAYDP_MLP_JIT=0 turns
    them off (the ahead-of-time run-time-descriptor kernel is used instead)."""
    import os
    from raydp_amd.utils.config import get as conf_get
    return bool(conf_get("spark.ray.mi355x.mlp_jit"))


def wgrad_mode() -> int:
    """Where weight gradients are computed (``spark.ray.mi355x.mlp_wgrad``): ``opt`` (default,
    1): the step kernel exports X^T / G^T and the optimizer kernel's many workgroups compute
    dW = X^T G as they update; ``step`` (0): inside the single-workgroup step kernel."""
    from raydp_amd.utils.config import get as conf_get
    return 1 if conf_get("spark.ray.mi355x.mlp_wgrad") == "opt" else 0


W0S_N = 16 * 64 * 4 + 16 * 16 * 4   # csrc/hip/mlp_persist.h RX_W0S_N


def persistent_enabled() -> bool:
    """One-GPU epochs as one persistent launch (``spark.ray.mi355x.mlp_persistent``)."""
    from raydp_amd.utils.config import get as conf_get
    return bool(conf_get("spark.ray.mi355x.mlp_persistent"))


_ATTR = {"weight": "weight", "bias": "bias", "gamma": "weight", "beta": "bias", "emb": "weight"}


def pick_mt(batch: int) -> Optional[int]:
    """Row tiles of a single-workgroup step (batch <= 128), else None."""
    for mt in (2, 4, 8):
        if batch <= mt * 16:
            return mt
    return None


# Largest batch of the multi-workgroup step: every one of its ceil(batch / 16 mt) workgroups
# must be resident at once (one per CU at the step kernel's LDS size; the host also checks the
# occupancy on the device).
MAX_FUSED_BATCH = 16384


def fused_batch_ok(batch: int) -> bool:
    return 1 <= int(batch) <= MAX_FUSED_BATCH


def layout_candidates(batch: int):
    """(row tiles per workgroup, workgroups per step) to try, best first: one workgroup for a
    batch that fits its tile, else the multi-workgroup step with the widest tile whose LDS
    image fits (csrc/hip/mlp_core.h MwCtx)."""
    out = []
    single = pick_mt(batch)
    if single is not None:
        out.append((single, 1))
    order = (8, 4, 2)
    want = int(os.environ.get("RAYDP_MLP_MW_MT", "0") or 0)   # dev knob: prefer this tile
    if want in order:
        order = (want,) + tuple(m for m in order if m != want)
    for mt in order:
        if batch > 16 * mt:
            out.append((mt, -(-batch // (16 * mt))))
    return out


class FusedMLPTrainer:
    def __init__(self, spec: MlpSpec, opt_cfg: dict, loss: tuple, batch_size: int,
                 device: torch.device, lr_schedule: Optional[Callable[[int], float]] = None,
                 layout_only: bool = False, acc_thr: Optional[float] = None, world: int = 1,
                 share: int = 1):
        # layout_only: build the descriptors on the host (no GPU needed) -- used to warm the
        # specialised-kernel cache at build time
        # world > 1: gradients are exchanged inside the training launches (layer 0 is then not
        # updated by the persistent step workgroup: its gradient must be summed over the ranks
        # first); share: training ranks on this device (rehearsals), which size the in-launch
        # optimizer workgroups so every rank's grid is resident at once
        self.world, self.share = int(world), max(1, int(share))
        self.layout_only = layout_only
        self.spec, self.cfg, self.device = spec, opt_cfg, torch.device("cpu" if layout_only else device)
        self.batch = int(batch_size)
        if not fused_batch_ok(self.batch):
            raise ValueError(f"batch {self.batch} outside the fused trainer's range (1..{MAX_FUSED_BATCH})")
        self.loss_code, self.beta = loss
        self.lr_schedule = lr_schedule
        self.acc_thr = acc_thr           # binary accuracy threshold (None: not counted)
        self.record_steps = False        # per-step device times of persistent epochs
        self.step_count = 0
        self.lib = _hip.lib()
        err = None
        for mt, G in layout_candidates(self.batch):
            self.mt, self.G, self.bp = mt, G, mt * 16
            try:
                self._build()
                err = None
                break
            except ValueError as e:      # LDS / width limits of this tile: try the next layout
                err = e
        if err is not None:
            raise err

    # ----------------------------------------------------------------------- layout -------
    def _build(self):
        spec, dev, bp, mt = self.spec, self.device, self.bp, self.mt
        G = self.G
        bp_all = G * bp      # exported X^T / G^T columns: the whole (padded) batch
        if G > 1:
            if spec.front:
                raise ValueError("the multi-workgroup step has no embedding front")
            if self.loss_code == 4:
                raise ValueError("cross entropy's weight sum is per workgroup: one-workgroup batches only")
        L = len(spec.layers)
        ntw = 16 // mt
        flat: List[torch.Tensor] = []
        off = 0
        self.layout = []
        d = _hip.MlpDesc()
        o = _hip.OptDesc()
        d.L = L
        max_k = max_n = 0
        dims = []
        for ly in spec.layers:
            i, oo = ly.linear.in_features, ly.linear.out_features
            dims.append((i, oo, _ru(i, 32), _ru(oo, 32), _ru(i, 16), _ru(oo, 16)))
            max_k = max(max_k, _ru(i, 32), _ru(oo, 32))
            max_n = max(max_n, _ru(oo, 16))
            if _ru(oo, 16) // 16 > ntw * 8 or _ru(i, 16) // 16 > ntw * 8:
                raise ValueError("layer too wide for this batch size in the fused trainer")
        self.run_bufs = []
        img_off = 0       # bf16 elements: W_l [out_n][in_k] then Wt_l [in_n][out_k], per layer
        rs_total = 0      # fp32 running statistics [mean | var] per BN layer
        rs_init = []
        xs = bp          # transposed-image stride: Tile<MT>::XS (csrc/hip/mlp_core.h)
        lds = 0

        def alloc(nbytes):
            nonlocal lds
            start = lds
            lds = _ru(lds + nbytes, 16)
            return start

        wmode = wgrad_mode() if G == 1 else 1   # multi-workgroup: dW over the whole batch
        # T mode (csrc/hip/mlp_core.h AOp): with the weight gradients on the optimizer side
        # (wgrad_mode 1) no layer's transposed image outlives the next publish, so ONE transposed
        # image serves as every X^T_l and as G^T, and the GEMMs read their A operands from it by
        # transposed LDS reads -- no row-major R image. The freed LDS keeps the saved BN inputs
        # on chip (sv_lds).
        tmode = wmode == 1 and not spec.front and mt >= 2
        if tmode:
            d.r_lds_off = -1
            t_off = alloc(max_k * xs * 2)          # rows up to every layer's K padding
            d.gt_lds_off = t_off
        else:
            d.r_lds_off = alloc(bp * (max_k + 16) * 2)   # row stride max_k + RX_RPAD (csrc/hip/mlp_core.h)
            d.gt_lds_off = alloc(max_n * xs * 2)
        stat_total = sum(2 * dm[5] for dm in dims)
        d.stats_lds_off = alloc(stat_total * 4)
        scratch_off = 0
        stat_off = 0
        pr_total = 0
        mw_total = 0
        nseg = 0
        seg_images = []
        act = 0           # bf16 elements of the exported X^T_l / G^T_l area (wgrad_mode 1)

        def vseg(start, n):
            # bias / BN gamma+beta vectors: plain element-wise optimizer segments
            nonlocal nseg
            sg = o.seg[nseg]
            sg.start, sg.len, sg.kind = start, n, 0
            nseg += 1

        def pad4():
            # every flat segment starts 16-B aligned (vectorised gradient stores)
            nonlocal off
            if off % 4:
                flat.append(torch.zeros(4 - off % 4))
                off += 4 - off % 4

        for li, (ly, dm) in enumerate(zip(spec.layers, dims)):
            i, oo, in_k, out_k, in_n, out_n = dm
            lin = ly.linear
            x = d.layer[li]
            x.in_, x.out, x.in_k, x.out_k, x.in_n, x.out_n = i, oo, in_k, out_k, in_n, out_n
            x.w_img = img_off
            img_off += _ru(out_n * in_k, 8)
            x.wt_img = img_off
            img_off += _ru(in_n * out_k, 8)
            pad4()
            x.w_off = off
            flat.append(lin.weight.detach().reshape(-1).float())
            seg = o.seg[nseg]
            seg.start, seg.len, seg.kind = off, oo * i, 1
            seg.out, seg.in_, seg.in_k, seg.out_k = oo, i, in_k, out_k
            x.xg_off = seg.xg_off = act
            act += in_n * bp_all
            x.gg_off = seg.gg_off = act
            act += out_n * bp_all
            seg.in_n, seg.out_n = in_n, out_n
            seg_images.append((nseg, x.w_img, x.wt_img))
            nseg += 1
            self.layout.append(("weight", lin, off, oo * i))
            off += oo * i
            if lin.bias is not None:
                pad4()
                x.b_off = off
                flat.append(lin.bias.detach().reshape(-1).float())
                self.layout.append(("bias", lin, off, oo))
                vseg(off, oo)
                off += oo
            else:
                x.b_off = -1
            x.act, x.bn = ly.act, ly.bn
            x.g_off = x.be_off = -1
            x.rs_off = -1
            if ly.bn:
                bn = ly.bn_module
                if bn.affine:
                    pad4()
                    x.g_off = off
                    flat.append(bn.weight.detach().reshape(-1).float())
                    self.layout.append(("gamma", bn, off, oo))
                    x.be_off = off + oo
                    flat.append(bn.bias.detach().reshape(-1).float())
                    self.layout.append(("beta", bn, off + oo, oo))
                    vseg(off, 2 * oo)
                    off += 2 * oo
                if bn.running_mean is not None:
                    x.rs_off = rs_total
                    rs_init.append((bn, rs_total, oo))
                    rs_total += 2 * oo
                x.eps, x.momentum = float(bn.eps), float(bn.momentum if bn.momentum is not None else 0.1)
            x.xt_off = t_off if tmode else alloc(in_n * xs * 2)
            x.sv_lds = -1
            x.stat_off = stat_off
            stat_off += 2 * out_n
            x.r_off = scratch_off
            scratch_off += bp * out_n
            x.pr_off = pr_total
            pr_total += 5 * out_n
            # multi-workgroup partials: [fwd 2 out_n | bwd 2 out_n | bias out_n], each region on
            # its own 128-B lines (csrc/hip/mlp_core.h mw_fwd)
            x.mw_off = mw_total
            # [forward pairs | backward pairs | bias singles] as tagged granules (csrc/hip/mlp_core.h
            # mw_put_pair): 4 and 2 floats per column
            mw_total += 2 * _ru(4 * out_n, 32) + _ru(2 * out_n, 32)
        # embedding front: every table is one contiguous run of the flat vector (element-wise
        # optimizer segment); front column k reads element [id][j] at poff + id * stride
        front = spec.front or []
        if len(front) > _hip.MAXF:
            raise ValueError("embedding front wider than the kernel's column table")
        d.front_n = len(front)
        if front:
            tab_off = {}
            pad4()
            emb_start = off
            for e in spec.embeddings():
                tab_off[id(e)] = off
                flat.append(e.weight.detach().reshape(-1).float())
                self.layout.append(("emb", e, off, e.weight.numel()))
                off += e.weight.numel()
            vseg(emb_start, off - emb_start)
            q = 0
            for k, c in enumerate(front):
                fc = d.front[k]
                fc.src = c.src
                d.front_qbase[k] = q
                if c.emb is None:
                    fc.poff, fc.stride, fc.rows = -1, 0, 0
                else:
                    fc.poff = tab_off[id(c.emb)] + c.j
                    fc.stride, fc.rows = c.emb.embedding_dim, c.emb.num_embeddings
                    q += fc.rows
            d.front_q = q
            l0 = d.layer[0]
            if bp * l0.in_n * 4 + bp * len(front) * 2 > max_n * xs * 2:
                raise ValueError("embedding front's backward scratch exceeds the G^T area")
        d.acc_mode = 1 if self.acc_thr is not None else 0
        d.acc_thr = float(self.acc_thr) if self.acc_thr is not None else 0.5
        d.pr_lds_off = alloc(pr_total * 4)
        d.pr_total = pr_total
        # one output column, regression / BCE loss, one workgroup: the loss runs a row per lane
        # through a BP-float LDS area (csrc/hip/mlp_core.h MlpDesc::loss_lds_off)
        d.loss_lds_off = -1
        if G == 1 and spec.layers[-1].linear.out_features == 1 and self.loss_code != 4 \
                and lds + bp * 4 <= 160 * 1024 - 1536:
            d.loss_lds_off = alloc(bp * 4)
        # persistent epoch: layer 0 updated by the step workgroup itself (csrc/hip/mlp_persist.h
        # ps_l0_update) -- its fp32 master + both moments (RX_W0S_N floats each) and a copy of
        # X^T_0 in LDS; layer 0's saved BN inputs then go to the global scratch buffer instead
        d.w0s_lds_off = d.x0c_lds_off = -1
        l00 = spec.layers[0].linear
        # (decided without looking at whether epochs run persistent: every kernel of the model then
        # runs layer 0 in the same k order, so the persistent epoch and the step loop agree bit for bit)
        l0_inline = (G == 1 and tmode and wmode == 1 and not front and self.world == 1
                     and l00.in_features <= 20 and dims[0][2] == 32 and l00.out_features % 16 == 0
                     and l00.out_features <= 256 and L > 1
                     and lds + 32 * xs * 2 + 3 * W0S_N * 4 <= 160 * 1024 - 1536)
        if l0_inline:
            d.x0c_lds_off = alloc(32 * xs * 2)
            d.w0s_lds_off = alloc(3 * W0S_N * 4)
        self.l0_inline = l0_inline
        # saved BN inputs / ReLU sources in LDS, largest first, while they fit (the rest stays in
        # the global scratch buffer); T mode only (R mode has no room for them)
        if tmode:
            budget = 160 * 1024 - 1536     # static LDS of the kernels (2 x BP row indices, flags)
            saves = [(bp * d.layer[li].out_n * 4, li) for li, ly in enumerate(spec.layers)
                     if (ly.bn or li != L - 1) and not (li == 0 and l0_inline)]
            for nbytes, li in sorted(saves, reverse=True):
                if lds + nbytes <= budget:
                    d.layer[li].sv_lds = alloc(nbytes)
        d.lds_bytes = lds
        d.max_k, d.max_n = max_k, max_n
        d.loss, d.beta = self.loss_code, self.beta
        d.out_dim = spec.out_features
        d.feat_k = _ru(spec.raw_features, 8) if front else dims[0][2]
        if lds > 160 * 1024:
            raise ValueError(f"fused MLP needs {lds} B of LDS (> 160 KiB)")
        self.desc = d
        self.feat_k = d.feat_k
        total = off
        # gradient buffer = [flat gradient (total) | exported activation area]; in xGMI mode the
        # whole buffer is the exchange slot, so peers read each other's X^T / G^T from it
        act_off = _ru(total, 4)
        act_floats = _ru((act + 1) // 2, 4)
        d.act_off, d.wgrad_mode = act_off, wmode
        self.total = total
        # ONE device arena for every buffer of the trainer: [params | rstats | descriptors] are
        # uploaded from one pinned host image in one copy, [grads | m | v | scratch | metrics |
        # img] are zeroed by one fill (a fit's engine set-up is on the headline's critical path)
        params_h = torch.cat([f.detach().reshape(-1).cpu().float() for f in flat]) if flat else \
            torch.zeros(0)
        rs_h = torch.zeros(max(1, rs_total), dtype=torch.float32)
        for bn, ro, n_ in rs_init:
            rs_h[ro:ro + n_] = bn.running_mean.detach().cpu().float()
            rs_h[ro + n_:ro + 2 * n_] = bn.running_var.detach().cpu().float()
        self._arena_plan = {"params": (params_h.numel(), torch.float32), "rstats": (rs_h.numel(), torch.float32)}
        self._arena_host = {"params": params_h, "rstats": rs_h}
        self._arena_zero = [("grads", act_off + act_floats, torch.float32), ("m", params_h.numel(), torch.float32),
                            ("v", params_h.numel(), torch.float32),
                            ("scratch", max(1, scratch_off) * G, torch.float32),
                            ("metrics", 8, torch.float64), ("img", max(8, img_off), torch.bfloat16),
                            ("mw_part", mw_total * G if G > 1 else 1, torch.float32),
                            ("mw_ctl", 4, torch.int32)]
        self._scratch_stride = max(1, scratch_off)
        self._mw_stride = mw_total
        self._arena_dev = dev
        self._seg_images = seg_images
        cfg = self.cfg
        o.nseg, o.total, o.algo = nseg, total, cfg["algo"]
        o.b1, o.b2, o.eps = cfg.get("b1", 0.9), cfg.get("b2", 0.999), cfg.get("eps", 1e-8)
        o.wd, o.momentum, o.dampening = cfg.get("wd", 0.0), cfg.get("momentum", 0.0), cfg.get("dampening", 0.0)
        o.nesterov, o.maximize = int(cfg.get("nesterov", False)), int(cfg.get("maximize", False))
        o.act_off, o.act_floats, o.bp, o.wgrad_mode = act_off, act_floats, bp_all, wmode
        o.ps_l0_inline = int(self.l0_inline)
        self.opt = o
        self._mw_nopt = 0
        if G > 1 and wmode == 1:
            # split-K weight-gradient partials + per-tile arrival counters of the multi-workgroup
            # optimizer (csrc/hip/fused_mlp.hip mw_wgrad_opt_kernel, RX_WSPLIT_K rows per split)
            splits = -(-int(bp_all) // 256)
            tiles = sum(((sg.out + 31) // 32) * ((sg.in_ + 31) // 32) for sg in o.seg[:o.nseg] if sg.kind == 1)
            self._arena_zero += [("mw_wpart", max(1, tiles * splits * 1024), torch.float32),
                                 ("mw_wctr", max(1, tiles), torch.int32), ("mw_lcnt", 8 * 32, torch.int32)]
            # optimizer workgroups inside the step's launch (csrc/hip/mlp_mwopt.h), two tasks each
            # (RAYDP_MLP_MW_FUSED_OPT: 0 = the separate launch, N > 1 = at most N workgroups; dev knob)
            cap = int(os.environ.get("RAYDP_MLP_MW_FUSED_OPT", "1"))
            self._mw_nopt = 0 if cap == 0 else min(-(-tiles * splits // 2), cap if cap > 1 else 1 << 30)
        self.lds_bytes = lds
        # descriptors live in device memory: the kernels index them with runtime layer ids
        from raydp_amd.utils import tracing
        with tracing.span("trainer arena", cat="train"):
            self._materialize(bytes(d), bytes(o), rs_init)
        self._dd = ctypes.c_void_p(self._desc_buf.data_ptr())
        self._od = ctypes.c_void_p(self._opt_buf.data_ptr())
        b = _hip.StepBufs()
        b.d_dev, b.img, b.rstats = self._desc_buf.data_ptr(), self.img.data_ptr(), self.rstats.data_ptr()
        b.params, b.grads = self.params.data_ptr(), self.grads.data_ptr()
        b.scratch, b.metrics = self.scratch.data_ptr(), self.metrics.data_ptr()
        self.bufs = b
        self.jit = None
        self._mw_args = None
        if G > 1:
            a = _hip.MwArgs()
            a.part, a.ctl, a.G = self.mw_part.data_ptr(), self.mw_ctl.data_ptr(), G
            a.stride = self._mw_stride
            a.scratch_stride = self._scratch_stride
            if self.mw_wpart is not None:
                a.wpart, a.wctr = self.mw_wpart.data_ptr(), self.mw_wctr.data_ptr()
                a.lcnt, a.nopt = self.mw_lcnt.data_ptr(), self._mw_nopt
            from raydp_amd.utils.config import get as conf_get
            khz = 100000
            a.ticks = int(float(conf_get("spark.ray.mi355x.mlp_persistent.timeout_s")) * khz * 1000)
            a.share = self.share
            a.resident_ok = 0
            if not self.layout_only:
                if int(self.lib.rx_mw_resident(mt, lds, G)) != 0:
                    raise ValueError(f"{G} step workgroups of {lds} B LDS cannot be resident at once")
                a.resident_ok = 1
            self._mw_args = a
            b.mw = ctypes.addressof(a)
        if self.layout_only:
            return
        if jit_enabled():
            from raydp_amd.ops import mlp_jit
            with tracing.span("jit load", cat="train"):
                self.jit = mlp_jit.load_specialized(self)
        self.refresh_images()

    def _materialize(self, desc_bytes: bytes, opt_bytes: bytes, rs_init):
        """Allocate the arena, point the optimizer descriptor's segments at their bf16 images,
        and fill the arena with one zero fill + one host-to-device copy."""
        dev = self._arena_dev
        A = 256

        def nbytes(n, dt):
            return _ru(n * torch.tensor([], dtype=dt).element_size(), A)
        up = [("params",) + self._arena_plan["params"], ("rstats",) + self._arena_plan["rstats"]]
        off, where = 0, {}
        for name, n, dt in up:
            where[name] = (off, n, dt)
            off += nbytes(n, dt)
        desc_off = off
        off += _ru(len(desc_bytes), A)
        opt_off = off
        off += _ru(len(opt_bytes), A)
        up_end = off
        for name, n, dt in self._arena_zero:
            where[name] = (off, n, dt)
            off += nbytes(n, dt)
        arena = torch.empty(max(A, off), dtype=torch.uint8, device=dev)
        self._arena = arena

        def view(name):
            o_, n, dt = where[name]
            return arena[o_:o_ + n * torch.tensor([], dtype=dt).element_size()].view(dt)
        self.params, self.rstats = view("params"), view("rstats")
        self.grads, self.m, self.v = view("grads"), view("m"), view("v")
        self.scratch, self.metrics, self.img = view("scratch"), view("metrics"), view("img")
        self.mw_part, self.mw_ctl = view("mw_part"), view("mw_ctl")
        self.mw_wpart = view("mw_wpart") if "mw_wpart" in where else None
        self.mw_wctr = view("mw_wctr") if "mw_wctr" in where else None
        self.mw_lcnt = view("mw_lcnt") if "mw_lcnt" in where else None
        self._desc_buf = arena[desc_off:desc_off + len(desc_bytes)]
        base = self.img.data_ptr()
        o = self.opt
        for si, wi, wti in self._seg_images:
            o.seg[si].W, o.seg[si].Wt = base + 2 * wi, base + 2 * wti
        opt_bytes = bytes(o)
        self._opt_buf = arena[opt_off:opt_off + len(opt_bytes)]
        # host image of the uploaded part, pinned: one asynchronous copy
        host = torch.empty(up_end, dtype=torch.uint8, pin_memory=dev.type == "cuda")
        for name in ("params", "rstats"):
            o_, n, dt = where[name]
            src = self._arena_host[name]
            host[o_:o_ + src.numel() * src.element_size()].view(dt).copy_(src)
        host[desc_off:desc_off + len(desc_bytes)] = torch.frombuffer(bytearray(desc_bytes), dtype=torch.uint8)
        host[opt_off:opt_off + len(opt_bytes)] = torch.frombuffer(bytearray(opt_bytes), dtype=torch.uint8)
        arena[:up_end].copy_(host, non_blocking=True)
        arena[up_end:].zero_()
        self._arena_upload = host          # kept alive until the copy has run
        self._arena_host = None
        for bn, ro, n_ in rs_init:
            self.run_bufs.append((bn, self.rstats[ro:ro + n_], self.rstats[ro + n_:ro + 2 * n_]))

    # ------------------------------------------------------------------- optimizer state ----
    def _param_of(self, kind, mod):
        return getattr(mod, _ATTR[kind])

    @torch.no_grad()
    def load_optimizer_state(self, opt: torch.optim.Optimizer) -> bool:
        """Start from a torch optimizer's state (Adam/AdamW ``exp_avg``/``exp_avg_sq``/``step``,
        SGD ``momentum_buffer``) -- a resumed fit or an optimizer handed in mid-training."""
        if not opt.state:
            return False
        m_h, v_h = self.m.cpu(), self.v.cpu()
        step = None
        for kind, mod, off, n in self.layout:
            st = opt.state.get(self._param_of(kind, mod))
            if not st:
                continue
            if "exp_avg" in st:
                m_h[off:off + n] = st["exp_avg"].detach().reshape(-1).float().cpu()
                v_h[off:off + n] = st["exp_avg_sq"].detach().reshape(-1).float().cpu()
                step = int(st["step"].item() if torch.is_tensor(st["step"]) else st["step"])
            elif st.get("momentum_buffer") is not None:
                m_h[off:off + n] = st["momentum_buffer"].detach().reshape(-1).float().cpu()
                step = max(step or 0, 1)
        self.m.copy_(m_h)
        self.v.copy_(v_h)
        if step is not None:
            self.step_count = step
        return True

    @torch.no_grad()
    def export_optimizer_state(self, opt: torch.optim.Optimizer) -> dict:
        """Write the device moments / step into ``opt`` (whose params are the user's module
        parameters) and return ``opt.state_dict()`` -- the ``optim.pt`` of a checkpoint."""
        m_h, v_h = self.m.cpu(), self.v.cpu()
        algo = self.cfg["algo"]
        for kind, mod, off, n in self.layout:
            p = self._param_of(kind, mod)
            if algo in (0, 1):
                opt.state[p] = {"step": torch.tensor(float(self.step_count)),
                                "exp_avg": m_h[off:off + n].view_as(p).clone(),
                                "exp_avg_sq": v_h[off:off + n].view_as(p).clone()}
            elif self.cfg.get("momentum", 0.0):
                opt.state[p] = {"momentum_buffer": m_h[off:off + n].view_as(p).clone()}
        return opt.state_dict()

    def refresh_images(self):
        """Rebuild the bf16 W/Wt images from the fp32 master parameters."""
        _hip.check(self.lib.rx_mlp_refresh_images(ctypes.byref(self.opt), self._od,
                                                   ctypes.c_void_p(self.params.data_ptr()),
                                                   _hip.stream_ptr(self.device)), "refresh_images")

    def opt_step(self, lr: float, bc1: float, bc2: float, gscale: float = 1.0, first: bool = False):
        pp = ctypes.c_void_p
        _hip.check(self.lib.rx_opt_step(ctypes.byref(self.opt), self._od, pp(self.params.data_ptr()),
                                        pp(self.grads.data_ptr()), pp(self.m.data_ptr()),
                                        pp(self.v.data_ptr()), ctypes.c_float(lr), ctypes.c_float(bc1),
                                        ctypes.c_float(bc2), ctypes.c_float(gscale), int(first),
                                        _hip.stream_ptr(self.device)), "rx_opt_step")

    # ----------------------------------------------------------------------- running ------
    def _lr(self, t: int) -> float:
        return float(self.lr_schedule(t)) if self.lr_schedule is not None else float(self.cfg["lr"])

    def train_epoch(self, feats: torch.Tensor, labels: torch.Tensor, n_rows: int,
                    perm: Optional[torch.Tensor], allreduce: Optional[Callable] = None,
                    world_size: int = 1, drop_last: bool = False, comm=None,
                    max_steps: Optional[int] = None, xg=None) -> Dict[str, float]:
        """Run one epoch. Multi-GPU: ``comm`` (a :class:`raydp_amd.ops.comm.NativeComm`) puts
        the gradient all-reduce inside the native step loop; otherwise ``allreduce(grads)``
        (sum) is called from Python between backward and step. ``xg`` (a
        :class:`raydp_amd.ops.comm.XgmiComm`) instead fuses a one-shot xGMI all-reduce into the
        optimizer kernel. ``max_steps`` caps the step count (ranks agree on it so every
        collective is matched)."""
        self._check_operands(feats, labels, n_rows, perm)
        nsteps = n_rows // self.batch if drop_last else -(-n_rows // self.batch)
        if max_steps is not None:
            nsteps = min(nsteps, int(max_steps))
        self.metrics.zero_()
        if nsteps == 0:
            return self._read_metrics()
        b1, b2 = self.opt.b1, self.opt.b2
        # per-step learning rate and Adam bias corrections, vectorised (a Python loop here costs
        # ~5 us per step of host time in front of the epoch's first launch)
        t = np.arange(self.step_count + 1, self.step_count + nsteps + 1, dtype=np.float64)
        if self.lr_schedule is None:
            lr_np = np.full(nsteps, float(self.cfg["lr"]), dtype=np.float32)
        else:
            lr_np = np.array([self._lr(self.step_count + s) for s in range(nsteps)], dtype=np.float32)
        bc1_np = (1.0 - np.power(float(b1), t)).astype(np.float32)
        bc2_np = (1.0 - np.power(float(b2), t)).astype(np.float32)
        fptr = ctypes.POINTER(ctypes.c_float)
        lrs, bc1, bc2 = (a.ctypes.data_as(fptr) for a in (lr_np, bc1_np, bc2_np))
        stream = _hip.stream_ptr(self.device)
        pp = ctypes.c_void_p
        perm_p = pp(perm.data_ptr()) if perm is not None else pp(0)
        gscale = 1.0 / world_size
        mw_snap = None
        if self.G > 1:
            # device snapshot of what the epoch mutates (one multi-tensor copy into kept buffers):
            # a grid-barrier timeout rolls the epoch back (see below)
            live = self._mw_live()
            mw_snap = getattr(self, "_mw_snap", None)
            if mw_snap is None:
                mw_snap = self._mw_snap = [torch.empty_like(t) for t in live]
            torch._foreach_copy_(mw_snap, live)
        if comm is None and allreduce is None and (xg is not None or world_size == 1) and \
                self._run_persistent(feats, labels, n_rows, perm_p, nsteps, lr_np, bc1_np, bc2_np, stream, xg):
            self.last_path = "persistent_xgmi_tiles" if xg is not None else "persistent"
        elif xg is not None:
            # multi-workgroup step: per-tile gradient exchange in the optimizer tasks; one workgroup:
            # the optimizer kernel reduces from the peers' exported activations
            self.last_path = "mw_xgmi_tiles" if self.G > 1 else "steps_xgmi_activations"
            mw_stamps = None
            if self.G > 1 and self.record_steps:
                mw_stamps = self._dev_buf("stamps", 32 + nsteps + 1 + _PS_LAYER_STAMPS, torch.int64)
                mw_stamps.zero_()
                self.bufs.stamps = mw_stamps.data_ptr()
            rc = self.lib.rx_mlp_train_steps_xg(
                ctypes.byref(self.desc), ctypes.byref(self.bufs), ctypes.byref(self.opt), self._od, self.mt,
                pp(self.m.data_ptr()), pp(self.v.data_ptr()),
                pp(feats.data_ptr()), pp(labels.data_ptr()), perm_p, n_rows, self.batch, 0, nsteps,
                lrs, bc1, bc2, ctypes.c_float(gscale), int(self.step_count == 0), stream, pp(xg.ctx))
            self.bufs.stamps = 0
            _hip.check(rc, "rx_mlp_train_steps_xg")
            if mw_stamps is not None:
                self._mw_stamps_dev = mw_stamps
        elif comm is not None or allreduce is None:
            self.last_path = "steps_rccl" if comm is not None else ("mw_steps" if self.G > 1 else "steps")
            mw_stamps = None
            if self.G > 1 and self.record_steps:
                # multi-workgroup epoch: workgroup 0 of every step stores the step's start time
                mw_stamps = self._dev_buf("stamps", 32 + nsteps + 1 + _PS_LAYER_STAMPS, torch.int64)
                mw_stamps.zero_()
                self.bufs.stamps = mw_stamps.data_ptr()
            ar_fn = comm.fn_ptr if comm is not None else pp(0)
            ar_ctx = pp(comm.ctx) if comm is not None else pp(0)
            rc = self.lib.rx_mlp_train_steps(
                ctypes.byref(self.desc), ctypes.byref(self.bufs), ctypes.byref(self.opt), self._od, self.mt,
                pp(self.m.data_ptr()), pp(self.v.data_ptr()),
                pp(feats.data_ptr()), pp(labels.data_ptr()), perm_p, n_rows, self.batch, 0, nsteps,
                lrs, bc1, bc2, ctypes.c_float(gscale), int(self.step_count == 0), stream, ar_fn, ar_ctx)
            self.bufs.stamps = 0
            _hip.check(rc, "rx_mlp_train_steps")
            if mw_stamps is not None:
                self._mw_stamps_dev = mw_stamps
        else:
            self.last_path = "steps_host_allreduce"
            for s in range(nsteps):
                rc = self.lib.rx_mlp_fwdbwd(
                    ctypes.byref(self.desc), ctypes.byref(self.bufs), self.mt,
                    pp(feats.data_ptr()), pp(labels.data_ptr()), perm_p, n_rows, self.batch, s, stream)
                _hip.check(rc, "rx_mlp_fwdbwd")
                _hip.check(self.lib.rx_mlp_wgrad(ctypes.byref(self.opt), self._od, ctypes.byref(self.bufs),
                                                 stream), "rx_mlp_wgrad")
                allreduce(self.grads[:self.total])
                rc = self.lib.rx_opt_step(ctypes.byref(self.opt), self._od, pp(self.params.data_ptr()),
                                          pp(self.grads.data_ptr()), pp(self.m.data_ptr()),
                                          pp(self.v.data_ptr()), ctypes.c_float(lrs[s]),
                                          ctypes.c_float(bc1[s]), ctypes.c_float(bc2[s]),
                                          ctypes.c_float(gscale), int(self.step_count + s == 0), stream)
                _hip.check(rc, "rx_opt_step")
        self.step_count += nsteps
        self.steps_in_epoch = nsteps
        if xg is not None and not getattr(self, "_voted", False):
            # epoch-end agreement over xGMI, read with the metrics (one D2H copy)
            xg.vote(self.metrics[7:8])
        self._voted = False
        pre, self._metrics_np = getattr(self, "_metrics_np", None), None
        if self.G > 1 and pre is None:
            # the multi-workgroup barriers' timeout word comes back with the metrics (one sync)
            mws = getattr(self, "_mw_stamps_dev", None)
            self._mw_stamps_dev = None
            back = self._readback([self.mw_ctl[2:3], self.metrics] + ([mws] if mws is not None else []))
            if mws is not None:
                # step starts only (no end stamp): the last step's time is not recorded
                st = back[2].copy()
                self._step_stamps = st[:32 + nsteps] if nsteps > 1 else None
                self._mw_layer_stamps = st[32 + nsteps + 1:]   # (RAYDP_MLP_LAYER_STAMPS builds)
            if int(back[0][0]) != 0:
                # from the timed-out step on, the steps stored no gradients and the optimizer
                # updated nothing; roll the whole epoch back and clear the control words so the
                # trainer is usable again
                if mw_snap is not None:
                    torch._foreach_copy_(self._mw_live(), mw_snap)
                    self.step_count -= nsteps
                self.mw_ctl.zero_()
                if self.mw_wctr is not None:
                    self.mw_wctr.zero_()
                if self.mw_lcnt is not None:   # the done counters restart with the launch count
                    self.mw_lcnt.zero_()
                    self._mw_args.fseq = 0
                self.metrics.zero_()
                raise RuntimeError("fused MLP multi-workgroup step: a grid barrier wait timed out "
                                   "(a step workgroup was not resident); the epoch was rolled back")
            pre = back[1].copy()
        out = self._read_metrics(pre)
        if xg is not None and out["xg_vote"] != 0.0:
            from raydp_amd.exceptions import CollectiveError
            raise CollectiveError("xGMI all-reduce: a peer did not arrive within the timeout "
                                  f"(vote {out['xg_vote']:g})")
        return out

    def _mw_live(self):
        return [self.params, self.m, self.v, self.rstats, self.img]

    def step_times_us(self) -> Optional[np.ndarray]:
        """Device time of every step of the last persistent epoch (microseconds; the 100 MHz
        wall clock), or None when it was not recorded (``record_steps``)."""
        st = getattr(self, "_step_stamps", None)
        if st is None:
            return None
        self._step_stamps = None
        t = np.asarray(st)[32:].astype(np.float64)
        if t.size > _PS_LAYER_STAMPS and not t[-_PS_LAYER_STAMPS:].any():
            t = t[:-_PS_LAYER_STAMPS]       # a persistent epoch's buffer: drop the layer-stamp tail
        t = t[t > 0] if t.size and (t <= 0).any() else t
        return np.diff(t) * 0.01 if t.size > 1 else None

    def snapshot(self):
        """Device copy of everything an epoch mutates (see :meth:`restore`)."""
        return ([t.clone() for t in (self.params, self.m, self.v, self.rstats, self.img)],
                self.step_count)

    def restore(self, snap):
        tensors, step = snap
        for dst, src in zip((self.params, self.m, self.v, self.rstats, self.img), tensors):
            dst.copy_(src)
        self.step_count = step
        self.metrics.zero_()

    def _run_persistent(self, feats, labels, n_rows, perm_p, nsteps, lr_np, bc1_np, bc2_np, stream, xg=None) -> bool:
        """The whole epoch as one persistent launch (csrc/hip/mlp_persist.h); False when this
        model / configuration cannot use it (the caller then runs the launch-per-step loop).
        ``xg`` (world > 1): the gradients are exchanged over xGMI inside the launch; every rank
        decides alike (same model, same device type), so ranks never mix the two loops."""
        if self.desc.wgrad_mode != 1 or not persistent_enabled() or self.desc.front_n or self.G > 1:
            # (an embedding front's tables are updated between steps by the optimizer kernel,
            # which the persistent epoch does not run)
            return False
        if getattr(self, "_ps_grid", None) is None:
            self._ps_grid = int(self.lib.rx_ps_grid_blocks(ctypes.byref(self.opt)))
            self._ps_sync = torch.zeros(int(self.lib.rx_ps_sync_words()), dtype=torch.int32, device=self.device)
            self._ps_err = int(self.lib.rx_ps_err_index())
            props = torch.cuda.get_device_properties(self.device)
            # ranks sharing the device (rehearsals) wait on each other inside their launches: all
            # of their grids must be resident together
            share = self.share if self.world > 1 else 1
            self._ps_ok = self._ps_grid * share <= int(props.multi_processor_count)
        if not self._ps_ok:
            return False
        pp = ctypes.c_void_p
        # the per-step schedule goes up from a pinned staging buffer (no synchronous copy)
        sched_h = self._host_buf("sched", 3 * nsteps, torch.float32)
        sched_np = sched_h.numpy()
        sched_np[:nsteps], sched_np[nsteps:2 * nsteps], sched_np[2 * nsteps:] = lr_np, bc1_np, bc2_np
        sched = sched_h.to(self.device, non_blocking=True)
        from raydp_amd.utils.config import get as conf_get
        timeout = float(conf_get("spark.ray.mi355x.mlp_persistent.timeout_s"))
        # device-side snapshot of the state the epoch mutates: a wait that times out (the grid was
        # admitted but a co-tenant still starved a workgroup) rolls back and reruns the epoch on
        # the launch-per-step loop instead of failing the fit. One multi-tensor copy into
        # buffers kept across epochs.
        live = [self.params, self.m, self.v, self.rstats, self.img]
        snap = getattr(self, "_snap", None)
        if xg is None:       # (world > 1 never reruns an epoch locally: nothing to roll back to)
            if snap is None:
                snap = self._snap = [torch.empty_like(t) for t in live]
            torch._foreach_copy_(snap, live)
        stamps = None
        if self.record_steps:
            # device wall clock at every step start (csrc/hip/mlp_persist.h RX_PS_STEP_STAMPS)
            stamps = self._dev_buf("stamps", 32 + nsteps + 1 + _PS_LAYER_STAMPS, torch.int64)
            stamps.zero_()
            self.bufs.stamps = stamps.data_ptr()
        rc = self.lib.rx_mlp_train_persistent(
            ctypes.byref(self.desc), ctypes.byref(self.bufs), ctypes.byref(self.opt), self._od, self.mt,
            pp(self.m.data_ptr()), pp(self.v.data_ptr()), pp(feats.data_ptr()), pp(labels.data_ptr()), perm_p,
            n_rows, self.batch, nsteps, pp(sched.data_ptr()), int(self.step_count == 0),
            pp(self._ps_sync.data_ptr()), ctypes.c_double(timeout), stream,
            pp(xg.ctx) if xg is not None else pp(0), ctypes.c_float(1.0 / max(1, self.world)),
            int(self.share if xg is not None else 1))
        self.bufs.stamps = 0
        if rc in (-2, -3, -4, -6):
            return False
        _hip.check(rc, "rx_mlp_train_persistent")
        self._ps_sched = sched   # kept alive until the launch has consumed it
        if xg is not None:
            # the epoch-end vote (every rank's xGMI error word) rides the same readback
            xg.vote(self.metrics[7:8])
            self._voted = True
        # ONE synchronisation for everything the epoch reports: the wait-timeout word, the
        # metrics and the step stamps come back together
        back = self._readback([self._ps_sync[self._ps_err:self._ps_err + 1], self.metrics] +
                              ([stamps] if stamps is not None else []))
        self._step_stamps = back[2].copy() if stamps is not None else None
        if int(back[0][0]) != 0 and xg is not None:
            # world > 1: no local rerun (the ranks would leave the same collective schedule). This
            # rank fails the epoch; its peers' waits on it time out and fail their votes: every rank
            # raises, and the worker group restarts from its newest checkpoint
            from raydp_amd.exceptions import CollectiveError
            xg._inject_error()
            raise CollectiveError("persistent fused-MLP epoch at world > 1: a wait timed out")
        if int(back[0][0]) != 0:
            import warnings
            warnings.warn("persistent fused-MLP epoch: a workgroup wait timed out; rolled back and "
                          "rerunning the epoch on the launch-per-step loop")
            torch._foreach_copy_(live, snap)
            self.metrics.zero_()
            self._step_stamps = None
            self._ps_ok = False          # this trainer stays on the step loop from now on
            self.persistent_fallbacks = getattr(self, "persistent_fallbacks", 0) + 1
            return False
        self._metrics_np = back[1].copy()
        return True

    def _host_buf(self, key, n, dtype) -> torch.Tensor:
        """A pinned host buffer of at least ``n`` elements kept across epochs (first ``n`` used)."""
        bufs = self.__dict__.setdefault("_host_bufs", {})
        b = bufs.get((key, dtype))
        if b is None or b.numel() < n:
            b = torch.empty(max(n, 64), dtype=dtype, pin_memory=self.device.type == "cuda")
            bufs[(key, dtype)] = b
        return b[:n]

    def _dev_buf(self, key, n, dtype) -> torch.Tensor:
        bufs = self.__dict__.setdefault("_dev_bufs", {})
        b = bufs.get((key, dtype))
        if b is None or b.numel() < n:
            b = torch.empty(max(n, 64), dtype=dtype, device=self.device)
            bufs[(key, dtype)] = b
        return b[:n]

    def _readback(self, tensors) -> List[np.ndarray]:
        """Copy device tensors into pinned host buffers and synchronise once; the returned
        arrays alias those buffers (valid until the next readback)."""
        hs = []
        for i, t in enumerate(tensors):
            h = self._host_buf(f"rb{i}", t.numel(), t.dtype)
            h.copy_(t.reshape(-1), non_blocking=True)
            hs.append(h)
        torch.cuda.current_stream(self.device).synchronize()
        return [h.numpy() for h in hs]

    def _check_operands(self, feats, labels, n_rows, perm=None):
        """Host-side guard: the kernels index rows [0, n_rows) of feats / labels (through perm)
        without bounds checks, so a mismatch must never reach the GPU."""
        def here(t):
            return t.device.type == self.device.type and (self.device.index is None or t.device.index is None
                                                          or t.device.index == self.device.index)
        if not here(feats) or not here(labels):
            raise ValueError("features / labels must live on the trainer's device")
        if feats.dtype != torch.bfloat16 or feats.dim() != 2 or feats.shape[1] != self.feat_k or \
                not feats.is_contiguous():
            raise ValueError(f"features must be a contiguous bf16 [rows, {self.feat_k}] matrix")
        if labels.dtype != torch.float32 or not labels.is_contiguous() or labels.numel() < n_rows * self.desc.out_dim:
            raise ValueError("labels must be contiguous fp32 with n_rows * out_dim elements")
        if n_rows < 0 or feats.shape[0] < n_rows:
            raise ValueError(f"n_rows={n_rows} exceeds the {feats.shape[0]} feature rows")
        if perm is not None and (perm.dtype != torch.int32 or perm.numel() < n_rows or not here(perm)):
            raise ValueError("perm must be an int32 permutation of n_rows on the trainer's device")

    def forward_backward(self, feats: torch.Tensor, labels: torch.Tensor, n_rows: int,
                         perm: Optional[torch.Tensor] = None, step: int = 0) -> torch.Tensor:
        """One fused fwd/bwd (no optimizer) — returns the flat fp32 gradient (for tests)."""
        self._check_operands(feats, labels, n_rows, perm)
        pp = ctypes.c_void_p
        self.metrics.zero_()
        rc = self.lib.rx_mlp_fwdbwd(
            ctypes.byref(self.desc), ctypes.byref(self.bufs), self.mt,
            pp(feats.data_ptr()), pp(labels.data_ptr()),
            pp(perm.data_ptr()) if perm is not None else pp(0), n_rows, self.batch, step,
            _hip.stream_ptr(self.device))
        _hip.check(rc, "rx_mlp_fwdbwd")
        _hip.check(self.lib.rx_mlp_wgrad(ctypes.byref(self.opt), self._od, ctypes.byref(self.bufs),
                                         _hip.stream_ptr(self.device)), "rx_mlp_wgrad")
        return self.grads[:self.total]

    def unflatten(self, flat: torch.Tensor) -> Dict[str, torch.Tensor]:
        """Map a flat vector (params/grads) onto ``{module_param_name: tensor}`` by identity."""
        out = {}
        for kind, mod, off, n in self.layout:
            attr = _ATTR[kind]
            out[(id(mod), attr)] = flat[off:off + n].view_as(getattr(mod, attr))
        return out

    def evaluate(self, feats: torch.Tensor, labels: torch.Tensor, n_rows: int) -> Dict[str, float]:
        self._check_operands(feats, labels, n_rows)
        self.metrics.zero_()
        pp = ctypes.c_void_p
        rc = self.lib.rx_mlp_eval(ctypes.byref(self.desc), ctypes.byref(self.bufs), self.mt,
                                  pp(feats.data_ptr()), pp(labels.data_ptr()), n_rows, self.batch,
                                  _hip.stream_ptr(self.device))
        _hip.check(rc, "rx_mlp_eval")
        return self._read_metrics()

    def _read_metrics(self, m: Optional[np.ndarray] = None) -> Dict[str, float]:
        if m is None:
            m = self.metrics.cpu().numpy()
        if m[6] > 0:
            raise IndexError("embedding id out of range in the fused trainer's input "
                             f"({int(m[6])} batch(es) clamped)")
        nb = max(m[4], 1.0)
        cnt = max(m[3], 1.0)
        return {"loss": float(m[0] / nb), "mae": float(m[1] / cnt), "mse": float(m[2] / cnt),
                "acc": float(m[5] / cnt), "count": float(m[3]), "batches": float(m[4]),
                "xg_vote": float(m[7])}

    # ----------------------------------------------------------------------- state --------
    @torch.no_grad()
    def write_back(self):
        """Copy fp32 master params / BN running stats back into the user's modules (one D2H
        copy of each flat buffer, then host-side slicing)."""
        p = self.params.detach().to("cpu", non_blocking=False)
        rs = self.rstats.detach().to("cpu", non_blocking=False) if self.run_bufs else None
        for kind, mod, off, n in self.layout:
            t = _ATTR[kind]
            dst = getattr(mod, t)
            dst.data.copy_(p[off:off + n].view_as(dst).to(dst.dtype))
        base = self.rstats.data_ptr()
        for bn, rm, rv in self.run_bufs:
            o = (rm.data_ptr() - base) // 4
            bn.running_mean.copy_(rs[o:o + rm.numel()])
            o = (rv.data_ptr() - base) // 4
            bn.running_var.copy_(rs[o:o + rv.numel()])
            if bn.num_batches_tracked is not None:
                bn.num_batches_tracked.add_(getattr(self, "_tracked_pending", 0))
        self._tracked_total = getattr(self, "_tracked_total", 0) + getattr(self, "_tracked_pending", 0)
        self._tracked_pending = 0

    @torch.no_grad()
    def state_dict_from_buffers(self, model: torch.nn.Module):
        """``model.state_dict()`` as :meth:`write_back` would leave it, built from the device
        buffers without touching ``model`` (whose modules the layout references): trained
        entries and running statistics are views of one host copy of each flat buffer (two
        storages in ``model.pt``), the rest are the module's own."""
        import collections
        names = {id(m): n for n, m in model.named_modules()}
        out = collections.OrderedDict(model.state_dict())
        p = self.params.detach().to("cpu")
        rs = self.rstats.detach().to("cpu") if self.run_bufs else None

        def key(mod, attr):
            n = names[id(mod)]
            return f"{n}.{attr}" if n else attr
        for kind, mod, off, n in self.layout:
            attr = _ATTR[kind]
            ref = getattr(mod, attr)
            out[key(mod, attr)] = p[off:off + n].view_as(ref).to(ref.dtype)
        base = self.rstats.data_ptr()
        tracked = getattr(self, "_tracked_total", 0) + getattr(self, "_tracked_pending", 0)
        for bn, rm, rv in self.run_bufs:
            o = (rm.data_ptr() - base) // 4
            out[key(bn, "running_mean")] = rs[o:o + rm.numel()]
            o = (rv.data_ptr() - base) // 4
            out[key(bn, "running_var")] = rs[o:o + rv.numel()]
            if bn.num_batches_tracked is not None:
                out[key(bn, "num_batches_tracked")] = bn.num_batches_tracked + tracked
        return out

    def note_steps(self, n):
        self._tracked_pending = getattr(self, "_tracked_pending", 0) + n
