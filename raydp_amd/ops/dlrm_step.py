"""The whole DLRM training step as one persistent HIP launch (``csrc/hip/dlrm_step.hip``).

Covers the reference notebook's training configuration (``examples/pytorch_dlrm.ipynb`` cells
9 and 14: ``Dlrm`` with replicated tables on one GPU, ``torch.optim.SGD`` without momentum or
weight decay, ``BCEWithLogitsLoss()``): forward, loss, backward, the dense SGD and the sparse
embedding SGD of one batch in 14 grid-wide phases of ONE kernel, instead of 21 dependent
launches (``raydp_amd.ops.linear_ops`` towers + ``raydp_amd.ops.dlrm_ops``). The fp32
``nn.Parameter`` storages are the masters and are updated in place, so ``state_dict`` is always
the trained model; the kernel keeps bf16 weight images (row-major and transposed, two parities)
of its own.

Numerics: the same bf16-operand / fp32-accumulate MFMA class as the fused towers; the last
layer (N = 1) and the loss run in fp32 on the fp32 weights.
"""
import ctypes
import math
import os
from typing import List, Optional

import torch

from raydp_amd.ops import _hip

PH_GEMM, PH_BOTTOM, PH_HEAD, PH_IBWD = 0, 1, 2, 3
EPI_FWD, EPI_DGRAD, EPI_WGRAD = 0, 1, 2
MAXPH, MAXBOT = 24, 4
_TILES = [(16, 16), (16, 32), (32, 16), (32, 32), (16, 64), (64, 16), (32, 64), (64, 32), (64, 64)]

vp, ll, i32 = ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int


class GSpec(ctypes.Structure):
    _fields_ = [("A", vp), ("Bm", vp * 2), ("lda", ll), ("ldb", ll),
                ("M", i32), ("N", i32), ("K", i32), ("tm", i32), ("tn", i32), ("epi", i32), ("relu", i32),
                ("pad0", i32),
                ("bias", vp), ("mask", vp), ("ldmask", ll), ("Y", vp), ("ldy", ll), ("YT", vp), ("ldyt", ll),
                ("Yf", vp), ("ldyf", ll),
                ("W", vp), ("kvalid", i32), ("pad1", i32), ("img", vp * 2), ("imgT", vp * 2),
                ("ldimg", ll), ("ldimgT", ll), ("b", vp), ("dyT", vp), ("lddyT", ll), ("brows", i32), ("pad2", i32)]


class Phase(ctypes.Structure):
    _fields_ = [("kind", i32), ("nspec", i32), ("s", GSpec * 2)]


class BotLayer(ctypes.Structure):
    _fields_ = [("img", vp * 2), ("bias", vp), ("N", i32), ("K", i32), ("Kp", i32), ("pad", i32),
                ("H", vp), ("HT", vp)]


class DlrmDesc(ctypes.Structure):
    _fields_ = [("B", i32), ("nph", i32), ("nbot", i32), ("F", i32), ("D", i32), ("ZP", i32), ("G", i32),
                ("pad0", i32),
                ("ph", Phase * MAXPH), ("bot", BotLayer * MAXBOT),
                ("dense", vp), ("ld_dense", ll), ("ndense", i32), ("pad1", i32),
                ("cats", vp), ("ld_cats", ll), ("labels", vp), ("ld_lab", ll),
                ("XdT", vp), ("emb", vp), ("offs", vp), ("emb_rows", ll),
                ("ximg", vp), ("Z", vp), ("ZT", vp),
                ("A_last", vp), ("K_last", i32), ("pad2", i32), ("w_last", vp), ("b_last", vp),
                ("dA", vp), ("dAT", vp), ("logits", vp), ("loss_acc", vp), ("step_loss", vp),
                ("dZ", vp), ("dmlp", vp), ("dmlpT", vp), ("lr", ctypes.c_float), ("pad3", i32),
                ("ctl", vp), ("ticks", ctypes.c_ulonglong), ("stamps", vp), ("head_part", vp),
                ("head_ld", i32), ("pad4", i32)]


_bound = None


def _lib():
    global _bound
    L = _hip.lib()
    if _bound is not L:
        for n in ("rx_dlrm_desc_size", "rx_dlrm_gspec_size", "rx_dlrm_phase_size", "rx_dlrm_max_phases",
                  "rx_dlrm_ctl_words", "rx_dlrm_err_index", "rx_dlrm_parity_index"):
            getattr(L, n).restype = i32
            getattr(L, n).argtypes = []
        for name, cls in (("rx_dlrm_desc_size", DlrmDesc), ("rx_dlrm_gspec_size", GSpec),
                          ("rx_dlrm_phase_size", Phase)):
            if getattr(L, name)() != ctypes.sizeof(cls):
                raise RuntimeError(f"ABI mismatch for {cls.__name__}: {getattr(L, name)()} != {ctypes.sizeof(cls)}")
        if L.rx_dlrm_max_phases() != MAXPH:
            raise RuntimeError("ABI mismatch: phase table size")
        L.rx_dlrm_resident.argtypes = [i32, i32, i32]
        L.rx_dlrm_resident.restype = i32
        L.rx_dlrm_train_steps.argtypes = [vp, i32, i32, i32, i32, vp, ll, i32, i32, vp]
        L.rx_dlrm_train_steps.restype = i32
        L.rx_dlrm_ticks.argtypes = [ctypes.c_double]
        L.rx_dlrm_ticks.restype = ctypes.c_ulonglong
        _bound = L
    return L


def _p(t: Optional[torch.Tensor]) -> int:
    return t.data_ptr() if t is not None else 0


def _ru(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def _job_cost(tm, tn, K):
    """Rough seconds of one tile job: its operand bytes at ~100 GB/s per CU plus one ~0.7 us
    round trip per load burst (a wave handles a quarter of the K steps)."""
    ms, ns = tm // 16, tn // 16
    kc = min(8, 32 // (ms + ns))
    bursts = math.ceil(math.ceil((K // 32) / 4) / kc)
    return (tm + tn) * K * 2 / 100e9 + 0.7e-6 * bursts


def plan_tiles(shapes, G):
    """Tile (tm, tn) per GEMM of one phase (``shapes`` = [(M, N, K), ...], all jobs of the phase
    share the G workgroups): minimises rounds x slowest job."""
    best = None
    options = [[t for t in _TILES if M % t[0] == 0 and N % t[1] == 0] for M, N, _ in shapes]
    if any(not o for o in options):
        raise ValueError(f"no tile divides {shapes}")

    def rec(i, chosen):
        nonlocal best
        if i == len(shapes):
            jobs = sum((M // tm) * (N // tn) for (M, N, _), (tm, tn) in zip(shapes, chosen))
            t = max(_job_cost(tm, tn, K) for (_, _, K), (tm, tn) in zip(shapes, chosen))
            cost = (math.ceil(jobs / G) * t, jobs)
            if best is None or cost < best[0]:
                best = (cost, list(chosen))
            return
        for t in options[i]:
            rec(i + 1, chosen + [t])
    rec(0, [])
    return best[1]


def supported(model, optimizer, loss, batch: int) -> Optional[str]:
    """None when the persistent step reproduces this configuration's training step, else why not."""
    from raydp_amd.models.dlrm import Dlrm
    from raydp_amd.ops.dlrm_ops import FusedEmbeddings
    if not isinstance(model, Dlrm):
        return "not a Dlrm model"
    if not isinstance(model.embeddings, FusedEmbeddings):
        return "sharded (model-parallel) tables"
    if batch % 32 or not 32 <= batch <= 256:
        return f"batch {batch} (the persistent step takes multiples of 32 up to 256)"
    if model.embedding_dim != 32 or len(model.embeddings.table_sizes) + 1 > 32:
        return "embedding dim != 32 or more than 31 tables"
    bot = model.bottom_mlp.linears
    top = model.top_mlp.linears + [model.out]
    if len(bot) > MAXBOT or bot[0].in_features > 32 or any(l.out_features % 32 for l in bot):
        return "bottom MLP shape"
    if top[-1].out_features != 1 or any(l.out_features % 32 for l in top[:-1]) or top[-1].in_features % 32 \
            or top[-1].in_features > 512:
        return "top MLP shape"
    if any(l.bias is None for l in bot + top):
        return "Linear without bias"
    if type(optimizer) is not torch.optim.SGD:
        return f"optimizer {type(optimizer).__name__}"
    lrs = set()
    for g in optimizer.param_groups:
        if float(g["momentum"]) != 0.0 or float(g["weight_decay"]) != 0.0 or g.get("maximize", False) \
                or g.get("nesterov", False) or isinstance(g["lr"], torch.Tensor):
            return "SGD with momentum / weight decay / tensor lr"
        lrs.add(float(g["lr"]))
    if len(lrs) != 1:
        return "several learning rates"
    covered = {id(p) for g in optimizer.param_groups for p in g["params"]}
    if any(id(p) not in covered for p in model.parameters() if p.requires_grad):
        return "a parameter the optimizer does not update"
    from raydp_amd.ops.fused_optim import fusable_bce, FusedBCEWithLogits
    if not (isinstance(loss, FusedBCEWithLogits) or fusable_bce(loss)):
        return "loss is not BCEWithLogitsLoss()"
    return None


class DlrmStep:
    """Persistent-step trainer bound to one ``Dlrm`` model and batch size on one GPU."""

    def __init__(self, model, lr: float, batch: int, device: torch.device, G: Optional[int] = None,
                 timeout_s: float = 10.0):
        self.model, self.lr, self.B, self.dev = model, float(lr), int(batch), device
        L = _lib()
        B = self.B
        bf = dict(dtype=torch.bfloat16, device=device)
        self.bot = model.bottom_mlp.linears
        self.top = model.top_mlp.linears + [model.out]
        emb = model.embeddings
        self.F = len(emb.table_sizes) + 1
        self.D = model.embedding_dim
        NZ = self.D + self.F * (self.F - 1) // 2 + 1
        self.ZP = _ru(NZ, 32)
        if self.top[0].in_features != NZ:
            raise ValueError("top MLP input width != interaction width")
        cus = torch.cuda.get_device_properties(device).multi_processor_count
        self.G = int(G or os.environ.get("RAYDP_DLRM_STEP_G", 0) or min(cus, 128))
        keep = self._keep = []

        def buf(*shape, dtype=torch.bfloat16):
            t = torch.zeros(*shape, dtype=dtype, device=device)
            keep.append(t)
            return t
        # weight images of every MFMA layer: [parity][N][Kp] and [parity][Kp][N]
        self.layers = []   # (linear, Kp, img, imgT)
        for lin in self.bot + self.top[:-1]:
            N, K = lin.out_features, lin.in_features
            Kp = _ru(K, 32)
            self.layers.append((lin, Kp, buf(2, N, Kp), buf(2, Kp, N)))
        nb = len(self.bot)
        D, ZP = self.D, self.ZP
        self.XdT = buf(self.layers[0][1], B)
        self.H = [(buf(B, l.out_features), buf(l.out_features, B)) if i < nb - 1 else (None, None)
                  for i, l in enumerate(self.bot)]
        self.ximg = buf(B, 32, D)
        self.Z, self.ZT = buf(B, ZP), buf(ZP, B)
        topm = self.top[:-1]
        self.A = [(buf(B, l.out_features), buf(l.out_features, B) if i < len(topm) - 1 else None)
                  for i, l in enumerate(topm)]
        self.dA = [(buf(B, l.out_features), buf(l.out_features, B)) for l in topm]
        self.dZ = buf(B, ZP, dtype=torch.float32)
        self.dmlp, self.dmlpT = buf(B, D), buf(D, B)
        self.dH = [(buf(B, l.in_features), buf(l.in_features, B)) for l in self.bot[1:]]  # grads of H_1..H_{nb-1}
        self.logits = buf(B, dtype=torch.float32)
        self.loss_acc = buf(1, dtype=torch.float64)
        self.step_loss = buf(1, dtype=torch.float32)
        self.head_ld = _ru(self.top[-1].in_features + 4, 4)
        self.head_part = buf(B // 16, self.head_ld, dtype=torch.float32)
        self.ctl = buf(int(L.rx_dlrm_ctl_words()), dtype=torch.int32)
        self._err, self._par = int(L.rx_dlrm_err_index()), int(L.rx_dlrm_parity_index())
        self.ticks = int(L.rx_dlrm_ticks(float(timeout_s)))
        self.desc = DlrmDesc()
        self._build_phases()
        self.lds = self._lds_bytes()
        rc = L.rx_dlrm_resident(D, self.lds, self.G)
        if rc:
            raise RuntimeError(f"persistent DLRM step: {self.G} workgroups with {self.lds} B of LDS are not "
                               f"co-resident (rc {rc})")
        self.desc_dev = None
        self._data_key = None
        self.parity = 0
        self.refresh_images()

    # ------------------------------------------------------------------ plan
    def _spec(self, s: GSpec, A, lda, Bm2, ldb, M, N, K, epi):
        s.A, s.lda, s.ldb = A, lda, ldb
        s.Bm[0], s.Bm[1] = Bm2
        s.M, s.N, s.K, s.epi = M, N, K, epi

    def _gemm_phase(self, specs):
        shapes = [(s.M, s.N, s.K) for s in specs]
        for s, (tm, tn) in zip(specs, plan_tiles(shapes, self.G)):
            s.tm, s.tn = tm, tn
        ph = Phase()
        ph.kind, ph.nspec = PH_GEMM, len(specs)
        for j, s in enumerate(specs):
            ph.s[j] = s
        return ph

    def _fwd(self, li, A, lda, Y, YT, relu=True):
        lin, Kp, img, imgT = self.layers[li]
        s = GSpec()
        self._spec(s, A, lda, (_p(img[0]), _p(img[1])), Kp, self.B, lin.out_features, Kp, EPI_FWD)
        s.bias, s.relu = _p(lin.bias), int(relu)
        s.Y, s.ldy = _p(Y), lin.out_features
        if YT is not None:
            s.YT, s.ldyt = _p(YT), self.B
        return s

    def _dgrad(self, li, dY, out_bf, out_T, out_f32, mask):
        """dX [B x Kp] = dY [B x N] . W (the transposed image [Kp][N])."""
        lin, Kp, img, imgT = self.layers[li]
        N = lin.out_features
        s = GSpec()
        self._spec(s, _p(dY), N, (_p(imgT[0]), _p(imgT[1])), N, self.B, Kp, N, EPI_DGRAD)
        if mask is not None:
            s.mask, s.ldmask = _p(mask), Kp
        if out_bf is not None:
            s.Y, s.ldy = _p(out_bf), Kp
        if out_T is not None:
            s.YT, s.ldyt = _p(out_T), self.B
        if out_f32 is not None:
            s.Yf, s.ldyf = _p(out_f32), out_f32.shape[1]
        return s

    def _wgrad(self, li, dYT, XT):
        """dW [N x Kp] = dY^T [N][B] . X^T [Kp][B]^T, SGD in the epilogue, new images of parity 1 - p."""
        lin, Kp, img, imgT = self.layers[li]
        N = lin.out_features
        s = GSpec()
        self._spec(s, _p(dYT), self.B, (_p(XT), _p(XT)), self.B, N, Kp, self.B, EPI_WGRAD)
        s.W, s.kvalid = _p(lin.weight), lin.in_features
        s.img[0], s.img[1], s.ldimg = _p(img[0]), _p(img[1]), Kp
        s.imgT[0], s.imgT[1], s.ldimgT = _p(imgT[0]), _p(imgT[1]), N
        s.b, s.dyT, s.lddyT, s.brows = _p(lin.bias), _p(dYT), self.B, self.B
        return s

    def _build_phases(self):
        d = self.desc
        B, nb = self.B, len(self.bot)
        d.B, d.nbot, d.F, d.D, d.ZP, d.G = B, nb, self.F, self.D, self.ZP, self.G
        for i, lin in enumerate(self.bot):
            _, Kp, img, _ = self.layers[i]
            bl = d.bot[i]
            bl.img[0], bl.img[1] = _p(img[0]), _p(img[1])
            bl.bias, bl.N, bl.K, bl.Kp = _p(lin.bias), lin.out_features, lin.in_features, Kp
            bl.H, bl.HT = _p(self.H[i][0]), _p(self.H[i][1])
        phases = []
        ph = Phase()
        ph.kind = PH_BOTTOM
        phases.append(ph)
        nt = len(self.top) - 1           # MFMA top layers (the last one runs in HEAD)
        prev, prevld = _p(self.Z), self.ZP
        for j in range(nt):
            li = nb + j
            Y, YT = self.A[j]
            phases.append(self._gemm_phase([self._fwd(li, prev, prevld, Y, YT)]))
            prev, prevld = _p(Y), self.top[j].out_features
        ph = Phase()
        ph.kind = PH_HEAD
        phases.append(ph)
        # top backward: layer j's dY = self.dA[j] (pre-activation gradient, row-major + T)
        for j in range(nt - 1, -1, -1):
            li = nb + j
            dY, dYT = self.dA[j]
            if j > 0:
                Xrow, XT = self.A[j - 1][0], self.A[j - 1][1]
                dg = self._dgrad(li, dY, self.dA[j - 1][0], self.dA[j - 1][1], None, Xrow)
            else:
                XT = self.ZT
                dg = self._dgrad(li, dY, None, None, self.dZ, None)
            phases.append(self._gemm_phase([dg, self._wgrad(li, dYT, XT)]))
        ph = Phase()
        ph.kind = PH_IBWD
        phases.append(ph)
        # bottom backward: layer i's dY: i = nb-1 -> dmlp; else dH[i]
        for i in range(nb - 1, -1, -1):
            dY, dYT = (self.dmlp, self.dmlpT) if i == nb - 1 else self.dH[i]
            XT = self.XdT if i == 0 else self.H[i - 1][1]
            specs = []
            if i > 0:
                specs.append(self._dgrad(i, dY, None, self.dH[i - 1][1], None, self.H[i - 1][0]))
                # dgrad output row-major is needed only as the next dgrad's operand
                if i - 1 > 0:
                    specs[0].Y, specs[0].ldy = _p(self.dH[i - 1][0]), self.layers[i][1]
            specs.append(self._wgrad(i, dYT, XT))
            phases.append(self._gemm_phase(specs))
        if len(phases) > MAXPH:
            raise ValueError("too many phases")
        d.nph = len(phases)
        for k, ph in enumerate(phases):
            d.ph[k] = ph
        d.ndense = self.bot[0].in_features
        emb = self.model.embeddings
        d.emb, d.offs, d.emb_rows = _p(emb.weight), _p(emb.offsets), emb.weight.shape[0]
        d.XdT, d.ximg, d.Z, d.ZT = _p(self.XdT), _p(self.ximg), _p(self.Z), _p(self.ZT)
        last = self.top[-1]
        d.A_last, d.K_last = _p(self.A[-1][0]), last.in_features
        d.w_last, d.b_last = _p(last.weight), _p(last.bias)
        d.dA, d.dAT = _p(self.dA[-1][0]), _p(self.dA[-1][1])
        d.logits, d.loss_acc, d.step_loss = _p(self.logits), _p(self.loss_acc), _p(self.step_loss)
        d.dZ, d.dmlp, d.dmlpT = _p(self.dZ), _p(self.dmlp), _p(self.dmlpT)
        d.lr, d.ctl, d.ticks = self.lr, _p(self.ctl), self.ticks
        d.head_part, d.head_ld = _p(self.head_part), self.head_ld

    def _lds_bytes(self):
        B, D, ZP = self.B, self.D, self.ZP
        need = 0
        d = self.desc
        for k in range(d.nph):
            ph = d.ph[k]
            if ph.kind == PH_GEMM:
                for j in range(ph.nspec):
                    s = ph.s[j]
                    need = max(need, 4 * s.tm * (s.tn + 4) * 4 + s.tm * (s.tn + 8) * 2)
            elif ph.kind == PH_BOTTOM:
                w = max([32] + [max(l.Kp, l.N) for l in d.bot[:d.nbot]])
                need = max(need, 16 * 32 * 8 + 2 * 16 * (w + 8) * 2 + 16 * 32 * (D + 8) * 2 + 16 * (ZP + 8) * 2)
            elif ph.kind == PH_HEAD:
                K = d.K_last
                need = max(need, 16 * (K + 8) * 2 + 4 * K * 4 + 48 * 4)
            else:
                need = max(need, 16 * ZP * 4 + 16 * D * 40 * 2 + 4 * 32 * 40 * 2 + 16 * 32 * 8 + 16 * (D + 8) * 2)
        return _ru(need, 16) + 64   # + the barrier's own __shared__ word

    # ------------------------------------------------------------------ state
    def refresh_images(self):
        """Rebuild the current-parity weight images from the fp32 masters (after any update the
        kernel did not make: an eager step, ``load_state_dict``)."""
        p = self.parity
        with torch.no_grad():
            for lin, Kp, img, imgT in self.layers:
                K = lin.in_features
                img[p].zero_()
                img[p][:, :K].copy_(lin.weight)
                imgT[p].zero_()
                imgT[p][:K].copy_(lin.weight.t())

    def sync_parity(self):
        """Read the device parity word (a sync point): the images of that parity are current."""
        self.parity = int(self.ctl[self._par].item()) & 1
        return self.parity

    def check(self):
        if int(self.ctl[self._err].item()) != 0:
            raise RuntimeError("persistent DLRM step: a grid barrier timed out (workgroups not co-resident?)")

    def bind_data(self, dense: torch.Tensor, cats: torch.Tensor, labels: torch.Tensor):
        """Point the step at a resident shard: dense [n][>=13] fp32, cats [n][T] int64, labels [n]."""
        key = (dense.data_ptr(), dense.stride(0), cats.data_ptr(), cats.stride(0), labels.data_ptr(),
               labels.stride(0))
        if key == self._data_key and self.desc_dev is not None:
            return
        if dense.dtype != torch.float32 or cats.dtype != torch.int64 or dense.stride(-1) != 1 \
                or cats.stride(-1) != 1 or cats.shape[1] != self.F - 1 or dense.shape[1] < self.desc.ndense:
            raise ValueError("persistent DLRM step: dense fp32 [n, 13] and cats int64 [n, T] expected")
        d = self.desc
        d.dense, d.ld_dense = dense.data_ptr(), dense.stride(0)
        d.cats, d.ld_cats = cats.data_ptr(), cats.stride(0)
        d.labels, d.ld_lab = labels.data_ptr(), labels.stride(0)
        self._upload()
        self._data_key = key
        self._bound_tensors = (dense, cats, labels)

    def _upload(self):
        raw = bytes(memoryview(self.desc).cast("B"))
        host = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
        if self.desc_dev is None:
            self.desc_dev = torch.empty(len(raw), dtype=torch.uint8, device=self.dev)
        self.desc_dev.copy_(host)

    def phase_profile(self, perm: torch.Tensor, row0: int = 0, reps: int = 20):
        """Per-phase microseconds of one step (workgroup 0's wall clock after each grid barrier,
        median over ``reps`` steps): [(kind, us), ...]. Trains ``reps`` steps."""
        nph = self.desc.nph
        st = torch.zeros(reps, nph + 1, dtype=torch.int64, device=self.dev)
        hz = float(_lib().rx_dlrm_ticks(1.0))
        try:
            for r in range(reps):
                self.desc.stamps = st[r].data_ptr()
                self._upload()
                self.steps(perm, row0, 1)
            torch.cuda.synchronize(self.dev)
        finally:
            self.desc.stamps = 0
            self._upload()
        d = (st[:, 1:] - st[:, :-1]).double().median(dim=0).values.cpu() * 1e6 / hz
        names = {PH_GEMM: "gemm", PH_BOTTOM: "bottom", PH_HEAD: "head", PH_IBWD: "ibwd"}
        return [(names[self.desc.ph[k].kind], round(float(d[k]), 2)) for k in range(nph)]

    def steps(self, perm: torch.Tensor, row0: int, nsteps: int, nvalid_last: Optional[int] = None):
        """Launch ``nsteps`` steps on rows ``perm[row0 + j * B ...]`` (int64 device permutation)."""
        if self.desc_dev is None:
            raise RuntimeError("bind_data first")
        if perm.dtype != torch.int64 or not perm.is_contiguous():
            raise ValueError("perm must be contiguous int64")
        nv = self.B if nvalid_last is None else int(nvalid_last)
        if nsteps <= 0:
            return
        if row0 + (nsteps - 1) * self.B + nv > perm.numel():
            raise ValueError("steps run past the permutation")
        _hip.check(_lib().rx_dlrm_train_steps(self.desc_dev.data_ptr(), self.D, self.B, self.G, self.lds,
                                              perm.data_ptr(), int(row0), int(nsteps), nv,
                                              _hip.stream_ptr(self.dev)), "rx_dlrm_train_steps")

    def after_training(self):
        """The kernel updated the fp32 masters in place (no ``_version`` bump): make every
        cached bf16 image of the model's own fused towers stale before its next forward."""
        for tower in (getattr(self.model.bottom_mlp, "_fused", None), getattr(self.model, "_top_fused", None)):
            if tower is not None:
                tower._versions = [None] * len(tower.linears)
                tower._managed = [False] * len(tower.linears)
