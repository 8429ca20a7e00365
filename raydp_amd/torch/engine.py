"""Per-worker training engines behind ``TorchEstimator``.

* ``FusedMLPEngine`` — MI355X fast path. The worker's whole data shard is ingested into HBM
  once (one pinned DMA + the ``arrow_ingest`` HIP kernel); every epoch is one native call that
  enqueues, per batch, the single-workgroup fused fwd/bwd kernel, the (optional) RCCL
  all-reduce and the fused optimizer kernel; the epoch shuffle is a device permutation read by
  the kernel's row gather. Used when the model is a fusable MLP (``models/mlp_spec.py``) --
  optionally behind an embedding front (per-column ``nn.Embedding`` lookups concatenated with
  dense columns, the stroke tutorial's NET_Model: the kernel gathers the table rows and stores
  their gradients itself) -- the loss is MSE/SmoothL1/L1/BCE-with-logits (metrics MAE/MSE/binary
  Accuracy) or class-weighted CrossEntropy over <= 16 classes (argmax Accuracy), the optimizer
  Adam/AdamW/SGD.
* ``TorchLoopEngine`` — any other model. Still device-resident (data ingested once, batches are
  device slices of a permuted index), loss and metrics accumulated on the device and read once
  per epoch; DDP via ``raydp_amd.parallel.ddp`` when ``world_size > 1``. On one GPU the whole
  step (gather, fwd, loss, metrics, bwd, optimizer) is replayed from a captured HIP graph
  (``raydp_amd/torch/graphs.py``).

Both report the reference's per-epoch dicts ``{epoch, train_res, train_loss}`` and
``{epoch, eval_res, test_loss}`` (``python/raydp/torch/estimator.py:245-253``).
"""
import copy
from typing import Any, Callable, Dict, List, Optional

import torch
import torch.nn as nn

from raydp_amd.train import session


def _epoch_seed_base(config) -> int:
    """Per-rank base of the epoch-permutation seeds (``shuffle_seed`` extra config, else 1234)."""
    base = config.get("shuffle_seed")
    base = 1234 if base is None else int(base)
    return (base * 1_000_003 + session.get_world_rank()) * 65_537


def random_permutation(n, seed, device):
    from raydp_amd.ops.ingest import random_permutation as rp
    return rp(n, seed, device)


def _to_tensor_spec(feature_columns, feature_types):
    """Normalise (feature_columns, feature_types) into groups of (cols, dtype)."""
    if feature_columns and isinstance(feature_columns[0], (list, tuple)):
        groups = [list(g) for g in feature_columns]
        if isinstance(feature_types, (list, tuple)):
            dts = list(feature_types)
        else:
            dts = [feature_types] * len(groups)
        return groups, [d or torch.float32 for d in dts], True
    dt = feature_types
    if isinstance(dt, (list, tuple)):
        uniq = {d for d in dt if d is not None}
        if len(uniq) > 1:
            # one tensor per column, each with its own dtype (DLRM-style multi-input models)
            return [[c] for c in feature_columns], [d or torch.float32 for d in dt], True
        dt = uniq.pop() if uniq else torch.float32
    return [list(feature_columns)], [dt or torch.float32], False


_INT_DTYPES = (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8)


class _ShardTensors:
    """A worker's shard, resident in HBM. Multi-input models (one tensor per column, as DLRM's
    13 dense + 26 categorical inputs) are ingested as ONE float matrix and ONE exact int64
    matrix (one DMA-fed ingest launch each), and a batch is one row gather per matrix whose
    column views are the model inputs."""

    def __init__(self, ds, feature_columns, feature_types, label_column, label_type, device,
                 fused_stride: Optional[int] = None, streamed: Optional[dict] = None):
        from raydp_amd.ops.ingest import ingest_columns
        self.groups, self.dtypes, self.multi = _to_tensor_spec(feature_columns, feature_types)
        self.device = device
        self.feats = None
        if streamed is not None and fused_stride is not None:
            self._from_stream(ds, streamed, label_column, label_type, fused_stride)
            return
        tables = ds._get_tables() if ds is not None else []
        self.n = int(sum(t.num_rows for t in tables))
        if fused_stride is not None:
            self.feats_bf16 = ingest_columns(tables, self.groups[0], device, True, fused_stride)
        elif self.multi and all(len(g) == 1 for g in self.groups):
            # one matrix per kind; group i -> (kind, column j)
            kinds = ["i" if d in _INT_DTYPES else "f" for d in self.dtypes]
            self.mats, self.where = {}, []
            for kind in ("f", "i"):
                cols = [g[0] for g, k in zip(self.groups, kinds) if k == kind]
                if cols:
                    self.mats[kind] = ingest_columns(tables, cols, device, False, out_i64=(kind == "i"))
            pos = {"f": 0, "i": 0}
            for k, d in zip(kinds, self.dtypes):
                self.where.append((k, pos[k], d))
                pos[k] += 1
            self.feats = self._views(self.mats)
        else:
            self.feats = [ingest_columns(tables, g, device, False, out_i64=d in _INT_DTYPES).to(d)
                          for g, d in zip(self.groups, self.dtypes)]
        lab = ingest_columns(tables, [label_column], device, False,
                             out_i64=(label_type in _INT_DTYPES)) if label_column is not None else None
        self.labels = lab.to(label_type or torch.float32) if lab is not None else None

    def _from_stream(self, ds, streamed, label_column, label_type, stride):
        """The fused matrix from blocks already ingested while the conversion ran
        (:func:`stream_ingest`), in partition order; a block that did not stream (or whose final
        reference differs: a retried task) is ingested now."""
        from raydp_amd.data.dataset import _resolve
        from raydp_amd.runtime.objects import ObjectRef
        fp, lp, n = [], [], 0
        for j, b in enumerate(ds._blocks):
            p = streamed.get(j)
            if p is None or not isinstance(b, ObjectRef) or p[0] != b.id:
                t = _resolve(b)
                p = _ingest_block(t, self.groups[0], label_column, self.device, stride)
            _, rows, f, lab = p
            fp.append(f)
            lp.append(lab)
            n += rows
        self.n = n
        self.feats_bf16 = fp[0] if len(fp) == 1 else torch.cat(fp)
        lab = lp[0] if len(lp) == 1 else torch.cat(lp)
        self.labels = lab.to(label_type or torch.float32)

    def _views(self, mats):
        out = []
        for k, j, d in self.where:
            v = mats[k][:, j:j + 1]
            out.append(v if v.dtype == d else v.to(d))
        return out

    def batch(self, sel):
        """Inputs and labels of rows ``sel`` (device index tensor) or of a slice."""
        if getattr(self, "mats", None) is not None:
            if isinstance(sel, slice):
                mats = {k: m[sel] for k, m in self.mats.items()}
            else:
                mats = {k: m.index_select(0, sel) for k, m in self.mats.items()}
            feats = self._views(mats)
        elif isinstance(sel, slice):
            feats = [f[sel] for f in self.feats]
        else:
            feats = [f.index_select(0, sel) for f in self.feats]
        lab = self.labels[sel] if isinstance(sel, slice) else self.labels.index_select(0, sel)
        return feats, lab


def _ingest_block(t, cols, label_column, device, stride):
    """(object id, rows, bf16 features [rows, stride], fp32 labels [rows, 1]) of one Arrow block."""
    from raydp_amd.ops.ingest import ingest_columns
    f = ingest_columns([t], cols, device, True, stride)
    lab = ingest_columns([t], [label_column], device, False)
    return None, t.num_rows, f, lab


def stream_ingest(ds, cols, label_column, device, stride) -> dict:
    """Ingest the blocks of a deferred dataset (``ds._stream``: ``(partition, ref)`` as each
    conversion task lands, raydp_amd/spark/cluster.py set_block_hook) while its conversion still
    runs; returns ``{partition: (object id, rows, features, labels)}`` once it finished. The DMA of
    a block overlaps the ETL of the later ones, so after the stage only its last block's copy is
    left (reference: the per-partition fetch tasks of python/raydp/spark/dataset.py:203-222 feed
    Ray Data blocks to the trainer the same way, block by block)."""
    import queue
    from raydp_amd.data.dataset import _resolve
    q, fut = ds._stream, ds._pending
    parts = {}
    while True:
        # blocking get: the conversion thread ends the stream with None (no polling loop taking
        # the GIL from the conversion's own Python)
        try:
            item = q.get(timeout=0.25)
        except queue.Empty:
            if fut is None or fut.done():     # (a conversion that died before its sentinel)
                break
            continue
        if item is None:
            break
        i, ref = item
        t = _resolve(ref)
        parts[i] = (ref.id,) + _ingest_block(t, cols, label_column, device, stride)[1:]
    return parts


class FusedMLPEngine:
    name = "fused_mlp_hip"

    @staticmethod
    def applicable(model, optimizer, loss, metrics, device, batch_size, feature_columns,
                   feature_types) -> Optional[tuple]:
        if device.type != "cuda":
            return None
        from raydp_amd.models.mlp_spec import extract_mlp_spec
        from raydp_amd.ops.fused_mlp import fused_batch_ok, loss_code, optimizer_config, pick_mt
        if not fused_batch_ok(batch_size):
            return None
        if feature_columns and isinstance(feature_columns[0], (list, tuple)):
            return None
        if isinstance(feature_types, (list, tuple)) and len({t for t in feature_types}) > 1:
            return None
        spec = extract_mlp_spec(model)
        lc = loss_code(loss)
        oc = optimizer_config(optimizer)
        if spec is None or lc is None or oc is None:
            return None
        if (spec.raw_features or spec.in_features) != len(feature_columns):
            return None
        if pick_mt(batch_size) is None and (spec.front or lc[0] == 4):
            return None     # the multi-workgroup step (batch > 128) has neither
        if lc[0] == 4:
            # cross entropy: the classes of one 16-wide output tile; accuracy is the argmax,
            # counted by the kernel (regression metrics do not apply)
            if not 2 <= spec.out_features <= 16 or not _argmax_accuracy_only(metrics, spec.out_features):
                return None
            return spec, lc, oc, None
        acc_thr = _binary_accuracy_threshold(metrics)
        if acc_thr is False:
            return None
        if acc_thr is not None and spec.out_features != 1:
            return None
        return spec, lc, oc, acc_thr

    def __init__(self, model, optimizer, spec, lc, oc, acc_thr, metrics, device, config, lr_scheduler_fn,
                 detached: bool = False, loss=None):
        """``detached``: ``model`` / ``optimizer`` are the caller's own objects, only read here
        (parameters, running statistics, hyper-parameters and moments are copied to the device
        once); results are exported from the device buffers and the objects are never written."""
        from raydp_amd.ops.fused_mlp import FusedMLPTrainer
        from raydp_amd.utils import tracing
        self.model, self.metrics_names, self.device = model, metrics.names, device
        self.detached = detached
        self.loss = loss if loss is not None else config.get("loss")   # label encoding (fused_labels)
        self.world = session.get_world_size()
        with tracing.span("fused trainer build", cat="train"):
            self.trainer = FusedMLPTrainer(spec, oc, lc, config["batch_size"], device, lr_scheduler_fn,
                                           acc_thr=acc_thr, world=session.get_world_size())
        from raydp_amd.utils.config import get as conf_get
        self.trainer.record_steps = bool(conf_get("spark.ray.mi355x.step_times"))
        self.last_step_times = None
        self.optimizer = optimizer
        self.trainer.load_optimizer_state(optimizer)
        self.xg, self.comm, self.ar = None, None, None
        self.allreduce_kind = None
        self.max_steps = None
        if self.world > 1:
            with tracing.span("collectives setup", cat="train", world=self.world):
                self._setup_collectives()
        self.drop_last = bool(config.get("drop_last", False))
        self.shuffle = bool(config.get("shuffle", True))
        self.seed = _epoch_seed_base(config)
        self.equal_shards = bool(config.get("_equal_shards", False))
        self.epoch = 0

    def _setup_collectives(self):
        """World > 1, once per fit: pick the gradient path (xGMI one-shot fused into the
        optimizer kernel, else the native RCCL communicator inside the C++ step loop, else
        ``torch.distributed``) and make every rank start from rank 0's parameters (DDP's
        constructor broadcast, reference ``train.torch.prepare_model`` at
        ``python/raydp/torch/estimator.py:243``) -- over xGMI that broadcast is one one-shot
        all-reduce where every rank but 0 contributes zeros (exact: x + 0 = x)."""
        import torch.distributed as dist
        from raydp_amd.ops.comm import NativeComm
        tr = self.trainer
        from raydp_amd.utils import tracing
        with tracing.span("xgmi communicator", cat="train"):
            self.xg = _xgmi_for(tr)
        if self.xg is not None:
            # gradients exchanged inside the training launches: the persistent epoch (batch <= 128)
            # and the multi-workgroup step's optimizer tasks send per-tile gradients
            self.allreduce_kind = "xgmi_tiles_in_launch" if (tr.G > 1 or persistent_layout(tr)) \
                else "xgmi_oneshot"
            tr.share = self.xg.share
            if tr._mw_args is not None:
                tr._mw_args.share = self.xg.share
            if tr.params.numel() <= self.xg.max_floats:
                if dist.get_rank() != 0:
                    tr.params.zero_()
                self.xg.allreduce_(tr.params)
            else:
                dist.broadcast(tr.params, 0)
        else:
            if dist.get_backend() == "nccl":
                self.comm = NativeComm.from_process_group()
            if self.comm is not None:
                self.allreduce_kind = "rccl_native"
                self.comm.broadcast_(tr.params, 0)
            else:
                self.allreduce_kind = f"torch.distributed:{dist.get_backend()}"
                dist.broadcast(tr.params, 0)

                def ar(g):
                    dist.all_reduce(g)
                self.ar = ar
        tr.refresh_images()

    def stream_ingest(self, train_ds, config):
        """Training blocks into HBM as the conversion lands them (world 1, in-process)."""
        if self.world != 1 or getattr(train_ds, "_stream", None) is None:
            return
        groups, _, _ = _to_tensor_spec(config["feature_columns"], config["feature_types"])
        self._streamed = stream_ingest(train_ds, groups[0], config["label_column"], self.device,
                                       self.trainer.feat_k)

    def load(self, train_ds, eval_ds, config):
        from raydp_amd.ops.fused_mlp import fused_labels
        fc, ft = config["feature_columns"], config["feature_types"]
        k = self.trainer.feat_k
        streamed, self._streamed = getattr(self, "_streamed", None), None
        self.train = _ShardTensors(train_ds, fc, ft, config["label_column"], torch.float32,
                                   self.device, fused_stride=k, streamed=streamed)
        self.eval = _ShardTensors(eval_ds, fc, ft, config["label_column"], torch.float32, self.device,
                                  fused_stride=k) if eval_ds is not None else None
        classes = self.trainer.desc.out_dim
        for sh in (self.train, self.eval):
            if sh is not None and sh.labels is not None:
                sh.labels = fused_labels(self.loss, sh.labels, classes)
        if self.world > 1 and not self.equal_shards:
            # ranks that brought their own data (SPMD local shards) agree once per fit on the
            # step count, so every per-step collective is matched; shards split by the trainer
            # are equal by construction and skip this
            import torch.distributed as dist
            b = self.trainer.batch
            mine = self.train.n // b if self.drop_last else -(-self.train.n // b)
            dev = self.device if dist.get_backend() == "nccl" else "cpu"
            s = torch.tensor([mine], device=dev, dtype=torch.int64)
            dist.all_reduce(s, op=dist.ReduceOp.MIN)
            self.max_steps = int(s.item())

    def _res(self, m):
        out = {}
        if "MeanAbsoluteError" in self.metrics_names:
            out["MeanAbsoluteError"] = m["mae"]
        if "MeanSquaredError" in self.metrics_names:
            out["MeanSquaredError"] = m["mse"]
        for n in ("Accuracy", "BinaryAccuracy"):
            if n in self.metrics_names:
                out[n] = m["acc"]
        return out

    def train_epoch(self):
        """One epoch = one native call. World > 1 adds no host synchronisation of its own: the
        only device read per epoch is the metrics vector, which on the xGMI path also carries
        the epoch-end vote (every rank's peer-timeout word, summed over xGMI). A nonzero vote
        -- seen identically by every rank -- fails this worker (``CollectiveError``): the group
        restarts from the newest epoch checkpoint, with the xGMI path disabled in this
        process (``FailureConfig`` semantics, reference ``torch/estimator.py:331-334``)."""
        t = self.train
        perm = None
        if self.shuffle:
            perm = random_permutation(t.n, self.seed + self.epoch, self.device)
        self.epoch += 1
        if self.xg is not None:
            from raydp_amd.exceptions import CollectiveError
            from raydp_amd.ops.comm import forget_xgmi
            try:
                m = self.trainer.train_epoch(t.feats_bf16, t.labels, t.n, perm, world_size=self.world,
                                             drop_last=self.drop_last, max_steps=self.max_steps, xg=self.xg)
            except CollectiveError:
                forget_xgmi(self.xg, disable=True)
                self.xg = None
                raise
        else:
            m = self.trainer.train_epoch(t.feats_bf16, t.labels, t.n, perm, allreduce=self.ar,
                                         world_size=self.world, drop_last=self.drop_last, comm=self.comm,
                                         max_steps=self.max_steps)
        self.trainer.note_steps(self.trainer.steps_in_epoch)
        st = self.trainer.step_times_us()
        if st is not None:
            from raydp_amd.utils.devmon import step_time_histogram
            self.last_step_times = step_time_histogram(st)
        return self._res(m), m["loss"]

    def evaluate_epoch(self):
        e = self.eval
        m = self.trainer.evaluate(e.feats_bf16, e.labels, e.n)
        return self._res(m), m["loss"]

    def state_dict(self):
        if self.detached:
            return self.trainer.state_dict_from_buffers(self.model)
        self.trainer.write_back()
        return self.model.state_dict()

    def optimizer_state_dict(self):
        opt = self.optimizer
        if self.detached:
            # export into a private optimizer over the same parameter groups, never the caller's
            # (its groups may cover a subset of the model, or several groups)
            priv = type(opt)([dict(g, params=list(g["params"])) for g in opt.param_groups])
            priv.load_state_dict(opt.state_dict())
            opt = priv
        return self.trainer.export_optimizer_state(opt)


def _argmax_accuracy_only(metrics, classes: int) -> bool:
    """Every requested metric is an Accuracy the fused cross-entropy epilogue counts (argmax of
    the logits == label): multiclass with ``classes`` classes, or unspecified."""
    from raydp_amd.torch import metrics as M
    for n in metrics.names:
        m = metrics._metrics.get(n)
        if n not in ("Accuracy", "MulticlassAccuracy") or type(m) not in (M.Accuracy,):
            return False
        kw = getattr(m, "kwargs", {})
        if kw.get("task", "multiclass") != "multiclass" or kw.get("num_classes") not in (None, classes) \
                or kw.get("average", "micro") != "micro" or kw.get("top_k", 1) != 1:
            return False
    return True


def _binary_accuracy_threshold(metrics):
    """The fused kernel computes MAE, MSE and single-output threshold accuracy (the built-in
    ``Accuracy``: ``(pred > threshold).long() == target.long()``). Returns the accuracy
    threshold (None when no accuracy metric is asked for) or False when some metric is
    something else."""
    from raydp_amd.torch import metrics as M
    thr = None
    for n in metrics.names:
        if n in ("MeanAbsoluteError", "MeanSquaredError"):
            continue
        m = metrics._metrics.get(n)
        if n in ("Accuracy", "BinaryAccuracy") and type(m) in (M.Accuracy, M.BinaryAccuracy):
            kw = getattr(m, "kwargs", {})
            if kw.get("task", "binary") != "binary" or kw.get("num_classes") not in (None, 2):
                return False
            thr = float(kw.get("threshold", 0.5))
            continue
        return False
    return thr


def persistent_layout(trainer) -> bool:
    """The trainer's epochs can run as the persistent launch (one-workgroup batch, wgrad mode 1)."""
    from raydp_amd.ops.fused_mlp import persistent_enabled
    return trainer.G == 1 and trainer.desc.wgrad_mode == 1 and not trainer.desc.front_n and persistent_enabled()


def _xgmi_for(trainer):
    """The one-shot xGMI communicator for this trainer's gradient, or None (RCCL instead).

    ``RAYDP_ALLREDUCE`` / ``spark.ray.mi355x.allreduce``: ``auto`` (default: xGMI when every
    rank of the group maps its peers and passes the self-test), ``xgmi`` (same, but failing
    the setup is an error), ``rccl`` (never)."""
    import torch.distributed as dist
    from raydp_amd.ops.comm import XgmiComm
    from raydp_amd.utils.config import get as conf_get
    mode = conf_get("spark.ray.mi355x.allreduce")
    if mode == "rccl" or not torch.cuda.is_available():
        return None
    # the exchange slot: the flat gradient for the in-launch tile exchange of the multi-workgroup
    # step; the whole gradient buffer (flat gradient + exported activations) for one-workgroup
    # batches, whose launch-per-step fallback reduces from the peers' activations
    nf = trainer.total if trainer.G > 1 else trainer.grads.numel()
    xg = XgmiComm.create(nf, timeout_s=conf_get("spark.ray.mi355x.allreduce.timeout_s"), host_seq=True)
    if xg is None and mode == "xgmi":
        raise RuntimeError("spark.ray.mi355x.allreduce=xgmi but the xGMI peer mapping is unavailable")
    return xg


class TorchLoopEngine:
    name = "torch_loop"

    def __init__(self, model, optimizer, loss, metrics, device, config, lr_scheduler):
        self.device = device
        self.world = session.get_world_size()
        self.raw_model = model.to(device)
        self.allreduce_kind = None
        # optimizer state may reference CPU tensors; move them
        for st in optimizer.state.values():
            for k, v in list(st.items()):
                if isinstance(v, torch.Tensor) and k != "step":
                    st[k] = v.to(device)
        self.optimizer, self.loss, self.metrics = optimizer, loss, metrics
        self.scheduler = lr_scheduler
        self._fused_sgd = None          # decided at the first step (needs the gradients)
        self.fusions = []
        if device.type == "cuda":
            self._fuse_hot_ops(config)  # before DDP sees which parameters have sparse gradients
        if self.world > 1:
            from raydp_amd.parallel.ddp import DistributedDataParallel
            self.model = DistributedDataParallel(self.raw_model)
            self.allreduce_kind = self.model._allreduce.kind
        else:
            self.model = self.raw_model
        self.batch = int(config["batch_size"])
        self.drop_last = bool(config.get("drop_last", False))
        self.shuffle = bool(config.get("shuffle", True))
        self.seed = _epoch_seed_base(config)
        self.epoch = 0
        self.graphed = None
        from raydp_amd.torch import graphs
        if graphs.graphs_requested():
            why = graphs.supported(self)
            if why is None:
                self.metrics.to(device)
                self.graphed = graphs.GraphedTrainLoop(self)
                self.name = "torch_loop_hipgraph"
            self.graph_status = why or "enabled"
        else:
            self.graph_status = "disabled (RAYDP_TORCH_GRAPHS=0)"

    def _fuse_hot_ops(self, config=None):
        """Swap the step's eager tails for HIP kernels where the semantics are identical:
        ``BCEWithLogitsLoss()`` -> :class:`raydp_amd.ops.fused_optim.FusedBCEWithLogits`;
        plain-SGD DLRM tables -> the sparse SGD fused into the embedding backward
        (``rx_emb_sgd``: no sparse gradient tensor, no index_add) -- on one GPU, for sharded
        tables, and for tables replicated over the ranks when the trainer's equal shards keep
        every rank's batch the same size: each step's ids and gradient rows are then
        all-gathered over xGMI on the device and every rank applies all of them (the DDP
        sparse all-reduce without its host round trips)."""
        from raydp_amd.ops import fused_optim
        if fused_optim.fusable_bce(self.loss):
            self.loss = fused_optim.FusedBCEWithLogits()
            self.fusions.append("bce_with_logits")
        opt = self.optimizer
        if type(opt) is torch.optim.SGD and self.scheduler is None and all(
                float(g["momentum"]) == 0.0 and float(g["weight_decay"]) == 0.0 and not g.get("maximize", False)
                and not isinstance(g["lr"], torch.Tensor) for g in opt.param_groups):
            from raydp_amd.ops.dlrm_ops import FusedEmbeddings
            lr_of = {id(p): float(g["lr"]) for g in opt.param_groups for p in g["params"]}
            for m in self.raw_model.modules():
                sharded = hasattr(m, "start") and hasattr(m, "finish")
                if isinstance(m, FusedEmbeddings) or sharded:
                    w = getattr(m, "weight", None)
                    if getattr(m, "fused_sgd_lr", 0) is not None or w is None or id(w) not in lr_of:
                        continue
                    if not sharded and self.world > 1:
                        # replicated tables updated locally would diverge: gather every rank's
                        # rows (fixed size per step only with equal shards)
                        sync = self._embedding_sync(m, config)
                        if sync is None:
                            continue
                        m.sync = sync
                        w._raydp_grad_synced = True
                    m.fused_sgd_lr = lr_of[id(w)]
                    w._raydp_sparse_grad = False
                    self.fusions.append("embedding_sgd" if sharded or self.world == 1 else "embedding_sgd_xgmi_gather")

    def _embedding_sync(self, m, config):
        """(xGMI communicator, world) for a replicated table's row all-gather, or None."""
        if not config or not config.get("_equal_shards") or not config.get("drop_last"):
            return None     # ragged last batches would gather rows of different sizes
        from raydp_amd.ops.comm import XgmiComm
        from raydp_amd.utils.config import get as conf_get
        if conf_get("spark.ray.mi355x.allreduce") == "rccl":
            return None
        b = int(config["batch_size"])
        words = b * (len(m.table_sizes) + 1) * m.dim + 64
        comm = XgmiComm.create(words, timeout_s=conf_get("spark.ray.mi355x.allreduce.timeout_s"))
        return (comm, self.world) if comm is not None else None

    def opt_step(self):
        """``optimizer.step()``, on the multi-tensor SGD kernel when it reproduces it (one launch
        per 24 tensors, fused-tower bf16 images written in the same pass)."""
        if self._fused_sgd is None:
            from raydp_amd.ops import fused_optim
            self._fused_sgd = self.device.type == "cuda" and fused_optim.sgd_supported(self.optimizer) is None
            if self._fused_sgd:
                self.fusions.append("multi_tensor_sgd")
        if self._fused_sgd:
            from raydp_amd.ops.fused_optim import sgd_step
            sgd_step(self.optimizer)
        else:
            self.optimizer.step()

    def zero_grad(self):
        """DDP: zero the gradient buckets in place (``.grad`` stays a bucket view, autograd
        accumulates straight into the all-reduced buffer); else drop the gradients."""
        if self.world > 1 and hasattr(self.model, "buckets"):
            self.model.zero_grad()
        else:
            self.optimizer.zero_grad(set_to_none=True)

    def load(self, train_ds, eval_ds, config):
        fc, ft = config["feature_columns"], config["feature_types"]
        lt = config.get("label_type") or torch.float32
        self.train = _ShardTensors(train_ds, fc, ft, config["label_column"], lt, self.device)
        self.eval = _ShardTensors(eval_ds, fc, ft, config["label_column"], lt, self.device) \
            if eval_ds is not None else None

    def _batches(self, data: _ShardTensors, shuffle: bool):
        n = data.n
        idx = None
        if shuffle:
            idx = random_permutation(n, self.seed + self.epoch, self.device).long()
            self.epoch += 1
        stop = n - n % self.batch if self.drop_last else n
        for s in range(0, stop, self.batch):
            feats, lab = data.batch(idx[s:s + self.batch] if idx is not None else slice(s, s + self.batch))
            yield (feats if data.multi else feats[0]), lab

    def _reset_metrics(self):
        if self.graphed is not None:
            self.metrics.zero_()   # captured updates keep pointing at this storage
        else:
            self.metrics.reset()

    def train_epoch(self):
        out = self.graphed.train_epoch() if self.graphed is not None else self._train_epoch_eager()
        if self.world > 1 and hasattr(self.model, "check_comm"):
            # the epoch's metrics readback synced the device already: a timed-out xGMI exchange
            # surfaces here as CollectiveError (the trainer restarts the group) instead of
            # replicas silently training on unsynchronised gradients
            self.model.check_comm()
        return out

    def _train_epoch_eager(self):
        self.model.train()
        total = torch.zeros((), dtype=torch.float64, device=self.device)
        nb = 0
        for inputs, targets in self._batches(self.train, self.shuffle):
            outputs = self.model(*inputs) if isinstance(inputs, list) else self.model(inputs)
            loss = self.loss(outputs, targets)
            total += loss.detach()
            self.metrics.update(outputs, targets)
            self.zero_grad()
            loss.backward()
            self.opt_step()
            if self.scheduler is not None:
                self.scheduler.step()
            nb += 1
        res = self.metrics.compute()
        self._reset_metrics()
        return res, (total / max(nb, 1)).item()

    @torch.no_grad()
    def evaluate_epoch(self):
        self.model.eval()
        total = torch.zeros((), dtype=torch.float64, device=self.device)
        nb = 0
        for inputs, targets in self._batches(self.eval, False):
            outputs = self.model(*inputs) if isinstance(inputs, list) else self.model(inputs)
            total += self.loss(outputs, targets).detach()
            self.metrics.update(outputs, targets)
            nb += 1
        res = self.metrics.compute()
        self._reset_metrics()
        return res, (total / max(nb, 1)).item()

    def state_dict(self):
        return self.raw_model.state_dict()

    def optimizer_state_dict(self):
        return self.optimizer.state_dict()

    def close(self):
        """End of the fit: destroy the captured graphs now. A warm worker keeps running fits;
        left to the garbage collector, a previous fit's graph could be destroyed while the next
        fit's capture is in progress, which HIP refuses (and torch turns into an abort)."""
        if self.graphed is not None:
            self.graphed.close()
