"""Native RCCL communicator for the fused trainer's C++ step loop (``csrc/comm/rccl_comm.cc``).

``NativeComm.from_process_group()`` builds one communicator per process group: rank 0 draws
an RCCL unique id, the id is broadcast over the existing ``torch.distributed`` group, and every
rank joins. ``fn_ptr`` / ``ctx`` are handed to ``rx_mlp_train_steps`` so each step's gradient
all-reduce is enqueued on the compute stream from C++ (kernel -> all-reduce -> Adam, no Python
between steps).
"""
import ctypes
import os
from typing import Optional

from raydp_amd.ops import _hip

_cache = {}


class NativeComm:
    def __init__(self, world: int, rank: int, uid: bytes, device: int):
        L = _hip.lib()
        L.rx_comm_init.restype = ctypes.c_void_p
        L.rx_comm_init.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        self.lib = L
        self.world, self.rank = world, rank
        self.ctx = L.rx_comm_init(world, rank, uid, device)
        if not self.ctx:
            raise RuntimeError("ncclCommInitRank failed for the native gradient communicator")
        self.fn_ptr = ctypes.cast(L.rx_comm_allreduce, ctypes.c_void_p)

    @staticmethod
    def available() -> bool:
        try:
            return bool(_hip.lib().rx_comm_available())
        except Exception:  # noqa: BLE001
            return False

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(128)
        rc = _hip.lib().rx_comm_unique_id(buf)
        if rc != 0:
            raise RuntimeError(f"ncclGetUniqueId failed ({rc})")
        return buf.raw

    @classmethod
    def from_process_group(cls, group=None) -> Optional["NativeComm"]:
        import torch
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()) or not cls.available():
            return None
        key = id(group) if group is not None else "world"
        if key in _cache:
            return _cache[key]
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        obj = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        comm = cls(world, rank, obj[0], torch.cuda.current_device())
        _cache[key] = comm
        return comm

    def allreduce_(self, t) -> None:
        """In-place sum of a contiguous fp32 CUDA tensor on the current stream."""
        rc = self.lib.rx_comm_allreduce(ctypes.c_void_p(t.data_ptr()), t.numel(), ctypes.c_void_p(self.ctx),
                                        _hip.stream_ptr(t.device))
        _hip.check(rc, "rx_comm_allreduce")

    def broadcast_(self, t, root: int = 0) -> None:
        rc = self.lib.rx_comm_broadcast(ctypes.c_void_p(t.data_ptr()), t.numel(), root, ctypes.c_void_p(self.ctx),
                                        _hip.stream_ptr(t.device))
        _hip.check(rc, "rx_comm_broadcast")

    def close(self):
        if self.ctx:
            self.lib.rx_comm_destroy(ctypes.c_void_p(self.ctx))
            self.ctx = None


def reset_cache():
    for c in _cache.values():
        c.close()
    _cache.clear()


class XgmiComm:
    """One-shot all-reduce over xGMI peer memory (``csrc/comm/xgmi_allreduce.hip``).

    Every rank of a single-node group maps every other rank's uncached exchange region
    (IPC handles exchanged over ``torch.distributed``); an all-reduce is then one flag exchange
    plus N-1 direct reads, which for the small gradient buckets of the reference's models
    (NYC: 194 KB) beats a ring of 2(N-1) hops. The fused NYC step loop reduces inside its
    optimizer kernel (``rx_mlp_train_steps_xg``); :meth:`allreduce_` serves other callers.

    ``create`` runs a self-test (sum of rank ids, both slots) and returns None on EVERY rank
    unless every rank passed it, so callers fall back to RCCL by construction when the peer
    mapping is unavailable (e.g. ranks on different hosts or GPUs hidden per process).
    """

    def __init__(self, world: int, rank: int, device: int, nfloats: int, timeout_s: float = 30.0,
                 host_seq: bool = False):
        L = _hip.lib()
        L.rx_xg_create.restype = ctypes.c_void_p
        L.rx_xg_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double]
        L.rx_xg_take_seq.restype = ctypes.c_uint
        self.lib, self.world, self.rank, self.nfloats = L, world, rank, nfloats
        self.host_seq = host_seq
        self.ctx = L.rx_xg_create(world, rank, device, nfloats, timeout_s)
        if not self.ctx:
            raise RuntimeError("rx_xg_create failed (uncached exchange region / IPC handle)")
        L.rx_xg_set_host_seq(ctypes.c_void_p(self.ctx), int(host_seq))
        self.max_floats = int(L.rx_xg_max_floats(ctypes.c_void_p(self.ctx)))
        self.fn_ptr = ctypes.cast(L.rx_xg_allreduce, ctypes.c_void_p)

    def handle(self) -> bytes:
        buf = ctypes.create_string_buffer(64)
        self.lib.rx_xg_handle(ctypes.c_void_p(self.ctx), buf)
        return buf.raw

    def open(self, handles) -> int:
        blob = b"".join(handles)
        return int(self.lib.rx_xg_open(ctypes.c_void_p(self.ctx), blob))

    def error(self) -> int:
        return int(self.lib.rx_xg_error(ctypes.c_void_p(self.ctx)))

    def _inject_error(self) -> None:
        """Test hook: mark this rank as having missed a peer (as a timed-out wait does)."""
        self.lib.rx_xg_set_error(ctypes.c_void_p(self.ctx), 1)

    def allreduce_(self, t, scale: float = 1.0) -> None:
        """In-place sum (times ``scale``) of a contiguous fp32 CUDA tensor (numel <= max_floats)
        on the current stream. A device-sequenced communicator (the default) launches the same
        kernel with the same arguments every call, so the call may be captured into a HIP graph
        and replayed."""
        if t.numel() > self.max_floats:
            raise ValueError(f"xGMI one-shot all-reduce of {t.numel()} floats > {self.max_floats}")
        rc = self.lib.rx_xg_allreduce_scaled(ctypes.c_void_p(t.data_ptr()), t.numel(), ctypes.c_float(scale),
                                             ctypes.c_void_p(self.ctx), _hip.stream_ptr(t.device))
        _hip.check(rc, "rx_xg_allreduce")

    def allreduce2_(self, t, scale: float = 1.0) -> bool:
        """Two-shot in-place sum (times ``scale``): all-pairs reduce-scatter + all-gather, 2S/N
        bytes per xGMI link instead of the one-shot kernel's S (device-sequenced, capturable).
        Needs a 16-B aligned tensor of a multiple of 4 floats; returns False (nothing launched)
        otherwise, so the caller can take :meth:`allreduce_`."""
        if t.numel() > self.max_floats:
            raise ValueError(f"xGMI two-shot all-reduce of {t.numel()} floats > {self.max_floats}")
        rc = self.lib.rx_xg_allreduce2_scaled(ctypes.c_void_p(t.data_ptr()), t.numel(), ctypes.c_float(scale),
                                              ctypes.c_void_p(self.ctx), _hip.stream_ptr(t.device))
        if rc == -4:
            return False
        _hip.check(rc, "rx_xg_allreduce2")
        return True

    def allgather_(self, src, dst) -> None:
        """``dst`` (``world * src`` bytes, contiguous, same dtype family of 4-byte words or
        int64) receives every rank's ``src`` in rank order: one device-sequenced launch
        (capturable). ``src`` must have the same size on every rank."""
        if src.element_size() * src.numel() % 4 or dst.numel() * dst.element_size() != \
                self.world * src.numel() * src.element_size():
            raise ValueError("allgather_: dst must hold world x src, in 4-byte words")
        words = src.numel() * src.element_size() // 4
        if words > self.max_floats:
            raise ValueError(f"xGMI all-gather of {words} words > {self.max_floats}")
        rc = self.lib.rx_xg_allgather(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()), words,
                                      ctypes.c_void_p(self.ctx), _hip.stream_ptr(src.device))
        _hip.check(rc, "rx_xg_allgather")

    def alltoallv_(self, src, dst, from_off, lens, dst_off) -> None:
        """Variable-split all-to-all in 4-byte words (device-sequenced: capturable). This rank
        publishes all of ``src``; it receives ``lens[p]`` words from rank ``p``, read at word
        ``from_off[p]`` of that rank's ``src`` and written at word ``dst_off[p]`` of ``dst``.
        Every rank must call it at the same point of its stream (like any collective)."""
        if src.element_size() * src.numel() % 4 or not (src.is_contiguous() and dst.is_contiguous()):
            raise ValueError("alltoallv_: contiguous tensors of whole 4-byte words")
        words = src.numel() * src.element_size() // 4
        if words > self.max_floats:
            raise ValueError(f"xGMI all-to-all of {words} words > {self.max_floats}")
        dwords = dst.numel() * dst.element_size() // 4
        if len(lens) != self.world or any(o + n > dwords for o, n in zip(dst_off, lens)):
            raise ValueError("alltoallv_: receive ranges outside dst")
        if not getattr(XgmiComm, "_a2a_checked", False):
            assert self.lib.rx_xg_a2a_size() == ctypes.sizeof(_XgA2A), "XgA2A layout mismatch"
            XgmiComm._a2a_checked = True
        a = _a2a_args(self.world, words, from_off, lens, dst_off)
        rc = self.lib.rx_xg_alltoallv(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()),
                                      ctypes.byref(a), ctypes.c_void_p(self.ctx), _hip.stream_ptr(src.device))
        _hip.check(rc, "rx_xg_alltoallv")

    def vote(self, out) -> None:
        """Epoch-end agreement (host-sequenced communicators): ``out`` (a device float64
        element) becomes the sum of every rank's error word, > 0 when any rank -- or this
        meeting -- timed out. Read it together with the epoch's metrics (one D2H copy)."""
        rc = self.lib.rx_xg_vote(ctypes.c_void_p(self.ctx), ctypes.c_void_p(out.data_ptr()),
                                 _hip.stream_ptr(out.device))
        _hip.check(rc, "rx_xg_vote")

    def check(self):
        """Raise ``CollectiveError`` (and retire this communicator in this process) when any
        exchange on it timed out. A set error word makes every later launch skip its exchange,
        so the callers read it at their sync points (epoch end) instead of letting replicas
        drift apart silently."""
        self._raise_for(self.error())

    def _raise_for(self, err: int):
        if err < 0:
            raise RuntimeError("xGMI communicator: reading its error word failed (device error)")
        if err:
            from raydp_amd.exceptions import CollectiveError
            forget_xgmi(self)
            raise CollectiveError("xGMI all-reduce: a peer did not arrive within the timeout")

    def check_async(self):
        """Non-blocking form of :meth:`check` for step loops: queue a stream-ordered copy of the
        error word into pinned host memory and examine the copy queued by the previous call
        (complete by then: its event is queried, never waited on). No device sync; legal
        inside a graph capture (the examination is skipped while capturing)."""
        import torch
        if not self.ctx:
            return
        if getattr(self, "_err_host", None) is None:
            self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            self._err_event = None
        capturing = torch.cuda.is_current_stream_capturing()
        ev = self._err_event
        if ev is not None and not capturing and ev.query():
            self._err_event = None
            self._raise_for(int(self._err_host[0]))
        if self._err_event is None and not capturing:
            rc = self.lib.rx_xg_error_async(ctypes.c_void_p(self.ctx), ctypes.c_void_p(self._err_host.data_ptr()),
                                            _hip.stream_ptr(torch.device("cuda", torch.cuda.current_device())))
            if rc != 0:
                raise RuntimeError(f"xGMI communicator: error-word copy failed ({rc})")
            self._err_event = torch.cuda.Event()
            self._err_event.record()

    def close(self):
        if self.ctx:
            self.lib.rx_xg_destroy(ctypes.c_void_p(self.ctx))
            self.ctx = None

    @classmethod
    def create(cls, nfloats: int, group=None, timeout_s: float = 30.0,
               host_seq: bool = False, tag: str = "") -> Optional["XgmiComm"]:
        """Collective: every rank of ``group`` calls it at the same point. ``tag`` keeps users
        that launch on different streams apart (a communicator's launches must be serialised:
        its sequence number lives on the device), e.g. the DDP buckets on the comm stream."""
        import socket

        import torch
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()):
            return None
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        if world < 2 or world > 16:
            return None
        # the two sequencing modes share the flag words, so they never share a communicator
        key = ("xg", id(group) if group is not None else "world", int(nfloats), bool(host_seq), tag)
        # Agree first, with one collective, whatever the local state: a rank that retired xGMI
        # (a peer timed out on it) or lost its cached communicator must not leave its peers in a
        # different collective than itself. Any disabled rank -> None everywhere; any miss -> every
        # rank rebuilds.
        disabled, cached = _XGMI_DISABLED, _cache.get(key)
        state = _agree_flags([int(disabled), int(cached is None)], group)
        if state[0] or state[1]:
            if cached is not None:
                _cache.pop(key, None)
                torch.cuda.synchronize()
                cached.close()
            if state[0]:
                return None
        else:
            return cached
        comm, err = None, None
        try:
            comm = cls(world, rank, torch.cuda.current_device(), nfloats, timeout_s, host_seq)
            h = comm.handle()
        except Exception as e:  # noqa: BLE001
            err, h = repr(e), b""
        info = [None] * world
        dist.all_gather_object(info, (socket.gethostname(), h, err, _device_identity()), group=group)
        ok = all(i[2] is None for i in info) and len({i[0] for i in info}) == 1
        if ok:
            ok = comm.open([i[1] for i in info]) == 0
        ok = _agree(ok, group)
        if ok:
            ok = _agree(comm._self_test(), group)
        if not ok:
            if comm is not None:
                torch.cuda.synchronize()
                comm.close()
            return None
        # ranks on the same device as this one (rehearsals put several on one GPU): kernels that
        # wait on their peers inside a launch size their grids so every rank's fits at once
        comm.share = max(1, sum(1 for i in info if i[3] == info[rank][3]))
        _cache[key] = comm
        return comm

    share = 1

    def _self_test(self) -> bool:
        import torch
        try:
            n = min(self.nfloats, 4096)
            for it in range(2):  # both slot parities
                t = torch.full((n,), float(self.rank + 1 + it), device="cuda", dtype=torch.float32)
                self.allreduce_(t)
                want = sum(r + 1 + it for r in range(self.world))
                torch.cuda.synchronize()
                if self.error() or not bool((t == want).all()):
                    return False
            return True
        except Exception:  # noqa: BLE001
            return False


_XGMI_DISABLED = False


def _device_identity() -> str:
    """A name of this process' current GPU that is the same in every process that uses it."""
    import torch
    dev = torch.cuda.current_device()
    p = torch.cuda.get_device_properties(dev)
    for attr in ("uuid", "pci_bus_id"):
        v = getattr(p, attr, None)
        if v is not None and str(v):
            return f"{attr}:{v}"
    return f"ordinal:{dev}:{os.environ.get('HIP_VISIBLE_DEVICES', os.environ.get('CUDA_VISIBLE_DEVICES', ''))}"


class _XgA2A(ctypes.Structure):
    """csrc/comm/xgmi_allreduce.hip XgA2A (RX_XG_MAXR = 16 ranks)."""
    _fields_ = [("src_words", ctypes.c_int), ("from_off", ctypes.c_int * 16), ("len", ctypes.c_int * 16),
                ("dst_off", ctypes.c_int * 16)]


def _a2a_args(world, words, from_off, lens, dst_off) -> _XgA2A:
    a = _XgA2A()
    a.src_words = int(words)
    for p in range(world):
        a.from_off[p], a.len[p], a.dst_off[p] = int(from_off[p]), int(lens[p]), int(dst_off[p])
    return a


def forget_xgmi(comm, disable: bool = True) -> None:
    """Retire a communicator whose peers missed a deadline. ``disable``: no xGMI communicator
    is created in this process any more (the retried fit runs over RCCL)."""
    global _XGMI_DISABLED
    for k, v in list(_cache.items()):
        if v is comm:
            _cache.pop(k, None)
    if disable:
        _XGMI_DISABLED = True


def _agree_flags(flags, group=None):
    """Element-wise max of small integer flags over the group (one collective)."""
    import torch
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor(list(flags), dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return [int(x) for x in t.tolist()]


def _agree(ok: bool, group=None) -> bool:
    """True on every rank iff ``ok`` on every rank."""
    import torch
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([0 if ok else 1], dtype=torch.int32, device=dev)
    dist.all_reduce(t, group=group)
    return int(t.item()) == 0


XG_BUCKET_MAX_BYTES = 16 << 20  # largest bucket the xGMI kernels are sized for


def oneshot_max_bytes() -> int:
    """Buckets up to this many bytes take an xGMI kernel (``spark.ray.mi355x.allreduce.
    oneshot_max_mb``, capped at the communicator's ``XG_BUCKET_MAX_BYTES``); larger ones RCCL."""
    from raydp_amd.utils.config import get as conf_get
    return int(min(float(conf_get("spark.ray.mi355x.allreduce.oneshot_max_mb")) * (1 << 20), XG_BUCKET_MAX_BYTES))


def twoshot_min_bytes() -> int:
    """Buckets from this size on take the two-shot kernel when world > 2
    (``spark.ray.mi355x.allreduce.twoshot_min_mb``). One-shot: every rank pulls the whole bucket
    from each peer, S bytes per xGMI link, one flag round. Two-shot: 2S/N per link, two flag
    rounds. At N = 8 the two-shot kernel moves 4x fewer bytes per link, which outweighs its
    second round from about a MiB on."""
    from raydp_amd.utils.config import get as conf_get
    return int(float(conf_get("spark.ray.mi355x.allreduce.twoshot_min_mb")) * (1 << 20))


class _Done:
    """Completed-work handle for a collective that is already ordered on the compute stream."""

    def wait(self):
        return True

    def is_completed(self):
        return True


class _Joined:
    """Handle of a bucket reduced on the comm stream: ``wait()`` makes the current stream wait
    for it (an event join, capturable: the comm stream forks from and joins the captured one)."""

    def __init__(self, stream):
        self.stream = stream

    def wait(self):
        import torch
        torch.cuda.current_stream().wait_stream(self.stream)
        return True

    def is_completed(self):
        return self.stream.query()


def _device_key():
    """(host, PCI location or uuid) of the current GPU: equal on two ranks iff they share it."""
    import socket
    import torch
    p = torch.cuda.get_device_properties(torch.cuda.current_device())
    loc = tuple(getattr(p, a, None) for a in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
    if all(v is None for v in loc):
        loc = (str(getattr(p, "uuid", "")), os.environ.get("HIP_VISIBLE_DEVICES", ""), torch.cuda.current_device())
    return (socket.gethostname(),) + tuple(loc)


def comm_stream_wanted(group=None) -> bool:
    """``spark.ray.mi355x.ddp.comm_stream``: on / off, or auto = on only when no two ranks of
    ``group`` share a GPU (collective: every rank calls it at the same point)."""
    import torch.distributed as dist
    from raydp_amd.utils.config import get as conf_get
    v = str(conf_get("spark.ray.mi355x.ddp.comm_stream")).lower()
    if v in ("on", "true", "1"):
        return True
    if v in ("off", "false", "0"):
        return False
    if not dist.is_initialized():
        return True
    keys = [None] * dist.get_world_size(group)
    dist.all_gather_object(keys, _device_key(), group=group)
    return len(set(keys)) == len(keys)


class BucketAllreduce:
    """All-reduce of gradient buckets for the DDP and Horovod wrappers.

    fp32 buckets up to :func:`oneshot_max_bytes` go through the xGMI kernels -- one-shot for small
    buckets (and always at world 2), two-shot (all-pairs reduce-scatter + all-gather) from
    :func:`twoshot_min_bytes` on -- with the 1/world average folded into the sum pass; larger
    buckets, other dtypes and non-xGMI groups use ``torch.distributed.all_reduce``.

    The xGMI launches go on a dedicated comm stream: a bucket that is ready forks the comm stream
    off the compute stream (event), its reduction runs while backward continues, and ``wait()``
    joins the comm stream back. Fork and join are events, so a captured HIP graph keeps the
    concurrency. The communicator is this object's own (``tag``), because its launches are
    ordered on the comm stream while other xGMI users (sharded embeddings) launch on the compute
    stream. Construct it on every rank at the same point (it runs the collective xGMI set-up)."""

    def __init__(self, group=None, overlap: Optional[bool] = None):
        import torch
        import torch.distributed as dist
        from raydp_amd.utils.config import get as conf_get
        self.group = group
        self.xg = None
        self.stream = None
        self.limit = oneshot_max_bytes()
        self.twoshot_min = twoshot_min_bytes()
        try:
            # gloo groups qualify too when the tensors are on the GPU (a rehearsal with several
            # ranks per device): the peer regions are bootstrapped over whatever group is given
            if (dist.is_initialized() and dist.get_backend(group) in ("nccl", "gloo") and torch.cuda.is_available()
                    and torch.cuda.is_initialized() and conf_get("spark.ray.mi355x.allreduce") != "rccl"
                    and self.limit > 0):
                self.xg = XgmiComm.create(XG_BUCKET_MAX_BYTES // 4, group=group,
                                          timeout_s=conf_get("spark.ray.mi355x.allreduce.timeout_s"),
                                          tag="buckets")
        except Exception:  # noqa: BLE001
            self.xg = None
        if overlap is None and self.xg is not None:
            overlap = comm_stream_wanted(group)
        if self.xg is not None and overlap:
            self.stream = torch.cuda.Stream()
        self.launched = {"oneshot": 0, "twoshot": 0, "torch": 0}

    @property
    def overlaps(self) -> bool:
        """True when a bucket reduction launched during backward runs BESIDE the rest of
        backward: the xGMI kernels on the comm stream, or torch.distributed's asynchronous
        collectives (RCCL's own stream / gloo's worker thread) when no xGMI communicator is up.
        False when the xGMI kernels are stream-ordered behind backward (ranks sharing a GPU)."""
        if self.xg is not None:
            return self.stream is not None
        return True

    @property
    def kind(self) -> str:
        """What the buckets ride on: the xGMI kernels for buckets up to the limit (when the peer
        mapping is up) and torch.distributed (RCCL / gloo) for the rest."""
        import torch.distributed as dist
        base = f"torch.distributed:{dist.get_backend(self.group)}" if dist.is_initialized() else "none"
        if self.xg is None:
            return base
        two = f",twoshot>={self.twoshot_min / (1 << 20):g}MiB" if self.xg.world > 2 else ""
        return f"xgmi_oneshot(<={self.limit / (1 << 20):g}MiB{two}{',comm_stream' if self.stream else ''})+{base}"

    def routes_to_xgmi(self, flat) -> bool:
        import torch
        return (self.xg is not None and flat.is_cuda and flat.dtype == torch.float32 and flat.is_contiguous()
                and flat.numel() * 4 <= self.limit and flat.numel() <= self.xg.max_floats)

    def _xg_launch(self, flat, scale):
        if self.xg.world > 2 and flat.numel() * 4 >= self.twoshot_min and self.xg.allreduce2_(flat, scale):
            self.launched["twoshot"] += 1
            return
        self.xg.allreduce_(flat, scale)
        self.launched["oneshot"] += 1

    def __call__(self, flat, scale: float = 1.0, overlap: bool = True):
        """Sum ``flat`` over ranks in place, times ``scale``. Returns a handle whose ``wait()``
        orders the result before later work on the current stream. ``overlap=False`` keeps the
        reduction on the current stream (the caller needs it at once)."""
        import torch
        import torch.distributed as dist
        if self.routes_to_xgmi(flat):
            if self.stream is not None and overlap:
                self.stream.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(self.stream):
                    self._xg_launch(flat, scale)
                return _Joined(self.stream)
            if self.stream is not None:
                # every launch of this communicator stays on one stream, in program order
                self.stream.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(self.stream):
                    self._xg_launch(flat, scale)
                torch.cuda.current_stream().wait_stream(self.stream)
                return _Done()
            self._xg_launch(flat, scale)
            return _Done()
        self.launched["torch"] += 1
        work = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        if scale == 1.0:
            return work
        return _Scaled(work, flat, scale)

    def check(self):
        """Raise ``CollectiveError`` when an xGMI exchange of these buckets timed out (host sync:
        call it where the caller syncs anyway, e.g. with the epoch's metrics)."""
        if self.xg is not None:
            try:
                self.xg.check()
            finally:
                if self.xg.ctx is None or _XGMI_DISABLED:
                    self.xg = None

    def check_async(self):
        """:meth:`check` without a device sync (``XgmiComm.check_async``): for step loops."""
        if self.xg is not None:
            try:
                self.xg.check_async()
            finally:
                if self.xg.ctx is None or _XGMI_DISABLED:
                    self.xg = None


class _Scaled:
    def __init__(self, work, flat, scale):
        self.work, self.flat, self.scale = work, flat, scale

    def wait(self):
        self.work.wait()
        self.flat.mul_(self.scale)
        return True

    def is_completed(self):
        return self.work.is_completed()
