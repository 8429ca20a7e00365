"""Native RCCL communicator for the fused trainer's C++ step loop (``csrc/comm/rccl_comm.cc``).

``NativeComm.from_process_group()`` builds one communicator per process group: rank 0 draws
an RCCL unique id, the id is broadcast over the existing ``torch.distributed`` group, and every
rank joins. ``fn_ptr`` / ``ctx`` are handed to ``rx_mlp_train_steps`` so each step's gradient
all-reduce is enqueued on the compute stream from C++ (kernel -> all-reduce -> Adam, no Python
between steps).
"""
import ctypes
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
